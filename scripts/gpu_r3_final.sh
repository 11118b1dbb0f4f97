#!/bin/bash
# Round-3 bench evidence on the current build (profiles/r3_pmc.json committed from scripts/gpu_r3_pmc.sh):
# smoke(), the driver's bench command (20 steps, 5 warm-up, CPU leg) timed, then configs[4] (--config 5).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3final}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
t0=$(date +%s.%N) && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $O/bench.log 2> $O/bench_progress.txt && \
t1=$(date +%s.%N) && echo "bench wall s: $(python -c "print($t1 - $t0)")" >> $O/bench_progress.txt && \
timeout -k 10 500 python -u bench.py --gpus 1 --config 5 --steps 2 --warmup 1 > $O/bench5.log 2> $O/bench5_progress.txt
rc=$?
tail -2 $O/smoke.log; grep '^{' $O/bench.log | cut -c1-300; tail -1 $O/bench_progress.txt; grep '^{' $O/bench5.log | cut -c1-300
exit $rc
