#!/bin/bash
# Last build of round 3: configs[2] PMC passes into profiles/r3_pmc.json, the VGA/step-depth parity tests,
# smoke, and the bench (STEPS/WARMUP, CPU leg).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
T=${TAG:-r3last}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
W2="synthetic-1000/50-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n"
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_nocaps.py tests/test_gpu_scale.py tests/test_merge_links.py -m gpu -k "(vga or tile or stepdepth or merge) and not 2000" \
  > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
TAG=$T/pmc2 bash scripts/gpu_pmc.sh > $OUT/pmc2.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/$T/pmc2 "$W2" profiles/r3_pmc.json > $OUT/pmc2_summary.log 2>&1 && \
cp profiles/r3_pmc.json $OUT/ && \
t0=$(date +%s.%N) && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARMUP:-2} > $OUT/bench.log 2> $OUT/bench_progress.txt && \
t1=$(date +%s.%N) && echo "bench wall s: $(python -c "print($t1 - $t0)")" >> $OUT/bench_progress.txt
rc=$?
tail -2 $OUT/tests.log; tail -1 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-250; tail -1 $OUT/bench_progress.txt
exit $rc
