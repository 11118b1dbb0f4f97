#!/bin/bash
# Final build: configs[2] PMC passes (merged into profiles/r3_pmc.json next to the configs[4] entry), the whole
# GPU suite, smoke, and the bench (STEPS/WARMUP, CPU leg).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
T=${TAG:-r3final2}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
W2="synthetic-1000/50-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n"
TAG=$T/pmc2 bash scripts/gpu_pmc.sh > $OUT/pmc2.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/$T/pmc2 "$W2" profiles/r3_pmc.json > $OUT/pmc2_summary.log 2>&1 && \
cp profiles/r3_pmc.json $OUT/ && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
t0=$(date +%s.%N) && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARMUP:-2} > $OUT/bench.log 2> $OUT/bench_progress.txt && \
t1=$(date +%s.%N) && echo "bench wall s: $(python -c "print($t1 - $t0)")" >> $OUT/bench_progress.txt && \
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -1 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-250; tail -1 $OUT/bench_progress.txt; tail -2 $OUT/pytest_gpu.log
# A/B probe of the next variant after the evidence (EXTRA_LIB under depthmapx_amd/_lib_ab/)
if [ $rc -eq 0 ] && [ -n "$EXTRA_LIB" ]; then
  timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $OUT/ab.log 2>> $OUT/ab.err && \
  DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $OUT/ab.log 2>> $OUT/ab.err
  cut -c1-200 $OUT/ab.log
fi
exit $rc
