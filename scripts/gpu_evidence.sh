#!/bin/bash
# Round evidence (ROUND, default 6): PART=2 -- configs[2] PMC passes -> profiles/r${RD}_pmc.json, smoke(), the bench (STEPS/WARMUP,
# CPU leg) under a kernel-trace + stats profile; PART=5 -- the configs[4] (bench --config 5) PMC passes and its
# bench line.  The PMC summary is written here on the box and merged back through gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
RD=${ROUND:-6}
T=${TAG:-r${RD}evidence}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
W2="synthetic-1000/50-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n"
W5="synthetic-1999/5000-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + STEPDEPTH -sdt metric -sdp 1000,1000 (cell 2001000)"
if [ "${PART:-2}" = 2 ]; then
  TAG=$T/pmc2 bash scripts/gpu_pmc.sh > $OUT/pmc2.log 2>&1
  rc=$?
  python3 scripts/pmc_summary.py gpurun_out/$T/pmc2 "$W2" $OUT/r${RD}_pmc.json > $OUT/pmc2_summary.log 2>&1
  cp $OUT/r${RD}_pmc.json profiles/r${RD}_pmc.json   # the bench below reads it
  [ $rc = 0 ] && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
  t0=$(date +%s.%N) && \
  timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-10} --warmup ${WARMUP:-2} > $OUT/bench.log 2> $OUT/bench_progress.txt && \
  t1=$(date +%s.%N) && echo "bench wall s: $(python -c "print($t1 - $t0)")" >> $OUT/bench_progress.txt
  rc=$?
  tail -5 $OUT/pmc2.log; tail -2 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-300; tail -1 $OUT/bench_progress.txt
else
  cp profiles/r${RD}_pmc.json $OUT/r${RD}_pmc.json 2>/dev/null
  TAG=$T/pmc5 BENCH_ARGS="--config 5" bash scripts/gpu_pmc.sh > $OUT/pmc5.log 2>&1
  rc=$?
  python3 scripts/pmc_summary.py gpurun_out/$T/pmc5 "$W5" $OUT/r${RD}_pmc.json > $OUT/pmc5_summary.log 2>&1
  cp $OUT/r${RD}_pmc.json profiles/r${RD}_pmc.json
  [ $rc = 0 ] && timeout -k 10 400 python -u bench.py --gpus 1 --config 5 --steps 2 --warmup 1 > $OUT/bench5.log 2> $OUT/bench5_progress.txt && \
  timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
    tests/test_gpu_scale.py -k "2000_vga_sources" > $OUT/vga2000_wide_tests.log 2>&1
  rc=$?
  # the 1000^2 step with the symmetry scatter left to the VGA preparation (the round-3 arrangement)
  [ $rc = 0 ] && DMX_MK_NOSYM=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/bench_nosym.log 2> $OUT/bench_nosym_progress.txt
  rc=$?
  tail -5 $OUT/pmc5.log; grep '^{' $OUT/bench5.log | cut -c1-300; tail -2 $OUT/vga2000_wide_tests.log
  grep '^{' $OUT/bench_nosym.log | cut -c1-300
fi
kill $HB
exit $rc
