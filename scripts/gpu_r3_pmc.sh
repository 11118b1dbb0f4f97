#!/bin/bash
# Round-3 PMC evidence: the rocprofv3 passes of scripts/gpu_pmc.sh over one step of configs[2] (1000^2 VGA)
# and of configs[4] (2000^2/5000 metric step depth), summarised into profiles/r3_pmc.json (read by bench.py;
# copied back under gpurun_out/TAG/).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
T=${TAG:-r3pmc}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
W2="synthetic-1000/50-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n"
W5="synthetic-1999/5000-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + STEPDEPTH -sdt metric -sdp 1000,1000 (cell 2001000)"
rm -f profiles/r3_pmc.json
TAG=$T/pmc2 bash scripts/gpu_pmc.sh > $OUT/pmc2.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/$T/pmc2 "$W2" profiles/r3_pmc.json > $OUT/pmc2_summary.log 2>&1 && \
TAG=$T/pmc5 BENCH_ARGS="--config 5" bash scripts/gpu_pmc.sh > $OUT/pmc5.log 2>&1 && \
python3 scripts/pmc_summary.py gpurun_out/$T/pmc5 "$W5" profiles/r3_pmc.json > $OUT/pmc5_summary.log 2>&1
rc=$?
cp profiles/r3_pmc.json $OUT/ 2>/dev/null
tail -3 $OUT/pmc2.log $OUT/pmc5.log
exit $rc
