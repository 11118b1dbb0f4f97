# configs[4] (2000^2 / 5000 occluders, makeGraph + metric step depth): PMC passes of one step, then the
# bench with its CPU leg; the VISPREP fill timing probe (host vs GPU) at 1000^2 and 2000^2.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-c5}
mkdir -p $OUT
cd $R && timeout -k 10 200 python -u scripts/probe_fill.py > $OUT/fill.log 2>&1 && \
TAG=${TAG:-c5}/pmc BENCH_ARGS="--config 5" bash $R/scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 && \
cd $R && python3 scripts/pmc_summary.py gpurun_out/${TAG:-c5}/pmc "synthetic-1999/5000-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + STEPDEPTH -sdt metric -sdp 1000,1000 (cell 2001000)" profiles/r2_pmc_1000.json > $OUT/pmc_summary.log 2>&1 && \
cp profiles/r2_pmc_1000.json $OUT/ && \
timeout -k 10 500 python -u bench.py --config 5 --steps 2 --warmup 1 > $OUT/bench.log 2> $OUT/bench_progress.txt
rc=$?
cat $OUT/fill.log | grep '^{'; tail -6 $OUT/pmc.log; grep '^{' $OUT/bench.log | cut -c1-300
exit $rc
