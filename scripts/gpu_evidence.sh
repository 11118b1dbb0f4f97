# Round evidence on one box: the rocprofv3 passes of scripts/gpu_pmc.sh over one 1000^2 step (same
# build as the bench), smoke(), then the driver's bench command (20 steps, 5 warm-up, CPU leg) timed.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-evidence}
mkdir -p $OUT
TAG=${TAG:-evidence}/pmc bash $R/scripts/gpu_pmc.sh > $OUT/pmc.log 2>&1 && \
cd $R && python3 scripts/pmc_summary.py gpurun_out/${TAG:-evidence}/pmc "synthetic-1000/50-occluders VISPREP -pg 1 -pp 0.5,0.5 -pm + VGA -vm visibility -vg -vr n" profiles/r2_pmc_1000.json > $OUT/pmc_summary.log 2>&1 && \
cp profiles/r2_pmc_1000.json $OUT/ && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
t0=$(date +%s.%N) && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $OUT/bench.log 2> $OUT/bench_progress.txt
rc=$?
t1=$(date +%s.%N)
echo "bench wall s: $(python -c "print($t1 - ${t0:-$t1})")" >> $OUT/bench_progress.txt
cat $OUT/pmc.log | tail -8; tail -2 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-400; tail -1 $OUT/bench_progress.txt
exit $rc
