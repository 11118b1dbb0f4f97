# Round-end evidence: the GPU suite, smoke(), and the driver's bench command (20 steps, 5 warm-up,
# CPU baseline included) with its wall time.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
t0=$(date +%s.%N) && \
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $OUT/bench.log 2>&1
rc=$?
t1=$(date +%s.%N)
echo "bench wall s: $(python -c "print($t1 - ${t0:-$t1})")" >> $OUT/bench.log
tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log; grep '^{' $OUT/bench.log | cut -c1-300; tail -1 $OUT/bench.log
exit $rc
