# One GPU-box call: smoke, GPU parity tests, default bench, rocprofv3 kernel-trace stats of the bench.
# Every GPU step has its own time limit; steps are chained with && so a failure ends the call.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${TAG:-r1}
mkdir -p $OUT/prof_$TAG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG/kt -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/prof_$TAG/kt.log 2>&1
rc=$?
echo "exit $rc"
tail -2 $OUT/smoke.log $OUT/pytest_gpu.log $OUT/bench.log 2>/dev/null
exit $rc
