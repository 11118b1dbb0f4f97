# Benchmark-size parity, the 1000^2 bench (no CPU leg) and the configs[4] bench.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-scale}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest_scale.log 2>&1 && \
DMX_VERBOSE=${VERBOSE:-0} timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --config 5 --steps 1 --warmup 1 > $OUT/bench_c5.log 2>&1
rc=$?
tail -12 $OUT/pytest_scale.log; grep '^{' $OUT/bench.log | cut -c1-400; grep '^{' $OUT/bench_c5.log | cut -c1-400
exit $rc
