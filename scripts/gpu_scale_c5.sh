# Benchmark-size parity (tests/test_gpu_scale.py) and the configs[4] bench (2000^2/5000, metric step depth).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-scale}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest_scale.log 2>&1 && \
timeout -k 10 500 python -u bench.py --config 5 --steps 1 --warmup 1 > $OUT/bench_c5.log 2>&1
rc=$?
tail -12 $OUT/pytest_scale.log; grep '^{' $OUT/bench_c5.log | cut -c1-400
exit $rc
