# Full GPU parity suite + a short 1000^2 bench (phase stats on stderr).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
DMX_VERBOSE=${VERBOSE:-1} timeout -k 10 400 python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; grep '^{' $OUT/bench.log | cut -c1-700
exit $rc
