# Round-2 baseline on a fresh box: smoke, full GPU parity suite, a short 1000^2 bench with phase stats.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r2base
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
echo "exit $rc"
tail -3 $OUT/smoke.log; tail -18 $OUT/pytest_gpu.log; grep -v amdgpu.ids $OUT/bench.log | tail -12 | cut -c1-600
exit $rc
