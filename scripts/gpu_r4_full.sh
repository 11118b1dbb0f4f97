# Round 4: the whole GPU suite with per-test durations, then smoke (what the driver runs at round end).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --durations=40 --timeout 400 --timeout-method thread ${PYARGS} \
  > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -45 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
exit $rc
