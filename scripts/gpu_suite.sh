# GPU suite + smoke on the current tree (no bench).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread ${PYARGS} > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
exit $rc
