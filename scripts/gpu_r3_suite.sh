# Round 3: merge-link tests first (fast feedback), then the whole GPU suite and smoke.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r3suite}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_merge_links.py tests/test_graphfile.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_merge.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYARGS} > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -5 $OUT/pytest_merge.log; tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
exit $rc
