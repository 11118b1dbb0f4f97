# Round 4: the tests this round touched first (fast feedback), then the whole GPU suite and smoke.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4suite}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_semifill.py tests/test_merge_links.py tests/test_graphfile.py \
  tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v -m gpu -k "${FIRST_K:-semi or mixed or link or merge or contextfilled or balance or targeted}" \
  --timeout 200 --timeout-method thread > $OUT/pytest_first.log 2>&1 && \
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYARGS} > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -5 $OUT/pytest_first.log; tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
exit $rc
