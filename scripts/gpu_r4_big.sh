# Round 4: the tests this round touched, then the 2000^2 VGA-global probe (tile BFS, frontier in HBM).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4big}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_semifill.py tests/test_merge_links.py tests/test_graphfile.py \
  tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v -m gpu --durations=20 \
  -k "${FIRST_K:-semi or mixed or link or merge or contextfilled or balance or targeted}" \
  --timeout 400 --timeout-method thread > $OUT/pytest_first.log 2>&1 && \
timeout -k 10 500 python -u scripts/probe_vga2000.py --nsrc ${NSRC:-4096} --blocks ${BLOCKS:-2} --check-do ${CHECK_DO:-16} \
  > $OUT/probe2000.jsonl 2> $OUT/probe2000_progress.txt
rc=$?
tail -4 $OUT/pytest_first.log; tail -5 $OUT/probe2000_progress.txt; tail -1 $OUT/probe2000.jsonl | cut -c1-600
exit $rc
