# Round 4: the tile kernel's level-reset race (context-filled radius-3 cases), then the 2000^2 VGA probe
# with the tvis row summaries.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-r4fix}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/diag_semi3b.py > $OUT/diagb.log 2>&1 || { tail -20 $OUT/diagb.log; exit 1; }
grep -v "^   " $OUT/diagb.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_graphfile.py \
  tests/test_semifill.py tests/test_merge_links.py tests/test_gpu_nocaps.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u scripts/probe_vga2000.py --nsrc 1024 --blocks 1 --check-do 16 > $OUT/probe2000.jsonl 2> $OUT/probe2000_progress.txt
rc=$?
grep -v amdgpu.ids $OUT/probe2000_progress.txt | cut -c1-700
exit $rc
