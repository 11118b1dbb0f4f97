# VGA tile kernel change: the VGA-side parity suites, then time + FETCH/WRITE at 1000^2 (gpu_vga_write.sh).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-vgaverify}
mkdir -p $OUT
timeout -k 10 ${TEST_TIMEOUT:-800} python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_merge_links.py tests/test_semifill.py tests/test_graphfile.py tests/test_gpu_nocaps.py tests/test_gpu_scale.py \
  -k "${K:-(vga or merge or contextfilled or special or asym or topdown or symmetry or visual or link or graph or long_grid or semi) and not 2000 and not makegraph}" \
  > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -2 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
TAG=${TAG:-vgaverify} bash $R/scripts/gpu_vga_write.sh
