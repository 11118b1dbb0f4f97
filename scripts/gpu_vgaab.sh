# VGA tile-kernel check: its GPU parity tests, then a 2-step 1000^2 bench.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-vgaab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_graphfile.py tests/test_progress_cancel.py -x -q -m gpu -k "${KSEL:-vga or visual or graph or progress or cancel}" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2> $OUT/bench.err
rc=$?
tail -2 $OUT/pytest.log; grep '^{' $OUT/bench.log | cut -c1-200
exit $rc
