set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/probe_big.py 256 65025 tile DMX_VGA_CHUNK=1 > $OUT/probe256.log 2>&1 && \
timeout -k 10 900 python scripts/probe_big.py 1000 16384 tile DMX_VGA_CHUNK=1 > $OUT/probe1000.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
cat $OUT/probe256.log $OUT/probe1000.log 2>/dev/null | grep -v amdgpu.ids
exit $rc
