# GPU parity tests, then the makeGraph phase profile at 256^2 and 1000^2.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 300 python scripts/probe_big.py 256 1024 > $OUT/mk256.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 600 python scripts/probe_big.py 1000 4096 > $OUT/mk1000.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
grep -h "phases\|attempt\|makegraph_kernel_s\|vga_kernel_s" $OUT/mk256.log $OUT/mk1000.log | cut -c1-400
exit $rc
