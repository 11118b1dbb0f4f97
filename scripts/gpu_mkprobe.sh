# makeGraph phase profile and LDS-occupancy sensitivity (256^2 default vs bcap 512), then 1000^2.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
DMX_VERBOSE=1 timeout -k 10 300 python scripts/probe_big.py 256 1024 > $OUT/mk256.log 2>&1 && \
DMX_MK_BCAP=512 DMX_VERBOSE=1 timeout -k 10 300 python scripts/probe_big.py 256 1024 > $OUT/mk256_b512.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 600 python scripts/probe_big.py 1000 4096 > $OUT/mk1000.log 2>&1
rc=$?
grep -h "phases\|attempt\|makegraph_kernel_s\|vga_kernel_s" $OUT/mk256.log $OUT/mk256_b512.log $OUT/mk1000.log | cut -c1-600
exit $rc
