# VGA kernel iteration: probe (middle block of 1000^2) first, then the VGA parity tests
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/vga_iter
mkdir -p $OUT
DMX_VERBOSE=1 timeout -k 10 300 python -u scripts/probe_big.py 1000 ${NSRC:-16384} "" ${PROBE_CONFIGS:-DMX_VGA_CHUNK=1} > $OUT/probe.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "vga_global or vga_kernels or vga_blocks or visual_stepdepth or smoke or tile" > $OUT/tests.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/probe.log | grep config | cut -c1-2500
tail -3 $OUT/tests.log
exit $rc
