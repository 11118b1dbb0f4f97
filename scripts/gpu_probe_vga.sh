# VGA tile-kernel work/phase breakdown at 1000^2 on a middle block of sources (+ kernel variants)
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/probe_vga
mkdir -p $OUT
DMX_VERBOSE=1 timeout -k 10 300 python -u scripts/probe_big.py 1000 ${NSRC:-16384} "" ${PROBE_CONFIGS:-DMX_VGA_CHUNK=1} > $OUT/probe.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/probe.log | tail -20
exit $rc
