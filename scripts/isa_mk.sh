# makeGraph ISA: the fixed first-pass kernel alone, compiled to assembly (spills, waitcnts, loop bodies).
# usage: scripts/isa_mk.sh [extra hipcc flags]  -> /tmp/mk_isa.s + resource usage
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
cat > /tmp/mk_only.hip <<HIP
#include "$R/depthmapx_amd/csrc/kernels/makegraph.hip"
template __global__ void dmx::makegraph_kernel<5, false, true, false, false, false>(const dmx::MakeGraphParams*);
HIP
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --cuda-device-only -S \
  -Wno-bitwise-instead-of-logical -Rpass-analysis=kernel-resource-usage "$@" /tmp/mk_only.hip -o /tmp/mk_isa.s 2>&1 | \
  grep -E "VGPRs|Spill|Scratch|Occupancy" | sed 's/.*remark: *//'
grep -cE "scratch_(load|store)|buffer_(load|store).*off, s\[0:3\]" /tmp/mk_isa.s || true
