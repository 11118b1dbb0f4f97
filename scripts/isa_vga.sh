# VGA tile kernel ISA: vga_tile_kernel<NT, SPECIAL, RBM, FG> alone, compiled to assembly (spills, loops).
# usage: scripts/isa_vga.sh [NT] [extra hipcc flags]  -> /tmp/vt_isa.s + resource usage
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NT=${1:-1024}; shift || true
cat > /tmp/vt_only.hip <<HIP
#include "$R/depthmapx_amd/csrc/kernels/vga.hip"
#include "$R/depthmapx_amd/csrc/kernels/vga_do.hip"
#include "$R/depthmapx_amd/csrc/kernels/vga_tile.hip"
template __global__ void dmx::vga_tile_kernel<$NT, ${VARIANT:-true, true, false}>(const dmx::VgaTileParams*);
HIP
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math --cuda-device-only -S \
  -Wno-bitwise-instead-of-logical -Rpass-analysis=kernel-resource-usage "$@" /tmp/vt_only.hip -o /tmp/vt_isa.s 2>&1 | \
  grep -A9 "Function Name: _ZN3dmx15vga_tile" | grep -E "VGPRs|Spill|Scratch|Occupancy" | sed 's/.*remark: *//'
