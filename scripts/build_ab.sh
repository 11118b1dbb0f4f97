# A/B build of libdmx.so with extra compiler flags into depthmapx_amd/_lib_ab/<name>/ (selected at run time
# with DMX_LIB=...).  Usage: scripts/build_ab.sh <name> [-DFLAG=value ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p $R/depthmapx_amd/_lib_ab/$name
C=${CSRC:-$R/depthmapx_amd/csrc}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -w "$@" \
  -o $R/depthmapx_amd/_lib_ab/$name/libdmx.so $C/dmx_api.hip $C/host/pointmap.cpp $C/host/graphio.cpp $C/host/graphfile.cpp
echo "built $name $*"
