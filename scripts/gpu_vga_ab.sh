#!/bin/bash
# A/B of VGA kernel builds (depthmapx_amd/_lib_ab/<variant>/libdmx.so): 1000^2 VGA global kernel time
set -o pipefail
O=gpurun_out/${TAG:-vga_ab}
mkdir -p $O
for v in ${VARIANTS:-c4 c8 c16}; do
  DMX_LIB=depthmapx_amd/_lib_ab/$v/libdmx.so timeout -k 10 150 python -u scripts/probe_vga_time.py >> $O/ab.log 2>> $O/ab.err || exit 1
done
