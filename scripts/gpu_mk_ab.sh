#!/bin/bash
# A/B of makeGraph kernel builds (depthmapx_amd/_lib_ab/<variant>/libdmx.so): whole-map kernel time
set -o pipefail
O=gpurun_out/${TAG:-mk_ab}
mkdir -p $O
for v in ${VARIANTS:-b0c0 b1c0 b0c1 b1c1}; do
  DMX_LIB=depthmapx_amd/_lib_ab/$v/libdmx.so timeout -k 10 120 python -u scripts/probe_mk_time.py --config ${CONFIG:-2} \
    >> $O/ab.log 2>> $O/ab.err || exit 1
done
