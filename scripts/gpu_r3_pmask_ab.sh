#!/bin/bash
# A/B of the phase-C partial-tile-mask builds (VARIANTS under depthmapx_amd/_lib_ab/): 1000^2 VGA global
# kernel time, prep wall time and output digest per build; then the VGA parity tests on TESTLIB.
set -o pipefail
O=gpurun_out/${TAG:-pmask_ab}
mkdir -p $O
for v in ${VARIANTS:-pm pmh}; do
  DMX_LIB=depthmapx_amd/_lib_ab/$v/libdmx.so timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err || exit 1
done
DMX_LIB=depthmapx_amd/_lib_ab/${TESTLIB:-pmh}/libdmx.so timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_nocaps.py tests/test_gpu_scale.py -k "(vga or tile or stepdepth) and not 2000" > $O/tests.log 2>&1
rc=$?
cut -c1-400 $O/ab.log; tail -3 $O/tests.log
exit $rc
