#!/bin/bash
# Phase-C partial-tile masks: 1000^2 VGA global (prep wall + kernel time, output digest) with the masks
# off and on, same build; then the VGA parity tests on the new build.
set -o pipefail
O=gpurun_out/${TAG:-pmask}
mkdir -p $O
export DMX_LIB=${LIB:-depthmapx_amd/_lib_ab/pm/libdmx.so}
DMX_VGA_PMASK=0 timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 2 >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 2 >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_nocaps.py tests/test_gpu_scale.py \
  -k "(vga or tile or stepdepth) and not 2000" > $O/tests.log 2>&1
rc=$?
cat $O/ab.log | cut -c1-600; tail -3 $O/tests.log
exit $rc
