#!/bin/bash
# A/B: the main build against EXTRA_LIB (1000^2 VGA time and digest), then the VGA parity tests on EXTRA_LIB.
set -o pipefail
O=gpurun_out/${TAG:-ab_default}
mkdir -p $O
timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err && \
DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err && \
DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_nocaps.py tests/test_gpu_scale.py tests/test_merge_links.py -m gpu \
  -k "(vga or tile or stepdepth or merge) and not 2000" > $O/tests.log 2>&1
rc=$?
cut -c1-200 $O/ab.log; tail -2 $O/tests.log
exit $rc
