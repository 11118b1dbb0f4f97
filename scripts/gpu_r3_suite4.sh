#!/bin/bash
# Final build: the whole GPU suite and smoke, then the A/B probe of EXTRA_LIB against it (1000^2 VGA).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3suite4}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log; tail -1 $O/smoke.log
if [ $rc -eq 0 ] && [ -n "$EXTRA_LIB" ]; then
  timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err && \
  DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err
  cut -c1-200 $O/ab.log
fi
exit $rc
