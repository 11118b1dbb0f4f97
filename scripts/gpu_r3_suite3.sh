#!/bin/bash
# Main build: phase-B run budget sweep (1000^2 VGA, DMX_VGA_BEXT), then the whole GPU suite and smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3suite3}
mkdir -p $O
for e in DMX_VGA_BEXT=4 DMX_VGA_BEXT=0 DMX_VGA_BEXT=2; do
  env $e timeout -k 10 200 python -u scripts/probe_vga_time.py --reps 1 >> $O/ab.log 2>> $O/ab.err || exit 1
done
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
cut -c1-250 $O/ab.log; tail -2 $O/pytest_gpu.log; tail -1 $O/smoke.log
exit $rc
