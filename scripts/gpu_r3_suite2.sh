#!/bin/bash
# The whole GPU suite and smoke on the current build, then the 2000^2 VGA-global timing probe.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3suite2}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python -u scripts/probe_vga2000.py --nsrc ${NSRC:-512} --blocks 4 > $O/vga2000.jsonl 2> $O/vga2000.err
rc=$?
tail -3 $O/pytest_gpu.log; tail -2 $O/smoke.log; cut -c1-600 $O/vga2000.jsonl
exit $rc
