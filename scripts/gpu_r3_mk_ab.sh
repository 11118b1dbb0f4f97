#!/bin/bash
# makeGraph A/B: the main build against EXTRA_LIB (1000^2 and configs[4] kernel time, pairs/runs), then the
# makeGraph parity tests on EXTRA_LIB (reference fixtures, seeded oracle blocks incl. 1000^2 and 2000^2).
set -o pipefail
O=gpurun_out/${TAG:-mk_ab}
mkdir -p $O
timeout -k 10 150 python -u scripts/probe_mk_time.py --reps 2 >> $O/ab.log 2>> $O/ab.err && \
DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 150 python -u scripts/probe_mk_time.py --reps 2 >> $O/ab.log 2>> $O/ab.err && \
DMX_LIB=depthmapx_amd/_lib_ab/$EXTRA_LIB/libdmx.so timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -k "makegraph or maxdist or far_rows or shard or chunk_bytes or random_occluders" \
  > $O/tests.log 2>&1
rc=$?
cat $O/ab.log; tail -2 $O/tests.log
exit $rc
