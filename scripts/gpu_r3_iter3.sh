#!/bin/bash
# makeGraph: previous build (_lib_ab/c4) vs the current one, then makeGraph parity incl. maxdist
set -o pipefail
O=gpurun_out/${TAG:-iter3}
mkdir -p $O
DMX_LIB=depthmapx_amd/_lib_ab/c4/libdmx.so timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
CONFIG=5 timeout -k 10 150 python -u scripts/probe_mk_time.py --config 5 >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "makegraph or maxdist or shard or chunk_bytes or random_occluders" > $O/tests.log 2>&1
