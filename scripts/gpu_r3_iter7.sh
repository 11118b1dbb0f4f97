#!/bin/bash
# makeGraph with far rows in scratch memory: timings (1000^2, config 5), parity incl. the corridor case and
# the 2000^2 blocks vs the oracle
set -o pipefail
O=gpurun_out/${TAG:-iter7}
mkdir -p $O
timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 150 python -u scripts/probe_mk_time.py --config 5 >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "makegraph or maxdist or far_rows or shard or chunk_bytes or random_occluders" > $O/tests.log 2>&1 && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 480 --timeout-method thread tests/test_gpu_scale.py \
  -k "makegraph" > $O/scale.log 2>&1
