#!/bin/bash
# makeGraph variant A/B (env switches), then the cancel / balance / makeGraph parity tests
set -o pipefail
O=gpurun_out/${TAG:-iter2}
mkdir -p $O
run() { echo "== $*" >> $O/ab.log; env "$@" timeout -k 10 150 python -u scripts/probe_mk_time.py --config ${CONFIG:-2} >> $O/ab.log 2>> $O/ab.err; }
run X=1 && run DMX_MK_NOFIXED=1 && run DMX_MK_WPE=4 && run DMX_MK_WPE=6 && \
CONFIG=5 run X=1 && CONFIG=5 run DMX_MK_NOFIXED=1 && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_progress_cancel.py \
  tests/test_gpu_parity.py -k "cancel or progress or makegraph or shard or chunk_bytes or random_occluders" > $O/tests.log 2>&1
