#!/bin/bash
# makeGraph kernel-variant A/B through environment switches of one build (DMX_MK_WPE, DMX_MK_NOFIXED)
set -o pipefail
O=gpurun_out/${TAG:-mk_env_ab}
mkdir -p $O
run() { echo "== $*" >> $O/ab.log; env "$@" timeout -k 10 150 python -u scripts/probe_mk_time.py --config ${CONFIG:-2} >> $O/ab.log 2>> $O/ab.err; }
run X=1 && run DMX_MK_NOFIXED=1 && run DMX_MK_WPE=4 && run DMX_MK_WPE=6 && \
CONFIG=5 run X=1 && CONFIG=5 run DMX_MK_NOFIXED=1
