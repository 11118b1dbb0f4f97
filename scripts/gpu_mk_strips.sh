#!/bin/bash
# makeGraph per x-strip on config 5 (edge-shard imbalance), with the attempt log
set -o pipefail
mkdir -p gpurun_out/mk_strips
DMX_VERBOSE=1 timeout -k 10 400 python -u scripts/probe_mk_strips.py --config 5 --width 50 --strips 0,1,2,3,4,5,6,10,20,30,39 \
  > gpurun_out/mk_strips/strips5.log 2> gpurun_out/mk_strips/strips5.err
