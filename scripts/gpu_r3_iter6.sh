#!/bin/bash
# makeGraph: first-pass block capacity 64 (FIXED) vs 32 (generic kernel with DMX_MK_BCAP=32 / NOFIXED)
set -o pipefail
O=gpurun_out/${TAG:-iter6}
mkdir -p $O
timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
DMX_MK_NOFIXED=1 timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
DMX_MK_NOFIXED=1 DMX_MK_BCAP=32 timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
DMX_MK_NOFIXED=1 DMX_MK_BCAP=128 timeout -k 10 150 python -u scripts/probe_mk_time.py >> $O/ab.log 2>> $O/ab.err && \
timeout -k 10 150 python -u scripts/probe_mk_time.py --config 5 >> $O/ab.log 2>> $O/ab.err
