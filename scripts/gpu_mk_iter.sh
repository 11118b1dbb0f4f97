#!/bin/bash
# makeGraph iteration: parity (reference fixtures, retries, certified moments, balanced shard bounds, 1000^2
# blocks vs the oracle), then per-strip kernel times + work counts (cost-model fit) and shard balance probes
set -o pipefail
O=gpurun_out/${TAG:-mk_iter}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "makegraph or shards_assemble or shard_bounds or chunk_bytes or random_occluders" > $O/parity.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_scale.py \
  -k "1000_makegraph" > $O/scale.log 2>&1 && \
timeout -k 10 300 python -u scripts/probe_mk_strips.py --config 5 --width 100 > $O/strips5.log 2> $O/strips5.err && \
timeout -k 10 200 python -u scripts/probe_mk_strips.py --config 2 --width 50 > $O/strips2.log 2> $O/strips2.err && \
timeout -k 10 200 python -u scripts/probe_shard_balance.py --config 2 > $O/bal2.log 2> $O/bal2.err && \
timeout -k 10 300 python -u scripts/probe_shard_balance.py --config 5 --balanced > $O/bal5b.log 2> $O/bal5b.err
