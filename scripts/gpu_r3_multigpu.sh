# Multi-GPU readiness on one GPU: makeGraph per shard range at W = 2/4/8 and the
# one-rank sharded exchange (device peak) at 1000^2 and 2000^2/5000.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r3multi}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/probe_shard_balance.py --config 2 > $OUT/balance_1000.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --mk-mode shard --no-cpu-baseline > $OUT/shard_1000.jsonl 2> $OUT/shard_1000.err && \
timeout -k 10 300 python -u scripts/probe_shard_balance.py --config 5 > $OUT/balance_2000.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config 5 --steps 1 --warmup 1 --mk-mode shard --no-cpu-baseline > $OUT/shard_2000.jsonl 2> $OUT/shard_2000.err
rc=$?
cat $OUT/balance_1000.log $OUT/balance_2000.log | grep "^W="
python -c "
import json
for f in ['shard_1000', 'shard_2000']:
    try:
        r = json.loads(open('$OUT/%s.jsonl' % f).read().strip().splitlines()[-1])
        print(f, r['ms_per_step'], r['kernels'].get('graph_exchange'))
    except Exception as e:
        print(f, 'n/a', e)
"
exit $rc
