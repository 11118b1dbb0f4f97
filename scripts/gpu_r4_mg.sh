# Round 4: configs[4] one-rank memory budget (8-rank emulation), per-rank makeGraph time and blob sizes at
# W = 2/4/8 for configs[2]/[4], and the 2000^2 VGA-global direction-switch sweep.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4mg}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded_2000.py -x -v -s -m gpu --timeout 450 --timeout-method thread \
  > $OUT/pytest_sharded2000.log 2>&1 && \
timeout -k 10 300 python -u scripts/probe_shard_balance.py --config 5 --balanced > $OUT/balance_config5.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe_shard_balance.py --config 2 --balanced > $OUT/balance_config2.log 2>&1 && \
timeout -k 10 400 python -u scripts/probe_vga2000.py --nsrc 1024 --blocks 1 --alphas ${ALPHAS:-15,240,2000} \
  > $OUT/probe2000_alpha.jsonl 2> $OUT/probe2000_alpha_progress.txt
rc=$?
tail -3 $OUT/pytest_sharded2000.log; grep "one-rank budget" $OUT/pytest_sharded2000.log; tail -4 $OUT/balance_config5.log | cut -c1-300; tail -4 $OUT/balance_config2.log | cut -c1-300; cat $OUT/probe2000_alpha_progress.txt | cut -c1-400
exit $rc
