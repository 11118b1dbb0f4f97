# 1000^2 bench with the CPU baseline, then the one-rank rehearsal of the sharded makeGraph exchange.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-bench}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --steps ${STEPS:-2} --warmup 1 > $OUT/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --mk-mode shard --no-cpu-baseline > $OUT/bench_shard1.log 2>&1
rc=$?
grep '^{' $OUT/bench.log | cut -c1-300; grep '^{' $OUT/bench_shard1.log | cut -c1-200
exit $rc
