# makeGraph A/B at 1000^2 (probe_mk: kernel time per env setting) + a 2-step bench.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-mkab}
mkdir -p $OUT
timeout -k 10 400 python -u scripts/probe_mk.py 1000 ${PROBE:-DMX_MK_NOSAMPLE=1} > $OUT/probe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?
grep '^{' $OUT/probe.log | cut -c1-300; grep '^{' $OUT/bench.log | cut -c1-300
exit $rc
