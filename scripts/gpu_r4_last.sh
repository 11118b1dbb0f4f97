# Round 4, last build: the whole GPU suite and smoke, then one short bench step per headline config (the
# bench's JSON line, as the driver reads it).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-r4last}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench1.log 2> $OUT/bench1.err && \
timeout -k 10 300 python -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench5.log 2> $OUT/bench5.err
rc=$?
kill $HB
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head; tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
grep '^{' $OUT/bench1.log | cut -c1-200; grep '^{' $OUT/bench5.log | cut -c1-200; tail -3 $OUT/bench5.err
exit $rc
