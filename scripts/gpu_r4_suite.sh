# Round 4: the whole GPU suite (per-test durations) and smoke.  A heartbeat file under gpurun_out/ marks the
# run alive through the long at-size oracle tests (each prints nothing for up to ~3 minutes).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4suite}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
timeout -k 10 1080 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread --durations=30 ${PYARGS} \
  > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
kill $HB
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; tail -40 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
exit $rc
