# BASELINE.json configs[4] on one MI355X: 2000^2 grid, 5000 occluders, makeGraph + metric step depth
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/c5
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat.txt; sleep 30; done) &
HB=$!
DMX_VERBOSE=1 timeout -k 10 ${C5_LIMIT:-1000} python -u bench.py --config 5 --warmup 0 --steps 1 --cpu-budget 10 > $OUT/bench.log 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -n "$C5_PROF" ]; then
  timeout -k 10 ${C5_LIMIT:-1000} rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --config 5 --warmup 0 --steps 1 --no-cpu-baseline > $OUT/kt.log 2>&1
  rc=$?
fi
kill $HB
grep -v amdgpu.ids $OUT/bench.log | tail -30
exit $rc
