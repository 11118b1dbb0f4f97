# configs[3] emulated 8-rank choreography at 1000^2 and configs[4] step depth against the oracle at size.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r3scale}
mkdir -p $OUT
(while true; do date >> $OUT/heartbeat.txt; sleep 45; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_1000.py -x -v -s -m gpu --timeout 500 --timeout-method thread > $OUT/sharded1000.log 2>&1
rc1=$?
echo "sharded1000 rc=$rc1"; tail -5 $OUT/sharded1000.log
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then exit $rc1; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -x -v -s -m gpu -k "2000" --timeout 800 --timeout-method thread > $OUT/scale2000.log 2>&1
rc2=$?
echo "scale2000 rc=$rc2"; grep -h "oracle metric\|PASS\|FAIL\|passed\|failed" $OUT/scale2000.log | tail -12
exit $(( rc1 | rc2 ))
