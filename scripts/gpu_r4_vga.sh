# Round 4: 1000^2 VGA time and the VGA parity tests on the current build.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-r4vga}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
run() {
  for v in default ${VARIANTS}; do
    if [ $v = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$v/libdmx.so; fi
    timeout -k 10 300 python -u scripts/probe_vga_time.py >> $OUT/vga1000.jsonl 2>> $OUT/vga1000.err || { tail -5 $OUT/vga1000.err; return 1; }
  done
  cut -c1-300 $OUT/vga1000.jsonl
  timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_scale.py tests/test_merge_links.py tests/test_semifill.py -k "${K:-vga or merge or contextfilled or special or asym}" \
    > $OUT/pytest.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -3 $OUT/pytest.log
  return $rc
}
run
rc=$?
kill $HB
exit $rc
