# A/B runs: VGA time at 1000^2 per build variant, makeGraph time per variant, then the VGA and makeGraph
# parity tests on the last variant (all changes).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
lib() { if [ $1 = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$1/libdmx.so; fi; }
run() {
  if [ -n "${PRETEST}" ]; then
    timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${PRETEST} -k "${PRETEST_K:-makegraph}" > $OUT/pretest.log 2>&1 \
      || { grep -E "FAILED|ERROR|Error" $OUT/pretest.log | head -20; tail -5 $OUT/pretest.log; return 1; }
    tail -2 $OUT/pretest.log
  fi
  [ -z "${NO_VGA}" ] && for v in default ${VGA_VARIANTS}; do
    lib $v
    timeout -k 10 300 python -u scripts/probe_vga_time.py ${VGA_ARGS} >> $OUT/vga1000.jsonl 2>> $OUT/vga1000.err || { tail -5 $OUT/vga1000.err; return 1; }
  done
  [ -z "${NO_VGA}" ] && cut -c1-260 $OUT/vga1000.jsonl
  [ -n "${MK_VARIANTS}" ] && for v in default ${MK_VARIANTS}; do
    lib $v
    timeout -k 10 200 python -u scripts/probe_mk_time.py --config 2 --reps 2 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; return 1; }
    if [ -n "${MK5}" ]; then
      timeout -k 10 200 python -u scripts/probe_mk_time.py --config 5 --reps 1 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; return 1; }
    fi
  done
  [ -n "${MK_VARIANTS}" ] && cut -c1-200 $OUT/mk.jsonl
  [ -n "${BENCH_VARIANTS}" ] && for v in default ${BENCH_VARIANTS}; do
    lib $v
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>> $OUT/bench.err | grep '^{' | \
      python -c "import sys, json; d = json.loads(sys.stdin.read()); print(json.dumps({'lib': '$v', 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'parts': {k: v for k, v in d.get('kernels', {}).items() if k.endswith('_s')}}))" >> $OUT/bench_ab.jsonl || { tail -5 $OUT/bench.err; return 1; }
  done
  [ -n "${BENCH_VARIANTS}" ] && cat $OUT/bench_ab.jsonl | cut -c1-400
  [ -n "${NO_TESTS}" ] && return 0
  lib ${TEST_VARIANT:-default}
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py \
    tests/test_gpu_scale.py tests/test_merge_links.py tests/test_semifill.py tests/test_graphfile.py tests/test_gpu_nocaps.py} \
    -k "${K:-(vga or merge or contextfilled or special or asym or makegraph or random_occluders or graph_regression or topdown or symmetry) and not 2000}" \
    > $OUT/pytest.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/pytest.log | head; tail -3 $OUT/pytest.log
  return $rc
}
run
rc=$?
kill $HB
exit $rc
