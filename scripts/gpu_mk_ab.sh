# makeGraph A/B: a parity subset on the default build first, then kernel time per variant (DMX_LIB) at
# configs[2] (and configs[4] with MK5=1).  Variants: "default" plus names under depthmapx_amd/_lib_ab/.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-mkab}
mkdir -p $OUT
lib() { if [ $1 = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$1/libdmx.so; fi; }
if [ -z "${NO_PRETEST}" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "${PRETEST_K:-makegraph or random_occluders or far_rows or maxdist or shards or symmetry}" > $OUT/pretest.log 2>&1 \
    || { grep -E "FAILED|ERROR|Error" $OUT/pretest.log | head -20; tail -5 $OUT/pretest.log; exit 1; }
  tail -n 1 $OUT/pretest.log
fi
for v in ${VARIANTS:-default}; do
  lib $v
  timeout -k 10 200 python3 -u scripts/probe_mk_time.py --config 2 --reps 2 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }
  [ -n "${MK5}" ] && { timeout -k 10 200 python3 -u scripts/probe_mk_time.py --config 5 --reps 1 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }; }
done
python3 -c "
import json
for l in open('$OUT/mk.jsonl'):
    d = json.loads(l); print(d['lib'].split('/')[-2] if '/' in d['lib'] else d['lib'], d['config'], [round(x, 3) for x in d['mk_s']], d['reruns'])
"
