# makeGraph spans (span.hpp): the makeGraph parity subset, then the whole-map kernel time per variant at
# configs[2] and configs[4] (CONFIGS), then optionally the phase clocks with span statistics (PHASES=1).
# RUNS: space-separated name=lib:ENV=VAL,ENV=VAL entries (lib "default" or a name under depthmapx_amd/_lib_ab/).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-span}
mkdir -p $OUT
if [ -z "${NO_PRETEST}" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "${PRETEST_K:-makegraph or random_occluders or far_rows or maxdist or shards or symmetry}" > $OUT/pretest.log 2>&1 \
    || { grep -E "FAILED|ERROR|Error" $OUT/pretest.log | head -20; tail -5 $OUT/pretest.log; exit 1; }
  tail -n 1 $OUT/pretest.log
fi
run() {   # name lib envlist config reps
  local envs=$(echo "$3" | tr ',' ' ')
  if [ "$2" = default ]; then L=""; else L="DMX_LIB=$R/depthmapx_amd/_lib_ab/$2/libdmx.so"; fi
  env $L $envs timeout -k 10 300 python3 -u scripts/probe_mk_time.py --config $4 --reps $5 --tag $1 >> $OUT/mk.jsonl 2>> $OUT/mk.err
}
for c in ${CONFIGS:-2 5}; do
  for spec in ${RUNS:-span=default:}; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=${rest#*:}
    run $name $lib "$envs" $c ${REPS:-2} || { tail -5 $OUT/mk.err; exit 1; }
  done
done
if [ -n "${PHASES}" ]; then
  for c in ${CONFIGS:-2 5}; do
    DMX_VERBOSE=1 timeout -k 10 300 python3 -u scripts/probe_mk_time.py --config $c --reps 1 > $OUT/ph_$c.log 2>&1 || { tail -5 $OUT/ph_$c.log; exit 1; }
    grep -h "makegraph phases\|makegraph spans\|makegraph merges" $OUT/ph_$c.log | tail -n 3
  done
fi
python3 -c "
import json
for l in open('$OUT/mk.jsonl'):
    d = json.loads(l); print(d.get('tag', ''), d['config'], [round(x, 3) for x in d['mk_s']], d['reruns'], d['pairs'], d['runs'])
"
