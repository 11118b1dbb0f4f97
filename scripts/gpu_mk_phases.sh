# makeGraph per-phase wave clocks (DMX_VERBOSE=1 selects the PROF kernel) at configs[2], per build variant.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-mkphases}
mkdir -p $OUT
lib() { if [ $1 = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$1/libdmx.so; fi; }
for v in ${VARIANTS:-default}; do
  lib $v
  DMX_VERBOSE=1 timeout -k 10 200 python3 -u $R/scripts/probe_mk_time.py --config 2 --reps 1 > $OUT/ph_$v.log 2>&1 || { tail -5 $OUT/ph_$v.log; exit 1; }
  echo "$v: $(grep -h 'makegraph phases' $OUT/ph_$v.log | tail -n 1)"
done
