# makeGraph A/B at configs[2]: kernel time per build variant (DMX_LIB) and one PMC pass of the instruction mix
# (SQ counters) per variant.  Variants: "default" plus the names of depthmapx_amd/_lib_ab/<name>.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-mkpmc}
mkdir -p $OUT
cd /tmp
lib() { if [ $1 = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$1/libdmx.so; fi; }
for v in ${VARIANTS:-default}; do
  lib $v
  timeout -k 10 200 python3 -u $R/scripts/probe_mk_time.py --config 2 --reps 2 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }
  [ -n "${MK5}" ] && { timeout -k 10 200 python3 -u $R/scripts/probe_mk_time.py --config 5 --reps 1 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }; }
  if [ -n "${PMC}" ]; then
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_$v -o pmc --output-format csv \
      -- python3 $R/scripts/probe_mk_time.py --config 2 --reps 1 > $OUT/pmc_$v.log 2>&1 || { tail -5 $OUT/pmc_$v.log; exit 1; }
  fi
done
cut -c1-200 $OUT/mk.jsonl
