# rocprofv3 passes over one 1000^2 bench step (configs[2]): kernel trace + stats, then the PMC passes
# summarised by scripts/pmc_summary.py (HBM bytes, VALU issue, FP64 op counts).  One pass per run:
# rocprofv3 does not split counters over passes (SQ 8 / TCC 4 / GRBM 2 slots).
set -o pipefail
export TMPDIR=/tmp
cd /tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-pmc}
mkdir -p $OUT
B="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
pass() {
  name=$1; shift
  timeout -s KILL 420 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $B > $OUT/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc"
  return $rc
}
pass stats --kernel-trace --stats && \
pass fetch --pmc FETCH_SIZE && \
pass write --pmc WRITE_SIZE && \
pass l2 --pmc TCC_HIT_sum TCC_MISS_sum && \
pass issue --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
pass mix --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
  SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE && \
pass lds --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE
