# PMC passes over the 1000^2 VGA probe (one pass per counter group, each under its own time limit).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_${TAG:-probe}
mkdir -p $OUT
W=${W:-1000}; NS=${NS:-8192}
P1="SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LEVEL_WAVES SQ_INSTS_SMEM"
timeout -s KILL 400 rocprofv3 --pmc $P1 -d $OUT/p1 -o p --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/p1.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc $P2 -d $OUT/p2 -o p --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/p2.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p3 -o p --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/p3.log 2>&1
rc=$?
for f in $(find $OUT -name "*counter_collection.csv"); do echo "== $f"; python3 -c "
import csv,collections
acc=collections.defaultdict(float)
for r in csv.DictReader(open('$f')):
    k=r['Kernel_Name']
    if 'vga_tile_kernel' in k and 'ELb1ELb1' in k or ('vga_tile_kernel' in k): acc[('vga',r['Counter_Name'])]+=float(r['Counter_Value'])
    if 'makegraph_kernel' in k: acc[('mk',r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(acc.items()): print(k, '%.4g'%v)"; done
exit $rc
