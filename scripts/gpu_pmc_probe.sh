# PMC passes over the 1000^2 VGA probe (one pass per counter group, each under its own time limit).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc_${TAG:-probe}
mkdir -p $OUT
W=${W:-1000}; NS=${NS:-8192}
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/fetch.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $OUT/sq -o s --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/sq.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o t --output-format csv -- python3 scripts/probe_big.py $W $NS tile > $OUT/tcc.log 2>&1
rc=$?
find $OUT -name "*counter_collection.csv" | while read f; do echo "== $f"; python3 -c "
import csv,sys,collections
acc=collections.defaultdict(float)
for r in csv.DictReader(open('$f')):
    if 'vga_tile_kernel' in r['Kernel_Name']: acc[r['Counter_Name']]+=float(r['Counter_Value'])
print(dict(acc))"; done
exit $rc
