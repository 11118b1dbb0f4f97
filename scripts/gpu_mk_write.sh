# makeGraph at configs[2]: parity subset (makeGraph, symmetry, VGA around special nodes), time, and the
# FETCH_SIZE / WRITE_SIZE passes of one makeGraph (probe_mk_time.py, whole-graph build with the fused scatter).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-mkwrite}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "${PRETEST_K:-makegraph or random_occluders or far_rows or maxdist or shards or symmetry or vga}" > $OUT/pretest.log 2>&1 \
  || { grep -E "FAILED|ERROR|Error" $OUT/pretest.log | head -20; tail -5 $OUT/pretest.log; exit 1; }
tail -n 1 $OUT/pretest.log
timeout -k 10 200 python3 -u scripts/probe_mk_time.py --config 2 --reps 2 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }
timeout -k 10 200 python3 -u scripts/probe_mk_time.py --config 5 --reps 1 >> $OUT/mk.jsonl 2>> $OUT/mk.err || { tail -5 $OUT/mk.err; exit 1; }
cut -c1-200 $OUT/mk.jsonl
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmc_$c -o pmc --output-format csv \
    -- python3 $R/scripts/probe_mk_time.py --config 2 --reps 1 > $OUT/pmc_$c.log 2>&1 || { tail -5 $OUT/pmc_$c.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for c in ["FETCH_SIZE", "WRITE_SIZE"]:
    acc = collections.defaultdict(float)
    for f in glob.glob("$OUT/pmc_%s/**/*counter_collection.csv" % c, recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"].split("(")[0][-40:]] += float(r["Counter_Value"]) * 1024
    for k, v in sorted(acc.items(), key=lambda t: -t[1])[:4]:
        print(c, k, "%.1f GB" % (v / 1e9))
PY
