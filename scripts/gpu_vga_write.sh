# VGA global at 1000^2 per build variant (DMX_LIB): kernel time (probe_vga_time.py) and the FETCH_SIZE /
# WRITE_SIZE passes per kernel, to split the tile kernel's writes (e.g. against a spill-free NT=512 build).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-vgawrite}
mkdir -p $OUT
lib() { if [ $1 = default ]; then unset DMX_LIB; else export DMX_LIB=$R/depthmapx_amd/_lib_ab/$1/libdmx.so; fi; }
cd /tmp
for v in ${VARIANTS:-default}; do
  lib $v
  timeout -k 10 300 python3 -u $R/scripts/probe_vga_time.py >> $OUT/vga.jsonl 2>> $OUT/vga.err || { tail -5 $OUT/vga.err; exit 1; }
  for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
    timeout -s KILL 400 rocprofv3 --pmc $c -d $OUT/pmc_${v}_$c -o pmc --output-format csv \
      -- python3 $R/scripts/probe_vga_time.py > $OUT/pmc_${v}_$c.log 2>&1 || { tail -5 $OUT/pmc_${v}_$c.log; exit 1; }
  done
done
cut -c1-300 $OUT/vga.jsonl
python3 - <<PY
import csv, glob, collections
for d in sorted(glob.glob("$OUT/pmc_*")):
    if d.endswith(".log"): continue
    acc = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"].split("(")[0][-48:]] += float(r["Counter_Value"]) * 1024
    for k, v in sorted(acc.items(), key=lambda t: -t[1])[:3]:
        print(d.split("/")[-1], k, "%.1f GB" % (v / 1e9))
PY
