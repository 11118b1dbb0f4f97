# A/B of the XCD-grouped VGA source dispatch (DMX_VGA_XCD) on 131072 middle sources of 1000^2 (A B A B),
# then the configs[4] bench line (2 steps, CPU leg) with the per-step PMC roofline fields.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-xcd}
mkdir -p $OUT
cd $R && timeout -k 10 300 python -u scripts/probe_big.py 1000 ${NSRC:-131072} "" DMX_VGA_XCD=0 DMX_VGA_XCD=1 DMX_VGA_XCD=0 DMX_VGA_XCD=1 > $OUT/probe.log 2>&1 && \
timeout -k 10 500 python -u bench.py --config 5 --steps 2 --warmup 1 > $OUT/bench_c5.log 2> $OUT/bench_c5_progress.txt
rc=$?
grep -v amdgpu.ids $OUT/probe.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print({k: d[k] for k in d if k in ('config', 'same_as_first', 'vga_kernel_s', 'est_full_vga_s', 'makegraph_kernel_s', 'prep_wall_s')})
"
grep '^{' $OUT/bench_c5.log | cut -c1-200
exit $rc
