# A/B of the permuted node order of sym_scatter_kernel (DMX_SYM_PERM=0: x-major order) on the 1000^2
# graph: kernel-trace stats of a short probe each way.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-symab}
mkdir -p $OUT
cd /tmp
DMX_SYM_PERM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/off -o off --output-format csv -- python3 $R/scripts/probe_big.py 1000 4096 > $OUT/off.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/on -o on --output-format csv -- python3 $R/scripts/probe_big.py 1000 4096 > $OUT/on.log 2>&1
rc=$?
for m in off on; do echo "== $m"; grep -h "sym_scatter\|tile_vis\|prep_wall" $OUT/$m.log $(find $OUT/$m -name "*kernel_stats.csv") | cut -c1-160; done
exit $rc
