# Round 4: PC sampling of configs[2] makeGraph + VGA global (a -gline-tables-only build of the same sources,
# depthmapx_amd/_lib_ab/prof), to attribute the kernels' issue and stall cycles to source lines.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${TAG:-r4pcs}
mkdir -p $OUT
export DMX_LIB=$R/depthmapx_amd/_lib_ab/prof/libdmx.so
cd /tmp
timeout -k 10 ${PCS_TIMEOUT:-240} rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} \
  --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-1048576} -d $OUT/pcs -o pcs \
  --output-format csv -- python3 $R/scripts/probe_pcsample.py --nsrc ${NSRC:-65536} > $OUT/pcs.log 2>&1
rc=$?
tail -5 $OUT/pcs.log
find $OUT/pcs -type f | head; du -sh $OUT/pcs
exit $rc
