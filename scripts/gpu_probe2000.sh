# The 2000^2 VGA-global probe (configs[4] map): NSRC sources in BLOCKS blocks spread over the node range,
# every block in the per-source rate; 16 sources of the first block checked against the direction-optimising kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-v2000}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
timeout -k 10 ${PROBE_TIMEOUT:-700} python -u scripts/probe_vga2000.py --nsrc ${NSRC:-4096} --blocks ${BLOCKS:-4} ${PROBE_ARGS:---check-do 16} > $OUT/probe2000.jsonl 2> $OUT/progress.txt
rc=$?
kill $HB
grep -v amdgpu.ids $OUT/progress.txt | cut -c1-300
python3 -c "import json; d = json.loads(open('$OUT/probe2000.jsonl').read().strip().splitlines()[-1]); print({k: d[k] for k in ('kernel_s_per_source', 'ms_per_source_by_block', 'extrapolated_whole_map_s', 'makegraph_s')})" || true
exit $rc
