# Round 4: the 2000^2 VGA-global probe (HBM-frontier tile BFS) on the current build, checked against the
# direction-optimising kernel on 16 sources.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4v2000}
mkdir -p $OUT
( while true; do sleep 45; date +%s >> $OUT/heartbeat; done ) > /dev/null 2>&1 &
HB=$!
timeout -k 10 500 python -u scripts/probe_vga2000.py --nsrc 1024 --blocks 1 --check-do 16 > $OUT/probe2000.jsonl 2> $OUT/progress.txt
rc=$?
kill $HB
grep -v amdgpu.ids $OUT/progress.txt | cut -c1-300
exit $rc
