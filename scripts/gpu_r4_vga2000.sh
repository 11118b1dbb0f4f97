# Round 4: 2000^2 VGA global with the tile-visibility miss certificate (tvis alone) in front of phase C's run scan.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-r4v2k}
mkdir -p $OUT
timeout -k 10 600 python -u scripts/probe_vga2000.py --nsrc ${NSRC:-2048} --blocks ${BLOCKS:-2} --check-do ${CHECK_DO:-16} \
  > $OUT/probe2000.jsonl 2> $OUT/probe2000_progress.txt
rc=$?
cat $OUT/probe2000_progress.txt | cut -c1-700
exit $rc
