# Bisect the 4-rank one-GPU gloo abort: variants run in order; the script stops at the first failure
# (a host abort ends the call, as the pool rules require).  VARIANTS: "devt:prep:mk" triples.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-rehearse4_bisect}
mkdir -p $OUT
i=0
VARIANTS=${VARIANTS:-0:shard:shard 0:shard:shard 1:replicate:shard}
for v in $VARIANTS; do
  i=$((i+1))
  IFS=: read devt prep mk <<< "$v"
  DMX_ABORT_BACKTRACE=1 PYTHONFAULTHANDLER=1 DMX_GLOO_DEVICE_TENSORS=$devt DMX_DIST_BACKEND=gloo DMX_FORCE_DEVICE=0 \
  timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-4} --master-addr 127.0.0.1 \
    --master-port $((29700 + i)) bench.py --gpus ${NPROC:-4} --grid ${W:-256} --steps 1 --warmup 1 --no-cpu-baseline \
    --mk-mode $mk --prep-mode $prep > $OUT/v$i.log 2>&1
  rc=$?
  echo "variant $i devt=$devt prep=$prep mk=$mk rc=$rc"
  grep -n "native backtrace\|libdmx\|libgloo\|libc.so\|Fatal Python\|double free\|corruption\|Segmentation\|in vga_\|in step\|in exchange\|in assemble\|in cb\|exitcode" $OUT/v$i.log | head -40
  if [ $rc -ne 0 ]; then break; fi
done
exit 0
