# 4 ranks sharing cuda:0 over gloo (bench.py --mk-mode shard at 256^2), gloo collectives on DEVICE
# tensors (DMX_GLOO_DEVICE_TENSORS=1, the pre-5b56724 path), with Python fault handlers (a SIGSEGV /
# SIGABRT prints every thread's Python stack) and glibc's malloc checks; repeated REPS times.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-rehearse4_diag}
mkdir -p $OUT
for i in $(seq 1 ${REPS:-3}); do
  PYTHONFAULTHANDLER=1 MALLOC_CHECK_=3 DMX_GLOO_DEVICE_TENSORS=${DEVT:-1} DMX_DIST_BACKEND=gloo DMX_FORCE_DEVICE=0 \
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-4} --master-addr 127.0.0.1 \
    --master-port $((29600 + i)) bench.py --gpus ${NPROC:-4} --grid ${W:-256} --steps 1 --warmup 1 --no-cpu-baseline \
    --mk-mode ${MK:-shard} > $OUT/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  grep -n "Fatal Python\|double free\|corruption\|Segmentation\|exitcode\|File \"" $OUT/run$i.log | head -40
  if [ $rc -ne 0 ]; then break; fi
done
exit 0
