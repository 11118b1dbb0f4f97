# 4 ranks sharing cuda:0 over gloo, pure torch (scripts/gloo_cuda_repro.py): CUDA tensors first, then
# the same collectives on host tensors.  Each run logs under gpurun_out/$TAG.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-gloo_repro}
mkdir -p $OUT
MODE=cuda ITERS=${ITERS:-12} timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-4} \
  --master-addr 127.0.0.1 --master-port 29541 scripts/gloo_cuda_repro.py > $OUT/cuda.log 2>&1
rc_cuda=$?
echo "cuda rc=$rc_cuda"; grep -h "REPRO_DONE\|double free\|corruption\|exitcode\|Segmentation\|Root Cause" $OUT/cuda.log | head -12
if [ $rc_cuda -eq 0 ]; then
MODE=host ITERS=${ITERS:-12} timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-4} \
  --master-addr 127.0.0.1 --master-port 29542 scripts/gloo_cuda_repro.py > $OUT/host.log 2>&1
echo "host rc=$?"; grep -h "REPRO_DONE" $OUT/host.log
fi
exit 0
