# Multi-rank rehearsal on a one-GPU box: 2 ranks share cuda:0 over gloo and run the sharded path
# (makeGraph shards -> blob all-gather -> assemble -> interleaved VGA sources -> chunked row gather);
# the gathered columns must equal a single-process run bit for bit.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-multi}
mkdir -p $OUT
W=${W:-256}
timeout -k 10 300 python bench.py --grid $W --steps 1 --warmup 0 --no-cpu-baseline --dump-out $OUT/one.npy > $OUT/one.log 2>&1 && \
DMX_DIST_BACKEND=gloo DMX_FORCE_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus ${NPROC:-2} --grid $W --steps 1 --warmup 1 --no-cpu-baseline \
  --dump-out $OUT/two.npy ${EXTRA:-} > $OUT/two.log 2>&1 && \
python -c "
import numpy as np
a = np.load('$OUT/one.npy'); b = np.load('$OUT/two.npy')
print('rows', a.shape, 'bit-identical', bool((a.view(np.uint32) == b.view(np.uint32)).all()), 'unset', int((b == -1).all(axis=1).sum()))
"
rc=$?
grep -h '"metric"' $OUT/one.log $OUT/two.log | cut -c1-300
tail -3 $OUT/two.log
exit $rc
