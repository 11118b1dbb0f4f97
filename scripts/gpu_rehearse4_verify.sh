# After the stream fix: the 4-rank one-GPU rehearsal on the un-staged gloo path (device tensors) REPS
# times, each run's gathered columns compared bit for bit with the one-process run.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-rehearse4_verify}
mkdir -p $OUT
W=${W:-256}
timeout -k 10 200 python bench.py --grid $W --steps 1 --warmup 0 --no-cpu-baseline --dump-out $OUT/one.npy > $OUT/one.log 2>&1 || exit 1
for i in $(seq 1 ${REPS:-5}); do
  DMX_ABORT_BACKTRACE=1 PYTHONFAULTHANDLER=1 DMX_GLOO_DEVICE_TENSORS=${DEVT:-1} DMX_DIST_BACKEND=gloo DMX_FORCE_DEVICE=0 \
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-4} --master-addr 127.0.0.1 \
    --master-port $((29800 + i)) bench.py --gpus ${NPROC:-4} --grid $W --steps 1 --warmup 1 --no-cpu-baseline \
    --mk-mode ${MK:-shard} --dump-out $OUT/four$i.npy > $OUT/four$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  if [ $rc -ne 0 ]; then grep -n "native backtrace\|libdmx\|double free\|corruption\|exitcode" $OUT/four$i.log | head -20; exit $rc; fi
  python -c "
import numpy as np
a = np.load('$OUT/one.npy'); b = np.load('$OUT/four$i.npy')
print('rows', a.shape, 'bit-identical', bool((a.view(np.uint32) == b.view(np.uint32)).all()))
"
done
