# config 5 (2000^2 / 5000 occluders, makeGraph + metric step depth), one step
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${TAG:-c5}
mkdir -p $OUT
DMX_VERBOSE=1 timeout -k 10 500 python -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c5.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/c5.log | grep -E "attempt|kernels|^\{" | cut -c1-600
exit $rc
