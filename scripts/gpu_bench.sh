# bench on the GPU box: default (256^2) and the 1000^2 headline config, plus rocprofv3 kernel stats
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${TAG:-r1}
mkdir -p $OUT/prof_$TAG
timeout -k 10 600 python bench.py > $OUT/bench256.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 900 python bench.py --grid 1000 --steps 1 --warmup 0 --cpu-budget 30 > $OUT/bench1000.log 2>&1 && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG/k1000 -o kt --output-format csv -- python3 bench.py --grid 1000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/prof_$TAG/k1000.log 2>&1
rc=$?
grep -v amdgpu.ids $OUT/bench256.log $OUT/bench1000.log | tail -30
exit $rc
