# rocprofv3 passes for the bench workload (run on the GPU box).  Kernel trace + stats, then one
# PMC pass per TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof_${TAG:-r1}
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
rc=$?
find $OUT -name "*.csv" | head -20
exit $rc
