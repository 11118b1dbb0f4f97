# Round artifacts on the GPU box: parity tests, smoke, the default bench (1000^2), its rocprofv3 kernel
# stats, and the FETCH_SIZE / WRITE_SIZE passes for the HBM traffic per launch.  Each GPU step has its
# own time limit; the steps are chained with && so a failure ends the call.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/final_${TAG:-r1}
mkdir -p $OUT
BA="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $BA > $OUT/kt.log 2>&1 && \
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o f --output-format csv -- python3 bench.py $BA > $OUT/fetch.log 2>&1 && \
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o w --output-format csv -- python3 bench.py $BA > $OUT/write.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log $OUT/smoke.log
grep -h '"metric"' $OUT/bench.log | cut -c1-600
exit $rc
