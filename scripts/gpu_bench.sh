# bench on the GPU box (default config); output under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/bench.log
exit $rc
