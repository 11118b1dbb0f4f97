# GPU parity tests, smoke, PMC traffic passes on the 256^2 bench, and the 1000^2 bench.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${TAG:-r1}
P=$OUT/prof_$TAG
mkdir -p $P
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch256 -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/fetch256.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write256 -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/write256.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $P/tcc256 -o tcc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $P/tcc256.log 2>&1 && \
DMX_VERBOSE=1 timeout -k 10 900 python bench.py --grid 1000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench1000.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
grep -v amdgpu.ids $OUT/smoke.log | tail -2
grep -h '^{\|attempt\|kernels' $OUT/bench1000.log | cut -c1-400
exit $rc
