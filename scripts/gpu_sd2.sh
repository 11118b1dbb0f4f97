# batched metric step depth: parity vs the serial kernel and the reference fixtures, then config 5
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/sd2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "metric_stepdepth" > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
C5_LIMIT=400 bash scripts/gpu_config5.sh
