# benchmark-size parity tests (1000^2, 2000^2/5000) + the syn128 reference VGA case
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/scale
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "scale or 1000 or 2000 or syn128" --durations=0 > $OUT/tests.log 2>&1
rc=$?
tail -30 $OUT/tests.log
exit $rc
