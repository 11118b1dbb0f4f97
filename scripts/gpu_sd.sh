# step-depth / VGA metric / angular GPU parity, then the config-5 bench
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/sd
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "step or metric or angular or cli" > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
C5_LIMIT=900 bash scripts/gpu_config5.sh
