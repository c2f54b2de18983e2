set -o pipefail
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f/mixed.log 2>&1; rc=$?
tail -30 gpurun_out/r04f/mixed.log
[ $rc -eq 0 ] || exit $rc
bash tools/check.sh r04f
