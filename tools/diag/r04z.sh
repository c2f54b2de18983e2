set -o pipefail
mkdir -p gpurun_out/r04z
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ingest.py tests/test_gpu_large.py > gpurun_out/r04z/tests.log 2>&1 && tail -1 gpurun_out/r04z/tests.log &&
bash tools/measure.sh r04z prof,fixup
