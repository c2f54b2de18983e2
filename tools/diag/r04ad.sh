set -o pipefail
mkdir -p gpurun_out/r04ad
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mixed.py > gpurun_out/r04ad/tests.log 2>&1 && tail -1 gpurun_out/r04ad/tests.log &&
bash tools/ab.sh r04ad 2 'python tools/shape_bench.py 1024x1280 1536x2048 960x1024' twlds notw:FCD_MR_TWLDS=0
