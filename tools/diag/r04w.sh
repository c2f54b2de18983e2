set -o pipefail
mkdir -p gpurun_out/r04w
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mixed.py tests/test_gpu_parity.py -k "mixed or non_square or unsupported" > gpurun_out/r04w/tests.log 2>&1 && tail -3 gpurun_out/r04w/tests.log &&
FCD_GENERIC_SCATTER=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mixed.py -k "mixed_frames" > gpurun_out/r04w/tests_scatter.log 2>&1 && tail -1 gpurun_out/r04w/tests_scatter.log &&
bash tools/ab.sh r04w 2 'python tools/shape_bench.py 1024x1280 1536x2048 960x1024' gather scatter:FCD_GENERIC_SCATTER=1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04w/shapeprof -o run -- python3 tools/shape_bench.py 1024x1280 --steps 3 > gpurun_out/r04w/shapeprof.log 2>&1
