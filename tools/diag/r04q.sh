set -o pipefail
mkdir -p gpurun_out/r04q
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py -k "4096 or fused or census" > gpurun_out/r04q/tests.log 2>&1 && tail -3 gpurun_out/r04q/tests.log &&
bash tools/ab.sh r04q 3 'python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames' zt16 zt4@ &&
bash tools/traffic.sh r04q/traffic4096 "--size 4096 --batch 16"
