set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fused or 4096 or 2048" > gpurun_out/r04j/tests.log 2>&1 && tail -3 gpurun_out/r04j/tests.log &&
bash tools/ab.sh r04j 3 'python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames' base ztnt@ &&
bash tools/traffic.sh r04j/traffic4096 "--size 4096 --batch 16"
