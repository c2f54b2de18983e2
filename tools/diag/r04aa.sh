set -o pipefail
mkdir -p gpurun_out/r04aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_parity.py -k "early or census or fused or seam or batch or null_stream or pending" > gpurun_out/r04aa/tests.log 2>&1 && tail -1 gpurun_out/r04aa/tests.log &&
bash tools/ab.sh r04aa 3 'python bench.py --no-cpu-baseline --no-real-frames' side noside:FCD_SIDE_SEAM=0 &&
bash tools/ab.sh r04aa 2 'python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline' side2048 noside2048:FCD_SIDE_SEAM=0 &&
bash tools/ab.sh r04aa 2 'python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline' side4096 noside4096:FCD_SIDE_SEAM=0
