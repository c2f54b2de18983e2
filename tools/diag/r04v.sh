set -o pipefail
mkdir -p gpurun_out/r04v
bash tools/check.sh r04v &&
timeout -k 10 300 python tools/shape_bench.py 1024x1280 1536x2048 960x1024 1024x1024 > gpurun_out/r04v/shapes.log 2>&1 && cat gpurun_out/r04v/shapes.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04v/shapeprof -o run -- python3 tools/shape_bench.py 1024x1280 --steps 3 > gpurun_out/r04v/shapeprof.log 2>&1
