set -o pipefail
bash tools/measure.sh r04u bench,prof,fixup,c3,c5 &&
timeout -k 10 300 python tools/shape_bench.py 1024x1280 1536x2048 960x1024 1024x1024 > gpurun_out/r04u/shapes.log 2>&1 && cat gpurun_out/r04u/shapes.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04u/shapeprof -o run -- python3 tools/shape_bench.py 1024x1280 --steps 3 > gpurun_out/r04u/shapeprof.log 2>&1
