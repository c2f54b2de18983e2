set -o pipefail
mkdir -p gpurun_out/r04r
bash tools/ab.sh r04r 3 'python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames' zt16 zt4@ &&
bash tools/traffic.sh r04r/traffic4096 "--size 4096 --batch 16"
