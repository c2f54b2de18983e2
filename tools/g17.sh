# kernel stats at 2048^2 and 4096^2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r01g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r01g/prof2048 -o run -- python3 bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01g/prof2048.log 2>&1 || { tail -20 gpurun_out/r01g/prof2048.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r01g/prof4096 -o run -- python3 bench.py --size 4096 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01g/prof4096.log 2>&1 || { tail -20 gpurun_out/r01g/prof4096.log; exit 1; }
echo ok
