# 4096 band-pruned inverse: parity + bench
set -o pipefail
mkdir -p gpurun_out/r01g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "4096 or 2048 or fft2" > gpurun_out/r01g/pytest_4096.log 2>&1 || { tail -30 gpurun_out/r01g/pytest_4096.log; exit 1; }
grep -E "passed|failed" gpurun_out/r01g/pytest_4096.log
timeout -k 10 300 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01g/bench4096b.log 2>&1 || { tail -20 gpurun_out/r01g/bench4096b.log; exit 1; }
tail -1 gpurun_out/r01g/bench4096b.log
