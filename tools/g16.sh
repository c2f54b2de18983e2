# large-size parity tests + c3 / c5 bench lines
set -o pipefail
mkdir -p gpurun_out/r01g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "2048 or 4096 or empty" > gpurun_out/r01g/pytest_big.log 2>&1 || { tail -30 gpurun_out/r01g/pytest_big.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r01g/pytest_big.log
timeout -k 10 400 python bench.py --size 2048 --batch 1024 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01g/bench2048.log 2>&1 || { tail -20 gpurun_out/r01g/bench2048.log; exit 1; }
tail -1 gpurun_out/r01g/bench2048.log
timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01g/bench4096.log 2>&1 || { tail -20 gpurun_out/r01g/bench4096.log; exit 1; }
tail -1 gpurun_out/r01g/bench4096.log
