set -o pipefail
mkdir -p gpurun_out/r01z
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01z/pytest.log 2>&1 || { tail -30 gpurun_out/r01z/pytest.log; exit 1; }
tail -1 gpurun_out/r01z/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r01z/p2048 -o run -- python3 bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01z/p2048.log 2>&1 || { tail -20 gpurun_out/r01z/p2048.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r01z/p4096 -o run -- python3 bench.py --size 4096 --batch 64 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r01z/p4096.log 2>&1 || { tail -20 gpurun_out/r01z/p4096.log; exit 1; }
echo ok
