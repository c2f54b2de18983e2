# ingest / pipeline / folder tests, full GPU suite, host-path throughput
set -o pipefail
mkdir -p gpurun_out/r01h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r01h/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r01h/pytest_gpu.log; exit 1; }
grep -E "passed|failed" gpurun_out/r01h/pytest_gpu.log
timeout -k 10 300 python tools/host_bench.py > gpurun_out/r01h/host_bench.log 2>&1 || { tail -20 gpurun_out/r01h/host_bench.log; exit 1; }
tail -1 gpurun_out/r01h/host_bench.log
