mkdir -p gpurun_out/r02j
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02j/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02j/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02j/pytest_gpu.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r02j/prof -o run -- python3 tools/fixup_bench.py 96 > gpurun_out/r02j/log 2>&1; grep metric gpurun_out/r02j/log
