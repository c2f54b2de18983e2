set -o pipefail
mkdir -p gpurun_out/r1c
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 8 20 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r1c/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/r1c/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r1c/bench.log 2>&1 || { tail -20 gpurun_out/r1c/bench.log; exit 1; }
tail -1 gpurun_out/r1c/bench.log
