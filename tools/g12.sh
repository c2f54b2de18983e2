set -o pipefail
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 32 5 | grep -E "demod_rows|demod_cols|band_phase|int_rows|int_cols|c2r|phase_rows" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c 1-300
