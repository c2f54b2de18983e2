set -o pipefail
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 32 5 | grep -E "band|phase_rows|int_rows k1|colk" || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "fused or real_df" > gpurun_out/pytest_fused.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_fused.log; exit 1; }
FCD_FUSED=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1 || { tail -20 gpurun_out/bench_fused.log; exit 1; }
tail -1 gpurun_out/bench_fused.log | cut -c 1-400
