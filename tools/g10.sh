set -o pipefail
timeout -k 10 300 python bench.py --size 2048 --batch 64 --steps 5 --no-cpu-baseline > gpurun_out/b2048.log 2>&1 || { tail -20 gpurun_out/b2048.log; exit 1; }
tail -1 gpurun_out/b2048.log
timeout -k 10 300 python bench.py --size 4096 --batch 16 --steps 5 --no-cpu-baseline > gpurun_out/b4096.log 2>&1 || { tail -20 gpurun_out/b4096.log; exit 1; }
tail -1 gpurun_out/b4096.log
timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 2048 16 5 || exit 1
timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 4096 4 5 || exit 1
