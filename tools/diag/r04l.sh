set -o pipefail
mkdir -p gpurun_out/r04l
bash tools/ab.sh r04l 2 'python tools/fixup_bench.py 96' t64 t6432:FCD_MST_TILE=6432 t6432r1:FCD_MST_TILE=6432,FCD_T0_ROUNDS=1 t6432r3:FCD_MST_TILE=6432,FCD_T0_ROUNDS=3 t32:FCD_MST_TILE=32 t32r1:FCD_MST_TILE=32,FCD_T0_ROUNDS=1
