set -o pipefail
mkdir -p gpurun_out/r04ah
bash tools/ab.sh r04ah 3 'python tools/fixup_bench.py 96' c2 c1:FCD_T0_ROUNDS=1 c3:FCD_T0_ROUNDS=3 f7:FCD_CG_FIRST=7
