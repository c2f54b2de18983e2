set -o pipefail
bash tools/check.sh r04d || exit 1
bash tools/ab.sh r04d_icx 3 'trapped-modes-ltg_amd/tools/bin/kbench_base 1024 256 10' x1 || exit 1
for v in base icx0; do for n in 1024 2048; do nb=256; [ $n = 2048 ] && nb=64; timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_$v $n $nb 10 > gpurun_out/r04d_icx/kb_${v}_$n.txt 2>&1 || exit 1; done; done
for r in 1 2; do for v in base icx0; do timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_$v 1024 256 10 > gpurun_out/r04d_icx/kb_${v}_1024_$r.txt 2>&1 || exit 1; done; done
grep -h int_cols gpurun_out/r04d_icx/kb_*.txt
