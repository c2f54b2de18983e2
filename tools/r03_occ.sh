#!/bin/bash
# A/B of the wide-row kernel variants (kbench_occ<V>, tools/kvar.sh builds), interleaved,
# at 4096^2 x 16 and 2048^2 x 64; then optionally the 2048^2 / 4096^2 bench lines and
# the GPU parity suite of the product build.
# Usage: bash tools/r03_occ.sh TAG "A B C" [bench+tests: 1]
set -o pipefail
out=gpurun_out/${1:-r03v}; vars=${2:-"A B"}; full=${3:-1}
mkdir -p $out
for rep in 1 2; do
  for cfg in "4096 16" "2048 64"; do
    set -- $cfg
    for v in $vars; do
      timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_occ$v $1 $2 10 > $out/kb_${v}_$1_$rep.txt 2>&1 || { echo "kbench $v $1 failed"; tail -5 $out/kb_${v}_$1_$rep.txt; exit 1; }
    done
  done
done
echo kbench done
[ "$full" = 1 ] || exit 0
timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench4096.log 2>&1 || { tail -20 $out/bench4096.log; exit 1; }
grep '^{' $out/bench4096.log | cut -c1-300
timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench2048.log 2>&1 || { tail -20 $out/bench2048.log; exit 1; }
grep '^{' $out/bench2048.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
