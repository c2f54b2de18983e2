#!/bin/bash
# A/B of the atan2 reduction (FCD_ATAN_FORM 0 = octant, 1 = quadrant) on the phase
# kernels (kbench, interleaved runs), then the GPU parity suite on the product build.
set -o pipefail
out=gpurun_out/${1:-r03s}
mkdir -p $out
for rep in 1 2; do
  for cfg in "1024 256" "2048 64" "4096 16"; do
    set -- $cfg
    for v in 0 1; do
      timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_atan$v $1 $2 10 > $out/kb_${v}_$1_$rep.txt 2>&1 || { echo "kbench $v $1 failed"; tail -5 $out/kb_${v}_$1_$rep.txt; exit 1; }
    done
  done
done
echo kbench done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | cut -c1-600
