#!/bin/bash
# Round-3 closing measurement on one MI355X: the lean 2048 k_int_cols A/B (kbench),
# the GPU parity suite + smoke, then tools/r03_measure.sh (bench with CPU baseline,
# rocprofv3 stats, PMC traffic, real frames + their stats, c3, c5).
set -o pipefail
tag=${1:-r03w}
out=gpurun_out/$tag
mkdir -p $out
for rep in 1 2; do
  for v in A E; do
    timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_occ$v 2048 64 10 > $out/kb_${v}_2048_$rep.txt 2>&1 || { echo "kbench $v failed"; exit 1; }
  done
done
echo kbench done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash tools/r03_measure.sh $tag
