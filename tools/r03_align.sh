#!/bin/bash
# k_int_cols column-range alignment: kbench A/B (al0 = unaligned, al1 = aligned, al2 = aligned
# with 2 workgroups per CU in the grid) at 1024 (128 frames, the headline launch) and 2048,
# then FETCH_SIZE of k_int_cols for al0 / al1 at 1024.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03align; mkdir -p $out
bash tools/r03_kb_ab.sh r03align "al0 al1 al2" 1024 128 3 || exit 1
bash tools/r03_kb_ab.sh r03align "al0 al1 al2" 2048 64 2 || exit 1
grep -h "^int_cols" $out/kb_*_1.txt
for v in al0 al1; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex 'k_int_cols' -f csv -d $out/pmc_$v -o run -- trapped-modes-ltg_amd/tools/bin/kbench_$v 1024 128 3 > $out/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $out/pmc_$v.log; exit 1; }
done
echo pmc done
