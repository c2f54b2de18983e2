#!/bin/bash
# k_int_cols with 16 elements per lane at 2048 / 4096 points vs 8 (kbench A/B).
set -o pipefail
export TMPDIR=/tmp
bash tools/r03_kb_ab.sh r03icw "icW16 icW0" 4096 16 3 || exit 1
bash tools/r03_kb_ab.sh r03icw "icW16 icW0" 2048 64 3 || exit 1
grep -h "int_cols\|int_c2r" gpurun_out/r03icw/kb_*_1.txt
