#!/bin/bash
# Build kbench variants of the fused kernel with FCD_PR_ABL ablations (diagnostic only).
set -e
cd "$(dirname "$0")/.."
for a in "$@"; do
  EXTRA=""; case $a in *_s) EXTRA="-DFCD_STAMPS";; *_r4) EXTRA="-DFCD_PR_ROWS=4";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -fno-slp-vectorize -fvisibility=hidden -I../include \
    -DFCD_DIAGNOSTIC -DFCD_PR_ABL=${a%%_*} ${EXTRA} -x hip -c csrc/kernels_phase_rows.hip -o build/pr_abl_$a.o
  objs=$(ls build/*.hip.o | grep -v phase_rows)
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include ${EXTRA} -x hip tools/kbench.cpp -x none build/pr_abl_$a.o $objs -o tools/kbench_abl_$a
done
