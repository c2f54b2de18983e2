#!/bin/bash
# Device assembly of every engine source into $1 (for checking that a source edit leaves
# the compiled kernels unchanged: diff -r two dumps).  Same flags as the Makefile.
set -e
out=${1:?out dir}
mkdir -p $out
cd "$(dirname "$0")/../trapped-modes-ltg_amd"
flags="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Wall -Werror -Wno-unused-function -fvisibility=hidden -Wno-unused-command-line-argument -I../include"
pids=()
for s in csrc/*.hip csrc/fcd_engine.cpp; do
  b=$(basename $s)
  fp=""
  case $b in kernels_phase_rows.hip|kernels_phase_rows_wide.hip|kernels_band.hip|kernels_fast.hip|kernels_integ.hip) fp="-ffp-contract=fast";; esac
  /opt/rocm/bin/hipcc $flags $fp -x hip --cuda-device-only -S -o $out/$b.s $s &
  pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
wait
# drop the compiler identification lines
sed -i -e '/\.ident\|clang version/d' -e 's/__hip_cuid_[0-9a-f]*/__hip_cuid_X/g' $out/*.s
