#!/bin/bash
# Build a kbench variant with extra compile definitions on every kernel object
# (tuning tool).  Usage: tools/kvar.sh NAME "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p build_var/$name
objs=""
for src in csrc/kernels_phase_rows.hip csrc/kernels_phase_rows_wide.hip csrc/kernels_band.hip csrc/kernels_fast.hip csrc/kernels_fft.hip csrc/kernels_unwrap.hip csrc/kernels_integ.hip csrc/kernels_ingest.hip csrc/kernels_temporal.hip csrc/kernels_tfft.hip csrc/kernels_pocketfft.hip csrc/kernels_mr.hip; do
  fp=""; case $src in *phase_rows*|*band*|*fast*|*integ*) fp="-ffp-contract=fast";; esac
  o=build_var/$name/$(basename $src).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fvisibility=hidden -I../include $fp $flags -x hip -c $src -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include $flags -x hip tools/kbench.cpp -x none $objs -o tools/bin/kbench_$name
