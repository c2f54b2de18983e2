#!/bin/bash
# The engine with the MST tile pass's per-phase cycle stamps (-DFCD_T0_STAMPS) as
# build_stamps/libfcd_stamps.so (diagnostic; read by tools/t0_stamps.py via FCD_LIB).
set -e
cd "$(dirname "$0")/.."
mkdir -p build_stamps
objs=""
for src in csrc/kernels_phase_rows.hip csrc/kernels_phase_rows_wide.hip csrc/kernels_band.hip csrc/kernels_fast.hip csrc/kernels_fft.hip csrc/kernels_unwrap.hip csrc/kernels_integ.hip csrc/kernels_ingest.hip csrc/kernels_temporal.hip csrc/kernels_tfft.hip csrc/kernels_pocketfft.hip csrc/kernels_mr.hip csrc/fcd_engine.cpp; do
  fp=""; case $src in *phase_rows*|*band*|*fast*|*integ*) fp="-ffp-contract=fast";; esac
  o=build_stamps/$(basename $src).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fvisibility=hidden -I../include $fp -DFCD_T0_STAMPS -x hip -c $src -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_stamps/libfcd_stamps.so $objs
