#!/bin/bash
# Interleaved headline bench: product library vs a tools/libvar.sh build (FCD_LIB),
# then the GPU parity suite on the product library.
# Usage: bash tools/r03_lib_ab.sh TAG VARIANT [reps]
set -o pipefail
out=gpurun_out/$1; v=$2; reps=${3:-3}
mkdir -p $out
for r in $(seq $reps); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-real-frames > $out/bench_new_$r.log 2>&1 || { tail -5 $out/bench_new_$r.log; exit 1; }
  FCD_LIB=trapped-modes-ltg_amd/build_libvar/$v/libfcd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-real-frames > $out/bench_${v}_$r.log 2>&1 || { tail -5 $out/bench_${v}_$r.log; exit 1; }
  for x in new $v; do echo "$x $(grep '^{' $out/bench_${x}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_us_per_frame"])')"; done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
