#!/bin/bash
# A/B of the exact (MST) chain on real camera frames: tools/fixup_bench.py with the
# product library against a tools/libvar.sh build (FCD_LIB), interleaved.
# Usage: bash tools/r03_fix_ab.sh TAG VARIANT [reps]
set -o pipefail
out=gpurun_out/$1; v=$2; reps=${3:-3}
mkdir -p $out
for r in $(seq $reps); do
  timeout -k 10 200 python tools/fixup_bench.py 96 > $out/fix_new_$r.log 2>&1 || { tail -5 $out/fix_new_$r.log; exit 1; }
  FCD_LIB=trapped-modes-ltg_amd/build_libvar/$v/libfcd.so timeout -k 10 200 python tools/fixup_bench.py 96 > $out/fix_${v}_$r.log 2>&1 || { tail -5 $out/fix_${v}_$r.log; exit 1; }
  echo "new $(grep '^{' $out/fix_new_$r.log | cut -c1-160)"
  echo "$v $(grep '^{' $out/fix_${v}_$r.log | cut -c1-160)"
done
