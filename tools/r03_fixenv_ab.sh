#!/bin/bash
# Interleaved A/B of runtime switches on the real-frame (exact MST) bench.
# Usage: bash tools/r03_fixenv_ab.sh TAG "ENV_A;ENV_B" [reps]
set -o pipefail
out=gpurun_out/$1; IFS=';' read -ra V <<< "$2"; reps=${3:-3}
mkdir -p $out
for r in $(seq $reps); do
  for i in "${!V[@]}"; do
    env ${V[$i]} timeout -k 10 200 python tools/fixup_bench.py 96 > $out/fix_${i}_$r.log 2>&1 || { tail -5 $out/fix_${i}_$r.log; exit 1; }
    echo "$i [${V[$i]}] $(grep '^{' $out/fix_${i}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fixup_ms"])')"
  done
done
