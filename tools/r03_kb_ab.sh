#!/bin/bash
# Interleaved kbench runs of tools/kvar.sh variants at one size.
# Usage: bash tools/r03_kb_ab.sh TAG "V1 V2 ..." N FRAMES [reps]
set -o pipefail
out=gpurun_out/$1; vars=$2; n=$3; nb=$4; reps=${5:-2}
mkdir -p $out
for r in $(seq $reps); do
  for v in $vars; do
    timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_$v $n $nb 10 > $out/kb_${v}_${n}_$r.txt 2>&1 || { echo "kbench $v failed"; tail -5 $out/kb_${v}_${n}_$r.txt; exit 1; }
  done
done
for v in $vars; do echo "$v $(cat $out/kb_${v}_${n}_*.txt | awk '{printf "%s=%s ", $1, $(NF-3)}')"; done
