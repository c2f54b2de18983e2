#!/bin/bash
# Run every kbench variant in trapped-modes-ltg_amd/tools/bin twice (interleaved). Usage: bash tools/kvar_run.sh <tag> [N] [nb]
set -o pipefail
tag=$1; N=${2:-1024}; nb=${3:-64}
out=gpurun_out/$tag; mkdir -p $out
for rep in 1 2; do
  for k in trapped-modes-ltg_amd/tools/bin/kbench_*; do
    v=$(basename $k)
    timeout -k 10 120 $k $N $nb 10 > $out/$v.$rep.txt 2>&1 || { echo "$v failed"; tail -5 $out/$v.$rep.txt; exit 1; }
  done
done
for k in trapped-modes-ltg_amd/tools/bin/kbench_*; do v=$(basename $k); echo "== $v"; grep -hE "band_phase|phase_rows|int_cols|int_c2r|demod_rows|demod_cols|int_rows|demod_phase" $out/$v.1.txt $out/$v.2.txt | sort; done
