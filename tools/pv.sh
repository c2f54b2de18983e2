#!/bin/bash
# Parity suite + kbench variants (tuning pass).  Usage: bash tools/pv.sh <tag> [N] [nb]
set -o pipefail
tag=$1; N=${2:-1024}; nb=${3:-256}
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
bash tools/kvar_run.sh $tag $N $nb
