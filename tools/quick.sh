#!/bin/bash
# Quick GPU pass: parity suite + one bench line.  Usage: bash tools/quick.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 400 python bench.py "$@" > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log
