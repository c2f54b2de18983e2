#!/bin/bash
# k_demod_cols at 16 elements per lane at 4096 points: GPU suite, then c5 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03dc2; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for r in 1 2; do
timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames > $out/c5_$r.log 2>&1 || { tail -20 $out/c5_$r.log; exit 1; }
grep '^{' $out/c5_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_us_per_frame"])'
done
