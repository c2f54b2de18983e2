#!/bin/bash
# k_int_c2r with 8-row blocks at 2048 points: GPU suite, then c3 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03c2r8; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for r in 1 2; do
timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-real-frames > $out/c3_$r.log 2>&1 || { tail -20 $out/c3_$r.log; exit 1; }
grep '^{' $out/c3_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_us_per_frame"])'
done
