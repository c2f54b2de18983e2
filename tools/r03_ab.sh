#!/bin/bash
# Interleaved A/B/... of engine runtime switches on the headline bench (no CPU
# baseline, no real-frame side measurement), then the GPU parity suite.
# Usage: bash tools/r03_ab.sh TAG "ENV_A;ENV_B;..." [reps]   (an empty ENV = defaults)
set -o pipefail
out=gpurun_out/$1; IFS=';' read -ra V <<< "$2"; reps=${3:-3}
mkdir -p $out
for r in $(seq $reps); do
  for i in "${!V[@]}"; do
    e=${V[$i]}
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-real-frames > $out/bench_${i}_$r.log 2>&1 || { echo "bench $i failed"; tail -20 $out/bench_${i}_$r.log; exit 1; }
    echo "$i [$e] $(grep '^{' $out/bench_${i}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
fi
