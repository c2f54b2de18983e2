#!/bin/bash
# Wide k_int_cols at 16 elements per lane: GPU suite on the product library, then c3 / c5
# benches interleaved with the 8-element build (build_libvar/icW0).
set -o pipefail
out=gpurun_out/r03icw2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
for r in 1 2; do
  for v in new icW0; do
    if [ $v = icW0 ]; then export FCD_LIB=trapped-modes-ltg_amd/build_libvar/icW0/libfcd.so; else unset FCD_LIB; fi
    timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-real-frames > $out/c3_${v}_$r.log 2>&1 || { tail -20 $out/c3_${v}_$r.log; exit 1; }
    timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames > $out/c5_${v}_$r.log 2>&1 || { tail -20 $out/c5_${v}_$r.log; exit 1; }
    for c in c3 c5; do echo "$c $v $(grep '^{' $out/${c}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_us_per_frame"])')"; done
  done
done
