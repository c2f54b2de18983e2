#!/bin/bash
# Tile shapes of the MST tile pass: parity, then residue-frame bench per shape.
set -o pipefail
out=gpurun_out/r03cg5; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "unwrap or real" > $out/pytest_unwrap.log 2>&1 || { tail -30 $out/pytest_unwrap.log; exit 1; }
tail -1 $out/pytest_unwrap.log
for rep in 1 2; do
  for t in 64 6432 32; do
    FCD_MST_TILE=$t timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix$t.$rep.log 2>&1 || { tail -20 $out/fix$t.$rep.log; exit 1; }
  done
done
for f in $out/fix*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fixup_ms"])')"; done
FCD_MST_TILE=6432 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/p6432 -o run -- python3 tools/fixup_bench.py 96 > $out/p6432.log 2>&1 || { tail -20 $out/p6432.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/p64 -o run -- python3 tools/fixup_bench.py 96 > $out/p64.log 2>&1 || { tail -20 $out/p64.log; exit 1; }
echo done
