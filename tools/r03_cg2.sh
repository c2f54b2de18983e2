#!/bin/bash
# Component-graph MST: sizes per round, 64 vs 32 tiles, tile-pass phase split.
set -o pipefail
out=gpurun_out/r03cg2; mkdir -p $out
export TMPDIR=/tmp
FCD_MST_DEBUG=1 timeout -k 10 180 python tools/fixup_bench.py 96 > $out/dbg.log 2>&1 || { tail -20 $out/dbg.log; exit 1; }
grep "mst-cg" $out/dbg.log | head -24
for rep in 1 2; do
  timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix64.$rep.log 2>&1 || { tail -20 $out/fix64.$rep.log; exit 1; }
  FCD_MST_TILE=32 timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix32.$rep.log 2>&1 || { tail -20 $out/fix32.$rep.log; exit 1; }
done
for f in $out/fix*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fixup_ms"])')"; done
FCD_LIB=trapped-modes-ltg_amd/build_stamps/libfcd_stamps.so timeout -k 10 180 python tools/t0_stamps.py > $out/stamps.log 2>&1 || { tail -20 $out/stamps.log; exit 1; }
cat $out/stamps.log
