#!/bin/bash
set -o pipefail
out=gpurun_out/r03cg6; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "unwrap or real" > $out/pytest_unwrap.log 2>&1 || { tail -30 $out/pytest_unwrap.log; exit 1; }
tail -1 $out/pytest_unwrap.log
for rep in 1 2; do
  timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_pre.$rep.log 2>&1 || { tail -20 $out/fix_pre.$rep.log; exit 1; }
  FCD_LIB=trapped-modes-ltg_amd/build_libvar/nopre/libfcd.so timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_nopre.$rep.log 2>&1 || { tail -20 $out/fix_nopre.$rep.log; exit 1; }
done
for f in $out/fix*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fixup_ms"])')"; done
