#!/bin/bash
set -o pipefail
out=gpurun_out/r03ef; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_auto.$rep.log 2>&1 || { tail -20 $out/fix_auto.$rep.log; exit 1; }
  FCD_EXACT_FIRST=0 timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_two.$rep.log 2>&1 || { tail -20 $out/fix_two.$rep.log; exit 1; }
done
for f in $out/fix*.log; do echo "$f: $(grep '^{' $f)"; done
