#!/bin/bash
set -o pipefail
out=gpurun_out/r03cg7; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ingest.py tests/test_analyze_ref.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix.$rep.log 2>&1 || { tail -20 $out/fix.$rep.log; exit 1; }; done
for f in $out/fix*.log; do echo "$f: $(grep '^{' $f)"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/p -o run -- python3 tools/fixup_bench.py 96 > $out/p.log 2>&1 || { tail -20 $out/p.log; exit 1; }
echo done
