#!/bin/bash
# Component-graph MST rounds: unwrap parity first, then the whole GPU suite, the
# residue-frame bench A/B (default vs FCD_MST_LEVEL=2) and its kernel profile.
set -o pipefail
out=gpurun_out/r03cg; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "unwrap" > $out/pytest_unwrap.log 2>&1 || { tail -30 $out/pytest_unwrap.log; exit 1; }
tail -1 $out/pytest_unwrap.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_cg.$rep.log 2>&1 || { tail -20 $out/fix_cg.$rep.log; exit 1; }
  FCD_MST_LEVEL=2 timeout -k 10 180 python tools/fixup_bench.py 96 > $out/fix_l2.$rep.log 2>&1 || { tail -20 $out/fix_l2.$rep.log; exit 1; }
done
for f in $out/fix_*.log; do echo "$f: $(grep '^{' $f | head -c 300)"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/fixprof -o run -- python3 tools/fixup_bench.py 96 > $out/fixprof.log 2>&1 || { tail -20 $out/fixprof.log; exit 1; }
echo prof done
