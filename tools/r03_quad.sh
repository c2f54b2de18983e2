#!/bin/bash
# k_int_cols quad item order at 4096 (4-row Zt tiles): parity, kbench A/B at 4096 and
# 1024, and PMC Zt reads of the quad build at 4096.
set -o pipefail
out=gpurun_out/r03q; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for v in quad noquad; do
    timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_$v 4096 16 10 > $out/kb4096_$v.$rep.txt 2>&1 || { echo "$v failed"; tail -5 $out/kb4096_$v.$rep.txt; exit 1; }
  done
done
for v in quad noquad; do echo "== $v"; grep -h int_cols $out/kb4096_$v.*.txt; done
KB=trapped-modes-ltg_amd/tools/bin/kbench_quad bash tools/traffic_kb.sh r03q/traffic 4096 16 || exit 1
