#!/bin/bash
set -o pipefail
out=gpurun_out/r03cg4; mkdir -p $out
export TMPDIR=/tmp
FCD_LIB=trapped-modes-ltg_amd/build_stamps/libfcd_stamps.so FCD_MST_LEVEL=2 timeout -k 10 180 python tools/t0_stamps.py > $out/stamps_l2.log 2>&1 || { tail -20 $out/stamps_l2.log; exit 1; }
cat $out/stamps_l2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/p3 -o run -- python3 tools/fixup_bench.py 96 > $out/p3.log 2>&1 || { tail -20 $out/p3.log; exit 1; }
FCD_MST_LEVEL=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/p2 -o run -- python3 tools/fixup_bench.py 96 > $out/p2.log 2>&1 || { tail -20 $out/p2.log; exit 1; }
echo done
