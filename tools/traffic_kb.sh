#!/bin/bash
# HBM traffic of the engine's kernels from rocprofv3 PMC counters over the kernel
# micro-benchmark (full 256-frame launches at 1024^2, no torch / reference setup in
# the profiled process): FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel
# trace only), plus the membench calibration copies of known byte counts.
# Then: python tools/traffic_summary.py gpurun_out/<tag> --chunk 256
set -o pipefail
tag=${1:-traffic_kb}; N=${2:-1024}; nb=${3:-256}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
kb=${KB:-trapped-modes-ltg_amd/tools/kbench}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -f csv -d $out/$c -o run -- $kb $N $nb 1 > $out/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $out/$c.log; exit 1; }
  echo "pmc $c done"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $out/cal_$c -o run -- trapped-modes-ltg_amd/tools/membench cal > $out/cal_$c.log 2>&1 || { echo "calibration $c failed"; tail -5 $out/cal_$c.log; exit 1; }
done
echo traffic passes done
