#!/bin/bash
# HBM traffic of the bench command from rocprofv3 PMC counters (MI355X_MICROARCH.md
# §HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel
# trace only), plus a calibration pass over streaming copies of known byte counts
# at 4 / 8 / 16 B per lane.  Then: python tools/traffic_summary.py gpurun_out/<tag>
# Usage: bash tools/traffic.sh TAG [extra bench.py args, e.g. "--size 2048 --batch 64"]
set -o pipefail
tag=${1:-traffic}
extra=${2:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
# heartbeat: PMC passes serialise every dispatch and can stay silent for minutes
( while sleep 30; do date +%T >> $out/heartbeat.txt; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for c in FETCH_SIZE WRITE_SIZE; do
  # counters on the engine's kernels only: the on-device frame generator's thousands of
  # small torch kernels are left out of the (dispatch-serialising) counter collection
  timeout -k 10 420 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex 'fcdk' -f csv -d $out/$c -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-real-frames $extra > $out/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $out/$c.log; exit 1; }
  echo "pmc $c done"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $out/cal_$c -o run -- trapped-modes-ltg_amd/tools/membench cal > $out/cal_$c.log 2>&1 || { echo "calibration $c failed"; tail -5 $out/cal_$c.log; exit 1; }
done
echo traffic passes done
