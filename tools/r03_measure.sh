#!/bin/bash
# Round-3 measurement pass on one MI355X: headline bench (with the CPU baseline),
# its rocprofv3 kernel stats, the PMC traffic passes over the same command, the
# residue-bearing real-frame bench with its kernel stats, and the c3 / c5 frame sizes.
# Usage (repo root on the box): bash tools/r03_measure.sh <tag>
set -o pipefail
tag=${1:-r03m}
steps=${2:-bench,prof,traffic,fixup,c3,c5}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
want() { [[ ",$steps," == *",$1,"* ]]; }
if want bench; then
step bench
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
fi
if want prof; then
step prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o run -- python3 bench.py --no-cpu-baseline > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
grep '^{' $out/prof.log > $out/prof_bench.json
fi
if want traffic; then
step traffic
bash tools/traffic.sh $tag/traffic || exit 1
fi
if want fixup; then
step fixup
timeout -k 10 300 python tools/fixup_bench.py 96 > $out/fixup.log 2>&1 || { tail -20 $out/fixup.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/fixprof -o run -- python3 tools/fixup_bench.py 96 > $out/fixprof.log 2>&1 || { tail -20 $out/fixprof.log; exit 1; }
fi
if want c3; then
step c3
timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench2048.log 2>&1 || { tail -20 $out/bench2048.log; exit 1; }
fi
if want c5; then
step c5
timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench4096.log 2>&1 || { tail -20 $out/bench4096.log; exit 1; }
fi
step done
for f in bench fixup bench2048 bench4096; do [ -f $out/$f.log ] && grep '^{' $out/$f.log | tail -1 | cut -c1-400; done; true
