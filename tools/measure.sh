#!/bin/bash
# Measurement pass on one MI355X (round 4): headline bench with the CPU baseline, its
# rocprofv3 kernel stats, PMC traffic (FETCH_SIZE / WRITE_SIZE passes), the real-frame
# (exact MST) bench with its kernel stats, and the c3 / c5 frame sizes with their own
# kernel stats and PMC traffic passes.
# Usage (repo root on the box): bash tools/measure.sh TAG [steps]
#   steps: comma list of bench,prof,traffic,fixup,c3,c3prof,c3traffic,c5,c5prof,c5traffic
set -o pipefail
tag=${1:-r04m}
steps=${2:-bench,prof,traffic,fixup,c3,c3prof,c3traffic,c5,c5prof,c5traffic}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
want() { [[ ",$steps," == *",$1,"* ]]; }
C3="--size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline"
C5="--size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline"
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
for cfg in c3 c5; do
  args=$C3; [ $cfg = c5 ] && args=$C5
  n=2048; [ $cfg = c5 ] && n=4096
  if want $cfg; then
    step $cfg
    timeout -k 10 500 python bench.py $args > $out/bench$n.log 2>&1 || { tail -20 $out/bench$n.log; exit 1; }
  fi
  if want ${cfg}prof; then
    step ${cfg}prof
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $out/prof$n -o run -- python3 bench.py $args > $out/prof$n.log 2>&1 || { tail -20 $out/prof$n.log; exit 1; }
    grep '^{' $out/prof$n.log > $out/prof_bench$n.json
  fi
  if want ${cfg}traffic; then
    step ${cfg}traffic
    # one launch chunk per step (64 frames at 2048^2, 16 at 4096^2)
    b=64; [ $cfg = c5 ] && b=16
    bash tools/traffic.sh $tag/traffic$n "--size $n --batch $b" || exit 1
  fi
done
step done
for f in bench fixup bench2048 bench4096; do [ -f $out/$f.log ] && grep '^{' $out/$f.log | tail -1 | cut -c1-400; done; true
