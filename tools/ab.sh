#!/bin/bash
# Interleaved A/B runs on the GPU box (replaces round 3's one-off r03_*.sh scripts).
#
#   bash tools/ab.sh TAG REPS 'COMMAND' VARIANT...
#
# VARIANT is NAME (the product build, no extra environment), NAME:VAR=v[,VAR=v...]
# (environment switches), or NAME@ (the library build_libvar/NAME/libfcd.so made by
# trapped-modes-ltg_amd/tools/libvar.sh NAME "-D..." on the CPU side, through FCD_LIB).
# COMMAND runs REPS times per variant, variants interleaved within each repetition,
# each run under its own 300 s limit; its output goes to gpurun_out/TAG/NAME_REP.log and
# the last line of each is echoed.  Examples:
#   bash tools/ab.sh r04x 3 'python bench.py --no-cpu-baseline --no-real-frames' base one:FCD_STREAMS=1
#   bash tools/ab.sh r04y 2 'trapped-modes-ltg_amd/tools/kbench 1024 256 10' base v2@
set -o pipefail
tag=$1; reps=$2; cmd=$3; shift 3
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq $reps); do
  for v in "$@"; do
    name=${v%%[:@]*}
    envs=()
    case $v in
      *@) envs=(FCD_LIB=trapped-modes-ltg_amd/build_libvar/$name/libfcd.so) ;;
      *:*) IFS=, read -ra envs <<< "${v#*:}" ;;
    esac
    log=$out/${name}_$r.log
    env "${envs[@]}" timeout -k 10 300 $cmd > $log 2>&1 || { echo "$name run $r failed"; tail -20 $log; exit 1; }
    echo "$name $r: $(tail -1 $log | cut -c1-400)"
  done
done
