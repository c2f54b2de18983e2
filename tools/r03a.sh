#!/bin/bash
# Round-3 GPU pass: parity suite (verbose, per-test timeout), smoke, bench N=1, and the
# self-launched 2-rank bench (gloo, ranks sharing the box's one GPU) with the gather.
# Usage (repo root on the box): bash tools/r03a.sh <tag>
set -o pipefail
tag=${1:-r03a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider \
    > $out/pytest_gpu.log 2>&1
rc=$?
tail -3 $out/pytest_gpu.log
grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20
case $rc in 0|1) ;; *) echo "pytest rc $rc: stop"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log
FCD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --batch 64 --steps 10 --gather > $out/bench_n2.log 2>&1 || { tail -30 $out/bench_n2.log; exit 1; }
grep '^{' $out/bench_n2.log
exit $rc
