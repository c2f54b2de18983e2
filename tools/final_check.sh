#!/bin/bash
# Round-end style GPU pass without the (flaky) PMC traffic passes:
# parity suite, smoke, bench (with CPU baselines), rocprofv3 kernel stats, residue-frame bench.
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -40 $out/bench.log; exit 1; }
tail -1 $out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o run -- python3 bench.py --no-cpu-baseline > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -40 $out/prof.log; exit 1; }
grep '^{' $out/prof.log > $out/prof_bench.json
timeout -k 10 300 python tools/fixup_bench.py 96 > $out/fixup.log 2>&1 || { echo "fixup bench failed"; tail -20 $out/fixup.log; exit 1; }
tail -1 $out/fixup.log
