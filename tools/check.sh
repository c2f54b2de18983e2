#!/bin/bash
# GPU pass: parity suite (or a -k subset), smoke, bench.
# Usage: bash tools/check.sh TAG [pytest -k expr]
set -o pipefail
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
sel=()
[ -n "$2" ] && sel=(-k "$2")
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" > $out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -60 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
[ -n "$2" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -40 $out/bench.log; exit 1; }
tail -1 $out/bench.log
