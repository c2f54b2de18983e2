#!/bin/bash
# GPU pass for a kernel change: parity suite, kbench variants (tools/bin/kbench_*, each
# twice, interleaved), and the bench.  Usage: bash tools/r03_kvar.sh <tag> [N] [nb] [pytest-k]
set -o pipefail
tag=$1; N=${2:-1024}; nb=${3:-256}; sel=${4:-}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$sel" ]; then kopt=(-k "$sel"); else kopt=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider "${kopt[@]}" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for k in trapped-modes-ltg_amd/tools/bin/kbench_*; do
    v=$(basename $k)
    timeout -k 10 120 $k $N $nb 10 > $out/$v.$rep.txt 2>&1 || { echo "$v failed"; tail -5 $out/$v.$rep.txt; exit 1; }
  done
done
for k in trapped-modes-ltg_amd/tools/bin/kbench_*; do v=$(basename $k); echo "== $v"; grep -hE "band_phase|phase_rows|int_cols|int_c2r|demod_rows|demod_cols|int_rows" $out/$v.1.txt $out/$v.2.txt | sort; done
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); print('bench', b['value'], b['roofline']['frac'], b['stage_us_per_frame'])"
