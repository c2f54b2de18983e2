#!/bin/bash
# Fused 4096 kernel: parity (2048 + 4096 fused tests), kbench at 4096, c5 bench fused vs unfused.
set -o pipefail
out=gpurun_out/r03f4; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "fused or 2048 or 4096" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $out/pytest.log | tail -14
timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 4096 16 10 > $out/kb4096.txt 2>&1 || { tail -5 $out/kb4096.txt; exit 1; }
grep -E "phase_rows|demod_phase|int_rows k1" $out/kb4096.txt
timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench4096.log 2>&1 || { tail -20 $out/bench4096.log; exit 1; }
FCD_FUSED_4096=0 timeout -k 10 400 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench4096_unfused.log 2>&1 || { tail -20 $out/bench4096_unfused.log; exit 1; }
for f in bench4096 bench4096_unfused; do grep '^{' $out/$f.log | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); print('$f', b['value'], b['stage_us_per_frame'])"; done
