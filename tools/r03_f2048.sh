#!/bin/bash
# Fused 2048 kernel: parity first, then kbench at 2048 and the c3 bench (fused vs unfused).
set -o pipefail
out=gpurun_out/r03f; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "fused or 2048" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $out/pytest.log | tail -12
timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 2048 64 10 > $out/kb2048.txt 2>&1 || { tail -5 $out/kb2048.txt; exit 1; }
cat $out/kb2048.txt
timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench2048.log 2>&1 || { tail -20 $out/bench2048.log; exit 1; }
FCD_FUSED_2048=0 timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench2048_unfused.log 2>&1 || { tail -20 $out/bench2048_unfused.log; exit 1; }
for f in bench2048 bench2048_unfused; do grep '^{' $out/$f.log | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); print('$f', b['value'], b['stage_us_per_frame'])"; done
