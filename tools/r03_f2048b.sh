#!/bin/bash
set -o pipefail
out=gpurun_out/r03f2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fused or 2048" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 2048 64 10 > $out/kb2048.$rep.txt 2>&1 || { tail -5 $out/kb2048.$rep.txt; exit 1; }; done
grep -h "phase_rows" $out/kb2048.*.txt
timeout -k 10 500 python bench.py --size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench2048.log 2>&1 || { tail -20 $out/bench2048.log; exit 1; }
grep '^{' $out/bench2048.log | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); print('bench2048', b['value'], b['stage_us_per_frame'])"
