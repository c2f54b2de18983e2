set -o pipefail
mkdir -p gpurun_out/r01au
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01au/pytest.log 2>&1 || { tail -30 gpurun_out/r01au/pytest.log; exit 1; }
tail -1 gpurun_out/r01au/pytest.log
timeout -k 10 300 python bench.py --size 2048 --batch 1024 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01au/b2048.log 2>&1 || { tail -20 gpurun_out/r01au/b2048.log; exit 1; }
grep '^{' gpurun_out/r01au/b2048.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['stage_us_per_frame'])"
timeout -k 10 300 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r01au/b4096.log 2>&1 || { tail -20 gpurun_out/r01au/b4096.log; exit 1; }
grep '^{' gpurun_out/r01au/b4096.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['stage_us_per_frame'])"
