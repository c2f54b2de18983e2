set -o pipefail
out=gpurun_out/r06e; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames > $out/bench4096.log 2>&1 || { tail -30 $out/bench4096.log; exit 1; }
tail -1 $out/bench4096.log | cut -c1-200
TAG=r06e bash tools/diag/demod_sq.sh > $out/sq_run.log 2>&1 || { tail -20 $out/sq_run.log; exit 1; }
tail -3 $out/sq_run.log
