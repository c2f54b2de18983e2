# Kernel trace of the c2 headline steps (tools/diag/timeline.py).  TAG=... bash tools/diag/timeline.sh
set -o pipefail
out=gpurun_out/${TAG:-r06tl}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $out/tr -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-real-frames > $out/tr.log 2>&1 || { tail -20 $out/tr.log; exit 1; }
python3 tools/diag/timeline.py $out/tr/run_kernel_trace.csv --steps 6 --warmup 2 | tee $out/timeline.txt
