# SQ counters of the c3 / c5 demod launch groups (tools/diag/demod_sq.sh per size)
set -o pipefail
TAG=${TAG:-r06g}
TAG=${TAG}_2048 bash tools/diag/demod_sq.sh --size 2048 --batch 128 --steps 2 --warmup 1 --no-cpu-baseline --no-real-frames > /dev/null 2>&1 || { echo c3 failed; exit 1; }
python3 tools/diag/sq_md.py gpurun_out/${TAG}_2048 128 > gpurun_out/${TAG}_2048/sq.md
TAG=${TAG}_4096 bash tools/diag/demod_sq.sh --size 4096 --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --no-real-frames > /dev/null 2>&1 || { echo c5 failed; exit 1; }
python3 tools/diag/sq_md.py gpurun_out/${TAG}_4096 32 > gpurun_out/${TAG}_4096/sq.md
echo done
