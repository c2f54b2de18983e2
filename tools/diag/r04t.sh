set -o pipefail
mkdir -p gpurun_out/r04t
bash tools/ab.sh r04t 3 'python tools/fixup_bench.py 96' ru5 ru1@ ru2@
