set -o pipefail
mkdir -p gpurun_out/r04ak
bash tools/ab.sh r04ak 3 'python bench.py --no-cpu-baseline --no-real-frames' s2 s1:FCD_STREAMS=1 ec0:FCD_EARLY_CENSUS=0 s1ec0:FCD_STREAMS=1,FCD_EARLY_CENSUS=0
