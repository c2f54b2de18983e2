set -o pipefail
mkdir -p gpurun_out/r03kb
for cfg in "2048 64" "4096 16" "1024 256"; do
  set -- $cfg
  timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_base $1 $2 10 > gpurun_out/r03kb/kb_$1.txt 2>&1 || { echo "kbench $1 failed"; tail -5 gpurun_out/r03kb/kb_$1.txt; exit 1; }
  echo "== $1"; cat gpurun_out/r03kb/kb_$1.txt
done
