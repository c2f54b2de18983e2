set -o pipefail
for a in ${ABLS:-0 0_d 8_d}; do
  echo "abl $a"; timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench_abl_$a 1024 32 5 | grep -E "phase_rows|wave" || exit 1
done
