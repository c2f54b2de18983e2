set -o pipefail
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 32 5 | grep -E "band|phase_rows|chain x1" || exit 1
