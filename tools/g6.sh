set -o pipefail
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 8 20 || exit 1
timeout -k 10 60 trapped-modes-ltg_amd/tools/kbench 1024 16 10 | grep chain || exit 1
