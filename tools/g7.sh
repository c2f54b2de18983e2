set -o pipefail
for nb in 8 16 32 64; do echo "nb $nb"; timeout -k 10 120 trapped-modes-ltg_amd/tools/kbench 1024 $nb 5 | grep -E "chain x1|band|int_rows k1|int_cols|int_c2r|demod_rows|demod_cols" || exit 1; done
