set -o pipefail
for v in zt16_1024 zt8_512 zt4_256 zt8_1024; do echo "== $v"; timeout -k 10 120 trapped-modes-ltg_amd/tools/bin/kbench_$v 1024 32 5 | grep -E "chain x1|int_rows k1|int_cols" || exit 1; done
