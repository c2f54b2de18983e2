#!/bin/bash
# Direct-load k_int_c2r for wide rows: kbench A/B (direct vs staged) at 2048 and 4096,
# then the wide-size parity tests on the product library.
set -o pipefail
out=gpurun_out/r03c2r; mkdir -p $out
export TMPDIR=/tmp
bash tools/r03_kb_ab.sh r03c2r "c2rD c2rS" 4096 16 3 || exit 1
bash tools/r03_kb_ab.sh r03c2r "c2rD c2rS" 2048 64 3 || exit 1
grep -h "int_c2r" $out/kb_*_4096_1.txt $out/kb_*_2048_1.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "2048 or 4096 or wide or fused" > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
