set -o pipefail
mkdir -p gpurun_out/r04y
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "two_level or real_df or unwrap" > gpurun_out/r04y/tests.log 2>&1 && tail -1 gpurun_out/r04y/tests.log &&
bash tools/ab.sh r04y 3 'python tools/fixup_bench.py 96' r1 head@
