set -o pipefail
mkdir -p gpurun_out/r04af
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_ingest.py -k "real_df or unwrap or large or exact or fixup" > gpurun_out/r04af/tests.log 2>&1 && tail -1 gpurun_out/r04af/tests.log &&
for i in 1 2 3; do timeout -k 10 120 python tools/fixup_bench.py 96 | tail -1; done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04af/fixprof -o run -- python3 tools/fixup_bench.py 96 > gpurun_out/r04af/fixprof.log 2>&1
