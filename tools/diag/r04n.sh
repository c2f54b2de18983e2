set -o pipefail
mkdir -p gpurun_out/r04n
L=trapped-modes-ltg_amd/build_libvar/zt16/libfcd.so
FCD_LIB=$L timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ingest.py -k "fused or batch_equals or full_size_1024 or exact_first or real_df or early" > gpurun_out/r04n/tests.log 2>&1 && tail -3 gpurun_out/r04n/tests.log &&
bash tools/ab.sh r04n 3 'python bench.py --no-cpu-baseline --no-real-frames' base zt16@ &&
bash tools/ab.sh r04n 2 'python tools/fixup_bench.py 96' fbase zt16@ &&
FCD_LIB=$L bash tools/traffic.sh r04n/traffic_zt16
