set -o pipefail
mkdir -p gpurun_out/r04s
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py -k "two_level or real_df or unwrap or large_frames" > gpurun_out/r04s/tests.log 2>&1 && tail -2 gpurun_out/r04s/tests.log &&
FCD_LIB=trapped-modes-ltg_amd/build_stamps/libfcd_stamps.so timeout -k 10 200 python tools/t0_stamps.py > gpurun_out/r04s/stamps.log 2>&1 && cat gpurun_out/r04s/stamps.log &&
bash tools/ab.sh r04s 3 'python tools/fixup_bench.py 96' batch loop@
