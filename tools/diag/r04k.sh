set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_mixed.py -k "two_level or real_df or unwrap or residue or census or large or mixed_frames" > gpurun_out/r04k/tests.log 2>&1 && tail -3 gpurun_out/r04k/tests.log &&
bash tools/measure.sh r04k fixup &&
FCD_MST_DEBUG=1 timeout -k 10 200 python tools/fixup_bench.py 96 > gpurun_out/r04k/mstdebug.log 2>&1 &&
FCD_LIB=trapped-modes-ltg_amd/build_stamps/libfcd_stamps.so timeout -k 10 200 python tools/t0_stamps.py > gpurun_out/r04k/stamps.log 2>&1 &&
bash tools/ab.sh r04k 2 'python tools/fixup_bench.py 96' f9 f6:FCD_CG_FIRST=6 f12:FCD_CG_FIRST=12 f7:FCD_CG_FIRST=7
