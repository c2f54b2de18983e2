set -o pipefail
mkdir -p gpurun_out/r04aj
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ingest.py -k "exact_first" > gpurun_out/r04aj/tests_ef.log 2>&1 && tail -1 gpurun_out/r04aj/tests_ef.log &&
FCD_LIB=trapped-modes-ltg_amd/build_libvar/jump/libfcd.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "two_level or real_df or unwrap" > gpurun_out/r04aj/tests.log 2>&1 && tail -1 gpurun_out/r04aj/tests.log &&
bash tools/ab.sh r04aj 3 'python tools/fixup_bench.py 96' walk jump@
