set -o pipefail
mkdir -p gpurun_out/r04ac
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_mixed.py tests/test_gpu_ingest.py -k "two_level or real_df or unwrap or large or mixed_frames or exact or fixup or census" > gpurun_out/r04ac/tests.log 2>&1 && tail -1 gpurun_out/r04ac/tests.log &&
bash tools/ab.sh r04ac 3 'python tools/fixup_bench.py 96' kfused fin@
