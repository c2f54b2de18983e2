set -o pipefail
mkdir -p gpurun_out/r04ag
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_mixed.py -k "two_level or real_df or unwrap or large or mixed_frames or exact" > gpurun_out/r04ag/tests.log 2>&1 && tail -1 gpurun_out/r04ag/tests.log &&
bash tools/ab.sh r04ag 3 'python tools/fixup_bench.py 96' hash nohash@ &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04ag/fixprof -o run -- python3 tools/fixup_bench.py 96 > gpurun_out/r04ag/fixprof.log 2>&1
