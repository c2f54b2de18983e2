set -o pipefail
mkdir -p gpurun_out/r01an
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01an/pytest.log 2>&1 || { tail -30 gpurun_out/r01an/pytest.log; exit 1; }
tail -1 gpurun_out/r01an/pytest.log
timeout -k 10 300 python tools/fixup_bench.py 96 > gpurun_out/r01an/fixup.log 2>&1 || { tail -20 gpurun_out/r01an/fixup.log; exit 1; }
tail -1 gpurun_out/r01an/fixup.log
