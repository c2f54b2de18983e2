mkdir -p gpurun_out/r02h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02h/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02h/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02h/pytest_gpu.log
timeout -k 10 300 python tools/fixup_bench.py 96 > gpurun_out/r02h/fixup_new.log 2>&1 && tail -1 gpurun_out/r02h/fixup_new.log
FCD_MST_LEVEL=0 timeout -k 10 300 python tools/fixup_bench.py 96 > gpurun_out/r02h/fixup_old.log 2>&1 && tail -1 gpurun_out/r02h/fixup_old.log
