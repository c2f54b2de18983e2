set -o pipefail
out=gpurun_out/r06h; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
L=trapped-modes-ltg_amd/build_libvar
bash tools/ab2.sh r06h FCD_LIB=$L/nt1/libfcd.so FCD_X=0 2 "1024 2048" && bash tools/ab2.sh r06h2 FCD_LIB=$L/pr0/libfcd.so FCD_X=0 2 "1024"
