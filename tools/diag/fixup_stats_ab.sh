# rocprof kernel stats of the real-frame pass for two library builds (FCD_LIB), hook kernels
set -o pipefail
out=gpurun_out/${TAG:-r04ba}
mkdir -p $out
export TMPDIR=/tmp
for v in base new; do
  FCD_LIB=trapped-modes-ltg_amd/build_libvar/$v/libfcd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/$v -o run -- python3 tools/fixup_bench.py 96 > $out/$v.log 2>&1 || { tail -5 $out/$v.log; exit 1; }
  grep -h "cg_hook\|mst_tile0\|cg_cand\"" $out/$v/run_kernel_stats.csv | cut -c1-200
done
