set -o pipefail
L=$PWD/trapped-modes-ltg_amd/build_libvar/r05/libfcd.so
for r in 1 2 3; do
  for v in cur r05; do
    if [ $v = r05 ]; then e="FCD_LIB=$L"; else e="FCD_X=1"; fi
    env $e timeout -k 10 120 python tools/fixup_bench.py 96 > gpurun_out/fx_${v}_$r.log 2>&1 || { tail -5 gpurun_out/fx_${v}_$r.log; exit 1; }
    echo $v $r $(grep -o '"value": [0-9.]*' gpurun_out/fx_${v}_$r.log | tail -1)
  done
done
