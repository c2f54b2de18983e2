set -o pipefail
out=gpurun_out/${TAG:-r04ay}
mkdir -p $out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex 'fcdk' -f csv -d $out/$c -o run -- python3 tools/fixup_bench.py 96 > $out/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $out/$c.log; exit 1; }
  echo "pmc $c done"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $out/cal_$c -o run -- trapped-modes-ltg_amd/tools/membench cal > $out/cal_$c.log 2>&1 || { echo "cal $c failed"; exit 1; }
done
echo done
