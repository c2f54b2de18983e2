# bench at several fast-path chunk sizes (FCD_CHUNK_MAX): MALL residency vs launch tails
mkdir -p gpurun_out/$1
for c in 256 64 32 16; do
  FCD_CHUNK_MAX=$c timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/$1/bench_$c.log 2>&1 || exit 1
  echo "chunk $c: $(tail -1 gpurun_out/$1/bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_us_per_frame"])')"
done
