set -o pipefail
for c in ${CHUNKS:-8 16 32}; do
  FCD_CHUNK_MB=8192 FCD_CHUNK_MAX=$c timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c$c.log 2>&1 || { tail -5 gpurun_out/bench_c$c.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_c$c.log').read().strip().splitlines()[-1]);print('chunk $c', d['value'], d['stage_us_per_frame'])"
done
