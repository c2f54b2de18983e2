# A/B/n of environment switches on one bench size, interleaved.
# Usage (repo root on the box): bash tools/abn.sh TAG SIZE RUNS "ENV_1" "ENV_2" ...
set -o pipefail
tag=$1; n=$2; runs=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
case $n in
  1024) args="--no-cpu-baseline --no-real-frames";;
  2048) args="--size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-real-frames";;
  4096) args="--size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames";;
esac
for r in $(seq $runs); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py $args > $out/${n}_${i}_$r.log 2>&1 || { tail -20 $out/${n}_${i}_$r.log; exit 1; }
    python - $out/${n}_${i}_$r.log "$n v$i r$r [$e]" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "value", d["value"], "frac", d["roofline"]["frac"], "us/launch", d["roofline"]["us_per_launch"])
PY
  done
done
