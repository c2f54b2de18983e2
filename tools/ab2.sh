# A/B of an environment switch on the c2 bench (and optionally c3 / c5), interleaved.
# Usage (repo root on the box): bash tools/ab2.sh TAG "ENV_A" "ENV_B" [runs] [sizes]
set -o pipefail
tag=$1; A=$2; B=$3; runs=${4:-2}; sizes=${5:-1024}
out=gpurun_out/$tag; mkdir -p $out
for n in $sizes; do
  case $n in
    1024) args="--no-cpu-baseline --no-real-frames";;
    2048) args="--size 2048 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-real-frames";;
    4096) args="--size 4096 --batch 64 --steps 5 --warmup 1 --no-cpu-baseline --no-real-frames";;
  esac
  for r in $(seq $runs); do
    for v in A B; do
      e=$A; [ $v = B ] && e=$B
      env $e timeout -k 10 300 python bench.py $args > $out/${n}_${v}_$r.log 2>&1 || { tail -20 $out/${n}_${v}_$r.log; exit 1; }
      python - $out/${n}_${v}_$r.log "$n $v $r [$e]" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "value", d["value"], "frac", d["roofline"]["frac"], "us/launch", d["roofline"]["us_per_launch"], "stages", d.get("stage_us_per_frame"))
PY
    done
  done
done
