# The bench line's residue_frames / generic_hd_frames under the current library and an
# alternative environment (e.g. FCD_LIB=... or a switch), interleaved.
# Usage (repo root on the box): bash tools/diag/resid_ab.sh "ENV_ALT" [runs]
set -o pipefail
ALT=$1; runs=${2:-2}
mkdir -p gpurun_out/resid
for r in $(seq $runs); do
  for v in cur alt; do
    e="FCD_X=1"; [ $v = alt ] && e="$ALT"
    env $e timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/resid/${v}_$r.log 2>&1 || { tail -5 gpurun_out/resid/${v}_$r.log; exit 1; }
    python - gpurun_out/resid/${v}_$r.log $v $r <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], sys.argv[3], "value", d["value"], "residue", d["residue_frames"]["value"], "generic", d["generic_hd_frames"]["value"])
PY
  done
done
