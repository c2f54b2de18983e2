"""Wrapped-phase error of the engine against the f64 oracle (tuning tool, GPU):
max / 99.99th percentile / median |wrap(ours - oracle)| over synthetic 1024^2 frames,
for the library named by FCD_LIB (e.g. builds with different FCD_ATAN_TERMS)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]

from bench_data import make_frames_numpy  # noqa: E402
from oracle import fcd_oracle as O  # noqa: E402
from pyfcd import _lib  # noqa: E402


def main():
    n, count = 1024, int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ref, frames = make_frames_numpy(n, count, seed=3, rotate_deg=5.0)
    eng = _lib.Engine((n, n))
    eng.set_reference(ref, 0.001)
    _, w, _ = eng.process(frames, 1.0, unwrap=True, want_phases=True)
    errs = []
    for f in range(count):
        wo = O.compute_height_map(ref, frames[f], 0.001, height=1.0)[3]["wrapped"]
        for m in range(2):
            d = np.asarray(w[f, m], np.float64) - np.asarray(wo[m], np.float64)
            errs.append(np.abs((d + np.pi) % (2 * np.pi) - np.pi).ravel())
    e = np.concatenate(errs)
    print(json.dumps({"lib": os.environ.get("FCD_LIB", "default"), "frames": count, "max": float(e.max()),
                      "p9999": float(np.quantile(e, 0.9999)), "p99": float(np.quantile(e, 0.99)),
                      "median": float(np.median(e))}))


if __name__ == "__main__":
    main()
