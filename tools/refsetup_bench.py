"""Many-reference setup throughput: fcd_find_peaks over a stack of
1024^2 references (rotated boards with seeded warps), batched on the device (means, FFTs,
|F| * highpass, candidates, 8-connected labelling, peak pick), against the host
labelling of the same device candidates (FCD_HOST_LABEL=1) and the CPU oracle's
fourier.find_peaks on one core.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    from pyfcd import _lib
    from bench_data import make_frames_numpy
    from oracle import fcd_oracle as O
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ref, frames = make_frames_numpy(1024, n, seed=1, rotate_deg=5.0)
    eng = _lib.Engine(ref.shape)
    eng.find_peaks(frames[:2], 0.001)  # warm-up (workspace, code objects)
    out = {"metric": "reference setups/s (fcd_find_peaks, 1024x1024, host stack in)", "images": n}
    for label, env in (("device_labelling", None), ("host_labelling", "1")):
        if env:
            os.environ["FCD_HOST_LABEL"] = env
        t0 = time.perf_counter()
        infos = eng.find_peaks(frames, 0.001)
        dt = time.perf_counter() - t0
        os.environ.pop("FCD_HOST_LABEL", None)
        out[label] = round(n / dt, 1)
        out[label + "_peaks0"] = np.ctypeslib.as_array(infos[0].peaks).tolist()
    m = min(n, 8)
    t0 = time.perf_counter()
    for f in frames[:m]:
        O.find_peaks(f)
    out["cpu_oracle_1core"] = round(m / (time.perf_counter() - t0), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
