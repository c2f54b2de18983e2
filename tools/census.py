"""Residue census of the bench recipe on the GPU: frames [0, total) in chunks."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]
import torch  # must load before the engine library (shared HIP runtime SONAME)
import numpy as np
import bench_data
from pyfcd import _lib
n, total = 1024, int(sys.argv[1])
for amp in [float(a) for a in sys.argv[2:]]:
    bench_data.AMP = amp
    bad = []
    eng = _lib.Engine((n, n))
    for b0 in range(0, total, 128):
        ref_t, frames = bench_data.make_frames_torch(n, 128, seed=b0, device="cuda")
        if b0 == 0:
            eng.set_reference(ref_t.cpu().numpy(), bench_data.SQUARE_SIZE)
        _, w, _ = eng.process(frames.cpu().numpy(), 1.0, unwrap=False)
        _, res = eng.unwrap(w.reshape(-1, n, n))
        bad += [b0 + i for i, r in enumerate(res.reshape(-1, 2)) if r.any()]
    print(f"amp {amp}: {len(bad)} of {total} frames with residues {bad[:20]}", flush=True)
