"""Diagnostic (GPU): which bench frames does the fast path send to the exact
fix-up pass, and do they really carry residues?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]
import numpy as np, torch
from pyfcd import _lib
from bench_data import make_frames_torch, SQUARE_SIZE
n, B = 1024, int(sys.argv[1]) if len(sys.argv) > 1 else 64
ref_t, frames = make_frames_torch(n, B, seed=0, device="cuda")
eng = _lib.Engine((n, n))
eng.set_reference(ref_t.cpu().numpy(), SQUARE_SIZE)
fr = frames.cpu().numpy()
eng.profile(True)
h, w, k = eng.process(fr, 1.0, unwrap=True)
st, nf = eng.stage_times()
print("fixup frames", st["fixup_frames"], "of", nf)
kk, res = eng.unwrap(w.reshape(-1, n, n))
res = res.reshape(B, 2)
print("frames with residues (exact census):", [(i, r.tolist()) for i, r in enumerate(res) if r.any()])
