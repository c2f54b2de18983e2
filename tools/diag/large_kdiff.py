"""Diagnose a k-field mismatch of the engine against large.npz (GPU box): where, and whether
the engine's unwrap of its OWN wrapped phases equals the oracle's Herraez restatement."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: F401
import numpy as np
from bench_data import make_residue_frame
from oracle import fcd_oracle as O
from pyfcd import _lib
tag = sys.argv[1] if len(sys.argv) > 1 else "r4096"
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/kdiff"
os.makedirs(out, exist_ok=True)
g = np.load(os.path.join(ROOT, "tests/golden/large.npz"))
n = int(g[f"{tag}_n"])
ref, frame = make_residue_frame(n, [tuple(p) for p in g[f"{tag}_pairs"]], seed=int(g[f"{tag}_seed"]), rotate_deg=5.0, quantum=4096)
eng = _lib.Engine(ref.shape)
eng.set_reference(ref, 0.001)
h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
rep = {}
for m in range(2):
    d = k[0][m].astype(np.int64) - g[f"{tag}_k"][m]
    c = d[1:-1, 1:-1].flat[0]
    bad = np.argwhere(d != c)
    _, ko = O.unwrap(w[0][m])
    de = k[0][m].astype(np.int64) - ko
    rep[m] = {"mismatch": bad[:20].tolist(), "count": int(len(bad)),
              "engine_vs_oracle_on_engine_w": int((de != de.flat[0]).sum()),
              "residues_engine_w": O.count_residues(w[0][m])}
    for i, (r, cc) in enumerate(bad[:4]):
        r0, c0 = max(r - 8, 0), max(cc - 8, 0)
        np.save(f"{out}/{tag}_m{m}_w_{r}_{cc}.npy", w[0][m][r0:r0 + 17, c0:c0 + 17])
        np.save(f"{out}/{tag}_m{m}_k_{r}_{cc}.npy", k[0][m][r0:r0 + 17, c0:c0 + 17])
print(json.dumps(rep))
json.dump(rep, open(f"{out}/{tag}.json", "w"))
