"""Engine vs oracle at one frame shape: wrapped phases, k-fields, heights (where they differ)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]
from bench_data import make_residue_frame  # noqa: E402
from oracle import fcd_oracle as O  # noqa: E402
from pyfcd import _lib  # noqa: E402


def wrapd(a):
    return np.abs((a + np.pi) % (2 * np.pi) - np.pi)


for arg in sys.argv[1:]:
    rows, cols = (int(v) for v in arg.split("x"))
    pairs = [(rows // 2 + 0.5, min(cols // 3, 40) + 0.25)]
    ref, frame = make_residue_frame(rows, pairs, seed=3, rotate_deg=5.0, quantum=4096, cols=cols)
    eng = _lib.Engine((rows, cols))
    eng.set_reference(ref, 0.001)
    h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    ho, _, _, ex = O.compute_height_map(ref, frame, 0.001, height=1.0)
    print(arg, "rel_l2 h", float(np.linalg.norm(h[0] - ho) / np.linalg.norm(ho)))
    for m in range(2):
        wd = wrapd(w[0][m] - ex["wrapped"][m])
        _, ko = O.unwrap(w[0][m])
        d = k[0][m].astype(np.int64) - ko
        bad = np.argwhere(d != d.flat[0])
        print(" map", m, "wrap max", float(wd.max()), "at", np.unravel_index(wd.argmax(), wd.shape),
              "k mismatches", len(bad), bad[:5].tolist())
        _, ko2 = O.unwrap(ex["wrapped"][m])
        d2 = ko2 - ko
        print("   oracle k on own vs engine phases: mismatches", int((d2 != d2.flat[0]).sum()))
    e = np.abs(h[0] - ho)
    print(" h max err", float(e.max()), "at", np.unravel_index(e.argmax(), e.shape), "max|h|", float(np.abs(ho).max()))
    eng.close()
