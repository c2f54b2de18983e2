"""Diagnostic (CPU, numpy): how the 64 x 64 tile pass's Boruvka rounds shrink the camera
frames' graphs.  After each tile round r: level-0 components, distinct adjacent component
pairs inside tiles (the contracted graph's intra-tile edges), and the per-tile maxima (the
capacities a tile pass that stops after r rounds would need).  Same hook rule as
k_mst_tile0 (kernels_unwrap.hip): a component hooks along its lightest edge (weight, edge
index) over all its edges when that edge stays inside the tile; of a mutual pair the
smaller root stays.

    python tools/diag/t0_rounds_sim.py [frames]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import fcd_oracle as O  # noqa: E402

T = 64


def edges(rel):
    H, W = rel.shape
    ii, jj = np.mgrid[0:H, 0:W - 1]
    hu = (ii * W + jj).ravel()
    hv = hu + 1
    hwt = (rel[:, :-1] + rel[:, 1:]).ravel()
    ii, jj = np.mgrid[0:H - 1, 0:W]
    vu = (ii * W + jj).ravel()
    vv = vu + W
    vwt = (rel[:-1, :] + rel[1:, :]).ravel()
    eu = np.concatenate([hu, vu])
    ev = np.concatenate([hv, vv])
    ew = np.concatenate([hwt, vwt])
    ec = np.arange(len(eu))
    return eu, ev, ew, ec


def simulate(w):
    H, W = w.shape
    rel = O.reliability(w)
    eu, ev, ew, ec = edges(rel)
    tile = lambda p: (p // W // T) * (W // T) + (p % W) // T  # noqa: E731
    tu = tile(eu)
    intra = tu == tile(ev)
    lab = np.arange(H * W)
    out = []
    r = 0
    while True:
        cu, cv = lab[eu], lab[ev]
        m = cu != cv
        comps = np.concatenate([cu[m], cv[m]])
        other = np.concatenate([cv[m], cu[m]])
        w2 = np.concatenate([ew[m], ew[m]])
        c2 = np.concatenate([ec[m], ec[m]])
        in2 = np.concatenate([intra[m], intra[m]])
        order = np.lexsort((c2, w2, comps))
        cs = comps[order]
        first = np.ones(len(cs), bool)
        first[1:] = cs[1:] != cs[:-1]
        sel = order[first]
        parent = np.arange(H * W)
        hook = in2[sel]
        hc, ho, he = comps[sel][hook], other[sel][hook], c2[sel][hook]
        parent[hc] = ho
        # mutual pairs: the smaller root stays
        best_e = np.full(H * W, -1)
        best_e[comps[sel]] = c2[sel]
        mutual = (best_e[ho] == he) & (hc < ho)
        parent[hc[mutual]] = hc[mutual]
        if not np.any(parent[hc] != hc):
            break
        r += 1
        while True:
            p2 = parent[parent]
            if np.array_equal(p2, parent):
                break
            parent = p2
        lab = parent[lab]
        cu, cv = lab[eu], lab[ev]
        d = (cu != cv)
        pairs = np.unique(np.minimum(cu, cv)[d & intra] * (H * W) + np.maximum(cu, cv)[d & intra])
        roots = np.unique(lab)
        ctile = np.bincount(tile(roots), minlength=(H // T) * (W // T))
        ptile = np.bincount(tile(pairs // (H * W)), minlength=len(ctile))
        out.append((r, len(roots), len(pairs), int(ctile.max()), int(ptile.max()), int((d & ~intra).sum())))
    return out


def main():
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    d = np.load(os.path.join(ROOT, "tests", "golden", "real_df.npz"))
    ref = d["ref_u16"].astype(np.float32)
    carriers, _ = O.compute_carriers(ref, float(d["square_size"]) if "square_size" in d else 0.002)
    for f in range(nfr):
        frame = d["frames_u16"][f].astype(np.float32)
        D = np.fft.fft2(frame.astype(np.float64)).astype(np.complex64)
        ws = O.wrapped_phases(D, carriers)
        for mi in range(2):
            print(f"frame {f} map {mi}: residues {O.count_residues(ws[mi])}")
            print("  round  comps  intra-pairs  max-comps/tile  max-pairs/tile  cross-edges")
            for row in simulate(ws[mi]):
                print("  %5d %7d %12d %15d %15d %12d" % row)


if __name__ == "__main__":
    main()
