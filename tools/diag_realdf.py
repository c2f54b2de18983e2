"""Diagnostic (GPU): where do the engine's wrapped phases on the real_df golden
frames differ most from the reference's, and how well-conditioned is that
pixel (band amplitude relative to the map's median, f64 recomputation)?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]
import numpy as np
from pyfcd import _lib
from oracle import fcd_oracle as O
d = np.load(os.path.join(ROOT, "tests/golden/real_df.npz"))
ref = d["ref_u16"].astype(np.float32)
fr = d["frames_u16"].astype(np.float32)
eng = _lib.Engine(ref.shape)
eng.set_reference(ref, float(d["square_size"]))
_, wr, _ = eng.process(fr, 1.0, unwrap=False)
carriers, cf = O.compute_carriers(ref, float(d["square_size"]))
R64 = np.fft.fft2(ref.astype(np.float64))
for f in range(fr.shape[0]):
    D64 = np.fft.fft2(fr[f].astype(np.float64))
    for m in range(2):
        mk = carriers[m].mask
        A = np.fft.ifft2(D64 * mk)[::8, ::8]
        Rr = np.fft.ifft2(R64 * mk)[::8, ::8]
        w64 = -np.angle(A * np.conj(Rr))
        wrapd = lambda a, b: np.abs((a - b + np.pi) % (2 * np.pi) - np.pi)
        g = d["wrapped_sub"][f][m].astype(np.float64)
        ours = wr[f, m][::8, ::8].astype(np.float64)
        e, eg, eo = wrapd(ours, g), wrapd(g, w64), wrapd(ours, w64)
        i = np.unravel_index(np.argmax(e), e.shape)
        print(f"frame {f} map {m}: ours-vs-ref max {e.max():.2e} p99.9 {np.quantile(e, 0.999):.2e} | "
              f"ref-vs-f64 max {eg.max():.2e} | ours-vs-f64 max {eo.max():.2e} | worst pixel {i}: "
              f"|A|/med {abs(A[i]) / np.median(abs(A)):.2e} |R|/med {abs(Rr[i]) / np.median(abs(Rr)):.2e} "
              f"ref err there {eg[i]:.2e} ours err there {eo[i]:.2e}", flush=True)
