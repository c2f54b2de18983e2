"""Minimax fits of atan(r) = r P(r^2) on [0, 1] with 7 / 8 / 9 terms (Lawson's
iteratively reweighted least squares) and their max |error| evaluated in float32:
the coefficients of gfft.hpp atan_coef (FCD_ATAN_TERMS).  Tuning tool, CPU only."""
import numpy as np
# minimax fit of atan(r) ~ r * P(r^2), r in [0,1], absolute error, via iterative reweighted LS (Lawson)
def fit(nterms, iters=300):
    r = np.cos(np.linspace(0, np.pi/2, 4000))  # dense in [0,1]
    r = np.concatenate([r, np.linspace(0,1,4000)])
    s = r*r
    A = np.stack([r * s**k for k in range(nterms)], 1)
    y = np.arctan(r)
    w = np.ones_like(r)/len(r)
    for _ in range(iters):
        sw = np.sqrt(w)
        c, *_ = np.linalg.lstsq(A*sw[:,None], y*sw, rcond=None)
        e = np.abs(A@c - y)
        w = w*e; w /= w.sum()
    return c
def eval32(c, r):
    r = r.astype(np.float32); s = (r*r).astype(np.float32)
    p = np.float32(c[-1])
    for k in range(len(c)-2, -1, -1):
        p = (p*s + np.float32(c[k])).astype(np.float32)  # fma-less; close enough
    return (r*p).astype(np.float32)
rt = np.linspace(0,1,2000001).astype(np.float32)
ref = np.arctan(rt.astype(np.float64))
cur = [0.9999998807907104,-0.33332598209381104,0.19985906779766083,-0.14161229133605957,0.10498946160078049,-0.07234858721494675,0.03978124260902405,-0.014401371590793133,0.0024567286018282175]
print("current 9-term", np.abs(eval32(np.array(cur), rt)-ref).max())
for n in (7,8,9):
    c = fit(n)
    print(n, "terms: f64 err", np.abs((rt.astype(np.float64)*np.polyval(c[::-1], rt.astype(np.float64)**2))-ref).max(), "f32 err", np.abs(eval32(c, rt)-ref).max())
    print("   ", ", ".join(repr(float(np.float32(x))) for x in c))
