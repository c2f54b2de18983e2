"""Diagnostic: which stage of the engine's exact reference spectrum differs from the
oracle (oracle/pocketfft.py) on a golden reference image.  GPU box only."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from oracle import pocketfft as P, fcd_oracle as O  # noqa: E402
from pyfcd import _lib  # noqa: E402

for name, key in (("real_pair", "ref_u8"), ("real_df", "ref_u16")):
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    img = g[key].astype(np.float32)
    eng = _lib.Engine(img.shape)
    m = P.mean_f32(img)
    c = (img - m).astype(np.float32)
    Fd = eng.fft2(c)
    Fo = P.fft2(c)
    print(name, "fft2(centered) mismatches", int((Fd != Fo).sum()))
    kr, kc = O.wavenumber_meshgrid(img.shape, shifted=True)
    hp = (kr ** 2 + kc ** 2) > (4 * np.pi / min(img.shape)) ** 2
    so = np.fft.fftshift(P.abs_c64(Fo)) * hp
    info = eng.set_reference(img, 0.001)
    print(name, "oracle max", so.max(), "engine threshold*2", 2 * info.threshold, "fixture", 2 * float(g["threshold"]))
    # the engine's own centring: its fft2 of (img - mean) equals which mean?
    for mm in (m, np.float32(img.astype(np.float64).mean())):
        s2 = np.fft.fftshift(P.abs_c64(P.fft2((img - mm).astype(np.float32)))) * hp
        print("   mean", repr(mm), "max", s2.max())
    # magnitude formula on the device spectrum
    sd = np.fft.fftshift(P.abs_c64(Fd)) * hp
    print("   abs of device fft2 max", sd.max(), "hypot", (np.fft.fftshift(np.hypot(Fd.real, Fd.imag)) * hp).max())
