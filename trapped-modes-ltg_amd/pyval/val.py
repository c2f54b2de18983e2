"""Synthetic known-answer validation of the height reconstruction, as the reference's
`pyval.val` (/root/reference/pyval/val.py:38-136), run through the MI355X engine.

A height field h is turned into the displacement u = -H grad h (spectral or finite
differences, val.py:116-131), a sinusoidal checker I0 is warped by it with bilinear
interpolation (val.py:96-106), and `fcd.compute_height_map(I0, I, N / (2 n), height=H)`
(val.py:108) must give back h.  examples/val_example.py runs unchanged against this
module; the README's "< 0.52 %" (max |h_fcd - h| / max |h_fcd|) is checked in
tests/test_gpu_parity.py.

Host-side synthesis in numpy / scipy (the harness is not on the hot path); the
reconstruction is the product path (pyfcd.fcd -> C ABI -> HIP kernels).
"""
import numpy as np
from scipy.interpolate import RegularGridInterpolator

from pyfcd.fcd import fcd, fourier


def h_grad(h, x, y, k=0):
    """(dh/dx, dh/dy) stacked on the last axis: k = 0 spectral derivative of the
    zero-mean field (val.py:117-126), k = 1 np.gradient (val.py:127-129)."""
    if k == 0:
        kx, ky = fourier.wavenumber_meshgrid(h.shape)
        spec = np.fft.fft2(h - np.mean(h))
        gx = np.fft.ifft2(1j * kx * spec).real
        gy = np.fft.ifft2(1j * ky * spec).real
    elif k == 1:
        gx, gy = np.gradient(h, x, y, axis=(0, 1))
    else:
        raise ValueError('Parameter k must be an integer between 0 (pseudoespectral) and 1 (finite differences)')
    return np.stack((gx, gy), axis=-1)


def centrado(v):
    """Map v to [-1, 1] around its mid-range (val.py:133-136)."""
    mid = (np.max(v) + np.min(v)) * 0.5
    half = (np.max(v) - np.min(v)) * 0.5
    return (v - mid) / half


def val(k, func=None, h=None, N=1024, H=1, n=60, centrado_si=False, *args, **kwargs):
    """(X, Y, h, I, height_map, I0, calibration_factor) of the reference's harness
    (val.py:38-114): ij-meshgrid of N points, square size N / (2 n) so the calibration
    factor is 1, checker I0 = 0.5 + sin(X kx) sin(Y ky) / 2 with kx = ky = 2 pi n / N."""
    square_size = N / (2 * n)
    axis = np.linspace(0, N, N, endpoint=False)
    X, Y = np.meshgrid(axis, axis, indexing="ij")
    if func is not None:
        if h is not None:
            raise Warning("Provide either h or func, not both.")
        h = func(X, Y, *args, **kwargs)
    elif h is None:
        raise Warning("Provide either h or func, not empty.")
    u = -H * h_grad(h, axis, axis, k=k)
    kc = 2 * np.pi * n / N
    I0 = 0.5 + np.sin(X * kc) * np.sin(Y * kc) / 2
    # sample I0 at r - u (clipped to the grid), bilinear, zero outside
    src = np.stack((X, Y), axis=-1) - u
    np.clip(src, axis.min(), axis.max(), out=src)
    sampler = RegularGridInterpolator((axis, axis), I0, bounds_error=False, fill_value=0)
    I = sampler(src.reshape(-1, 2)).reshape(N, N)
    height_map, _, calibration_factor = fcd.compute_height_map(I0, I, square_size=square_size, height=H)
    if centrado_si:
        height_map = centrado(height_map)
    return X, Y, h, I, height_map, I0, calibration_factor
