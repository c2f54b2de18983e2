"""TEST INFRASTRUCTURE ONLY (the checker, never the product): the float32 names of the
restated reference spectrum.  The restatement itself (any frame shape, float32 and
float64) is oracle/pocketfft.py; this module keeps the float32 entry points the tests
and tools have always imported (fourier.py:18 for a float32 image: scipy 1.7.1's fft2,
numpy 1.26.4's mean and complex64 abs).
"""
import numpy as np

from oracle import pocketfft as _P

rfactors = _P.rfactors
cfactors = _P.cfactors


def fft2(x):
    """scipy.fft.fft2 of a real float32 image: complex64 [H, W]."""
    return _P.fft2(np.ascontiguousarray(x, np.float32))


def sum_f32(x):
    return _P.sum_T(x, np.float32)


def mean_f32(x):
    return _P.mean_T(x, np.float32)


def abs_c64(z):
    return _P.abs_c(np.asarray(z, np.complex64))


def find_peaks_spectrum(image):
    """|fftshift(fft2(image - mean(image)))| of a float32 image, as fourier.py:18."""
    return _P.find_peaks_spectrum(np.ascontiguousarray(image, np.float32))


def rtwiddles(n, fact):
    """rfftp::comp_twiddle<float>: per pass its (ip - 1) * (ido - 1) floats."""
    return [tw for tw, _ in _P.rtwiddles(n, fact, np.float32)]


def ctwiddles(n, fact):
    """cfftp::comp_twiddle<float>: per pass (re, im) of its (ip - 1) * (ido - 1) twiddles."""
    out = []
    for (tr, ti), _ in _P.ctwiddles(n, fact, np.float32):
        out.append((np.ascontiguousarray(tr).ravel(), np.ascontiguousarray(ti).ravel()))
    return out
