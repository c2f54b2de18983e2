"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's FCD hot path (/root/reference/pyfcd/*.py),
written from SURVEY.md §8a, used as the parity checker by tests/, by
__graft_entry__.smoke() and as bench.py's cpu_baseline ("port").  The product
(trapped-modes-ltg_amd/) never imports this module.

Pinning: tests/test_oracle_golden.py checks this restatement against the
golden vectors the reference itself produced (tests/golden/make_golden.py,
numpy 1.26.4 / scipy 1.7.1 / scikit-image 0.18.3): peaks, radius, calibration
factor and interior k-fields bit-exact; wrapped phases / heights to float32
FFT tolerance.

Third-party pieces restated here (absent from /root/reference):
  * scipy.fft (pocketfft)   -> scipy.fft of the interpreter at hand (same
    library family; float32 in -> complex64 out, as in the reference);
  * skimage.measure.label / regionprops (0.18.3) -> scipy.ndimage.label with
    the 8-connected structure (labels in raster order of first pixel, coords
    row-major, as regionprops reports them);
  * skimage.draw.disk (0.18.3) -> explicit strict-inequality raster below;
  * skimage.restoration.unwrap_phase (0.18.3) -> oracle/herraez_unwrap.c.
"""
import ctypes
import os

import numpy as np
from scipy import ndimage
from scipy.fft import fft2, ifft2

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

PI = 3.141592653589793
TWOPI = 6.283185307179586


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liboracle_unwrap.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = ctypes.CDLL(path)
        lib.orc_unwrap2d.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        lib.orc_unwrap2d.restype = ctypes.c_int
        lib.orc_count_residues.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.orc_count_residues.restype = ctypes.c_long
        lib.orc_reliability.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        lib.orc_reliability.restype = None
        _LIB = lib
    return _LIB


# ---------------------------------------------------------------- wavenumbers
def wavenumber(n, cf=1.0, shifted=False):
    """fourier.wavenumber (fourier.py:43-56): fftfreq(n, cf/2pi) = m * (1/(n*d))."""
    d = cf / (2 * np.pi)
    val = 1.0 / (n * d)
    m = np.concatenate([np.arange(0, (n - 1) // 2 + 1), np.arange(-(n // 2), 0)])
    k = m * val
    return np.fft.fftshift(k) if shifted else k


def wavenumber_meshgrid(shape, cf=1.0, shifted=False):
    """fourier.wavenumber_meshgrid (fourier.py:58-73), 'ij' indexing -> (k_rows, k_cols)."""
    return np.meshgrid(wavenumber(shape[0], cf, shifted), wavenumber(shape[1], cf, shifted), indexing="ij")


def pixel_to_wavenumber(shape, loc, cf=1.0):
    """fourier.pixel_to_wavenumber (fourier.py:94-113) for one (row, col) index."""
    return np.array([wavenumber(shape[0], cf, True)[loc[0]], wavenumber(shape[1], cf, True)[loc[1]]])


# ---------------------------------------------------------------- peak finding
def find_peak_locations(image, threshold, no_peaks):
    """fourier.find_peak_locations (fourier.py:139-168): dimmest `no_peaks` blobs above threshold."""
    blob = np.array(image > threshold)
    blob[0] = False
    blob[-1] = False
    blob[:, 0] = False
    blob[:, -1] = False
    labels, n = ndimage.label(blob, structure=np.ones((3, 3), bool))
    peaks = []
    for lab in range(1, n + 1):
        rr, cc = np.nonzero(labels == lab)          # row-major, like regionprops().coords
        vals = image[rr, cc]
        i = int(np.argmax(vals))                     # first of equal maxima
        peaks.append((vals[i], np.array([rr[i], cc[i]])))
    peaks.sort(key=lambda t: t[0])                   # stable ascending
    return [p[1] for p in peaks[:no_peaks]]


def find_peaks(image, exact=False):
    """fourier.find_peaks (fourier.py:7-41).  exact: the spectrum with the reference's own
    rounding in the image's precision (oracle/pocketfft.py: scipy 1.7.1's pocketfft, numpy
    1.26.4's mean and abs), which decides the picks where blobs tie in exact arithmetic;
    otherwise the interpreter's scipy.fft (a faster stand-in for the CPU baseline)."""
    if exact:
        from oracle import pocketfft
        spec = pocketfft.find_peaks_spectrum(image)
    else:
        spec = np.fft.fftshift(np.abs(fft2(image - np.mean(image))))
    kr, kc = wavenumber_meshgrid(spec.shape, shifted=True)
    kmin = 4 * np.pi / min(image.shape)
    spec *= (kr ** 2 + kc ** 2) > kmin ** 2
    thr = 0.5 * np.max(spec)
    locs = find_peak_locations(spec, thr, 4)

    def angle_key(p):
        k = pixel_to_wavenumber(spec.shape, p)
        return abs(np.arctan2(k[0], k[1]))

    right = min(locs, key=angle_key)
    k0 = pixel_to_wavenumber(spec.shape, right)

    def dep_key(p):
        k = pixel_to_wavenumber(spec.shape, p)
        return abs(np.dot(k0, k))

    perp = min(locs, key=dep_key)
    return right, perp


def calibration_factor(square_size, reference, exact=False):
    """fcd.compute_calibration_factor (fcd.py:72-101): 2*sq / (2pi / mean|k_pix|)."""
    peaks = find_peaks(reference, exact)
    kp = np.array([pixel_to_wavenumber(reference.shape, p) for p in peaks])
    pixel_wavelength = 2 * np.pi / np.mean(np.abs(kp))
    return 2 * square_size / pixel_wavelength, peaks


# ---------------------------------------------------------------- carriers
def disk_mask(shape, center, radius):
    """skimage.draw.disk(center, radius, shape) raster: strict ((dr/R)^2 + (dc/R)^2 < 1), clipped."""
    out = np.zeros(shape, bool)
    r0, c0 = int(center[0]), int(center[1])
    lo_r = max(int(np.ceil(r0 - radius)), 0)
    hi_r = min(int(np.floor(r0 + radius)), shape[0] - 1)
    lo_c = max(int(np.ceil(c0 - radius)), 0)
    hi_c = min(int(np.floor(c0 + radius)), shape[1] - 1)
    rr = np.arange(lo_r, hi_r + 1, dtype=np.float64)[:, None] - r0
    cc = np.arange(lo_c, hi_c + 1, dtype=np.float64)[None, :] - c0
    d = (rr / radius) ** 2 + (cc / radius) ** 2
    out[lo_r:hi_r + 1, lo_c:hi_c + 1] = d < 1
    return out


class Carrier:
    """carriers.Carrier (carriers.py:9-24)."""

    def __init__(self, reference, cf, peak, radius):
        self.pixels = peak
        self.frequencies = pixel_to_wavenumber(reference.shape, peak, cf)
        self.radius = radius
        self.mask = np.fft.ifftshift(disk_mask(reference.shape, peak, radius))
        self.ccsgn = np.conj(ifft2(fft2(reference) * self.mask))


def compute_carriers(reference, square_size):
    """fcd.compute_carriers (fcd.py:53-70)."""
    cf, peaks = calibration_factor(square_size, reference)
    radius = np.linalg.norm(np.asarray(peaks[0]) - np.asarray(peaks[1])) / 2
    return [Carrier(reference, cf, p, radius) for p in peaks], cf


# ---------------------------------------------------------------- unwrap
def unwrap(wrapped):
    """skimage unwrap_phase restated (oracle/herraez_unwrap.c). Returns (f64 unwrapped, int32 k)."""
    w = np.ascontiguousarray(wrapped, dtype=np.float32)
    k = np.zeros(w.shape, np.int32)
    u = np.zeros(w.shape, np.float64)
    if _lib().orc_unwrap2d(w.ctypes.data, w.shape[0], w.shape[1], k.ctypes.data, u.ctypes.data) != 0:
        raise MemoryError("oracle unwrap")
    return u, k


def count_residues(wrapped):
    w = np.ascontiguousarray(wrapped, dtype=np.float32)
    return int(_lib().orc_count_residues(w.ctypes.data, w.shape[0], w.shape[1]))


def reliability(wrapped):
    w = np.ascontiguousarray(wrapped, dtype=np.float64)
    rel = np.zeros(w.shape, np.float64)
    _lib().orc_reliability(w.ctypes.data, w.shape[0], w.shape[1], rel.ctypes.data)
    return rel


# ---------------------------------------------------------------- pipeline
def wrapped_phases(displaced_fft, carriers):
    """fcd.compute_phases without unwrap (fcd.py:116-118): -angle(ifft2(D*mask) * ccsgn), float32."""
    return np.stack([(-np.angle(ifft2(displaced_fft * c.mask) * c.ccsgn)).astype(np.float32) for c in carriers])


def displacement_field(phases, carriers):
    """fcd.compute_displacement_field (fcd.py:122-138)."""
    f0, f1 = carriers[0].frequencies, carriers[1].frequencies
    det = f0[1] * f1[0] - f0[0] * f1[1]
    u = (f1[0] * phases[0] - f0[0] * phases[1]) / det
    v = (f0[1] * phases[1] - f1[1] * phases[0]) / det
    return np.array([u, v])


def integrate_in_fourier(gx, gy, cf=1.0):
    """fourier.integrate_in_fourier (fourier.py:115-137), incl. remove_degeneracy's index N/2+1 (fourier.py:75-92)."""
    ky, kx = wavenumber_meshgrid(gx.shape, cf)
    k2 = kx ** 2 + ky ** 2
    k2[0, 0] = 1
    if gx.shape[1] % 2 == 0:
        kx[:, gx.shape[1] // 2 + 1] = 0
    if gx.shape[0] % 2 == 0:
        ky[gx.shape[0] // 2 + 1, :] = 0
    hat = (-1.0j * kx * fft2(gx) + -1.0j * ky * fft2(gy)) / k2
    return np.real(ifft2(hat))


def height_from_layers(layers):
    """fcd.height_from_layers / effective_height (fcd.py:37-51); layers[2][1] hard-coded as in the reference."""
    alpha = 1 - layers[-1][1] / layers[-2][1]
    h = 0
    for i in range(len(layers) - 1):
        h += layers[2][1] * (layers[i][0] / layers[i][1])
    return alpha * h


def compute_height_map(reference, displaced, square_size, layers=None, height=None, unwrap_phases=True,
                       carriers=None):
    """fcd.compute_height_map (fcd.py:13-35). Returns (height f64, phases f64 [2,H,W], cf, extras)."""
    if height is not None and layers is not None:
        raise Warning("Provide either height or layers, not both.")
    if height is None:
        height = 1 if layers is None else height_from_layers(layers)
    if carriers is None:
        carriers, cf = compute_carriers(reference, square_size)
    else:
        carriers, cf = carriers
    D = fft2(displaced)
    wrapped = wrapped_phases(D, carriers)
    ks = np.zeros(wrapped.shape, np.int32)
    if unwrap_phases:
        phases = np.zeros(wrapped.shape, np.float64)
        for i in range(2):
            phases[i], ks[i] = unwrap(wrapped[i])
    else:
        phases = wrapped.astype(np.float64)
    disp = displacement_field(phases, carriers)
    grad = -disp / height
    h = integrate_in_fourier(grad[0], grad[1], cf)
    return h, phases, cf, dict(wrapped=wrapped, k=ks, carriers=carriers)
