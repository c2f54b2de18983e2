"""Fourier-space helpers of the FCD pipeline — drop-in for
/root/reference/pyfcd/fourier.py (class `fourier`, same classmethod names,
arguments and return conventions).

The wavenumber tables are host-side scalar arithmetic (they are tiny and
computed exactly as the reference computes them).  The heavy operations run on
the MI355X engine: `find_peaks` (FFT + |F| + high-pass + threshold on the
device) and `integrate_in_fourier` (batched R2C/C2R-equivalent spectral
integration on the device).
"""
import numpy as np
from scipy import ndimage

from . import _lib


def _fftfreq(n, d):
    # numpy.fft.fftfreq: m * (1 / (n * d)) with m = 0..ceil(n/2)-1, -floor(n/2)..-1
    val = 1.0 / (n * d)
    m = np.empty(n, int)
    npos = (n - 1) // 2 + 1
    m[:npos] = np.arange(0, npos)
    m[npos:] = np.arange(-(n // 2), 0)
    return m * val


class fourier:
    """Spectral utilities; every method is a classmethod, as in the reference."""

    @classmethod
    def find_peaks(cls, image):
        """(rightmost_peak, perpendicular_peak) in fftshifted pixel coordinates.

        Reference: fourier.py:7-41.  Runs on the device (fcd_find_peaks); the
        engine's current reference is left in place.
        """
        img = np.asarray(image)
        eng = _lib.engine_for(img.shape)
        info = eng.find_peaks(img, 1.0)[0]
        return (np.array([info.peaks[0][0], info.peaks[0][1]]),
                np.array([info.peaks[1][0], info.peaks[1][1]]))

    @classmethod
    def wavenumber(cls, size, calibration_factor=1, shifted=False):
        """k = 2*pi*fftfreq(size)/calibration_factor (fourier.py:43-56)."""
        k = _fftfreq(size, calibration_factor / (2 * np.pi))
        return np.fft.fftshift(k) if shifted else k

    @classmethod
    def wavenumber_meshgrid(cls, shape, calibration_factor=1, shifted=False):
        """'ij' meshgrid of the row and column wavenumbers (fourier.py:58-73)."""
        rows = cls.wavenumber(shape[0], calibration_factor, shifted)
        cols = cls.wavenumber(shape[1], calibration_factor, shifted)
        return np.meshgrid(rows, cols, indexing="ij")

    @classmethod
    def remove_degeneracy(cls, kx, ky, shape):
        """Zero column N/2+1 of kx and row N/2+1 of ky in place (fourier.py:75-92, index kept literally)."""
        if shape[1] % 2 == 0:
            kx[:, shape[1] // 2 + 1] = 0
        if shape[0] % 2 == 0:
            ky[shape[0] // 2 + 1, :] = 0

    @classmethod
    def pixel_to_wavenumber(cls, image_shape, locations, calibration_factor=1):
        """Wavenumber (k_row, k_col) of fftshifted pixel index/indices (fourier.py:94-113)."""
        kr = cls.wavenumber(image_shape[0], calibration_factor, shifted=True)
        kc = cls.wavenumber(image_shape[1], calibration_factor, shifted=True)
        if isinstance(locations[0], np.ndarray):
            return np.array([[kr[p[0]], kc[p[1]]] for p in locations])
        return np.array([kr[locations[0]], kc[locations[1]]])

    @classmethod
    def integrate_in_fourier(cls, gradient_x, gradient_y, calibration_factor=1):
        """Height from its gradient by spectral inversion (fourier.py:115-137), on the device.

        float32 arithmetic (the reference promotes to complex128); returns float64
        like the reference.
        """
        gx = np.asarray(gradient_x)
        eng = _lib.engine_for(gx.shape)
        return eng.integrate(gx, gradient_y, calibration_factor).astype(np.float64)

    @classmethod
    def find_peak_locations(cls, image, threshold, no_peaks):
        """The `no_peaks` dimmest above-threshold 8-connected blobs' peak pixels (fourier.py:139-168).

        Generic host helper kept for API completeness; the engine's find_peaks
        performs the same selection on its device-side candidate list.
        """
        img = np.asarray(image)
        blob = img > threshold
        blob[[0, -1], :] = False
        blob[:, [0, -1]] = False
        labels, n = ndimage.label(blob, structure=np.ones((3, 3), bool))
        found = []
        for lab in range(1, n + 1):
            rr, cc = np.nonzero(labels == lab)
            vals = img[rr, cc]
            i = int(np.argmax(vals))
            found.append((vals[i], np.array([rr[i], cc[i]])))
        found.sort(key=lambda t: t[0])
        return [p for _, p in found[:no_peaks]]
