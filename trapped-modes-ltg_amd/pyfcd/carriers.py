"""Carrier description — drop-in for /root/reference/pyfcd/carriers.py.

A `Carrier` is built by the engine from its device-side reference state: the
peak pixel, its physical wavenumber, the band-pass disk radius, the
ifftshifted disk mask (skimage.draw.disk raster) and ccsgn =
conj(ifft2(fft2(reference) * mask)), all computed on the MI355X.
"""
import numpy as np

from . import _lib


class Carrier:
    """One demodulation carrier (carriers.py:9-24).

    Construct it like the reference (reference image, calibration factor, peak,
    radius); the arrays come from the engine that holds this reference.
    """

    def __init__(self, reference_image, calibration_factor, peak, peak_radius, _index=None, _engine=None):
        ref = np.asarray(reference_image)
        self.pixels = np.asarray(peak)
        self.radius = peak_radius
        from .fourier import fourier
        self.frequencies = fourier.pixel_to_wavenumber(ref.shape, self.pixels, calibration_factor)
        eng = _engine
        if eng is None:
            raise TypeError("Carrier objects are created by fcd.compute_carriers on the MI355X engine")
        cc, masks = eng.carriers_arrays()
        i = _index
        if i is None:
            raise TypeError("Carrier index missing")
        self.mask = masks[i]
        self.ccsgn = cc[i]
        self._engine = eng
        self._index = i
