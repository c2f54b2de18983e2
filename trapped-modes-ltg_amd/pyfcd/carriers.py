"""Carrier description — drop-in for /root/reference/pyfcd/carriers.py.

A `Carrier` holds what the reference's does (carriers.py:9-24): the peak pixel,
its physical wavenumber, the band-pass disk radius, the ifftshifted disk mask
(skimage.draw.disk raster) and ccsgn = conj(ifft2(fft2(reference) * mask)), the
arrays computed on the MI355X.  It is a self-contained value, as in the
reference: it also keeps the reference image and the geometry it was built
from, so fcd.compute_phases can rebuild the engine's carrier state from the
carriers it is handed when the engine has since moved on to another reference.
"""
import numpy as np

from . import _lib


class Carrier:
    """One demodulation carrier (carriers.py:9-24).

    `Carrier(reference_image, calibration_factor, peak, peak_radius)` works as in
    the reference (carriers.py:10-15): the engine builds the disk and ccsgn for
    this peak and radius (fcd_set_carriers).  fcd.compute_carriers builds both
    carriers from one device pass instead (`_state`).
    """

    def __init__(self, reference_image, calibration_factor, peak, peak_radius, _state=None):
        from .fourier import fourier
        ref = np.asarray(reference_image)
        self.pixels = peak
        self.frequencies = fourier.pixel_to_wavenumber(ref.shape, peak, calibration_factor)
        self.radius = peak_radius
        if _state is None:
            if ref.ndim != 2:
                raise ValueError("reference_image must be a 2-D image")
            eng = _lib.engine_for(ref.shape)
            p = (int(peak[0]), int(peak[1]))
            eng.set_carriers(ref, None, calibration_factor, (p, p), (peak_radius, peak_radius))
            cc, masks = eng.carriers_arrays()
            index, ref_f32 = 0, eng.geometry[0]
        else:
            cc, masks, index, ref_f32 = _state
        self.mask = masks[index]
        self.ccsgn = cc[index]
        # identity of the carrier for fcd.compute_phases (float32, as the engine saw it)
        self._reference = ref_f32
        self._calibration_factor = float(calibration_factor)
