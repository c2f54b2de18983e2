"""FCD entry point — drop-in for /root/reference/pyfcd/fcd.py.

`from pyfcd.fcd import fcd, fourier` works exactly as in the reference
(pyval/val.py:36); every classmethod keeps its name, arguments and return
types.  The per-frame path of compute_height_map (FFT, disk band-pass, inverse
FFTs, phase extraction, unwrap, displacement solve and spectral integration)
runs as one batched pipeline of hand-written HIP kernels on the MI355X; the
reference-derived state (peaks, calibration factor, carriers) is computed on
the device once per reference and cached, instead of once per call.

Numerics: the engine computes in float32 (the reference's FFTs are float32
for float32 images, its unwrap and integration float64).  Outputs are returned
as float64 arrays like the reference's.  Phases are w + 2*pi*k with w the
float32 wrapped angle and k the integer unwrap field, the reference's own
composition (skimage unwrap: value + TWOPI * increment).
"""
import numpy as np

from . import _lib
from .carriers import Carrier
from .fourier import fourier

TWOPI = 6.283185307179586  # 2 * M_PI, skimage unwrap's TWOPI

__all__ = ["fcd", "fourier", "Carrier"]


def _engine_with_reference(reference, square_size):
    ref = np.asarray(reference)
    eng = _lib.engine_for(ref.shape)
    if not eng.matches(ref, square_size):
        eng.set_reference(ref, square_size)
    return eng


def _carriers_from_engine(eng, reference):
    info = eng.info
    cf = info.calibration_factor
    cc, masks = eng.carriers_arrays()
    carriers = [Carrier(reference, cf, np.array([info.peaks[i][0], info.peaks[i][1]]), info.radius,
                        _state=(cc, masks, i, eng.ref_copy)) for i in range(2)]
    return carriers, cf


class fcd:
    """Classmethod namespace, as in the reference (fcd() itself is not instantiable there either)."""

    def __init__(self):
        raise TypeError("fcd is a classmethod namespace")

    @classmethod
    def compute_height_map(cls, reference, displaced, square_size, layers=None, height=None, unwrap=True):
        """(height_map, phases, calibration_factor) — fcd.py:13-35.

        height_map float64 [H, W]; phases float64 [2, H, W]; calibration_factor float.
        """
        if height is not None:
            if layers is not None:
                raise Warning("Provide either height or layers, not both.")
        else:
            height = 1 if layers is None else cls.height_from_layers(layers)
        eng = _engine_with_reference(reference, square_size)
        hmap, wrapped, k = eng.process(np.asarray(displaced)[None], height, unwrap=unwrap, want_phases=True)
        phases = wrapped[0].astype(np.float64)
        if unwrap:
            phases += TWOPI * k[0]
        return hmap[0].astype(np.float64), phases, eng.info.calibration_factor

    @classmethod
    def compute_height_maps(cls, reference, displaced_stack, square_size, layers=None, height=None, unwrap=True,
                            return_phases=False):
        """Batched form of compute_height_map for a [B, H, W] stack (one device pass per chunk)."""
        if height is not None:
            if layers is not None:
                raise Warning("Provide either height or layers, not both.")
        else:
            height = 1 if layers is None else cls.height_from_layers(layers)
        eng = _engine_with_reference(reference, square_size)
        hmap, wrapped, k = eng.process(displaced_stack, height, unwrap=unwrap, want_phases=return_phases)
        if not return_phases:
            return hmap, eng.info.calibration_factor
        phases = wrapped.astype(np.float64)
        if unwrap:
            phases += TWOPI * k
        return hmap, phases, eng.info.calibration_factor

    @classmethod
    def height_from_layers(cls, layers):
        """Effective height of a layer stack (fcd.py:37-47): alpha * sum_i effective_height(i)."""
        alpha = 1 - layers[-1][1] / layers[-2][1]
        total = 0
        for i in range(len(layers) - 1):
            total += cls.effective_height(layers, i)
        return alpha * total

    @classmethod
    def effective_height(cls, layers, i):
        """layers[2][1] * t_i / n_i — the reference hard-codes layers[2][1] (fcd.py:49-51)."""
        return layers[2][1] * ((layers[i][0]) / (layers[i][1]))

    @classmethod
    def compute_carriers(cls, reference, square_size):
        """([Carrier, Carrier], calibration_factor) — fcd.py:53-70, computed on the device."""
        eng = _engine_with_reference(reference, square_size)
        return _carriers_from_engine(eng, reference)

    @classmethod
    def compute_calibration_factor(cls, square_size, reference, plot=False):
        """(calibration_factor, (peak0, peak1)) — fcd.py:72-101."""
        eng = _engine_with_reference(reference, square_size)
        info = eng.info
        peaks = (np.array([info.peaks[0][0], info.peaks[0][1]]), np.array([info.peaks[1][0], info.peaks[1][1]]))
        cf = info.calibration_factor
        if plot:
            import matplotlib.pyplot as plt
            ref = np.asarray(reference)
            pix_wl = 2 * square_size / cf
            fig, ax = plt.subplots()
            ax.imshow(ref, cmap="gray")
            ax.set_title(f"Calibration factor: \n {cf} dist/px")
            cy, cx = ref.shape[0] / 2, ref.shape[1] / 2
            ax.plot([cy, cy + pix_wl], [cx, cx], ".-", label=r"$\lambda$")
            ax.set_xlabel("X (pix)")
            ax.set_ylabel("Y (pix)")
            plt.legend()
            plt.tight_layout()
            plt.show()
        return cf, peaks

    @classmethod
    def compute_calibration_factors(cls, square_size, references):
        """[(calibration_factor, (peak0, peak1))] for a stack of references in one call
        (compute_calibration_factor, fcd.py:72-101, for many-reference workloads; the
        engine's current reference is left in place)."""
        refs = np.asarray(references)
        if refs.ndim == 2:
            refs = refs[None]
        eng = _lib.engine_for(refs.shape[1:])
        out = []
        for info in eng.find_peaks(refs, square_size):
            out.append((info.calibration_factor, (np.array([info.peaks[0][0], info.peaks[0][1]]),
                                                  np.array([info.peaks[1][0], info.peaks[1][1]]))))
        return out

    @classmethod
    def compute_phases(cls, displaced_fft, carriers, unwrap=True):
        """Phase maps [2, H, W] float64 from an unshifted spectrum (fcd.py:103-120), on the device.

        Demodulates against the carriers it is given, as the reference does: if the
        engine's carrier state was built from other carriers (another reference set
        since, or hand-made Carrier objects), it is rebuilt from these carriers'
        images and geometry first (fcd_set_carriers)."""
        if len(carriers) != 2:
            raise ValueError("compute_phases takes the two carriers of fcd.compute_carriers")
        c0, c1 = carriers[0], carriers[1]
        if not all(hasattr(c, "_reference") for c in (c0, c1)):
            raise TypeError("carriers must be pyfcd.carriers.Carrier objects")
        spec = np.asarray(displaced_fft)
        eng = _lib.engine_for(spec.shape[-2:])
        peaks = [(int(c.pixels[0]), int(c.pixels[1])) for c in (c0, c1)]
        radii = (float(c0.radius), float(c1.radius))
        if not eng.holds_carriers(c0._reference, c1._reference, peaks, radii, c0._calibration_factor):
            eng.set_carriers(c0._reference, c1._reference, c0._calibration_factor, peaks, radii)
        wrapped, k = eng.phases_from_spectrum(spec, unwrap=unwrap)
        phases = wrapped[0].astype(np.float64)
        if unwrap:
            phases += TWOPI * k[0]
        return phases

    @classmethod
    def compute_displacement_field(cls, phases, carriers):
        """[u, v] from the two phase maps by the 2x2 carrier solve (fcd.py:122-138).

        Elementwise host helper for API parity; inside compute_height_map this
        solve is folded into the device integration multiplier.
        """
        f0, f1 = carriers[0].frequencies, carriers[1].frequencies
        det = f0[1] * f1[0] - f0[0] * f1[1]
        u = (f1[0] * phases[0] - f0[0] * phases[1]) / det
        v = (f0[1] * phases[1] - f1[1] * phases[0]) / det
        return np.array([u, v])

    @staticmethod
    def fft_peaks(image):
        """Plot |FFT| with the detected blob peaks and the chosen carriers (fcd.py:141-175).

        The picks come from fcd_find_peaks, which leaves the engine's reference (and so the
        next compute_height_map's cached carriers) untouched."""
        import matplotlib.pyplot as plt
        img = np.asarray(image)
        eng = _lib.engine_for(img.shape)
        info = eng.find_peaks(img, 1.0)[0]
        spec = np.fft.fftshift(np.abs(eng.fft2(img - np.mean(img))))
        fig, ax = plt.subplots()
        ax.imshow(np.log1p(spec), origin="lower", cmap="magma")
        ax.set_title("FFT Spectrum with Peaks")
        ax.set_xlabel(r"$k_x$ (1/pix)")
        ax.set_ylabel(r"$k_y$ (1/pix)")
        for i in range(info.n_blobs):
            y, x = info.blob_peaks[i][0], info.blob_peaks[i][1]
            ax.plot(x, y, "k.", markersize=6)
            ax.text(x + 5, y + 5, f"peak {i + 1}", color="white", fontsize=9)
        ax.plot(info.peaks[0][1], info.peaks[0][0], "r.", label="Rightmost peak")
        ax.plot(info.peaks[1][1], info.peaks[1][0], "b.", label=r"$\perp$ peak")
        ax.legend()
        plt.tight_layout()
        plt.show()
