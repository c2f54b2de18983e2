"""ctypes binding of the MI355X FCD engine (include/fcd.h).

The engine is the in-tree shared library lib/libfcd_mi355x.so built from
csrc/ (HIP kernels for gfx950).  There is no fallback: if the library or a
HIP device is missing every entry point raises.
"""
import collections
import ctypes
import os
import threading

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FCD_LIB", os.path.join(_PKG_ROOT, "lib", "libfcd_mi355x.so"))

FCD_OK = 0
FCD_E_INVALID = -1
FCD_E_UNSUPPORTED = -2
FCD_E_HIP = -3
FCD_E_STATE = -4
FCD_E_NOPEAKS = -5
FCD_E_INTERNAL = -6
FCD_HOST_PTRS = 0
FCD_DEVICE_PTRS = 1
FCD_STACK_F64 = 2  # temporal calls: float64 samples
FCD_IMG_F64 = 4  # set_reference / find_peaks / fft2: float64 images (the reference's precision)
# frame sample formats (fcd_process_raw)
FCD_FMT_F32 = 0
FCD_FMT_U8 = 1
FCD_FMT_U16 = 2
FCD_FMT_P10 = 3

# Every symbol include/fcd.h declares (checked by tests/test_cpu_host.py::test_header_lists_bound_symbols).
EXPORTED = (
    "fcd_abi_version", "fcd_last_error", "fcd_create", "fcd_destroy", "fcd_synchronize",
    "fcd_set_reference", "fcd_set_carriers", "fcd_get_carriers", "fcd_process", "fcd_phases_from_spectrum",
    "fcd_unwrap", "fcd_integrate", "fcd_fft2", "fcd_profile", "fcd_stage_times",
    "fcd_process_raw", "fcd_frame_bytes", "fcd_host_alloc", "fcd_host_free", "fcd_find_peaks",
    "fcd_temporal_spectrum", "fcd_temporal_bins", "fcd_spectrogram",
)


class FcdRefInfo(ctypes.Structure):
    _fields_ = [
        ("peaks", (ctypes.c_int64 * 2) * 2),
        ("radius", ctypes.c_double),
        ("calibration_factor", ctypes.c_double),
        ("frequencies", (ctypes.c_double * 2) * 2),
        ("mask_count", ctypes.c_int32 * 2),
        ("n_blobs", ctypes.c_int32),
        ("blob_peaks", (ctypes.c_int64 * 2) * 4),
        ("threshold", ctypes.c_double),
    ]


class FcdError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fcd error {code}: {msg}")
        self.code = code


class FcdNoPeaksError(FcdError, ValueError):
    """FCD_E_NOPEAKS: the reference has fewer than two carrier peaks.  Also a ValueError,
    as the reference raises there (`min()` of an empty sequence, fourier.py:38), so a
    caller catching ValueError keeps working."""


_lib = None
_lib_lock = threading.Lock()


def load_library(path=None):
    """Load libfcd_mi355x.so and declare the ABI.  Raises OSError if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise OSError(f"MI355X FCD engine not built: {p} is missing (run __graft_entry__.build() or "
                          f"`make -C trapped-modes-ltg_amd`)")
        lib = ctypes.CDLL(p)
        vp, i32, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        sig = {
            "fcd_abi_version": ([], i32),
            "fcd_last_error": ([], ctypes.c_char_p),
            "fcd_create": ([i32, i32, i32, ctypes.POINTER(vp)], i32),
            "fcd_destroy": ([vp], i32),
            "fcd_synchronize": ([vp], i32),
            "fcd_set_reference": ([vp, vp, i32, f64, ctypes.POINTER(FcdRefInfo)], i32),
            "fcd_set_carriers": ([vp, vp, vp, i32, f64, vp, vp, ctypes.POINTER(FcdRefInfo)], i32),
            "fcd_get_carriers": ([vp, vp, vp], i32),
            "fcd_process": ([vp, vp, i32, i32, f64, i32, vp, vp, vp, vp], i32),
            "fcd_phases_from_spectrum": ([vp, vp, i32, i32, i32, vp, vp, vp], i32),
            "fcd_unwrap": ([vp, vp, i32, i32, vp, vp, vp], i32),
            "fcd_integrate": ([vp, vp, vp, i32, f64, i32, vp, vp], i32),
            "fcd_fft2": ([vp, vp, i32, i32, vp, vp], i32),
            "fcd_profile": ([vp, i32], i32),
            "fcd_stage_times": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)], i32),
            "fcd_process_raw": ([vp, vp, i32, i32, i32, f64, i32, vp, vp, vp, vp], i32),
            "fcd_frame_bytes": ([vp, i32, ctypes.POINTER(ctypes.c_int64)], i32),
            "fcd_host_alloc": ([ctypes.c_int64, ctypes.POINTER(vp)], i32),
            "fcd_host_free": ([vp], i32),
            "fcd_find_peaks": ([vp, vp, i32, i32, f64, ctypes.POINTER(FcdRefInfo)], i32),
            "fcd_temporal_spectrum": ([vp, vp] + [i32] * 9 + [vp, vp], i32),
            "fcd_temporal_bins": ([vp, vp] + [i32] * 8 + [vp, i32, vp, vp], i32),
            "fcd_spectrogram": ([vp, vp] + [i32] * 10 + [vp, f64, vp, vp], i32),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if path is None:
            _lib = lib
        return lib


def _check(rc):
    if rc != FCD_OK:
        cls = FcdNoPeaksError if rc == FCD_E_NOPEAKS else FcdError
        raise cls(rc, load_library().fcd_last_error().decode(errors="replace"))


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _spectrum_dtype(dtype):
    """The precision the reference computes an image's spectrum in (fourier.py:18, fcd.py:28):
    scipy's fft2 keeps float32 (and computes float16 in float32) and promotes everything
    else -- float64, bool, int, uint -- to float64 (scipy/fft/_pocketfft/helper.py:91-92,
    `_asfarray`); `image - np.mean(image)` of an integer image is float64 as well."""
    dt = np.dtype(dtype)
    return np.float32 if dt in (np.float32, np.float16) else np.float64


def _img(a):
    """An image in the precision the reference computes its spectrum in (_spectrum_dtype):
    a uint8 / uint16 reference (pattern.py's board, a raw camera frame) goes to the engine
    as float64 (FCD_IMG_F64) exactly as scipy promotes it, not rounded to float32."""
    a = np.asarray(a)
    if a.dtype.kind not in "biuf":
        raise TypeError(f"image dtype {a.dtype} is not real")
    return np.ascontiguousarray(a, dtype=_spectrum_dtype(a.dtype))


def _img_flag(a):
    return FCD_IMG_F64 if a.dtype == np.float64 else 0


def _ptr(a):
    return None if a is None else a.ctypes.data


def _peaks_of(info):
    return tuple((int(info.peaks[q][0]), int(info.peaks[q][1])) for q in range(2))


def _same_image(a, b):
    if a is b:
        return True
    a = np.asarray(a)
    return a.shape == b.shape and np.array_equal(_img(a), b) and _img(a).dtype == b.dtype


class Engine:
    """One engine context: a device, a frame shape, and (once set) a reference."""

    def __init__(self, shape, device=None):
        lib = load_library()
        if device is None:
            device = int(os.environ.get("FCD_DEVICE", "0"))
        self.shape = (int(shape[0]), int(shape[1]))
        self.device = device
        h = ctypes.c_void_p()
        _check(lib.fcd_create(device, self.shape[0], self.shape[1], ctypes.byref(h)))
        self._h = h
        self._lib = lib
        self.info = None
        self.ref_copy = None
        self.ref_square_size = None
        # what the context's carriers were built from, whichever call set them:
        # (image of carrier 0, image of carrier 1, ((r0, c0), (r1, c1)), (radius0, radius1),
        #  calibration factor)
        self.geometry = None
        self.explicit = False  # set by set_carriers (not by a find_peaks reference)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fcd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ reference
    def set_reference(self, reference, square_size):
        ref = _img(reference)
        if ref.shape != self.shape:
            raise ValueError(f"reference shape {ref.shape} != engine shape {self.shape}")
        info = FcdRefInfo()
        # a failed set_reference leaves the context without a reference: forget the
        # cached one first so the next call with the old reference re-uploads it
        self.ref_copy = None
        self.ref_square_size = None
        self.geometry = None
        _check(self._lib.fcd_set_reference(self._h, ref.ctypes.data, FCD_HOST_PTRS | _img_flag(ref),
                                           float(square_size), ctypes.byref(info)))
        self.info = info
        self.ref_copy = ref.copy()
        self.ref_square_size = float(square_size)
        self.explicit = False
        self.geometry = (self.ref_copy, self.ref_copy, _peaks_of(info), (info.radius, info.radius),
                         info.calibration_factor)
        return info

    def set_carriers(self, ref0, ref1, calibration_factor, peaks, radii):
        """fcd_set_carriers: both carriers from caller-given geometry (Carrier.__init__,
        carriers.py:10-24): peaks ((row, col), (row, col)) fftshifted, one radius per
        carrier, carrier q's ccsgn from image ref_q."""
        r0 = _f32(ref0)
        r1 = r0 if ref1 is None or ref1 is ref0 else _f32(ref1)
        for r in (r0, r1):
            if r.shape != self.shape:
                raise ValueError(f"reference shape {r.shape} != engine shape {self.shape}")
        pk = np.ascontiguousarray(np.asarray(peaks, dtype=np.int64).reshape(2, 2))
        rad = np.ascontiguousarray(np.asarray(radii, dtype=np.float64).reshape(2))
        info = FcdRefInfo()
        self.ref_copy = None
        self.ref_square_size = None
        self.geometry = None
        _check(self._lib.fcd_set_carriers(self._h, r0.ctypes.data, None if r1 is r0 else r1.ctypes.data,
                                          FCD_HOST_PTRS, float(calibration_factor), pk.ctypes.data, rad.ctypes.data,
                                          ctypes.byref(info)))
        self.info = info
        self.explicit = True
        # the images as given (their precision identifies them for holds_carriers); the
        # carrier signals themselves come from the float32 rounding
        c0 = _img(ref0).copy()
        c1 = c0 if r1 is r0 else _img(ref1).copy()
        self.geometry = (c0, c1, _peaks_of(info), (float(rad[0]), float(rad[1])), float(calibration_factor))
        return info

    def holds_carriers(self, ref0, ref1, peaks, radii, calibration_factor):
        """True if the context's carriers were built from these images, this geometry and
        this calibration factor (the phases depend on mask and ccsgn only, but the
        context's info -- calibration factor, frequencies -- must describe these carriers)."""
        if self.geometry is None:
            return False
        g0, g1, gp, gr, gcf = self.geometry
        pk = tuple(tuple(int(v) for v in p) for p in peaks)
        if pk != gp or tuple(float(r) for r in radii) != gr or float(calibration_factor) != gcf:
            return False
        return _same_image(ref0, g0) and _same_image(ref1, g1)

    def find_peaks(self, images, square_size=1.0):
        """fcd_find_peaks: FcdRefInfo per image of a [n, H, W] (or [H, W]) stack, the
        context's reference untouched."""
        imgs = _img(images)
        if imgs.ndim == 2:
            imgs = imgs[None]
        if imgs.shape[1:] != self.shape:
            raise ValueError(f"image shape {imgs.shape[1:]} != engine shape {self.shape}")
        infos = (FcdRefInfo * max(len(imgs), 1))()
        _check(self._lib.fcd_find_peaks(self._h, imgs.ctypes.data, len(imgs), FCD_HOST_PTRS | _img_flag(imgs),
                                        float(square_size), infos))
        return [infos[i] for i in range(len(imgs))]

    def matches(self, reference, square_size):
        if self.explicit or self.ref_copy is None or self.ref_square_size != float(square_size):
            return False
        ref = _img(reference)
        return ref.shape == self.ref_copy.shape and ref.dtype == self.ref_copy.dtype and np.array_equal(ref, self.ref_copy)

    def carriers_arrays(self):
        h, w = self.shape
        cc = np.empty((2, h, w), np.complex64)
        mask = np.empty((2, h, w), np.uint8)
        _check(self._lib.fcd_get_carriers(self._h, cc.ctypes.data, mask.ctypes.data))
        return cc, mask.astype(bool)

    # ------------------------------------------------------------ per frame
    def process(self, frames, height, unwrap=True, want_phases=True):
        fr = _f32(frames)
        if fr.ndim == 2:
            fr = fr[None]
        n = fr.shape[0]
        if fr.shape[1:] != self.shape:
            raise ValueError(f"frame shape {fr.shape[1:]} != engine shape {self.shape}")
        hmap = np.empty((n,) + self.shape, np.float32)
        wrapped = np.empty((n, 2) + self.shape, np.float32) if want_phases else None
        k = np.empty((n, 2) + self.shape, np.int32) if want_phases else None
        _check(self._lib.fcd_process(self._h, fr.ctypes.data, n, FCD_HOST_PTRS, float(height), int(bool(unwrap)),
                                     hmap.ctypes.data, _ptr(wrapped), _ptr(k), None))
        return hmap, wrapped, k

    def frame_bytes(self, fmt):
        b = ctypes.c_int64()
        _check(self._lib.fcd_frame_bytes(self._h, int(fmt), ctypes.byref(b)))
        return b.value

    def process_raw(self, raw, fmt, n, height, unwrap=True, out=None):
        """Heights of n frames stored as raw samples (FCD_FMT_*) in the host buffer `raw`
        (an ndarray of n * frame_bytes(fmt) bytes, e.g. a PinnedBuffer view); `out`: an
        optional float32 [n, H, W] array (pinned memory skips the staging copy)."""
        raw = np.ascontiguousarray(raw)
        if raw.nbytes < n * self.frame_bytes(fmt):
            raise ValueError(f"raw buffer holds {raw.nbytes} bytes, {n} frames need {n * self.frame_bytes(fmt)}")
        hmap = out if out is not None else np.empty((n,) + self.shape, np.float32)
        if hmap.dtype != np.float32 or hmap.shape[0] < n or hmap.shape[1:] != self.shape or not hmap.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float32 [n, H, W] array")
        _check(self._lib.fcd_process_raw(self._h, raw.ctypes.data, int(fmt), int(n), FCD_HOST_PTRS, float(height),
                                         int(bool(unwrap)), hmap.ctypes.data, None, None, None))
        return hmap[:n]

    def process_device(self, frames_ptr, n, height, unwrap, height_ptr, wrapped_ptr=None, k_ptr=None,
                       stream=None):
        """Device-pointer variant (e.g. torch tensors' data_ptr()); asynchronous on `stream`."""
        _check(self._lib.fcd_process(self._h, ctypes.c_void_p(frames_ptr), int(n), FCD_DEVICE_PTRS, float(height),
                                     int(bool(unwrap)), ctypes.c_void_p(height_ptr) if height_ptr else None,
                                     ctypes.c_void_p(wrapped_ptr) if wrapped_ptr else None,
                                     ctypes.c_void_p(k_ptr) if k_ptr else None,
                                     ctypes.c_void_p(stream) if stream else None))

    def profile(self, enable=True):
        _check(self._lib.fcd_profile(self._h, int(bool(enable))))

    def stage_times(self):
        """(ms dict {demod, unwrap, integrate, total, fixup, fixup_frames, launches, chunk}, frames) since the last call."""
        out = (ctypes.c_double * 8)()
        nf = ctypes.c_int64()
        _check(self._lib.fcd_stage_times(self._h, out, ctypes.byref(nf)))
        keys = ("demod", "unwrap", "integrate", "total", "fixup", "fixup_frames", "launches", "chunk")
        return dict(zip(keys, list(out))), nf.value

    def phases_from_spectrum(self, spectrum, unwrap=True):
        sp = np.ascontiguousarray(spectrum, dtype=np.complex64)
        if sp.ndim == 2:
            sp = sp[None]
        n = sp.shape[0]
        wrapped = np.empty((n, 2) + self.shape, np.float32)
        k = np.empty((n, 2) + self.shape, np.int32)
        _check(self._lib.fcd_phases_from_spectrum(self._h, sp.ctypes.data, n, FCD_HOST_PTRS, int(bool(unwrap)),
                                                  wrapped.ctypes.data, k.ctypes.data, None))
        return wrapped, k

    def unwrap(self, maps):
        m = _f32(maps)
        if m.ndim == 2:
            m = m[None]
        n = m.shape[0]
        k = np.empty(m.shape, np.int32)
        res = np.empty(n, np.int32)
        _check(self._lib.fcd_unwrap(self._h, m.ctypes.data, n, FCD_HOST_PTRS, k.ctypes.data, res.ctypes.data, None))
        return k, res

    def integrate(self, gx, gy, calibration_factor=1.0):
        x, y = _f32(gx), _f32(gy)
        squeeze = x.ndim == 2
        if squeeze:
            x, y = x[None], y[None]
        h = np.empty(x.shape, np.float32)
        _check(self._lib.fcd_integrate(self._h, x.ctypes.data, y.ctypes.data, x.shape[0], float(calibration_factor),
                                       FCD_HOST_PTRS, h.ctypes.data, None))
        return h[0] if squeeze else h

    def fft2(self, images):
        """scipy.fft.fft2 of real images, bit for bit: float32 -> complex64, float64 -> complex128."""
        x = _img(images)
        squeeze = x.ndim == 2
        if squeeze:
            x = x[None]
        out = np.empty(x.shape, np.complex128 if x.dtype == np.float64 else np.complex64)
        _check(self._lib.fcd_fft2(self._h, x.ctypes.data, x.shape[0], FCD_HOST_PTRS | _img_flag(x), out.ctypes.data,
                                  None))
        return out[0] if squeeze else out


    # ---- temporal analysis of a [T][rows][cols] float32 map stack
    @staticmethod
    def _stack(stack, block):
        """(contiguous stack, dims, flags): float64 stacks stay float64 (FCD_STACK_F64),
        as the reference hands them to numpy / scipy unchanged; everything else goes
        as float32."""
        st = np.asarray(stack)
        if st.ndim != 3:
            raise ValueError("stack must be [T, rows, cols]")
        dt = np.float64 if st.dtype == np.float64 else np.float32
        if st.dtype != dt or not st.flags.c_contiguous:
            st = np.ascontiguousarray(st, dtype=dt)
        T, rows, cols = st.shape
        r0, c0, bh, bw = block if block is not None else (0, 0, rows, cols)
        flags = FCD_HOST_PTRS | (FCD_STACK_F64 if dt == np.float64 else 0)
        return st, (int(T), int(rows), int(cols), int(r0), int(c0), int(bh), int(bw)), flags

    def temporal_spectrum(self, stack, nf, block=None):
        """(sum of |X(f)| over non-NaN pixels, their count) for bins f < nf of the
        temporal DFT of every pixel of the block (r0, c0, bh, bw)."""
        st, dims, flags = self._stack(stack, block)
        sc = np.empty((int(nf), 2), np.float64)
        _check(self._lib.fcd_temporal_spectrum(self._h, st.ctypes.data, *dims, flags, int(nf), sc.ctypes.data, None))
        return sc[:, 0], sc[:, 1]

    def temporal_bins(self, stack, bins, block=None):
        """complex128 [bh, bw, len(bins)]: the temporal DFT of every pixel at `bins`."""
        st, dims, flags = self._stack(stack, block)
        b = np.ascontiguousarray(bins, dtype=np.int32)
        out = np.empty((dims[5], dims[6], len(b)), np.complex128)
        _check(self._lib.fcd_temporal_bins(self._h, st.ctypes.data, *dims, flags, b.ctypes.data, len(b),
                                           out.ctypes.data, None))
        return out

    def spectrogram(self, stack, nperseg, noverlap, window, fs, block=None):
        """float64 [bh, bw, nperseg // 2 + 1, nseg] one-sided PSD of every pixel's series."""
        st, dims, flags = self._stack(stack, block)
        w = np.ascontiguousarray(window, dtype=np.float64)
        if w.shape != (int(nperseg),):
            raise ValueError("window length must equal nperseg")
        nseg = (dims[0] - nperseg) // (nperseg - noverlap) + 1
        out = np.empty((dims[5], dims[6], nperseg // 2 + 1, max(nseg, 0)), np.float64)
        _check(self._lib.fcd_spectrogram(self._h, st.ctypes.data, *dims, flags, int(nperseg), int(noverlap),
                                         w.ctypes.data, float(fs), out.ctypes.data, None))
        return out


_engines = collections.OrderedDict()  # (shape, device, thread) -> Engine, least recently used first
_engines_lock = threading.Lock()


def _engine_cache_size():
    return max(1, int(os.environ.get("FCD_ENGINE_CACHE", "4")))


def engine_for(shape, device=None):
    """Process-wide engine cache: one engine per (shape, device, host thread) -- a context
    is driven by one host thread at a time (fcd.h) -- and at most FCD_ENGINE_CACHE (4)
    shapes per thread and device, the least recently used closed first; the engines of
    threads that have ended are closed on the next miss.  A stateless drop-in call
    (fcd.py:13-35) therefore never accumulates device memory beyond that bound; each
    engine's chunk workspace is itself sized to the calls it has served (fcd_process)."""
    tid = threading.get_ident()
    key = (tuple(int(s) for s in shape), device, tid)
    stale = []
    with _engines_lock:
        e = _engines.pop(key, None)
        if e is None:
            alive = {t.ident for t in threading.enumerate()}
            for k in [k for k in _engines if k[2] not in alive]:
                stale.append(_engines.pop(k))
            mine = [k for k in _engines if k[1] == device and k[2] == tid]
            while len(mine) >= _engine_cache_size():
                stale.append(_engines.pop(mine.pop(0)))
            e = Engine(shape, device)
        _engines[key] = e  # most recently used last
    for old in stale:
        old.close()
    return e


def temporal_engine(device=None):
    """The engine context the temporal-analysis calls run on (any frame shape will
    do: they take the stack's own shape)."""
    return engine_for((64, 64), device)


class PinnedBuffer:
    """Page-locked host memory from the engine (fcd_host_alloc) viewed as a numpy
    array: frames decoded into it, or heights written to it, cross PCIe by DMA
    without a staging copy."""

    def __init__(self, shape, dtype):
        lib = load_library()
        self._lib = lib
        self.nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = ctypes.c_void_p()
        _check(lib.fcd_host_alloc(self.nbytes, ctypes.byref(p)))
        self._p = p
        buf = (ctypes.c_char * max(self.nbytes, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def free(self):
        if getattr(self, "_p", None):
            self.array = None
            self._lib.fcd_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
