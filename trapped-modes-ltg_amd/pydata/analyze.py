"""Drop-in for the hot-path part of `pydata.analyze` (/root/reference/pydata/analyze.py):
the frame loader, the floating-structure mask, and the batch driver `analyze.folder`
(SURVEY.md §8f rows 1-2), and the temporal post-analysis of the map stack
(`block_split`, `block_amplitude`, `spectrogram`; §8f row 4) on the device.  The other
post-analysis members of the reference class (video, polar warps, ...) are out of scope
(DESIGN.md §8).

`analyze.folder` keeps the reference's contract -- directory of `.tif` frames ->
`maps/{name}_map.npy` (float32) + `maps/calibration_factor.npy`, resumable at file
granularity, optional mask blend -- but runs it as a pipeline instead of one frame at a
time: the carriers are computed once per reference (the reference recomputes them for
every frame, fcd.py:26 via compute_height_map), frames are decoded by a thread pool
straight into page-locked buffers, unmasked frames cross PCIe as raw samples
(fcd_process_raw: 1.25 B/px for the 10-bit camera TIFFs instead of 4 B/px float32),
batches overlap upload / compute / download on the device, and an ordered writer
thread saves the maps.
"""
import os
import threading
from concurrent.futures import ThreadPoolExecutor
from queue import Queue

import numpy as np
from scipy import ndimage

from pyfcd import _lib
from pyfcd.fcd import fcd, _engine_with_reference
from pydata import images

_EIGHT = np.ones((3, 3), bool)  # skimage.measure.label's default full (8-) connectivity in 2-D


class analyze:
    """Classmethod namespace, as in the reference (analyze.py:24)."""

    @classmethod
    def load_image(cls, path):
        """io.imread(path, as_gray=True).astype(np.float32) (analyze.py:25-40)."""
        return np.asarray(images.read_gray(path)).astype(np.float32)

    @classmethod
    def mask(cls, image, smoothed=14, show_mask=False, find_center=False):
        """Largest connected region darker than the mean of the box-smoothed image
        (analyze.py:42-100): uniform_filter(size=smoothed) -> `< mean` -> 8-connected
        labels in raster order -> largest area (first label on ties, the reference's
        stable descending sort)."""
        smooth = ndimage.uniform_filter(image, size=smoothed)
        threshold = np.mean(smooth)
        dark = smooth < threshold
        labels, n = ndimage.label(dark, structure=_EIGHT)
        if n == 0:
            raise IndexError("list index out of range")  # regions_sorted[0] on an empty list
        areas = np.bincount(labels.ravel())[1:]
        mask = labels == (int(np.argmax(areas)) + 1)
        if show_mask:
            import matplotlib.pyplot as plt
            fig, ax = plt.subplots(1, 3, figsize=(10, 4))
            for a, im, t in zip(ax, (image, mask, image * mask), ("Original image", "Mask", "Masked image")):
                a.imshow(im, cmap="gray")
                a.set_title(t)
                a.axis("off")
            plt.tight_layout()
            plt.show()
        if find_center:
            return mask, cls.center(mask)
        return mask

    @classmethod
    def center(cls, mask):
        """(cy, cx) of the largest hole of the mask that does not touch the image border
        (analyze.py:102-139): 8-connected labels of ~mask, bbox strictly inside, max area
        (first on ties), centroid truncated to int."""
        labels, n = ndimage.label(~mask, structure=_EIGHT)
        rows, cols = mask.shape
        best, best_area = None, -1
        areas = np.bincount(labels.ravel(), minlength=n + 1)
        for k, sl in enumerate(ndimage.find_objects(labels), start=1):
            if sl is None:
                continue
            r0, r1, c0, c1 = sl[0].start, sl[0].stop, sl[1].start, sl[1].stop
            if r0 > 0 and c0 > 0 and r1 < rows and c1 < cols and areas[k] > best_area:
                best, best_area = k, areas[k]
        if best is None:
            # the reference reaches `return center` with `center` unbound
            raise UnboundLocalError("local variable 'center' referenced before assignment")
        coords = np.argwhere(labels == best)
        cy, cx = coords.mean(axis=0)
        return (int(cy), int(cx))

    @classmethod
    def folder(cls, reference_path, displaced_dir, layers, square_size, smoothed=None, polar=False, show_mask=False,
               batch=32, workers=8, **kwargs):
        """Height maps of every `.tif` frame of `displaced_dir` (analyze.py:142-286).

        Same files as the reference: sorted `*.tif` without 'reference' in the name;
        `maps/{name}_map.npy` float32, resuming after the maps already present;
        `maps/calibration_factor.npy` (np.array([cf])) written once per call;
        with `smoothed`, each frame's mask region is replaced by the reference
        before the demodulation, the height there is zeroed, and `maps/centers.txt`
        gets one `i\\t(cy, cx)` line per frame (resuming after its lines).
        `batch` frames go to the device per call (`workers` decoder threads).
        """
        if polar:
            raise NotImplementedError("polar maps (analyze.polar / cv2.fitEllipse) are outside the FCD hot path")
        if show_mask:
            if not smoothed:
                raise ValueError("If show_mask == True, expect smoothed too")
            raise NotImplementedError("interactive mask preview (analyze.py:184-203) is not provided")
        reference = cls.load_image(reference_path)
        tif_list = [f for f in sorted(os.listdir(displaced_dir)) if f.endswith(".tif") and "reference" not in f]
        output_dir = os.path.join(displaced_dir, "maps")
        os.makedirs(output_dir, exist_ok=True)
        start_index = len([f for f in os.listdir(output_dir) if f.endswith("_map.npy")])
        centers_path = os.path.join(output_dir, "centers.txt")
        if smoothed:
            if not os.path.exists(centers_path):
                open(centers_path, "w").close()
            with open(centers_path) as f:
                start_index = max(start_index, len(f.readlines()))
        todo = list(enumerate(tif_list))[start_index:]
        if not todo:
            return
        height = 1 if layers is None else fcd.height_from_layers(layers)
        eng = _engine_with_reference(reference, square_size)
        cf = eng.info.calibration_factor
        np.save(os.path.join(output_dir, "calibration_factor.npy"), np.array([cf]))
        shape = reference.shape
        # unmasked frames cross PCIe raw, in the first pending frame's layout (checked per frame)
        fmt = _lib.FCD_FMT_F32
        if not smoothed:
            fmts = {images.raw_info(os.path.join(displaced_dir, f))[2] for _, f in todo[:1]}
            fmt = fmts.pop()
        fb = eng.frame_bytes(fmt)
        nb = max(1, min(batch, len(todo)))
        in_bufs = [_lib.PinnedBuffer((nb * fb,), np.uint8) for _ in range(2)]
        out_bufs = [_lib.PinnedBuffer((nb,) + shape, np.float32) for _ in range(2)]
        writes = Queue(maxsize=2)
        err = []

        def writer():
            while True:
                item = writes.get()
                if item is None:
                    return
                slot, names, masks, centers, idx = item
                try:
                    for j, name in enumerate(names):
                        h = out_bufs[slot].array[j]
                        if masks is not None:
                            h = h * ~masks[j]
                        np.save(os.path.join(output_dir, name.replace(".tif", "") + "_map.npy"), h.astype(np.float32))
                        if centers is not None:
                            with open(centers_path, "a") as f:
                                f.write(f"{idx[j]}\t{centers[j]}\n")
                except Exception as e:  # surfaced after the loop
                    err.append(e)
                finally:
                    done[slot].set()

        done = [threading.Event(), threading.Event()]
        for d in done:
            d.set()
        wt = threading.Thread(target=writer, daemon=True)
        wt.start()

        def decode(args):
            slot, j, name = args
            path = os.path.join(displaced_dir, name)
            dst = in_bufs[slot].array[j * fb:(j + 1) * fb]
            if not smoothed:
                raw, f = images.read_raw(path, out=dst)
                if f != fmt or raw.size != fb:
                    raise ValueError(f"{name}: raw layout differs from the first frame's")
                return None, None
            disp = cls.load_image(path)
            m = cls.mask(disp, smoothed=smoothed)
            blend = np.where(m == 1, reference, disp).astype(np.float32)
            dst.view(np.float32)[:] = blend.ravel()
            return m, cls.center(m)

        batches = [todo[k:k + nb] for k in range(0, len(todo), nb)]
        try:
            with ThreadPoolExecutor(max_workers=workers) as pool:
                def submit(b):
                    return [pool.submit(decode, (b & 1, j, name)) for j, (_, name) in enumerate(batches[b])]

                pending = submit(0)
                for b, part in enumerate(batches):
                    slot = b & 1
                    res = [f.result() for f in pending]
                    if b + 1 < len(batches):
                        pending = submit(b + 1)  # decoded while this batch is on the device
                    done[slot].wait()  # the writer has saved this slot's previous batch
                    done[slot].clear()
                    eng.process_raw(in_bufs[slot].array, fmt, len(part), height, unwrap=True,
                                    out=out_bufs[slot].array)
                    masks = [r[0] for r in res] if smoothed else None
                    centers = [r[1] for r in res] if smoothed else None
                    writes.put((slot, [n for _, n in part], masks, centers, [i for i, _ in part]))
                    if err:
                        break
        finally:
            writes.put(None)
            wt.join()
            for buf in in_bufs + out_bufs:
                buf.free()
        if err:
            raise err[0]

    # ---- temporal post-analysis of the map stack
    @staticmethod
    def _map_files(map_folder, t_limit=None):
        files = sorted(f for f in os.listdir(map_folder) if f.endswith("_map.npy") and "calibration_factor" not in f)
        return files[:t_limit]

    @classmethod
    def _block_stack(cls, map_folder, t_limit=None, num_blocks=64, block_index=0, zero=0):
        """[T, size, size] block of every map (memory-mapped reads of just the block), NaN
        where the first map is 0 (analyze.py:386-417; `- zero` as analyze.py:557-567), in
        the dtype the reference's arithmetic gives: the maps' own float dtype (float32
        from analyze.folder, float64 kept float64), promoted by an array `zero` the way
        numpy promotes `m - zero` (a scalar `zero` does not promote, numpy 1.x value-based
        casting as in the reference's environment); non-float maps become float64 (the
        NaN fill)."""
        files = cls._map_files(map_folder, t_limit)
        first = np.load(os.path.join(map_folder, files[0]), mmap_mode="r")
        H, W = first.shape
        per_row = int(np.sqrt(num_blocks))
        n = H // per_row
        i0, j0 = (block_index // per_row) * n, (block_index % per_row) * n
        valid = np.asarray(first[i0:i0 + n, j0:j0 + n]) != 0
        z = zero
        dt = first.dtype if np.issubdtype(first.dtype, np.floating) else np.dtype(np.float64)
        if np.ndim(zero) == 2:
            z = np.asarray(zero)[i0:i0 + n, j0:j0 + n]
            dt = np.result_type(dt, z.dtype)
            if not np.issubdtype(dt, np.floating):
                dt = np.dtype(np.float64)
        out = np.empty((len(files), n, n), dt)
        for t, f in enumerate(files):
            m = np.load(os.path.join(map_folder, f), mmap_mode="r")[i0:i0 + n, j0:j0 + n]
            out[t] = np.where(valid, np.asarray(m) - z, np.nan)
        return out

    @classmethod
    def block_split(cls, map_folder, t_limit=None, num_blocks=64, block_index=0):
        """[size, size, T] series of one spatial block (analyze.py:364-417)."""
        return np.transpose(cls._block_stack(map_folder, t_limit, num_blocks, block_index), (1, 2, 0))

    @classmethod
    def block_amplitude(cls, map_folder, f0=None, tasa=500, mode=1, num_blocks=64, block_index=0, zero=0):
        """(harmonics, amps, phases, f0) of every pixel of a block (analyze.py:543-587).

        The temporal DFT runs on the device in f64 (fcd_temporal_spectrum for the
        nanmean |spectrum| that locates f0, fcd_temporal_bins for the harmonics); the
        reference's quirks are kept: amps / phases have mode + 1 columns of which
        the first `mode` are filled, and no spectral peak returns five values."""
        from scipy.signal import find_peaks
        stack = cls._block_stack(map_folder, None, num_blocks, block_index, zero)
        N, ny, nx = stack.shape
        eng = _lib.temporal_engine()
        freqs = np.fft.fftfreq(N, d=1 / tasa)
        freqs = freqs[freqs >= 0]
        if f0 is None:
            tot, cnt = eng.temporal_spectrum(stack, len(freqs))
            with np.errstate(invalid="ignore", divide="ignore"):
                mean_spectrum = tot / cnt
            peaks, _ = find_peaks(mean_spectrum)
            if len(peaks) == 0:
                return (np.zeros(mode), np.full((ny, nx, mode), None, dtype=object),
                        np.full((ny, nx, mode), None, dtype=object), None, None)
            f0 = freqs[peaks[np.argmax(mean_spectrum[peaks])]]
        harmonics = [f0 * n for n in range(0, mode)]
        idx = [int(np.argmin(np.abs(freqs - f))) for f in harmonics]
        X = eng.temporal_bins(stack, idx)
        amps = np.zeros((ny, nx, mode + 1))
        phases = np.zeros((ny, nx, mode + 1))
        amps[:, :, :mode] = np.abs(X) / N
        amps[:, :, 1:mode] *= 2
        phases[:, :, :mode] = np.angle(X)
        return harmonics, amps, phases, f0

    @staticmethod
    def _spectro_params(T, fs, kwargs):
        """scipy.signal.spectrogram's defaults: window ('tukey', .25), nperseg 256
        (clipped to the series length), noverlap nperseg // 8."""
        from scipy.signal import get_window
        window = kwargs.get("window", ("tukey", 0.25))
        nperseg = kwargs.get("nperseg")
        if isinstance(window, (str, tuple)):
            nperseg = 256 if nperseg is None else int(nperseg)
            if nperseg > T:
                nperseg = T
            win = get_window(window, nperseg)
        else:
            win = np.asarray(window, np.float64)
            if nperseg is None:
                nperseg = len(win)
            if len(win) != nperseg:
                raise ValueError("value specified for nperseg is different from length of window")
        noverlap = kwargs.get("noverlap")
        noverlap = nperseg // 8 if noverlap is None else int(noverlap)
        if noverlap >= nperseg:
            raise ValueError("noverlap must be less than nperseg.")
        f = np.fft.rfftfreq(nperseg, 1 / fs)
        t = np.arange(nperseg / 2, T - nperseg / 2 + 1, nperseg - noverlap) / float(fs)
        return nperseg, noverlap, np.asarray(win, np.float64), f, t

    @classmethod
    def spectrogram(cls, map_folder=None, array=None, fs=125, show=False, **kwargs):
        """analyze.spectrogram (analyze.py:419-531): (t, f, Sxx) of one series, or
        (t, f, Sxx_all [ny, nx, nf, nt], Sxx_avg) of every pixel of a block, one-sided
        PSD (scipy.signal.spectrogram's density scaling, constant detrend) computed on
        the device in f64.  Block pixels with NaN gaps are filled by np.interp first,
        all-NaN pixels give NaN, as in the reference."""
        block_kw = {k: kwargs[k] for k in ("t_limit", "num_blocks", "block_index") if k in kwargs}
        eng = _lib.temporal_engine()
        if map_folder is None:
            if array is None:
                raise ValueError("Any map_folder or array is needed")
            x = np.asarray(array)
            nperseg, noverlap, win, f, t = cls._spectro_params(len(x), fs, kwargs)
            # scipy keeps a float32 series in float32 and computes everything else in
            # float64: the series goes to the device in its own precision (float64 is
            # not rounded to float32 first) and S comes back in scipy's dtype
            dt = np.float32 if x.dtype == np.float32 else np.float64
            S = eng.spectrogram(x.astype(dt).reshape(-1, 1, 1), nperseg, noverlap, win, fs)[0, 0].astype(dt)
            if show:
                cls._show_spectrogram(t, f, S, "Spectrogram of some point")
            return t, f, S
        if array is not None:
            raise ValueError("map_folder or array is needed, not both")
        stack = cls._block_stack(map_folder, block_kw.get("t_limit"), block_kw.get("num_blocks", 64),
                                 block_kw.get("block_index", 0))
        N, ny, nx = stack.shape
        bad = np.isnan(stack)
        part = bad.any(axis=0) & ~bad.all(axis=0)
        if part.any():  # NaN gaps inside a pixel's series: linear fill (analyze.py:512-517)
            # np.interp returns float64 and the reference keeps those pixels in float64:
            # the whole stack goes to the device as float64 (exact for the float32 pixels)
            stack = stack.astype(np.float64)
            ar = np.arange(N)
            for iy, ix in zip(*np.nonzero(part)):
                ts = stack[:, iy, ix]
                ok = ~np.isnan(ts)
                stack[:, iy, ix] = np.interp(ar, ar[ok], ts[ok])
        nperseg, noverlap, win, f, t = cls._spectro_params(N, fs, kwargs)
        S = eng.spectrogram(stack, nperseg, noverlap, win, fs)
        with np.errstate(invalid="ignore"):
            avg = np.nanmean(S, axis=(0, 1))
        if show:
            cls._show_spectrogram(t, f, avg, "Average Spectrogram over block")
        return t, f, S, avg

    @staticmethod
    def _show_spectrogram(t, f, S, title):
        import matplotlib.pyplot as plt
        plt.figure(figsize=(8, 4))
        plt.pcolormesh(t, f, np.log10(S), shading="gouraud")
        plt.ylabel("Frequency [Hz]")
        plt.xlabel("Time [sec]")
        plt.title(title)
        plt.colorbar()
        plt.tight_layout()
        plt.show()
