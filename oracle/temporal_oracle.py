"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's temporal post-analysis of a map stack
(SURVEY.md §8f row 4), used as the parity checker by tests/ only; the product
(trapped-modes-ltg_amd/pydata/analyze.py) never imports it.

Follows /root/reference/pydata/analyze.py:
  * block_split      analyze.py:364-417  (block of every map, NaN where the first map is 0)
  * block_amplitude  analyze.py:543-587  (np.fft.fft over time in f64, f0 from the
                                          nanmean |spectrum| via scipy.signal.find_peaks)
  * spectrogram      analyze.py:419-531  (scipy.signal.spectrogram per pixel, NaN gaps
                                          filled by np.interp, all-NaN pixels -> NaN)

Pinned (round 3) to the reference module's own outputs: tests/golden/make_golden.py
imports analyze.py as shipped, with a placeholder for its module-level `import cv2`
(analyze.py:21; cv2 is used only on the polar paths, which no fixture runs), and
records block_split / block_amplitude / spectrogram on synthetic map folders
(tests/golden/analyze_ref.npz); tests/test_analyze_ref.py checks this restatement
against them at 1e-12.  The restatement uses the same numpy / scipy calls the
reference makes, on in-memory stacks instead of map folders.
"""
import numpy as np
from scipy import signal


def block_of(stack, num_blocks=64, block_index=0):
    """(i0, j0, size) of block `block_index` of a [T, H, W] stack (analyze.py:395-402)."""
    per_row = int(np.sqrt(num_blocks))
    size = stack.shape[1] // per_row
    return (block_index // per_row) * size, (block_index % per_row) * size, size


def block_split(stack, num_blocks=64, block_index=0, zero=0):
    """[size, size, T] block series, NaN where the FIRST map is exactly 0 (analyze.py:386-417,
    with analyze.py:557-567's `- zero` applied to every map first)."""
    stack = np.asarray(stack)
    valid = stack[0] != 0
    i0, j0, n = block_of(stack, num_blocks, block_index)
    maps = [np.where(valid[i0:i0 + n, j0:j0 + n], (m - zero)[i0:i0 + n, j0:j0 + n], np.nan) for m in stack]
    return np.transpose(np.stack(maps, axis=0), (1, 2, 0))


def block_amplitude(stack, f0=None, tasa=500, mode=1, num_blocks=64, block_index=0, zero=0):
    """(harmonics, amps, phases, f0) of analyze.block_amplitude (analyze.py:543-587)."""
    from scipy.signal import find_peaks
    maps = block_split(stack, num_blocks, block_index, zero)
    ny, nx, N = maps.shape
    spec = np.fft.fft(maps.astype(np.float64), axis=-1)
    freqs = np.fft.fftfreq(N, d=1 / tasa)
    keep = freqs >= 0
    spec, freqs = spec[:, :, keep], freqs[keep]
    if f0 is None:
        with np.errstate(invalid="ignore"):
            mean_spectrum = np.nanmean(np.abs(spec), axis=(0, 1))
        peaks, _ = find_peaks(mean_spectrum)
        if len(peaks) == 0:
            return (np.zeros(mode), np.full((ny, nx, mode), None, dtype=object),
                    np.full((ny, nx, mode), None, dtype=object), None, None)
        f0 = freqs[peaks[np.argmax(mean_spectrum[peaks])]]
    harmonics = [f0 * n for n in range(0, mode)]
    idx = [int(np.argmin(np.abs(freqs - f))) for f in harmonics]
    amps = np.zeros((ny, nx, mode + 1))
    phases = np.zeros((ny, nx, mode + 1))
    for k, i in enumerate(idx):
        v = spec[:, :, i]
        amps[:, :, k] = (1 if k == 0 else 2) * np.abs(v) / N
        phases[:, :, k] = np.angle(v)
    return harmonics, amps, phases, f0


def spectrogram_series(x, fs=125, **kw):
    """(t, f, Sxx) of scipy.signal.spectrogram on one series (analyze.py:486-497)."""
    f, t, sxx = signal.spectrogram(x, fs=fs, **kw)
    return t, f, sxx


def spectrogram_block(stack, fs=125, num_blocks=64, block_index=0, **kw):
    """(t, f, Sxx_all, Sxx_avg) of analyze.spectrogram on a block (analyze.py:499-527)."""
    maps = block_split(stack, num_blocks, block_index)
    ny, nx, N = maps.shape
    f, t, ex = signal.spectrogram(maps[0, 0, :], fs=fs, **kw)
    out = np.empty((ny, nx, len(f), len(t)))
    for iy in range(ny):
        for ix in range(nx):
            ts = maps[iy, ix, :]
            bad = np.isnan(ts)
            if bad.all():
                out[iy, ix] = np.nan
                continue
            if bad.any():
                ar = np.arange(len(ts))
                ts = np.interp(ar, ar[~bad], ts[~bad])
            out[iy, ix] = signal.spectrogram(ts, fs=fs, **kw)[2]
    with np.errstate(invalid="ignore"):
        avg = np.nanmean(out, axis=(0, 1))
    return t, f, out, avg
