"""Throughput of the temporal post-analysis on one MI355X.

Workload: a device-resident stack of T = 2000 height maps of 1024 x 1024 (8 GB float32,
random values: the DFTs are data-independent), one 128 x 128 block (num_blocks = 64,
the reference's default) per call:
  * block_amplitude's mean spectrum: the temporal DFT of 16384 pixel series at all
    1000 non-negative bins (fcd_temporal_spectrum), f64 accumulation;
  * the harmonic bins (fcd_temporal_bins, 3 bins);
  * spectrogram of every pixel (fcd_spectrogram, nperseg 256, noverlap 32, Tukey 0.25).
Roofline: 4 flops per (pixel, sample, bin) (two f64 FMAs) against 78.6 TFLOP/s, the
f64 peak of both the matrix cores (the mean-spectrum GEMM, k_tdft_mfma) and the vector
units (vendor spec).  CPU: the oracle's
numpy / scipy calls (the reference's own, analyze.py:497, :521, :574) on a sample of the block's series, 1 core.

The mean spectrum is timed on both paths (FCD_TDFT_FFT=0: the direct DFT, =1: the
Bluestein / four-step FFT of kernels_tfft.hip, two real series per transform, HBM-bound:
4 B x T + 2 x 16 B x M + 16 B x T per series, M = 2^ceil(log2(2T - 1))).

    python tools/temporal_bench.py [--T 2000] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")]

import torch  # noqa: E402  (first: the engine binds to torch's HIP runtime)
import numpy as np  # noqa: E402

from pyfcd import _lib  # noqa: E402

F64_PEAK = 78.6e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2000)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--block", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    T, n, b = a.T, a.n, a.block
    g = torch.Generator(device=dev).manual_seed(0)
    stack = torch.randn((T, n, n), generator=g, device=dev, dtype=torch.float32)
    torch.cuda.synchronize()
    eng = _lib.temporal_engine()
    lib = _lib.load_library()
    P, nf = b * b, (T + 1) // 2
    sc = np.empty((nf, 2), np.float64)
    dims = (T, n, n, 0, 0, b, b)

    def spectrum():
        _lib._check(lib.fcd_temporal_spectrum(eng.handle, ctypes.c_void_p(stack.data_ptr()), *dims,
                                              _lib.FCD_DEVICE_PTRS, nf, sc.ctypes.data, None))

    bins = np.array([0, 40, 80], np.int32)
    xb = torch.empty((P, len(bins), 2), dtype=torch.float64, device=dev)

    def harmonics():
        _lib._check(lib.fcd_temporal_bins(eng.handle, ctypes.c_void_p(stack.data_ptr()), *dims, _lib.FCD_DEVICE_PTRS,
                                          bins.ctypes.data, len(bins), ctypes.c_void_p(xb.data_ptr()), None))

    from scipy.signal import get_window
    nperseg, nover = 256, 32
    win = get_window(("tukey", 0.25), nperseg).astype(np.float64)
    nseg = (T - nperseg) // (nperseg - nover) + 1
    nfs = nperseg // 2 + 1
    sx = torch.empty((P, nfs, nseg), dtype=torch.float64, device=dev)

    def spectro():
        _lib._check(lib.fcd_spectrogram(eng.handle, ctypes.c_void_p(stack.data_ptr()), *dims, _lib.FCD_DEVICE_PTRS,
                                        nperseg, nover, win.ctypes.data, 500.0, ctypes.c_void_p(sx.data_ptr()), None))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps

    def with_env(val, fn):
        old = os.environ.get("FCD_TDFT_FFT")
        os.environ["FCD_TDFT_FFT"] = val
        try:
            return timed(fn)
        finally:
            if old is None:
                del os.environ["FCD_TDFT_FFT"]
            else:
                os.environ["FCD_TDFT_FFT"] = old

    t_spec = timed(spectrum)
    t_fft = with_env("1", spectrum)
    t_direct = with_env("0", spectrum)
    M = 1 << max(2, (2 * T - 2).bit_length())
    # stack read + 4 passes of the [M] f64 complex work per pixel pair + the pair's spectrum
    # written and read back (16 B x T per pixel pair each way)
    fft_bytes = P * (4.0 * T + 2 * 16.0 * M + 16.0 * T)
    t_harm = timed(harmonics)
    t_spg = timed(spectro)
    flops_spec = 4.0 * P * T * nf  # the direct DFT's count (the default path when T <= 8192)
    flops_spg = 4.0 * P * nseg * nperseg * nfs

    # CPU: the reference's calls on a sample of the block's series (1 core)
    from scipy import signal
    host = stack[:, :b, :b].cpu().numpy()
    ns = 1024
    series = host.reshape(T, -1)[:, :ns].T.astype(np.float64)
    c0 = time.perf_counter()
    np.abs(np.fft.fft(series, axis=-1))
    cpu_fft = ns / (time.perf_counter() - c0)
    ns2 = 256
    c0 = time.perf_counter()
    for i in range(ns2):
        signal.spectrogram(host.reshape(T, -1)[:, i], fs=500.0, nperseg=nperseg, noverlap=nover)
    cpu_spg = ns2 / (time.perf_counter() - c0)
    print(json.dumps({
        "metric": "temporal post-analysis of a map stack (block_amplitude / spectrogram), pixel series per second",
        "workload": f"{T} maps of {n}x{n} float32 in HBM, one {b}x{b} block per call (num_blocks=64)",
        "block_amplitude_spectrum": {"ms": t_spec * 1e3, "series_per_s": P / t_spec, "bins": nf},
        "direct_dft_roofline": {"bound": "f64 (matrix cores; FCD_TDFT_VALU=1 or T > 8192: vector)",
                                "achieved_tflops": flops_spec / t_direct / 1e12, "peak_tflops": F64_PEAK / 1e12,
                                "frac": flops_spec / t_direct / F64_PEAK},
        "block_amplitude_spectrum_paths": {
            "default": os.environ.get("FCD_TDFT_FFT_DEFAULT", "see kernels_tfft.hip"), "direct_ms": t_direct * 1e3, "fft_ms": t_fft * 1e3,
            "fft_roofline": {"bound": "hbm", "M": M, "bytes_per_series": fft_bytes / P,
                             "achieved_gbs": fft_bytes / t_fft / 1e9, "peak_gbs": 8000.0,
                             "frac": fft_bytes / t_fft / 8e12}},
        "block_amplitude_harmonics": {"ms": t_harm * 1e3, "bins": len(bins)},
        "spectrogram": {"ms": t_spg * 1e3, "series_per_s": P / t_spg, "nperseg": nperseg, "segments": nseg,
                        "achieved_tflops": flops_spg / t_spg / 1e12, "frac": flops_spg / t_spg / F64_PEAK},
        "cpu_baseline": {"kind": "port", "cores": 1,
                         "fft_series_per_s": cpu_fft, "fft_sample": f"np.fft.fft of {ns} series of {T} (f64)",
                         "spectrogram_series_per_s": cpu_spg,
                         "spectrogram_sample": f"scipy.signal.spectrogram of {ns2} float32 series (the reference's loop)"},
    }))


if __name__ == "__main__":
    main()
