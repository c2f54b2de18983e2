"""Temporal post-analysis of the map stack (analyze.py:364-587):
`analyze.block_split`, `analyze.block_amplitude`, `analyze.spectrogram`.

These tests check the device against oracle/temporal_oracle.py (the reference's numpy /
scipy calls restated on in-memory stacks) over many shapes and edge cases; the oracle
and the device path are pinned to the reference's OWN outputs in
tests/test_analyze_ref.py (analyze_ref.npz: block_split / block_amplitude / spectrogram
run by /root/reference/pydata/analyze.py itself).  The device DFTs accumulate in f64, so the
comparisons are at 1e-9 relative (the reference's np.fft is f64 as well; its
spectrogram of a float32 series runs in float32 inside scipy, which the f64 device
result beats — compared here against scipy on the f64 series).
"""
import os

import numpy as np
import pytest

from oracle import temporal_oracle as ora

TASA = 500.0


def make_stack(T, n=64, seed=0, f0=25.0, zero_corner=True, nan_pixels=()):
    """T maps of n x n: per-pixel harmonics of f0 (random amplitude / phase) + noise;
    the first map's top-left corner is 0 (masked block pixels), a few pixels carry
    NaN gaps in later maps (the spectrogram's interpolation path)."""
    rng = np.random.default_rng(seed)
    t = np.arange(T) / TASA
    a1 = rng.uniform(0.5, 1.5, (n, n))
    p1 = rng.uniform(-np.pi, np.pi, (n, n))
    a2 = rng.uniform(0.1, 0.3, (n, n))
    st = (a1[None] * np.cos(2 * np.pi * f0 * t[:, None, None] + p1[None])
          + a2[None] * np.cos(2 * np.pi * 2 * f0 * t[:, None, None] + 2 * p1[None])
          + 0.05 * rng.standard_normal((T, n, n)) + 0.2).astype(np.float32)
    if zero_corner:
        st[0, :5, :7] = 0.0
    for (i, j, t0, t1) in nan_pixels:
        st[t0:t1, i, j] = np.nan
    return st


def write_maps(folder, stack):
    os.makedirs(folder, exist_ok=True)
    for k, m in enumerate(stack):
        np.save(os.path.join(folder, f"frame{k:05d}_map.npy"), m)
    np.save(os.path.join(folder, "calibration_factor.npy"), np.array([1e-4]))


def close_nan(a, b, rtol=1e-9, atol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape
    assert np.array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(a)
    scale = np.abs(b[ok]).max() if ok.any() else 1.0
    np.testing.assert_allclose(a[ok], b[ok], rtol=0, atol=rtol * scale + atol)


# ---------------------------------------------------------------- CPU: oracle / host logic
def test_oracle_block_amplitude_recovers_harmonics():
    st = make_stack(500, n=16, zero_corner=False)
    harm, amps, phases, f0 = ora.block_amplitude(st, tasa=TASA, mode=3, num_blocks=4, block_index=0)
    assert f0 == 25.0 and harm == [0.0, 25.0, 50.0]
    assert np.allclose(amps[:, :, 0], 0.2, atol=0.01)  # mean
    assert np.all(amps[:, :, 3] == 0)                   # the reference's unused column


def test_spectro_params_match_scipy():
    from scipy import signal
    from pydata.analyze import analyze
    for T, kw in [(300, {}), (300, {"nperseg": 64}), (300, {"nperseg": 64, "noverlap": 40}), (100, {}),
                  (257, {"window": "hann", "nperseg": 32})]:
        x = np.random.default_rng(T).standard_normal(T)
        f_ref, t_ref, _ = signal.spectrogram(x, fs=125, **kw)
        nperseg, noverlap, win, f, t = analyze._spectro_params(T, 125, kw)
        assert np.array_equal(f, f_ref) and np.array_equal(t, t_ref), (T, kw)
        assert len(win) == nperseg


# ---------------------------------------------------------------- GPU: device vs oracle
@pytest.mark.gpu
@pytest.mark.parametrize("T,block", [(400, 0), (301, 3), (2000, 1)])
def test_block_amplitude_matches_oracle(tmp_path, T, block):
    """(2000 maps: the mean spectrum takes the FFT path by the engine's cost model.)"""
    from pydata.analyze import analyze
    st = make_stack(T, n=64, seed=T)
    write_maps(str(tmp_path), st)
    got = analyze.block_amplitude(str(tmp_path), tasa=TASA, mode=3, num_blocks=4, block_index=block)
    want = ora.block_amplitude(st, tasa=TASA, mode=3, num_blocks=4, block_index=block)
    assert got[3] == want[3] and got[0] == want[0]
    close_nan(got[1], want[1])
    ok = ~np.isnan(want[1][:, :, :3])
    np.testing.assert_allclose(got[2][:, :, :3][ok], want[2][:, :, :3][ok], atol=1e-7)
    if block == 0:
        assert np.isnan(got[1][0, 0, 0])  # masked pixel (first map 0)
    # given f0: only the harmonic bins are computed
    got2 = analyze.block_amplitude(str(tmp_path), f0=50.0, tasa=TASA, mode=2, num_blocks=4, block_index=block)
    want2 = ora.block_amplitude(st, f0=50.0, tasa=TASA, mode=2, num_blocks=4, block_index=block)
    assert got2[0] == want2[0]
    close_nan(got2[1], want2[1])


@pytest.mark.gpu
def test_block_amplitude_no_peak(tmp_path):
    from pydata.analyze import analyze
    # 3 maps: 2 non-negative bins, so find_peaks has no interior sample to report
    st = np.random.default_rng(0).uniform(1, 2, (3, 32, 32)).astype(np.float32)
    write_maps(str(tmp_path), st)
    got = analyze.block_amplitude(str(tmp_path), tasa=TASA, mode=2, num_blocks=4)
    want = ora.block_amplitude(st, tasa=TASA, mode=2, num_blocks=4)
    assert len(got) == len(want) == 5 and got[3] is None and got[4] is None
    assert np.array_equal(got[0], want[0]) and got[1].shape == want[1].shape


@pytest.mark.gpu
def test_temporal_engine_long_series():
    """T above the LDS table (the FFT path for the spectrum, the global-table kernel
    for the bins), odd T, a sub-block."""
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    st = make_stack(9001, n=16, seed=5, zero_corner=False)
    spec = np.fft.fft(st.astype(np.float64), axis=0)
    nf = 4501
    tot, cnt = eng.temporal_spectrum(st, nf)
    assert np.all(cnt == 256)
    np.testing.assert_allclose(tot, np.abs(spec[:nf]).sum(axis=(1, 2)), rtol=1e-9)
    bins = [0, 450, 900, 4500]
    X = eng.temporal_bins(st, bins, block=(4, 2, 8, 8))
    close_nan(X.real, np.transpose(spec[bins, 4:12, 2:10], (1, 2, 0)).real)
    close_nan(X.imag, np.transpose(spec[bins, 4:12, 2:10], (1, 2, 0)).imag)


def nan_spectrum(st, nf):
    """np.nanmean's numerator and denominator over the pixels of |np.fft.fft| (f64):
    a pixel with a NaN sample has every bin NaN and drops out."""
    spec = np.abs(np.fft.fft(st.astype(np.float64), axis=0)[:nf])
    ok = ~np.isnan(spec)
    return np.where(ok, spec, 0.0).sum(axis=(1, 2)), ok.sum(axis=(1, 2)).astype(np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("pair", ["1", "0"])
@pytest.mark.parametrize("T", [1, 2, 3, 5, 100, 257, 2000])
def test_temporal_fft_path_short_series(monkeypatch, T, pair):
    """The Bluestein / four-step FFT path (FCD_TDFT_FFT=1 forces it at any T): every
    sub-transform length from 2 up, odd and prime T, NaN pixels excluded as np.nanmean
    does, a sub-block addressed in place, against numpy's f64 FFT; two real series per
    transform (default) and one (FCD_TDFT_PAIR=0)."""
    from pyfcd import _lib
    monkeypatch.setenv("FCD_TDFT_FFT", "1")
    monkeypatch.setenv("FCD_TDFT_PAIR", pair)
    eng = _lib.temporal_engine()
    st = make_stack(T, n=20, seed=T, zero_corner=False, nan_pixels=[(3, 4, T // 2, T // 2 + 1)])
    nf = T // 2 + 1
    tot, cnt = eng.temporal_spectrum(st, nf)
    want_t, want_c = nan_spectrum(st, nf)
    assert np.array_equal(cnt, want_c) and cnt[0] == 399
    np.testing.assert_allclose(tot, want_t, rtol=1e-12)
    blk = (2, 5, 11, 13)
    tot, cnt = eng.temporal_spectrum(st, nf, block=blk)
    want_t, want_c = nan_spectrum(st[:, 2:13, 5:18], nf)
    assert np.array_equal(cnt, want_c)
    np.testing.assert_allclose(tot, want_t, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["0", "1"])
def test_temporal_spectrum_inf_sample_stays_in_its_pixel(monkeypatch, path):
    """A series holding an infinity (no NaN): np.fft gives it inf / NaN bins (which ones
    depends on the transform's butterflies: parity unpinned for non-finite input),
    np.nanmean keeps the inf ones.  Whichever path runs (direct DFT, or the FFT, which
    then takes one series per transform instead of pairing the pixel with a partner),
    every other pixel's contribution is unchanged: per bin either the pixel is left out
    (count P - 1, sum = the other pixels' sum) or it adds an infinite |X| (count P)."""
    from pyfcd import _lib
    monkeypatch.setenv("FCD_TDFT_FFT", path)
    eng = _lib.temporal_engine()
    T, n = 1200, 16
    st = make_stack(T, n=n, seed=21, zero_corner=False)
    P = n * n
    base = st.copy()
    base[:, 3, 9] = np.nan  # the pixel left out everywhere
    tb, cb = eng.temporal_spectrum(base, 300)
    assert (cb == P - 1).all()
    inf = st.copy()
    inf[T // 3, 3, 9] = np.inf
    ti, ci = eng.temporal_spectrum(inf, 300)
    left_out = ci == P - 1
    assert np.all(left_out | (ci == P))
    np.testing.assert_allclose(ti[left_out], tb[left_out], rtol=1e-12)
    assert np.all(np.isinf(ti[~left_out]))


@pytest.mark.gpu
def test_temporal_fft_equals_direct_dft(monkeypatch, tdft_family):
    """The FFT path and both direct-DFT kernel families agree to f64 rounding."""
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    st = make_stack(1500, n=40, seed=8, zero_corner=False)
    monkeypatch.setenv("FCD_TDFT_FFT", "0")
    direct = eng.temporal_spectrum(st, 751)
    monkeypatch.setenv("FCD_TDFT_FFT", "1")
    fft = eng.temporal_spectrum(st, 751)
    assert np.array_equal(direct[1], fft[1])
    np.testing.assert_allclose(fft[0], direct[0], rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("T,n", [(40000, 24), (300001, 8)])
def test_temporal_fft_long_series(T, n):
    """Long series (the default FFT range, T > 8192): 40000 maps of 576 pixels need two
    pixel batches of the work array; 300001 maps use the longest sub-transforms
    (M = 2^20 = 1024 x 1024).  Against numpy's f64 FFT, per bin."""
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    rng = np.random.default_rng(T)
    st = (rng.standard_normal((T, n, n)) + 3.0).astype(np.float32)
    nf = T // 2 + 1
    tot, cnt = eng.temporal_spectrum(st, nf)
    want_t, want_c = nan_spectrum(st, nf)
    assert np.array_equal(cnt, want_c)
    np.testing.assert_allclose(tot, want_t, rtol=1e-10)


@pytest.mark.gpu
def test_block_amplitude_zero_map(tmp_path):
    from pydata.analyze import analyze
    st = make_stack(256, n=32, seed=9)
    zero = st.mean(axis=0)
    write_maps(str(tmp_path), st)
    got = analyze.block_amplitude(str(tmp_path), tasa=TASA, mode=2, num_blocks=4, block_index=2, zero=zero)
    want = ora.block_amplitude(st, tasa=TASA, mode=2, num_blocks=4, block_index=2, zero=zero)
    assert got[3] == want[3]
    close_nan(got[1], want[1], rtol=1e-6)  # the maps minus a float32 mean, rounded to float32


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{"nperseg": 64}, {"nperseg": 50, "noverlap": 20, "window": "hann"}, {}])
def test_spectrogram_block_matches_oracle(tmp_path, kw):
    from pydata.analyze import analyze
    st = make_stack(300, n=32, seed=3, nan_pixels=[(10, 12, 40, 45), (20, 3, 100, 101)])
    write_maps(str(tmp_path), st)
    t, f, S, avg = analyze.spectrogram(map_folder=str(tmp_path), fs=TASA, num_blocks=4, block_index=0, **kw)
    # the oracle on the float64 series (scipy keeps float32 series in float32)
    t2, f2, S2, avg2 = ora.spectrogram_block(st.astype(np.float64), fs=TASA, num_blocks=4, block_index=0, **kw)
    assert np.array_equal(t, t2) and np.array_equal(f, f2)
    close_nan(S, S2)
    close_nan(avg, avg2)
    assert np.isnan(S[0, 0]).all() and not np.isnan(S[10, 12]).any()


@pytest.mark.gpu
def test_spectrogram_series():
    from pydata.analyze import analyze
    x = make_stack(1000, n=1, seed=1, zero_corner=False)[:, 0, 0]
    t, f, S = analyze.spectrogram(array=x, fs=TASA, nperseg=128)
    assert S.dtype == np.float32  # scipy's dtype for a float32 series
    t2, f2, S2 = ora.spectrogram_series(x.astype(np.float64), fs=TASA, nperseg=128)
    assert np.array_equal(t, t2) and np.array_equal(f, f2)
    close_nan(S, S2, rtol=1e-6)  # f64 on the device, rounded once to float32
    # and the reference's own float32 computation, to float32 accuracy
    t3, f3, S3 = ora.spectrogram_series(x, fs=TASA, nperseg=128)
    close_nan(S, S3, rtol=1e-5)


@pytest.fixture(params=["mfma", "valu"])
def tdft_family(request, monkeypatch):
    """Both kernel families: the f64 matrix-core kernels (default) and the vector-unit
    ones (FCD_TDFT_VALU=1, read by the engine on every call)."""
    if request.param == "valu":
        monkeypatch.setenv("FCD_TDFT_VALU", "1")
    else:
        monkeypatch.delenv("FCD_TDFT_VALU", raising=False)
    return request.param


def offset_series(T, dtype, dc=1000.0, amp=1e-4, seed=2):
    """A series whose mean is far larger than its fluctuation: the
    constant detrend must not lose the fluctuation's digits."""
    rng = np.random.default_rng(seed)
    t = np.arange(T) / TASA
    x = dc + amp * (np.sin(2 * np.pi * 31.0 * t) + 0.3 * rng.standard_normal(T))
    return x.astype(dtype)


@pytest.mark.gpu
def test_spectrogram_series_f64_large_offset(tdft_family):
    """A float64 series stays float64 on the device (the reference hands it to scipy
    unchanged): equal to scipy's float64 spectrogram at 1e-9, returned as float64."""
    from pydata.analyze import analyze
    x = offset_series(1000, np.float64)
    for kw in ({"nperseg": 128}, {}, {"nperseg": 100, "noverlap": 30, "window": "hann"}):
        t, f, S = analyze.spectrogram(array=x, fs=TASA, **kw)
        t2, f2, S2 = ora.spectrogram_series(x, fs=TASA, **kw)
        assert S.dtype == S2.dtype == np.float64
        assert np.array_equal(t, t2) and np.array_equal(f, f2)
        # the samples themselves carry the fluctuation to ulp(1000) / 1e-4 ~ 1e-9
        # relative, so two correct f64 detrends agree to a few 1e-9
        close_nan(S, S2, rtol=1e-8)


@pytest.mark.gpu
def test_spectrogram_series_f32_large_offset(tdft_family):
    """A float32 series with a large DC offset: the device detrends in f64, so it equals
    scipy on the same samples widened to float64 (to the float32 rounding of the
    result, which comes back float32 like scipy's)."""
    from pydata.analyze import analyze
    x = offset_series(1000, np.float32, amp=1e-2)
    t, f, S = analyze.spectrogram(array=x, fs=TASA, nperseg=128)
    assert S.dtype == np.float32
    t2, f2, S2 = ora.spectrogram_series(x.astype(np.float64), fs=TASA, nperseg=128)
    close_nan(S, S2, rtol=1e-6)


@pytest.mark.gpu
def test_spectrogram_block_large_offset(tmp_path, tdft_family):
    """Maps far from zero (a float32 block with a 1000 offset) with NaN gaps: the gap
    pixels are interpolated in float64 and the whole block runs as float64, as the
    reference's per-pixel loop does."""
    from pydata.analyze import analyze
    st = make_stack(300, n=32, seed=4, nan_pixels=[(3, 5, 20, 30), (9, 1, 200, 202)])
    st = st + np.float32(1000.0)
    st[0, :5, :7] = 0.0
    write_maps(str(tmp_path), st)
    t, f, S, avg = analyze.spectrogram(map_folder=str(tmp_path), fs=TASA, num_blocks=4, block_index=0, nperseg=64)
    t2, f2, S2, avg2 = ora.spectrogram_block(st.astype(np.float64), fs=TASA, num_blocks=4, block_index=0, nperseg=64)
    close_nan(S, S2)
    close_nan(avg, avg2)


@pytest.mark.gpu
def test_temporal_f64_stack_equals_widened_f32(tdft_family):
    """FCD_STACK_F64: a float64 stack holding float32 values gives the float32 call's
    results bit for bit (the arithmetic is f64 either way)."""
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    st = make_stack(257, n=24, seed=6, zero_corner=False)
    st64 = st.astype(np.float64)
    a = eng.temporal_spectrum(st, 129)
    b = eng.temporal_spectrum(st64, 129)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.array_equal(eng.temporal_bins(st, [0, 3, 128]), eng.temporal_bins(st64, [0, 3, 128]))
    win = np.hanning(64)
    assert np.array_equal(eng.spectrogram(st, 64, 8, win, TASA), eng.spectrogram(st64, 64, 8, win, TASA))


@pytest.mark.gpu
def test_fft_path_device_pointer_block(monkeypatch):
    """The FFT path on a device-resident stack, the block addressed in place through the
    stack's own pitches (float32 and float64 stacks), equals the host-pointer call and
    numpy."""
    import ctypes
    import torch
    from pyfcd import _lib
    monkeypatch.setenv("FCD_TDFT_FFT", "1")
    eng = _lib.temporal_engine()
    lib = _lib.load_library()
    st = make_stack(700, n=72, seed=12, zero_corner=False, nan_pixels=[(20, 30, 100, 101)])
    T, rows, cols = st.shape
    blk = (8, 20, 30, 40)  # r0, c0, bh, bw
    nf = 351
    want_t, want_c = nan_spectrum(st[:, 8:38, 20:60], nf)
    for arr, flag in ((st, 0), (st.astype(np.float64), _lib.FCD_STACK_F64)):
        sd = torch.from_numpy(arr).cuda()
        sc = np.empty((nf, 2))
        _lib._check(lib.fcd_temporal_spectrum(eng.handle, ctypes.c_void_p(sd.data_ptr()), T, rows, cols, *blk,
                                              _lib.FCD_DEVICE_PTRS | flag, nf, sc.ctypes.data, None))
        tot_h, cnt_h = eng.temporal_spectrum(arr, nf, block=blk)
        assert np.array_equal(sc[:, 0], tot_h) and np.array_equal(sc[:, 1], cnt_h)
        assert np.array_equal(cnt_h, want_c) and cnt_h[0] == 1199
        np.testing.assert_allclose(tot_h, want_t, rtol=1e-12)


@pytest.mark.gpu
def test_device_pointer_block_equals_host():
    """FCD_DEVICE_PTRS on a device-resident stack (the block addressed in place with the
    stack's own pitches, no staging) gives the host-pointer results bit for bit."""
    import ctypes
    import torch
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    lib = _lib.load_library()
    st = make_stack(300, n=96, seed=11, zero_corner=False)
    T, rows, cols = st.shape
    blk = (16, 40, 32, 24)  # r0, c0, bh, bw
    dims = (T, rows, cols) + blk
    sd = torch.from_numpy(st).cuda()
    nf = 150
    tot_h, cnt_h = eng.temporal_spectrum(st, nf, block=blk)
    sc = np.empty((nf, 2))
    _lib._check(lib.fcd_temporal_spectrum(eng.handle, ctypes.c_void_p(sd.data_ptr()), *dims, _lib.FCD_DEVICE_PTRS, nf,
                                          sc.ctypes.data, None))
    assert np.array_equal(sc[:, 0], tot_h) and np.array_equal(sc[:, 1], cnt_h)
    bins = np.array([0, 6, 12, 149], np.int32)
    X_h = eng.temporal_bins(st, bins, block=blk)
    xd = torch.empty((blk[2] * blk[3], len(bins), 2), dtype=torch.float64, device="cuda")
    _lib._check(lib.fcd_temporal_bins(eng.handle, ctypes.c_void_p(sd.data_ptr()), *dims, _lib.FCD_DEVICE_PTRS,
                                      bins.ctypes.data, len(bins), ctypes.c_void_p(xd.data_ptr()), None))
    Xd = xd.cpu().numpy()
    assert np.array_equal(Xd[..., 0].reshape(X_h.shape), X_h.real)
    assert np.array_equal(Xd[..., 1].reshape(X_h.shape), X_h.imag)
    from scipy.signal import get_window
    win = get_window(("tukey", 0.25), 64)
    S_h = eng.spectrogram(st, 64, 8, win, TASA, block=blk)
    sdv = torch.empty(S_h.shape, dtype=torch.float64, device="cuda")
    _lib._check(lib.fcd_spectrogram(eng.handle, ctypes.c_void_p(sd.data_ptr()), *dims, _lib.FCD_DEVICE_PTRS, 64, 8,
                                    win.ctypes.data, TASA, ctypes.c_void_p(sdv.data_ptr()), None))
    torch.cuda.synchronize()
    assert np.array_equal(sdv.cpu().numpy(), S_h)
    # and the block itself against numpy's f64 FFT
    ref = np.fft.fft(st[:, 16:48, 40:64].astype(np.float64), axis=0)
    close_nan(np.transpose(ref[bins], (1, 2, 0)).real, X_h.real)


@pytest.mark.gpu
def test_temporal_bad_arguments():
    from pyfcd import _lib
    eng = _lib.temporal_engine()
    st = make_stack(20, n=8, zero_corner=False)
    with pytest.raises(_lib.FcdError):
        eng.temporal_bins(st, [0, 20])  # bin out of range
    with pytest.raises(_lib.FcdError):
        eng.temporal_spectrum(st, 4, block=(4, 4, 8, 8))  # block outside the frame
    with pytest.raises(_lib.FcdError):
        eng.spectrogram(st, 32, 4, np.ones(32), TASA)  # nperseg > T
