"""GPU parity at the c3 / c5 frame sizes (BASELINE configs[2] 2048^2, configs[4] 4096^2)
against the reference ITSELF (tests/golden/large.npz, written by make_golden.py `large`:
/root/reference/pyfcd/fcd.py:13-35 compute_height_map, its skimage unwrap at fcd.py:119).

Per size one residue-free rotated-board frame and one frame whose maps carry residues
(bump field + three edge-dislocation pairs, bench_data.make_residue_frame), regenerated
here from the stored recipe and checked against the stored digest first.  Checked:

  * the reference setup (peaks, blobs, threshold, cf, radius, frequencies, disk counts):
    bit-exact;
  * wrapped phases on the fixture's 128^2 sub-grid: 2e-4 rad (synthetic tolerance);
  * the FULL unwrap k-field of both maps against the reference's, as unwrapped phases
    (w + 2 pi k) up to one global 2 pi c off the border ring (the reference seeds border
    reliabilities from rand()), with the two exceptions float32 rounding
    forces (assert_k_equal: wrapped values within 1e-3 of +-pi, and a branch cut between
    two residues moved by a pixel where last-bit phase differences swap two
    reliabilities; measured on r4096: one pixel per map) -- and the exact Boruvka MST
    pass (tile pass, component-graph rounds, per-tile capacities) bit for bit against
    the oracle's Herraez restatement fed the engine's own phases;
  * heights: rel-L2 <= 1e-5 on the 256^2 sub-grid and against the full map's norm, for
    the unfused chain (phases returned) and the fused height-only kernel
    (kernels_phase_rows_wide.hip), which must flag the residue frames and send them to
    the exact pass;
  * chunked batches: with FCD_CHUNK_MAX=2 a 5-frame batch [r, s, r, s, r] spans three
    launch chunks and the exact pass groups of 2; every copy equals the single-frame
    result bit for bit.
"""
import hashlib

import numpy as np
import pytest

from conftest import border_ring

pytestmark = pytest.mark.gpu

TWOPI = 2 * np.pi
CASES = ["s2048", "r2048", "s4096", "r4096"]


def wrap_diff(a, b):
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    return np.abs((d + np.pi) % TWOPI - np.pi)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


_frames = {}


def case_frames(g, tag):
    """(ref, frame) of a large.npz case, regenerated (bench_data.make_residue_frame with the
    displacement rounded to 1/4096 px: the same bytes under any numpy build)."""
    if tag not in _frames:
        from bench_data import make_residue_frame
        n = int(g[f"{tag}_n"])
        pairs = [tuple(p) for p in g[f"{tag}_pairs"]]
        ref, frame = make_residue_frame(n, pairs, seed=int(g[f"{tag}_seed"]), rotate_deg=5.0, quantum=4096)
        assert hashlib.sha256(ref.tobytes()).hexdigest() == str(g[f"{tag}_ref_sha"])
        assert hashlib.sha256(frame.tobytes()).hexdigest() == str(g[f"{tag}_frame_sha"])
        _frames.clear()  # keep one case (a 4096^2 pair is 128 MB)
        _frames[tag] = (ref, frame)
    return _frames[tag]


def residue_sites(w):
    """(row, col) of the plaquettes of a wrapped map with non-zero wrap circulation."""
    w = np.asarray(w, np.float64)
    wr = lambda d: (d + np.pi) % TWOPI - np.pi  # noqa: E731
    c = (wr(w[:-1, 1:] - w[:-1, :-1]) + wr(w[1:, 1:] - w[:-1, 1:]) + wr(w[1:, :-1] - w[1:, 1:])
         + wr(w[:-1, :-1] - w[1:, :-1]))
    return np.argwhere(np.abs(c) > 1)


def assert_k_equal(k, kref, w, tag, cut_margin=16, max_cut=4):
    """The engine's k-field against the reference's, as unwrapped phases w + 2 pi k, up to
    one global 2 pi c, off the border ring.  Two kinds of pixel may differ, and no other:

      * |w| within 1e-3 of pi: the float32 rounding of the two pipelines can put the
        wrapped value on either side of the cut, and k differs by the compensating -+1
        (same unwrapped phase);
      * pixels next to a branch cut between residues: which side of the cut a pixel
        falls on is decided by reliability ORDER, which last-bit differences of the
        wrapped phases can swap.  These must lie within `cut_margin` px of the bounding
        box of a residue pair (residues closer than 512 px clustered), and there are at
        most `max_cut` of them per map (measured: at most 1, at 4096^2).  The exact pass
        itself is checked against the oracle fed the engine's own phases (bit for bit,
        test_large_unwrap_equals_oracle_on_engine_phases).
    """
    k = np.asarray(k, np.int64)
    d = k - np.asarray(kref, np.int64)
    ring = border_ring(d.shape)
    c = np.bincount((d[~ring] - d[~ring].min())).argmax() + d[~ring].min()
    d = d - c
    flip = (np.abs(w) > np.pi - 1e-3) & (d == -np.sign(w).astype(np.int64))
    bad = (d != 0) & ~flip & ~ring
    if bad.any():
        sites = residue_sites(w)
        assert len(sites) > 0, f"{tag}: {int(bad.sum())} k mismatches in a residue-free map"
        near = np.zeros(d.shape, bool)
        used = np.zeros(len(sites), bool)
        for i in range(len(sites)):
            if used[i]:
                continue
            cl = np.abs(sites - sites[i]).max(axis=1) < 512
            used |= cl
            (r0, c0), (r1, c1) = sites[cl].min(axis=0), sites[cl].max(axis=0)
            r0, c0 = max(r0 - cut_margin, 0), max(c0 - cut_margin, 0)
            r1, c1 = min(r1 + cut_margin + 1, d.shape[0]), min(c1 + cut_margin + 1, d.shape[1])
            near[r0:r1, c0:c1] = True
        far = bad & ~near
        assert not far.any(), f"{tag}: {int(far.sum())} k mismatches away from residues, e.g. {np.argwhere(far)[:4].tolist()}"
        assert bad.sum() <= max_cut, f"{tag}: {int(bad.sum())} k mismatches next to branch cuts (cap {max_cut})"
    assert (d[ring] != 0).sum() <= 8, f"{tag}: {int((d[ring] != 0).sum())} border k mismatches"


@pytest.fixture(scope="module")
def large(golden):
    return golden("large")


@pytest.fixture
def fresh(monkeypatch):
    from pyfcd import _lib
    monkeypatch.delenv("FCD_UNFUSED", raising=False)
    _lib._engines.clear()
    yield
    _lib._engines.clear()


@pytest.mark.parametrize("tag", CASES)
def test_large_frames_match_reference_run(large, fresh, tag):
    from pyfcd import _lib
    g = large
    ref, frame = case_frames(g, tag)
    n = ref.shape[0]
    eng = _lib.Engine(ref.shape)
    info = eng.set_reference(ref, 0.001)
    peaks = np.array([[info.peaks[i][0], info.peaks[i][1]] for i in range(2)])
    assert np.array_equal(peaks, g[f"{tag}_peaks"])
    assert info.calibration_factor == float(g[f"{tag}_cf"])
    assert info.radius == float(g[f"{tag}_radius"])
    freqs = np.array([[info.frequencies[i][0], info.frequencies[i][1]] for i in range(2)])
    assert np.array_equal(freqs, g[f"{tag}_freqs"])
    assert [info.mask_count[0], info.mask_count[1]] == list(g[f"{tag}_mask_count"])
    blobs = np.array([[info.blob_peaks[i][0], info.blob_peaks[i][1]] for i in range(info.n_blobs)])
    assert np.array_equal(blobs, g[f"{tag}_blob_peaks"])
    assert info.threshold == np.float32(g[f"{tag}_threshold"])

    # unfused chain with phases and k-fields (the exact MST pass for residue frames)
    eng.profile(True)
    h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    st, _ = eng.stage_times()
    eng.profile(False)
    residues = g[f"{tag}_residues"]
    assert int(st["fixup_frames"]) == int(residues.any()), st
    s = n // 128
    assert wrap_diff(w[0][:, ::s, ::s], g[f"{tag}_wrapped_sub"]).max() < 2e-4
    for m in range(2):
        assert_k_equal(k[0][m], g[f"{tag}_k"][m], w[0][m], f"{tag} map {m}")
    sub = n // 256
    gs = g[f"{tag}_height_stats"]
    assert rel_l2(h[0][::sub, ::sub], g[f"{tag}_height_sub"]) < 1e-5
    assert abs(np.linalg.norm(h[0].astype(np.float64)) - gs[1]) < 1e-5 * gs[1]

    # fused height-only kernel: flags the residue frames, same heights
    eng.profile(True)
    hf, _, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=False)
    st, _ = eng.stage_times()
    eng.profile(False)
    assert int(st["fixup_frames"]) == int(residues.any()), st
    assert rel_l2(hf[0][::sub, ::sub], g[f"{tag}_height_sub"]) < 1e-5
    if residues.any():
        assert np.array_equal(hf[0], h[0])  # both from the exact pass
    else:
        assert rel_l2(hf[0], h[0]) < 1e-6
    eng.close()


@pytest.mark.parametrize("n", [2048, 4096])
def test_large_chunked_batches_equal_single(large, fresh, monkeypatch, n):
    """Several launch chunks and exact-pass groups per call at the c3 / c5 sizes: residue
    frames first, in the middle and last; every height bit-identical to its single-frame
    call (fused path) and within the reference's tolerance."""
    from pyfcd import _lib
    g = large
    ref, rf = case_frames(g, f"r{n}")
    rf = rf.copy()
    _, sf = case_frames(g, f"s{n}")
    sf = sf.copy()
    monkeypatch.setenv("FCD_CHUNK_MAX", "2")
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, 0.001)
    batch = np.stack([rf, sf, rf, sf, rf])
    eng.profile(True)
    hb, _, _ = eng.process(batch, 1.0, unwrap=True, want_phases=False)
    st, _ = eng.stage_times()
    eng.profile(False)
    assert int(st["fixup_frames"]) == 3, st
    hr, _, _ = eng.process(rf[None], 1.0, unwrap=True, want_phases=False)
    hs, _, _ = eng.process(sf[None], 1.0, unwrap=True, want_phases=False)
    for i in (0, 2, 4):  # all from the exact pass
        assert np.array_equal(hb[i], hr[0]), i
    # the residue-free copies came from the fused kernel, and so does the single call after
    # a residue-heavy one (FCD_EXACT_FIRST auto: the exact chain redoes residue-free frames
    # with the first pass's chain), so the heights do not depend on the call history
    assert np.array_equal(hb[1], hb[3])
    assert np.array_equal(hb[1], hs[0])
    sub = n // 256
    assert rel_l2(hr[0][::sub, ::sub], g[f"r{n}_height_sub"]) < 1e-5
    assert rel_l2(hs[0][::sub, ::sub], g[f"s{n}_height_sub"]) < 1e-5
    eng.close()


@pytest.mark.parametrize("n", [2048, 4096])
def test_large_unwrap_equals_oracle_on_engine_phases(large, fresh, n):
    """The exact Boruvka MST pass at the c3 / c5 sizes (64x64 tile pass, component-graph
    rounds, per-tile capacities) against the oracle's Herraez restatement
    (oracle/herraez_unwrap.c, pinned to skimage by test_oracle_golden) fed the engine's own
    wrapped phases: every pixel's k equal up to the anchor, border ring included (border
    reliabilities are the constant in both)."""
    from oracle import fcd_oracle as O
    from pyfcd import _lib
    ref, frame = case_frames(large, f"r{n}")
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, 0.001)
    _, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    for m in range(2):
        assert len(residue_sites(w[0][m])) > 0
        _, ko = O.unwrap(w[0][m])
        d = k[0][m].astype(np.int64) - ko
        assert np.all(d == d.flat[0]), (m, int((d != d.flat[0]).sum()))
    eng.close()


def test_single_call_device_memory_is_bounded(fresh):
    """A stateless drop-in call (fcd.py:13-35) sizes its workspace to the call: one 4096^2
    fcd.compute_height_map raises the device's memory use (hipMemGetInfo, through torch)
    by at most 2 GiB -- not the 16 GiB chunk budget a 32-frame batch uses --, a second
    call with the same reference adds nothing, and the engine cache stays bounded per
    thread and device."""
    import gc

    import torch
    from bench_data import checkerboard
    from pyfcd import _lib
    from pyfcd.fcd import fcd
    torch.cuda.init()
    gc.collect()
    free0, _ = torch.cuda.mem_get_info(0)
    ref = checkerboard(4096, 5.0)
    frame = np.roll(ref, 1, axis=1)
    h, ph, cf = fcd.compute_height_map(ref, frame, 0.001, height=1.0)
    assert np.isfinite(h).all()
    free1, _ = torch.cuda.mem_get_info(0)
    used = free0 - free1
    assert used <= 2 << 30, f"one 4096^2 call pinned {used / 2**30:.2f} GiB"
    fcd.compute_height_map(ref, frame, 0.001, height=1.0)
    free2, _ = torch.cuda.mem_get_info(0)
    assert free2 >= free1 - (64 << 20), "a repeated call grew the workspace"
    # the cache: at most FCD_ENGINE_CACHE shapes per thread and device, LRU closed
    for n in (64, 128, 256, 512, 1024):
        _lib.engine_for((n, n))
    mine = [k for k in _lib._engines if k[2] == __import__("threading").get_ident()]
    assert len(mine) <= _lib._engine_cache_size()
    assert (4096, 4096) not in [k[0] for k in mine]
    _lib._engines.clear()
    gc.collect()


def test_4096_folded_band_demod_equals_full_length(large, fresh, monkeypatch):
    """The phases chain at 4096 (fcd.compute_height_map's, fcd.py:63, 118): the folded
    band-pruned inverse (16 groups of 256 points per row, the 512-bin window's halves summed
    per group, kernels_band.hip FOLD) against the full-length inverse row transform
    (`FCD_WIDE_BAND=0`, k_demod_phase<4096>) on the same frame: the same wrapped phases up to
    float32 rounding, and the same residue-free heights."""
    from pyfcd import _lib
    ref, frame = case_frames(large, "s4096")
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, 0.001)
    h1, w1, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    monkeypatch.setenv("FCD_WIDE_BAND", "0")
    h0, w0, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    d = wrap_diff(w1[0], w0[0])
    assert d.max() < 2e-4 and float(np.median(d)) < 2e-6, (d.max(), float(np.median(d)))
    assert rel_l2(h1[0], h0[0]) < 1e-5
    eng.close()


def test_rectangular_4096_wide_frames_match_oracle(fresh):
    """4096-point rows on a short frame (256 x 4096): the folded band demod of the phases
    chain, the folded fused kernel of the height-only chain and its reference angles against
    the CPU oracle's chain (oracle/fcd_oracle.py, fcd.py:13-35): carriers, wrapped phases
    (2e-4 rad), the unwrap up to the anchor, heights (1e-5)."""
    from bench_data import make_residue_frame
    from oracle import fcd_oracle as O
    from pyfcd import _lib
    rows, cols = 256, 4096
    ref, frame = make_residue_frame(rows, [], seed=5, rotate_deg=5.0, quantum=4096, cols=cols)
    eng = _lib.Engine(ref.shape)
    info = eng.set_reference(ref, 0.001)
    (cars, cf) = O.compute_carriers(ref, 0.001)
    assert info.calibration_factor == cf
    assert sorted(tuple(info.peaks[i]) for i in range(2)) == sorted(tuple(int(v) for v in c.pixels) for c in cars)
    h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    hf, _, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=False)
    ho, _, _, ex = O.compute_height_map(ref, frame, 0.001, height=1.0)
    for m in range(2):
        assert wrap_diff(w[0][m], ex["wrapped"][m]).max() < 2e-4, m
        _, ko = O.unwrap(w[0][m])
        d = k[0][m].astype(np.int64) - ko
        assert np.all(d == d.flat[0]), m
    assert rel_l2(h[0], ho) < 1e-5, rel_l2(h[0], ho)
    assert rel_l2(hf[0], ho) < 1e-5, rel_l2(hf[0], ho)
    eng.close()
