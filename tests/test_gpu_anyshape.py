"""GPU parity for frame sides of ANY size against the reference ITSELF
(tests/golden/anyshape.npz, make_golden.py `anyshape`: compute_height_map, fcd.py:13-35,
with scipy's fft2 / ifft2 at fcd.py:28, 118 and carriers.py:23-24 and skimage's unwrap at
fcd.py:119): the HD camera format 1080 x 1920, 1000 x 1000 with residues, prime /
Bluestein sides 1023 x 1021 and 1021 x 1023, a 1000 x 1000 crop of the 10-bit camera pair.

The generic chain runs there: mixed-radix transforms with radix-7 / generic odd-prime
passes or Bluestein's convolution (kernels_mr.hip), the unwrap on maps padded to multiples
of 64 (pad pixels heavier than every frame edge, kernels_unwrap.hip), the exact reference
spectrum for the carrier picks (kernels_pocketfft.hip).  Assertions as test_gpu_mixed.py:
fft2 sha256-equal to scipy, setup bit-exact, wrapped phases 2e-4 rad (synthetic) / the
real-image rule (camera crop), k-fields against the reference's (assert_k_equal) and bit
for bit against the oracle fed the engine's phases, heights rel-L2 1e-5 (1e-4 camera).
"""
import hashlib

import numpy as np
import pytest

from test_gpu_large import assert_k_equal, rel_l2, residue_sites, wrap_diff
from test_gpu_parity import assert_phase_close, band_amplitude

pytestmark = pytest.mark.gpu

CASES = ["s1080x1920", "r1000x1000", "s1023x1021", "r1021x1023", "c1000x1000"]


@pytest.fixture(scope="module")
def anyshape(golden):
    return golden("anyshape")


def case_frames(g, golden, tag):
    if tag.startswith("c"):
        d = golden("real_df")
        ref = np.ascontiguousarray(d["ref_u16"][12:1012, 20:1020].astype(np.float32))
        frame = np.ascontiguousarray(d["frames_u16"][0][12:1012, 20:1020].astype(np.float32))
    else:
        from bench_data import make_residue_frame
        rows, cols = (int(v) for v in g[f"{tag}_shape"])
        ref, frame = make_residue_frame(rows, [tuple(p) for p in g[f"{tag}_pairs"]], seed=int(g[f"{tag}_seed"]),
                                        rotate_deg=5.0, quantum=4096, cols=cols)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == str(g[f"{tag}_ref_sha"])
    assert hashlib.sha256(frame.tobytes()).hexdigest() == str(g[f"{tag}_frame_sha"])
    return ref, frame, float(g[f"{tag}_sq"])


@pytest.mark.parametrize("tag", CASES)
def test_anyshape_frames_match_reference_run(anyshape, golden, tag):
    from oracle import fcd_oracle as O
    from pyfcd import _lib
    g = anyshape
    ref, frame, sq = case_frames(g, golden, tag)
    eng = _lib.Engine(ref.shape)
    F = eng.fft2(ref)
    assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{tag}_ref_fft2_sha"]), tag
    info = eng.set_reference(ref, sq)
    peaks = np.array([[info.peaks[i][0], info.peaks[i][1]] for i in range(2)])
    assert np.array_equal(peaks, g[f"{tag}_peaks"])
    assert info.calibration_factor == float(g[f"{tag}_cf"])
    assert info.radius == float(g[f"{tag}_radius"])
    freqs = np.array([[info.frequencies[i][0], info.frequencies[i][1]] for i in range(2)])
    assert np.array_equal(freqs, g[f"{tag}_freqs"])
    assert [info.mask_count[0], info.mask_count[1]] == list(g[f"{tag}_mask_count"])
    blobs = np.array([[info.blob_peaks[i][0], info.blob_peaks[i][1]] for i in range(info.n_blobs)])
    assert np.array_equal(blobs, g[f"{tag}_blob_peaks"])
    assert info.threshold == float(np.float32(g[f"{tag}_threshold"]))

    h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    ws, hs = int(g[f"{tag}_wrapped_step"]), int(g[f"{tag}_height_step"])
    camera = tag.startswith("c")
    if camera:
        masks = [c.mask for c in O.compute_carriers(ref, sq)[0]]
        assert_phase_close(w[0][:, ::ws, ::ws], g[f"{tag}_wrapped_sub"], band_amplitude(frame, masks, step=ws))
    else:
        assert wrap_diff(w[0][:, ::ws, ::ws], g[f"{tag}_wrapped_sub"]).max() < 2e-4
    for m in range(2):
        if not camera:  # (the camera crop's border pixels next to residues follow rand())
            assert_k_equal(k[0][m], g[f"{tag}_k"][m], w[0][m], f"{tag} map {m}")
        if len(residue_sites(w[0][m])):
            _, ko = O.unwrap(w[0][m])  # the exact pass against the oracle on the engine's phases
            d = k[0][m].astype(np.int64) - ko
            assert np.all(d == d.flat[0]), (m, int((d != d.flat[0]).sum()))
    assert rel_l2(h[0][::hs, ::hs], g[f"{tag}_height_sub"]) < (1e-4 if camera else 1e-5)
    hf, _, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=False)
    assert np.array_equal(hf, h)
    # fcd_unwrap on the same maps (skimage's unwrap_phase boundary, fcd.py:119)
    ku, res = eng.unwrap(w[0])
    for m in range(2):
        d = ku[m].astype(np.int64) - k[0][m]
        assert np.all(d == d.flat[0]), m
    eng.close()


def test_anyshape_batches_and_device_pointers(anyshape, golden):
    """A batch spanning several chunks equals the single-frame calls bit for bit, and
    device-pointer calls equal host-pointer calls (1021 x 1023: Bluestein rows / columns,
    maps padded for the unwrap)."""
    import torch
    from pyfcd import _lib
    g = anyshape
    ref, rf, sq = case_frames(g, golden, "r1021x1023")
    _, sf, _ = case_frames(g, golden, "s1023x1021")
    sf = np.ascontiguousarray(sf.T)  # another residue pattern of the same shape
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, sq)
    hr, _, _ = eng.process(rf[None], 1.0, want_phases=False)
    hs, _, _ = eng.process(sf[None], 1.0, want_phases=False)
    batch = np.stack([rf, sf] * 18 + [rf])  # 37 frames: more than one chunk
    hb, _, _ = eng.process(batch, 1.0, want_phases=False)
    for i in range(len(batch)):
        assert np.array_equal(hb[i], hr[0] if i % 2 == 0 else hs[0]), i
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(batch[:5]).to(dev)
    hd = torch.empty_like(fd)
    eng.process_device(fd.data_ptr(), 5, 1.0, True, hd.data_ptr())
    assert np.array_equal(hd.cpu().numpy(), hb[:5])
    eng.close()


def test_anyshape_raw_formats(anyshape, golden):
    """Raw 8-bit, 16-bit and 10-bit-packed frames of an odd width (1021 columns: the packed
    rows end mid-group) widen to the same heights as their float32 frames."""
    from pyfcd import _lib
    g = anyshape
    ref, frame, sq = case_frames(g, golden, "s1023x1021")
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, sq)
    q = np.clip(np.rint(frame / 65535.0 * 1023.0), 0, 1023).astype(np.uint16)
    f32 = q.astype(np.float32)
    want, _, _ = eng.process(f32[None], 1.0, want_phases=False)
    # 10-bit MSB-first rows, each padded to a whole byte (FCD_FMT_P10, any width)
    bits = ((q[..., None] >> np.arange(9, -1, -1, dtype=np.uint16)) & 1).astype(np.uint8).reshape(q.shape[0], -1)
    p10 = np.packbits(bits, axis=1).reshape(-1)
    assert p10.size == eng.frame_bytes(_lib.FCD_FMT_P10)
    for fmt, raw in ((_lib.FCD_FMT_U16, q.copy()), (_lib.FCD_FMT_U8, (q >> 2).astype(np.uint8)),
                     (_lib.FCD_FMT_P10, p10)):
        got = eng.process_raw(np.ascontiguousarray(raw), fmt, 1, 1.0)
        exp = want if fmt != _lib.FCD_FMT_U8 else eng.process((q >> 2).astype(np.float32)[None], 1.0,
                                                              want_phases=False)[0]
        assert np.array_equal(got, exp), fmt
    eng.close()


@pytest.mark.parametrize("tag", ["r1000x1000", "s1023x1021"])
def test_mst_levels_agree_on_odd_shapes(anyshape, golden, monkeypatch, tag):
    """The exact unwrap's other round structures (FCD_MST_LEVEL=2: tiles then boundary
    lists; 1: one pixel round then lists; 0: all-pixel rounds) on maps of odd shapes,
    padded to multiples of 64 for them: the same k-fields as the default tiles +
    component-graph rounds (the level-2 / 1 fallback of a tile graph over its capacity
    decodes pixels with the padded, not power-of-two, sides: ADVICE r04)."""
    from pyfcd import _lib
    g = anyshape
    ref, frame, sq = case_frames(g, golden, tag)
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, sq)
    _, w, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    k3, res = eng.unwrap(w[0])
    assert (res > 0).any()
    for level in ("2", "1", "0"):
        monkeypatch.setenv("FCD_MST_LEVEL", level)
        k, _ = eng.unwrap(w[0])
        assert np.array_equal(k, k3), level
    monkeypatch.delenv("FCD_MST_LEVEL")
    eng.close()


@pytest.mark.parametrize("shape", [(4099, 96), (96, 8200), (64, 16384)])
def test_long_sides_match_oracle(shape):
    """Sides the rows' LDS cannot hold (kernels_mr.hip global-scratch rows): 4099 (prime:
    Bluestein with M = 16384, the columns through the transpose route), 8200 (2^3 5^2 41:
    a generic radix-41 pass over 8200-point rows), 16384 (2^14).  Setup bit-exact against
    the oracle's restatement of the reference's spectrum, heights rel-L2 1e-5 against the
    oracle (fcd.compute_height_map with the unwrap, and the oracle's unwrap and integration on
    the engine's phases), the k-fields of the maps equal to the oracle's on the engine's phases (up to the
    constant)."""
    check_shape_against_oracle(shape)


@pytest.mark.parametrize("shape", [(509, 384), (97, 1000), (1200, 250), (1536, 160)])
def test_integration_column_paths_match_oracle(shape):
    """The generic integration's column kernel (kernels_mr.hip k_mr_int_cols) in each of its
    forms: one wave per column with Bluestein columns (509: M = 1024 with 4 columns per
    group; 97: M = 256 with 16), one wave per 1200-point mixed-radix column, and a
    multi-wave team per 1536-point column.  Same checks as test_long_sides_match_oracle (at
    509 x 384 one pixel next to a branch cut takes another k in the oracle's own chain -- its
    f32 phases' last bits on the other side of pi -- so there the heights are checked
    against the oracle's unwrap and integration of the engine's phases only)."""
    check_shape_against_oracle(shape)


def check_shape_against_oracle(shape):
    from bench_data import make_residue_frame
    from oracle import fcd_oracle as O
    from pyfcd import _lib
    rows, cols = shape
    pairs = [(rows // 2 + 0.5, min(cols // 3, 40) + 0.25)]
    ref, frame = make_residue_frame(rows, pairs, seed=3, rotate_deg=5.0, quantum=4096, cols=cols)
    eng = _lib.Engine(shape)
    info = eng.set_reference(ref, 0.001)
    (cars, cf) = O.compute_carriers(ref, 0.001)
    assert info.calibration_factor == cf
    got = sorted(tuple(info.peaks[i]) for i in range(2))
    want = sorted(tuple(int(v) for v in c.pixels) for c in cars)
    assert got == want, (got, want)
    h, w, k = eng.process(frame[None], 1.0, unwrap=True, want_phases=True)
    hf, _, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=False)
    assert np.array_equal(h, hf)
    ho, _, _, ex = O.compute_height_map(ref, frame, 0.001, height=1.0)
    flips = 0
    phases = np.zeros((2, rows, cols))
    for m in range(2):
        assert wrap_diff(w[0][m], ex["wrapped"][m]).max() < 2e-4
        phases[m], ko = O.unwrap(w[0][m])
        d = k[0][m].astype(np.int64) - ko
        assert np.all(d == d.flat[0]), m
        # the oracle's own k-field: it may differ at a pixel next to a branch cut, where the
        # two f32 phase chains' last bits fall on either side of +-pi (test_gpu_large)
        dk = ex["k"][m].astype(np.int64) - ko
        flips += int(np.count_nonzero(dk != dk.flat[0]))
    assert flips <= 2, flips
    if flips == 0:
        assert rel_l2(h[0], ho) < 1e-5, rel_l2(h[0], ho)
    # heights against the oracle's chain (its unwrap and integration) on the engine's phases
    disp = O.displacement_field(phases, ex["carriers"])
    he = O.integrate_in_fourier(-disp[0], -disp[1], info.calibration_factor)
    assert rel_l2(h[0], he) < 1e-5, rel_l2(h[0], he)
    eng.close()


def test_unsupported_shapes_raise():
    """Sides below 16 or above 16384 stay refused (FCD_E_UNSUPPORTED): the MST's 32-bit
    vertex ids bound a batch's pixels."""
    from pyfcd import _lib
    for shape in ((8, 64), (64, 16400), (16385, 64)):
        with pytest.raises(_lib.FcdError) as e:
            _lib.Engine(shape)
        assert e.value.code == _lib.FCD_E_UNSUPPORTED
