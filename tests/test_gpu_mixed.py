"""GPU parity for frame sides that are not powers of two (the engine's generic chain on
the mixed-radix transforms of kernels_mr.hip) against the reference ITSELF
(tests/golden/mixed.npz, make_golden.py `mixed`: compute_height_map, fcd.py:13-35, with
scipy's fft2 / ifft2 at fcd.py:28, 118 and carriers.py:23-24 and skimage's unwrap at
fcd.py:119, on 1024 x 1280 and 1536 x 2048 boards and a 960 x 1024 crop of the 10-bit
camera pair).

  * fcd_fft2 = scipy 1.7.1's float32 fft2 bit for bit at 5-smooth shapes (the restated
    radf3 / radf5 / pass3 / pass5 of kernels_pocketfft.hip): the carrier picks stay the
    reference's own, ties included;
  * reference setup bit-exact; wrapped phases 2e-4 rad (synthetic) / the real-image rule
    of test_gpu_parity.assert_phase_close (camera crop);
  * k-fields against the reference's as in test_gpu_large.assert_k_equal, and bit for bit
    against the oracle's Herraez restatement fed the engine's own phases;
  * heights rel-L2 <= 1e-5 (synthetic), 1e-4 on the camera crop (the reference seeds border
    reliabilities next to residues from rand());
  * batches equal single frames, height-only calls equal calls with phases, device
    pointers equal host pointers.
"""
import hashlib

import numpy as np
import pytest

from test_gpu_large import assert_k_equal, rel_l2, residue_sites, wrap_diff
from test_gpu_parity import assert_phase_close, band_amplitude

pytestmark = pytest.mark.gpu

CASES = ["s1024x1280", "r1024x1280", "s1536x2048", "c960x1024"]


@pytest.fixture(scope="module")
def mixed(golden):
    return golden("mixed")


def case_frames(g, golden, tag):
    if tag.startswith("c"):
        d = golden("real_df")
        r0, r1 = 32, 992
        ref = np.ascontiguousarray(d["ref_u16"][r0:r1].astype(np.float32))
        frame = np.ascontiguousarray(d["frames_u16"][0][r0:r1].astype(np.float32))
    else:
        from bench_data import make_residue_frame
        rows, cols = (int(v) for v in g[f"{tag}_shape"])
        ref, frame = make_residue_frame(rows, [tuple(p) for p in g[f"{tag}_pairs"]], seed=int(g[f"{tag}_seed"]),
                                        rotate_deg=5.0, quantum=4096, cols=cols)
    assert hashlib.sha256(ref.tobytes()).hexdigest() == str(g[f"{tag}_ref_sha"])
    assert hashlib.sha256(frame.tobytes()).hexdigest() == str(g[f"{tag}_frame_sha"])
    return ref, frame, float(g[f"{tag}_sq"])


def test_mixed_fft2_bit_exact_with_scipy(mixed, golden):
    """scipy.fft.fft2 (fcd.py:28, fourier.py:18) at 5-smooth shapes, bit for bit."""
    from pyfcd import _lib
    g = mixed
    for h, w in g["rand_shapes"]:
        img = g[f"rand_{h}x{w}_u16"].astype(np.float32) * np.float32(0.37)
        F = _lib.Engine(img.shape).fft2(img)
        assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"rand_{h}x{w}_fft2_sha"]), (h, w)
    for tag in CASES:
        ref, _, _ = case_frames(g, golden, tag)
        F = _lib.Engine(ref.shape).fft2(ref)
        assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{tag}_ref_fft2_sha"]), tag


@pytest.mark.parametrize("tag", CASES)
def test_mixed_frames_match_reference_run(mixed, golden, tag):
    from oracle import fcd_oracle as O
    from pyfcd import _lib
    g = mixed
    ref, frame, sq = case_frames(g, golden, tag)
    eng = _lib.Engine(ref.shape)
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
    assert info.threshold == np.float32(g[f"{tag}_threshold"])

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
    # the height-only call is the same chain
    hf, _, _ = eng.process(frame[None], 1.0, unwrap=True, want_phases=False)
    assert np.array_equal(hf, h)
    eng.close()


def test_mixed_batches_and_device_pointers(mixed, golden):
    """A batch spanning several chunks (frames in any order) equals the single-frame calls
    bit for bit, and device-pointer calls equal host-pointer calls."""
    import torch
    from pyfcd import _lib
    g = mixed
    ref, rf, sq = case_frames(g, golden, "r1024x1280")
    _, sf, _ = case_frames(g, golden, "s1024x1280")
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, sq)
    hr, _, _ = eng.process(rf[None], 1.0, want_phases=False)
    hs, _, _ = eng.process(sf[None], 1.0, want_phases=False)
    batch = np.stack([rf, sf] * 20 + [rf])  # 41 frames: two chunks and a remainder
    hb, _, _ = eng.process(batch, 1.0, want_phases=False)
    for i in range(len(batch)):
        assert np.array_equal(hb[i], hr[0] if i % 2 == 0 else hs[0]), i
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(batch[:5]).to(dev)
    hd = torch.empty_like(fd)
    eng.process_device(fd.data_ptr(), 5, 1.0, True, hd.data_ptr())
    assert np.array_equal(hd.cpu().numpy(), hb[:5])
    eng.close()


def test_mixed_high_level_api(mixed, golden):
    """fcd.compute_height_map / compute_phases / fourier.integrate on a 1024 x 1280 frame
    (the generic chain behind the reference's classmethods)."""
    from pyfcd.fcd import fcd
    g = mixed
    ref, frame, sq = case_frames(g, golden, "s1024x1280")
    hmap, phases, cf = fcd.compute_height_map(ref, frame, sq, height=1.0)
    assert cf == float(g["s1024x1280_cf"]) and hmap.shape == ref.shape and phases.shape == (2,) + ref.shape
    hs = int(g["s1024x1280_height_step"])
    assert rel_l2(hmap[::hs, ::hs], g["s1024x1280_height_sub"]) < 1e-5
    carriers, _ = fcd.compute_carriers(ref, sq)
    D = np.fft.fft2(frame.astype(np.float64)).astype(np.complex64)
    ph = fcd.compute_phases(D, carriers)
    assert wrap_diff(ph, phases).max() < 1e-4
