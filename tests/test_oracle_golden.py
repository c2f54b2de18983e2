"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden).

The oracle is the checker of every GPU parity test, so it must itself match
the golden vectors the reference produced (tests/golden/make_golden.py):
bit-exact peaks / calibration factor / unwrap k-fields, and float32-FFT
tolerance on phases and heights.
"""
import hashlib

import numpy as np
import pytest

from conftest import border_ring
from oracle import fcd_oracle as O

LAYERS = [[5.7e-2, 1.0003], [1.2e-2, 1.48899], [4.3e-2, 1.34], [80e-2, 1.0003]]


def test_height_from_layers(golden):
    g = golden("real_pair")
    assert O.height_from_layers(g["layers"].tolist()) == float(g["eff_height"])


def test_wavenumber_tables(golden):
    g = golden("integrate")
    for key in ("64x64", "128x64", "256x256"):
        h, w = (int(v) for v in key.split("x"))
        kr, kc = O.wavenumber_meshgrid((h, w), float(g[f"cf_{key}"]))
        assert np.array_equal(kr[:, 0], g[f"krow_{key}"])
        assert np.array_equal(kc[0, :], g[f"kcol_{key}"])


def test_integrate_in_fourier(golden):
    g = golden("integrate")
    for key in ("64x64", "128x64", "256x256"):
        h = O.integrate_in_fourier(g[f"gx_{key}"], g[f"gy_{key}"], float(g[f"cf_{key}"]))
        np.testing.assert_allclose(h, g[f"h_{key}"], rtol=0, atol=1e-12 * np.abs(g[f"h_{key}"]).max())


def test_integrate_symmetrised_tables_equivalence(golden):
    """The device form (odd-symmetrised kx/ky, real spectrum) equals the reference's real(ifft2(...))."""
    g = golden("integrate")
    for key in ("64x64", "128x64"):
        gx, gy, cf = g[f"gx_{key}"], g[f"gy_{key}"], float(g[f"cf_{key}"])
        H, W = gx.shape
        ky, kx = O.wavenumber_meshgrid((H, W), cf)
        k2 = kx ** 2 + ky ** 2
        k2[0, 0] = 1
        kxm, kym = kx.copy(), ky.copy()
        kxm[:, W // 2 + 1] = 0
        kym[H // 2 + 1, :] = 0
        kxe = (kxm - kxm[:, (-np.arange(W)) % W]) / 2
        kye = (kym - kym[(-np.arange(H)) % H, :]) / 2
        hat = (-1j * kxe * np.fft.fft2(gx) - 1j * kye * np.fft.fft2(gy)) / k2
        h = np.fft.ifft2(hat)
        assert np.abs(h.imag).max() < 1e-12 * np.abs(h.real).max()
        np.testing.assert_allclose(h.real, g[f"h_{key}"], atol=1e-12 * np.abs(g[f"h_{key}"]).max())


def test_real_pair_setup(golden):
    g = golden("real_pair")
    ref = g["ref_u8"].astype(np.float32)
    carriers, cf = O.compute_carriers(ref, float(g["square_size"]))
    assert cf == float(g["cf"])
    assert np.array_equal(np.array([np.asarray(c.pixels) for c in carriers]), g["peaks"])
    assert carriers[0].radius == float(g["radius"])
    assert np.array_equal(np.array([c.frequencies for c in carriers]), g["freqs"])
    assert [int(c.mask.sum()) for c in carriers] == list(g["mask_count"])


def test_real_df_committed_calibration(golden):
    d = golden("real_df")
    cf, peaks = O.calibration_factor(float(d["square_size"]), d["ref_u16"].astype(np.float32))
    assert cf == float(d["committed_cf"][0])  # examples/Pictures/mask/maps/calibration_factor.npy
    assert np.array_equal(np.array([np.asarray(p) for p in peaks]), d["peaks"])


def test_real_pair_end_to_end(golden):
    g = golden("real_pair")
    ref, disp = g["ref_u8"].astype(np.float32), g["disp_u8"].astype(np.float32)
    h, ph, cf, ex = O.compute_height_map(ref, disp, float(g["square_size"]), layers=g["layers"].tolist())
    assert np.array_equal(ex["wrapped"][:, ::8, ::8], g["wrapped_sub"])
    # k-fields: the reference draws border reliabilities from rand(); only border pixels may differ
    for i in range(2):
        bad = ex["k"][i] != g["k"][i]
        assert not bad[~border_ring(bad.shape)].any()
        assert bad.sum() <= 2
    rel = np.linalg.norm(h[::4, ::4] - g["height_sub"]) / np.linalg.norm(g["height_sub"])
    assert rel < 1e-4


def test_synthetic_bit_exact(golden):
    s = golden("synthetic")
    for c in s["cases"]:
        h, ph, cf, ex = O.compute_height_map(s[f"{c}_ref"], s[f"{c}_disp"], float(s[f"{c}_sq"]), height=1.0)
        assert cf == float(s[f"{c}_cf"])
        assert np.array_equal(ex["wrapped"], s[f"{c}_wrapped"]), c
        assert np.array_equal(ph, s[f"{c}_phases"]), c
        np.testing.assert_allclose(h, s[f"{c}_height"], rtol=0, atol=1e-12 * np.abs(s[f"{c}_height"]).max())


def test_unwrap_crops_exact(golden):
    u = golden("unwrap_crops")
    for w, k in zip(u["crops"], u["k_crops"]):
        _, ko = O.unwrap(w)
        bad = ko != k
        assert not bad[~border_ring(bad.shape)].any()
        assert bad.sum() <= 2
    _, ko = O.unwrap(u["rect"])
    assert (ko != u["k_rect"]).sum() <= 2


@pytest.mark.parametrize("which", [0])
def test_unwrap_full_map_exact(golden, which):
    u = golden("unwrap_crops")
    _, ko = O.unwrap(u["full"])
    bad = ko != u["k_full"]
    assert not bad[~border_ring(bad.shape)].any()
    assert bad.sum() <= 2


def test_val_accuracy_threshold(golden):
    """pyval.val(0, gauss_sin) (examples/val_example.py) — README's "< 0.52 %"."""
    v = golden("val")
    assert float(v["err_percent"]) < 0.52
    assert float(v["cf"]) == 1.0


def test_residue_counter_matches_definition():
    rng = np.random.default_rng(1)
    w = np.angle(np.exp(1j * rng.normal(0, 2.0, (40, 50)))).astype(np.float32)
    a = w[:-1, :-1].astype(np.float64)
    b, c, d = w[:-1, 1:], w[1:, 1:], w[1:, :-1]

    def fw(p, q):
        x = p - np.asarray(q, np.float64)
        return np.where(x > np.pi, -1, np.where(x < -np.pi, 1, 0))
    assert O.count_residues(w) == int(((fw(a, b) + fw(b, c) + fw(c, d) + fw(d, a)) != 0).sum())


def test_pocketfft_f32_matches_scipy_digests(golden):
    """oracle/pocketfft.py restates scipy 1.7.1's float32 fft2, numpy 1.26.4's float32
    mean and complex64 abs bit for bit: sha256 of every output equals the reference
    interpreter's (fourier.py:18's spectrum included)."""
    import hashlib
    from conftest import spectrum_images
    from oracle import pocketfft as P
    g, imgs = spectrum_images(golden)
    assert sorted(imgs) == sorted(str(n) for n in g["names"])
    for name, img in imgs.items():
        F = P.fft2(img)
        assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{name}_fft2_sha"]), name
        assert P.mean_f32(img) == g[f"{name}_mean"], name
        spec = P.find_peaks_spectrum(img)
        assert hashlib.sha256(spec.tobytes()).hexdigest() == str(g[f"{name}_spec_sha"]), name


@pytest.mark.parametrize("tag", ["s2048", "r2048"])
def test_oracle_large_frames_vs_reference_run(golden, tag):
    """The oracle at the c3 frame size against the reference's own run (large.npz): setup
    bit-exact, the full unwrap k-fields of a residue-free and a residue frame exact up to
    the anchor off the border ring, heights at float32-FFT tolerance (the GPU tests at
    2048^2 / 4096^2 compare the engine with the same fixture directly)."""
    import hashlib
    from bench_data import make_residue_frame
    g = golden("large")
    n = int(g[f"{tag}_n"])
    ref, frame = make_residue_frame(n, [tuple(p) for p in g[f"{tag}_pairs"]], seed=int(g[f"{tag}_seed"]),
                                    rotate_deg=5.0, quantum=4096)
    assert hashlib.sha256(frame.tobytes()).hexdigest() == str(g[f"{tag}_frame_sha"])
    h, ph, cf, ex = O.compute_height_map(ref, frame, 0.001, height=1.0)
    assert cf == float(g[f"{tag}_cf"])
    assert np.array_equal([np.asarray(c.pixels) for c in ex["carriers"]], g[f"{tag}_peaks"])
    assert [O.count_residues(w) for w in ex["wrapped"]] == list(g[f"{tag}_residues"])
    for m in range(2):
        d = ex["k"][m].astype(np.int64) - g[f"{tag}_k"][m]
        inner = d[1:-1, 1:-1]
        assert np.all(inner == inner.flat[0]), int((inner != inner.flat[0]).sum())
    sub = n // 256
    hs = h[::sub, ::sub]
    assert np.linalg.norm(hs - g[f"{tag}_height_sub"]) / np.linalg.norm(g[f"{tag}_height_sub"]) < 1e-5


def test_pocketfft_f32_mixed_radix_digests(golden):
    """oracle/pocketfft.py's radf3 / radf5 / pass3 / pass5 (5-smooth shapes) against
    scipy 1.7.1's float32 fft2, numpy's mean and the find_peaks spectrum, by digest."""
    import hashlib
    from oracle import pocketfft as P
    g = golden("mixed")
    for h, w in g["rand_shapes"]:
        img = g[f"rand_{h}x{w}_u16"].astype(np.float32) * np.float32(0.37)
        assert hashlib.sha256(P.fft2(img).tobytes()).hexdigest() == str(g[f"rand_{h}x{w}_fft2_sha"]), (h, w)
        assert P.mean_f32(img) == g[f"rand_{h}x{w}_mean"]
        assert hashlib.sha256(P.find_peaks_spectrum(img).tobytes()).hexdigest() == str(g[f"rand_{h}x{w}_spec_sha"])


@pytest.mark.parametrize("tag", ["r1024x1280", "c960x1024"])
def test_oracle_mixed_frames_vs_reference_run(golden, tag):
    """The oracle on frames whose sides are not powers of two against the reference's own
    run (mixed.npz): setup bit-exact, k-fields exact up to the anchor off the border ring
    (the camera crop: off the pixels next to residues on the border), heights at
    float32-FFT tolerance."""
    import hashlib
    g = golden("mixed")
    if tag.startswith("c"):
        d = golden("real_df")
        ref = np.ascontiguousarray(d["ref_u16"][32:992].astype(np.float32))
        frame = np.ascontiguousarray(d["frames_u16"][0][32:992].astype(np.float32))
    else:
        from bench_data import make_residue_frame
        rows, cols = (int(v) for v in g[f"{tag}_shape"])
        ref, frame = make_residue_frame(rows, [tuple(p) for p in g[f"{tag}_pairs"]], seed=int(g[f"{tag}_seed"]),
                                        rotate_deg=5.0, quantum=4096, cols=cols)
    assert hashlib.sha256(frame.tobytes()).hexdigest() == str(g[f"{tag}_frame_sha"])
    sq = float(g[f"{tag}_sq"])
    h, ph, cf, ex = O.compute_height_map(ref, frame, sq, height=1.0)
    assert cf == float(g[f"{tag}_cf"])
    assert np.array_equal([np.asarray(c.pixels) for c in ex["carriers"]], g[f"{tag}_peaks"])
    for m in range(2):
        d = ex["k"][m].astype(np.int64) - g[f"{tag}_k"][m]
        inner = d[1:-1, 1:-1]
        bad = inner != inner.flat[0]
        assert bad.sum() <= (0 if not tag.startswith("c") else 16), int(bad.sum())
    hs = int(g[f"{tag}_height_step"])
    sub = g[f"{tag}_height_sub"]
    assert np.linalg.norm(h[::hs, ::hs] - sub) / np.linalg.norm(sub) < (1e-5 if not tag.startswith("c") else 1e-4)


def test_pocketfft_any_shape_and_float64_digests(golden):
    """oracle/pocketfft.py against scipy 1.7.1 / numpy 1.26.4 themselves (shapes.npz): fft2,
    mean and the find_peaks spectrum of hashed integer images at odd, prime (radfg, pass7 /
    pass11 / passg), Bluestein and camera shapes, float32 and float64, bit for bit."""
    from bench_data import hash_image
    from oracle import pocketfft as P
    g = golden("shapes")
    for k, (h, w) in enumerate(g["fft_shapes"]):
        u = hash_image(int(h), int(w), seed=k)
        assert hashlib.sha256(u.tobytes()).hexdigest() == str(g[f"{h}x{w}_u16_sha"]), (h, w)
        for T, tag in ((np.float32, "f32"), (np.float64, "f64")):
            img = u.astype(T) * T(0.37)
            assert hashlib.sha256(P.fft2(img).tobytes()).hexdigest() == str(g[f"{h}x{w}_{tag}_fft2_sha"]), (h, w, tag)
            assert P.mean_T(img, T) == g[f"{h}x{w}_{tag}_mean"], (h, w, tag)
            spec = P.find_peaks_spectrum(img)
            assert hashlib.sha256(spec.tobytes()).hexdigest() == str(g[f"{h}x{w}_{tag}_spec_sha"]), (h, w, tag)


def f64_reference_image(g, tag):
    """The float64 references of shapes.npz, rebuilt exactly (make_golden.py F64_REFS)."""
    from bench_data import board_from_tables, checkerboard
    if f"{tag}_sx" in g:
        img = board_from_tables(g[f"{tag}_sx"], g[f"{tag}_sy"])
    else:
        spec = {"flat1024": (1024, 0.0, None), "rot768x1280": (768, 5.0, 1280)}[tag]
        img = checkerboard(spec[0], spec[1], cols=spec[2]).astype(np.float64)
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g[f"{tag}_sha"]), tag
    return img


def test_oracle_float64_reference_picks(golden):
    """find_peaks of a float64 reference decides its carriers from the complex128 spectrum
    (fourier.py:18; pyval/val.py:98): the oracle's exact spectrum reproduces the
    reference's picks, blobs and threshold in float64, and the different picks of the same
    image rounded to float32 (flat1024, val600x800)."""
    from oracle import fcd_oracle as O
    g = golden("shapes")
    for tag in g["f64_refs"]:
        img = f64_reference_image(g, str(tag))
        cf, peaks = O.calibration_factor(0.001, img, exact=True)
        assert np.array_equal(np.array(peaks), g[f"{tag}_peaks"]), tag
        assert cf == float(g[f"{tag}_cf"]), tag
        _, p32 = O.calibration_factor(0.001, img.astype(np.float32), exact=True)
        assert np.array_equal(np.array(p32), g[f"{tag}_peaks_f32"]), tag


def int_reference_image(golden, tag):
    """The integer-typed references of intref.npz, rebuilt exactly (make_golden.py INT_REFS):
    pattern.py's board as uint16 / int32 (bench_data.checkerboard) and the raw example
    pictures (real_pair.npz / real_df.npz)."""
    import hashlib
    from bench_data import checkerboard
    g = golden("intref")
    if tag == "ref2_u8":
        img = golden("real_pair")["ref_u8"]
    elif tag == "refdf_u16":
        img = golden("real_df")["ref_u16"]
    else:
        rows, rot, dt = {"board_u16": (1024, 0.0, np.uint16), "board_rot5_u16": (1024, 5.0, np.uint16),
                         "board_i32": (512, 0.0, np.int32)}[tag]
        img = checkerboard(rows, rot, dtype=dt)
    assert str(img.dtype) == str(g[f"{tag}_dtype"]), tag
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g[f"{tag}_sha"]), tag
    return img


INT_TAGS = ["board_u16", "board_rot5_u16", "board_i32", "ref2_u8", "refdf_u16"]


@pytest.mark.parametrize("tag", INT_TAGS)
def test_oracle_integer_reference_picks(golden, tag):
    """Integer-typed references take the complex128 spectrum (scipy's `_asfarray`,
    scipy/fft/_pocketfft/helper.py:91-92; fourier.py:18): the oracle's exact spectrum gives
    the reference's picks, cf, fft2 bits -- and on the unrotated board (uint16 as pattern.py
    writes it, and int32) picks that differ from the float32 rounding's."""
    import hashlib
    from oracle import fcd_oracle as O
    from oracle import pocketfft as P
    g = golden("intref")
    img = int_reference_image(golden, tag)
    if img.size <= 512 * 512:
        F = P.fft2(img)
        assert F.dtype == np.complex128
        assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{tag}_fft2_sha"])
    cf, peaks = O.calibration_factor(0.001, img, exact=True)
    assert np.array_equal(np.array(peaks), g[f"{tag}_peaks"]), tag
    assert cf == float(g[f"{tag}_cf"]), tag
    if tag in ("board_u16", "board_i32"):
        assert not np.array_equal(g[f"{tag}_peaks"], g[f"{tag}_peaks_f32"])


def test_image_precision_follows_scipy():
    """pyfcd._lib._img: the dtype an image reaches the engine in is scipy's fft2 type
    (float32 / float16 -> float32, float64 and every integer / bool type -> float64)."""
    from pyfcd import _lib
    from oracle import pocketfft as P
    for dt in (np.float32, np.float16, np.float64, np.uint8, np.uint16, np.int16, np.int32, np.int64, np.uint64,
               np.bool_):
        a = np.ones((4, 4), dt)
        assert _lib._img(a).dtype == P.spectrum_dtype(dt), dt
        assert _lib._img_flag(_lib._img(a)) == (_lib.FCD_IMG_F64 if P.spectrum_dtype(dt) == np.float64 else 0)
    with pytest.raises(TypeError):
        _lib._img(np.ones((4, 4), np.complex64))
