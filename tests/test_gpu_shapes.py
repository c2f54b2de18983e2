"""GPU parity of the reference setup for any frame shape and for float64 references,
against the reference's libraries themselves (tests/golden/shapes.npz, make_golden.py
`shapes`: scipy 1.7.1's fft2 and numpy 1.26.4's mean / abs at fourier.py:18, and
fcd.compute_calibration_factor / find_peaks of float64 images, fcd.py:72-101).

  * fcd_fft2 = scipy.fft.fft2 bit for bit at odd, prime (pocketfft's radfg / pass7 /
    pass11 / passg) and Bluestein sides and camera formats, float32 -> complex64 and
    float64 -> complex128 (kernels_pocketfft.hip + csrc/pocketfft.hpp);
  * the carrier picks, blob order, threshold and calibration factor of float64 references
    (pyval/val.py:98's I0, whose four blobs tie in exact arithmetic; the pattern.py board
    as float64) equal the reference's complex128 picks -- which differ from the float32
    picks of the same image for two of them.
"""
import hashlib

import numpy as np
import pytest

from test_oracle_golden import f64_reference_image

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def shapes(golden):
    return golden("shapes")


@pytest.mark.parametrize("tag", ["f32", "f64"])
def test_fft2_any_shape_bit_exact(shapes, tag):
    from bench_data import hash_image
    from pyfcd import _lib
    g = shapes
    T = np.float32 if tag == "f32" else np.float64
    tested = 0
    for k, (h, w) in enumerate(g["fft_shapes"]):
        h, w = int(h), int(w)
        if min(h, w) < 16:  # the engine's smallest frame side
            continue
        img = hash_image(h, w, seed=k).astype(T) * T(0.37)
        eng = _lib.Engine((h, w))  # (every side in [16, 16384] is taken, Bluestein sides above 4096 too)
        F = eng.fft2(img)
        assert F.dtype == (np.complex64 if T == np.float32 else np.complex128)
        assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{h}x{w}_{tag}_fft2_sha"]), (h, w, tag)
        eng.close()
        tested += 1
    assert tested >= 12


def test_float64_reference_picks(shapes):
    from pyfcd import _lib
    g = shapes
    for tag in g["f64_refs"]:
        tag = str(tag)
        img = f64_reference_image(g, tag)
        eng = _lib.Engine(img.shape)
        info = eng.set_reference(img, 0.001)
        peaks = np.array([[info.peaks[i][0], info.peaks[i][1]] for i in range(2)])
        assert np.array_equal(peaks, g[f"{tag}_peaks"]), tag
        assert info.calibration_factor == float(g[f"{tag}_cf"]), tag
        blobs = np.array([[info.blob_peaks[i][0], info.blob_peaks[i][1]] for i in range(info.n_blobs)])
        assert np.array_equal(blobs, g[f"{tag}_blob_peaks"]), tag
        assert info.threshold == float(g[f"{tag}_threshold"]), tag
        # the same image rounded to float32 takes the float32 spectrum's picks
        (i32,) = eng.find_peaks(img.astype(np.float32), 0.001)
        p32 = np.array([[i32.peaks[i][0], i32.peaks[i][1]] for i in range(2)])
        assert np.array_equal(p32, g[f"{tag}_peaks_f32"]), tag
        # and the batched float64 call agrees with set_reference
        (i64,) = eng.find_peaks(img, 0.001)
        assert [tuple(i64.peaks[i]) for i in range(2)] == [tuple(p) for p in peaks.tolist()], tag
        eng.close()


def test_float64_reference_high_level(shapes):
    """fcd.compute_calibration_factor / compute_carriers with pyval's float64 I0 (val.py:98)."""
    from pyfcd.fcd import fcd
    g = shapes
    img = f64_reference_image(g, "val1024")
    cf, (p0, p1) = fcd.compute_calibration_factor(0.001, img)
    assert cf == float(g["val1024_cf"])
    assert np.array_equal(np.array([p0, p1]), g["val1024_peaks"])


@pytest.mark.parametrize("tag", ["board_u16", "board_rot5_u16", "board_i32", "ref2_u8", "refdf_u16"])
def test_integer_reference_picks(golden, tag):
    """Integer-typed references (pattern.py:17-36 writes its board as uint16; raw uint8 /
    uint16 camera pictures) reach the engine as float64, the type scipy's fft2 promotes
    them to (scipy/fft/_pocketfft/helper.py:91-92, fourier.py:18), so set_reference,
    find_peaks and fft2 reproduce the reference's complex128 picks, blob order, threshold,
    cf and spectrum bits -- including the unrotated board's [[563, 563], [461, 563]], which
    the float32 rounding of the same board would not pick."""
    from test_oracle_golden import int_reference_image
    from pyfcd import _lib
    from pyfcd.fcd import fcd
    g = golden("intref")
    img = int_reference_image(golden, tag)
    eng = _lib.Engine(img.shape)
    info = eng.set_reference(img, 0.001)
    peaks = np.array([[info.peaks[i][0], info.peaks[i][1]] for i in range(2)])
    assert np.array_equal(peaks, g[f"{tag}_peaks"]), (tag, peaks.tolist())
    assert info.calibration_factor == float(g[f"{tag}_cf"]), tag
    blobs = np.array([[info.blob_peaks[i][0], info.blob_peaks[i][1]] for i in range(info.n_blobs)])
    assert np.array_equal(blobs, g[f"{tag}_blob_peaks"]), tag
    assert info.threshold == float(g[f"{tag}_threshold"]), tag
    (i2,) = eng.find_peaks(img, 0.001)
    assert [tuple(i2.peaks[i]) for i in range(2)] == [tuple(p) for p in peaks.tolist()], tag
    F = eng.fft2(img)
    assert F.dtype == np.complex128
    assert hashlib.sha256(F.tobytes()).hexdigest() == str(g[f"{tag}_fft2_sha"]), tag
    eng.close()
    # the drop-in classmethods with the integer image itself
    cf, (p0, p1) = fcd.compute_calibration_factor(0.001, img)
    assert cf == float(g[f"{tag}_cf"]) and np.array_equal(np.array([p0, p1]), g[f"{tag}_peaks"]), tag


def test_integer_reference_heights(golden):
    """fcd.compute_height_map with pattern.py's uint16 board as the reference (fcd.py:13-35):
    the reference's carriers, and heights within the float32 tolerance of its run."""
    from bench_data import make_frames_numpy
    from test_oracle_golden import int_reference_image
    from pyfcd.fcd import fcd
    g = golden("intref")
    ref = int_reference_image(golden, "board_u16")
    _, frames = make_frames_numpy(1024, 2, seed=0, rotate_deg=0.0)
    assert hashlib.sha256(frames.tobytes()).hexdigest() == str(g["board_u16_frames_sha"])
    for f in range(2):
        h, ph, cf = fcd.compute_height_map(ref, frames[f], 0.001, height=1.0)
        assert cf == float(g[f"board_u16_hcf{f}"])
        sub = g[f"board_u16_height_sub{f}"]
        assert np.linalg.norm(h[::4, ::4] - sub) / np.linalg.norm(sub) < 1e-5, f
