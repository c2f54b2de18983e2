"""The engine's host-side logic (trapped-modes-ltg_amd/csrc/host_logic.hpp: blob
labelling, carrier picks, calibration factor, disk raster, pocketfft plans, the pinned
pipeline's parallel copy) built with g++ under AddressSanitizer + UBSan and -Werror
 and checked against the oracle.  CPU only: the header has no HIP code."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "native", "host_logic_test.cpp")


@pytest.fixture(scope="module")
def hlt(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("native") / "host_logic_test")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-Wall", "-Wextra", "-Werror", "-pthread", SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr

    def run(*args, stdin=""):
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
        p = subprocess.run([exe] + list(args), input=stdin, capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode == 0, (args, p.returncode, p.stderr[-3000:])
        assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
        return p.stdout
    return run


def _cands(img, thr):
    H, W = img.shape
    inner = np.zeros(img.shape, bool)
    inner[1:-1, 1:-1] = True
    idx = np.flatnonzero((img > thr) & inner)
    rng = np.random.default_rng(len(idx))
    rng.shuffle(idx)  # the device hands candidates over in arbitrary order
    return f"{H} {W} {len(idx)}\n" + "".join(f"{i} {float(img.flat[i])!r}\n" for i in idx)


@pytest.mark.parametrize("seed", range(6))
def test_labelling_matches_oracle(hlt, seed):
    """fourier.find_peak_locations (fourier.py:139-168): 8-connected blobs, per blob the
    first maximum, the 4 dimmest in stable order -- ties included (integer intensities)."""
    from oracle import fcd_oracle as O
    rng = np.random.default_rng(seed)
    H, W = (64, 96) if seed % 2 else (128, 128)
    img = np.zeros((H, W), np.float32)
    for _ in range(12):
        r, c = rng.integers(1, H - 4), rng.integers(1, W - 4)
        img[r:r + rng.integers(1, 4), c:c + rng.integers(1, 5)] = rng.integers(2, 6)
    img[rng.random((H, W)) < 0.02] = 3.0
    got = [tuple(int(v) for v in ln.split()) for ln in hlt("labels", stdin=_cands(img, 1.5)).splitlines()]
    want = [tuple(int(v) for v in p) for p in O.find_peak_locations(img, 1.5, 4)]
    assert got == want


@pytest.mark.parametrize("shape", [(1024, 1024), (512, 1024), (256, 128)])
def test_disk_raster_matches_oracle(hlt, shape):
    """skimage.draw.disk's strict-inequality raster (carriers.py:17-20) per carrier, each
    with its own radius, clipped at the image border."""
    from oracle import fcd_oracle as O
    H, W = shape
    rng = np.random.default_rng(H + W)
    for _ in range(8):
        pr = rng.integers(0, H, 2)
        pc = rng.integers(0, W, 2)
        R = rng.uniform(0.5, H / 6, 2)
        out = hlt("geometry", stdin=f"{H} {W} 0.37 {pr[0]} {pc[0]} {pr[1]} {pc[1]} {float(R[0])!r} {float(R[1])!r}\n").splitlines()
        counts = [int(v) for v in out[0].split()]
        rows = np.array([int(v) for v in out[1].split()]).reshape(2, W, 2)
        for q in range(2):
            m = O.disk_mask((H, W), (pr[q], pc[q]), R[q])
            assert counts[q] == int(m.sum())
            for j in range(W):
                rr = np.flatnonzero(m[:, j])
                lo, hi = rows[q, j]
                if rr.size:
                    assert (lo, hi) == (rr[0], rr[-1]) and rr.size == hi - lo + 1
                else:
                    assert lo > hi


def test_carrier_pick_and_calibration(hlt, golden):
    """fourier.find_peaks' rightmost / perpendicular picks (fourier.py:38-39), the
    calibration factor (fcd.py:85-101) and radius (fcd.py:68) from the golden blob lists,
    bit-exact against the reference's own outputs."""
    for name in ("real_pair", "real_df"):
        g = golden(name)
        blobs = [int(r) * 1024 + int(c) for r, c in g["blob_peaks"]]
        out = hlt("setup", stdin=f"1024 1024 {float(g['square_size'])!r} {len(blobs)} " + " ".join(map(str, blobs)))
        lines = out.splitlines()
        peaks = np.array([int(v) for v in lines[0].split()]).reshape(2, 2)
        cf, radius = (float(v) for v in lines[1].split())
        freqs = np.array([float(v) for v in lines[2].split()]).reshape(2, 2)
        assert np.array_equal(peaks, g["peaks"]), name
        assert cf == float(g["cf"]) and radius == float(g["radius"]), name
        assert np.array_equal(freqs, g["freqs"]), name
        assert [int(v) for v in lines[3].split()] == list(g["mask_count"]), name


def test_no_blobs_is_an_error(hlt):
    out = hlt("setup", stdin="64 64 1.0 0\n")
    assert out.startswith("error -5")  # FCD_E_NOPEAKS, as the reference's min() of an empty list raises


PF_LENGTHS = [1, 2, 3, 5, 7, 8, 11, 12, 13, 17, 31, 49, 60, 64, 93, 121, 128, 186, 189, 227, 257, 289, 343, 377,
              1000, 1021, 1023, 1080, 1920, 2048, 2448]


@pytest.mark.parametrize("f64", [0, 1])
@pytest.mark.parametrize("real", [1, 0])
def test_pocketfft_passes_match_oracle(hlt, real, f64):
    """csrc/pocketfft.hpp -- the exact passes the device runs (rfftp radf2/3/4/5/g, cfftp
    pass2/3/4/5/7/8/11/g, Bluestein), its plans and sincos_2pibyn twiddles -- run on the
    host under the sanitizers, bit for bit against oracle/pocketfft.py (itself pinned to
    scipy 1.7.1 on every length 1..400, tests/golden/shapes.npz) in both precisions."""
    from oracle import pocketfft as P
    T = np.float64 if f64 else np.float32
    rng = np.random.default_rng(11 + real + 2 * f64)
    for n in PF_LENGTHS:
        rows = 2
        if real:
            x = rng.standard_normal((rows, n)).astype(T)
            want_r, want_i = P.rfft_rows(x, T)
            vals = x.astype(np.float64).ravel()
        else:
            z = (rng.standard_normal((rows, n)) + 1j * rng.standard_normal((rows, n)))
            zr, zi = z.real.astype(T), z.imag.astype(T)
            want_r, want_i = P.cfft((zr.copy(), zi.copy()), True, T)
            vals = np.stack([zr, zi], -1).astype(np.float64).ravel()
        stdin = f"{n} {real} {f64} {rows}\n" + " ".join(float(v).hex() for v in vals) + "\n"
        lines = hlt("pfrun", stdin=stdin).splitlines()
        blue, n2, nf = (int(v) for v in lines[0].split()[1:])
        assert bool(blue) == P.use_bluestein(n, bool(real)), n
        got = np.array([[float.fromhex(a) for a in ln.split()] for ln in lines[1:]], np.float64).astype(T)
        got = got.reshape(rows, -1, 2)
        assert np.array_equal(got[..., 0], want_r) and np.array_equal(got[..., 1], want_i), (n, real, f64)


@pytest.mark.parametrize("nbytes", [0, 1, 4095, 8 << 20, (8 << 20) + 7, 77_777_777])
def test_parallel_copy(hlt, nbytes):
    assert hlt("parcopy", stdin=f"{nbytes}\n").strip() == "ok"
