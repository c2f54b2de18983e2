"""The §8f rows around the hot path against fixtures the reference's own
pydata/analyze.py produced (tests/golden/analyze_ref.npz, make_golden.py
`analyze_ref`: the module imported as shipped, with a placeholder for its
`import cv2` that raises on any use; cv2 is only reached by the polar paths,
analyze.py:237-241, 674-676, which no fixture runs):

* analyze.mask / center (analyze.py:43-140) on camera frames and crops: bit-exact
  masks and centres (CPU, the host path);
* analyze.block_split (analyze.py:365-417): exact, float32 and float64 map folders
  (CPU, host path);
* analyze.block_amplitude / spectrogram (analyze.py:420-587) through the device
  kernels: f0 and harmonics exact, amplitudes at 1e-9 of the block maximum (the
  reference's np.fft is float64), phases at 1e-7 rad where the amplitude is not
  negligible; spectrograms at 1e-9 for float64 maps and 2e-6 for float32 maps (scipy
  computes a float32 series in float32, the device in float64);
* analyze.folder (analyze.py:143-286), plain and with the mask blend, on the frames
  the reference's own folder run saw: same files, maps at height rel-L2 1e-4 (these
  camera frames carry residues; the reference seeds border reliabilities from
  rand()), the same zeroed pixels, the same centers.txt and calibration_factor.npy.
"""
import os

import numpy as np
import pytest

LAYERS = [[5.7e-2, 1.0003], [1.2e-2, 1.48899], [4.3e-2, 1.34], [80e-2, 1.0003]]  # fcd_example.py:17


@pytest.fixture(scope="module")
def A(golden):
    return golden("analyze_ref")


def _mask_inputs(A, golden):
    """(kind, frame index, smoothed, float32 image) per mask case."""
    df = golden("real_df")
    mnames = [str(n) for n in A["mask_names"]]
    assert os.path.basename(str(df["names"][1])) == mnames[4]
    full = {4: df["frames_u16"][1], 5: A["frame5_u16"]}
    out = []
    for kind, idx, sm in A["mask_cases"].tolist():
        idx, sm = int(idx), int(sm)
        img = full[idx] if kind == "full" else A[f"crop{idx}_u16"]
        out.append((kind, idx, sm, img.astype(np.float32)))
    return out


def _masks(A):
    bits, lens = A["mask_bits"], A["mask_bits_len"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [bits[offs[i]:offs[i + 1]] for i in range(len(lens))]


def test_mask_and_center_match_reference_run(A, golden):
    from pydata.analyze import analyze
    packed = _masks(A)
    for k, (kind, idx, sm, img) in enumerate(_mask_inputs(A, golden)):
        m, c = analyze.mask(img, smoothed=sm, find_center=True)
        want = np.unpackbits(packed[k])[: m.size].reshape(m.shape).astype(bool)
        assert np.array_equal(m, want), (kind, idx, sm)
        assert c == tuple(int(v) for v in A["mask_centers"][k]), (kind, idx, sm)


def _write_maps(folder, stack):
    os.makedirs(folder, exist_ok=True)
    for t in range(stack.shape[0]):
        np.save(os.path.join(folder, f"f{t:05d}_map.npy"), stack[t])
    np.save(os.path.join(folder, "calibration_factor.npy"), np.array([0.001]))
    return folder


@pytest.fixture(scope="module")
def map_folders(A, tmp_path_factory):
    base = tmp_path_factory.mktemp("maps")
    return {dt: _write_maps(str(base / dt), A[f"{dt}_stack"]) for dt in ("float32", "float64")}


@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_block_split_matches_reference_run(A, map_folders, dt):
    from pydata.analyze import analyze
    T = A[f"{dt}_stack"].shape[0]
    got = analyze.block_split(map_folders[dt], t_limit=T - 7, num_blocks=4, block_index=1)
    want = A[f"{dt}_split"]
    assert got.dtype == want.dtype and got.shape == want.shape
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    assert np.array_equal(got[ok], want[ok])


def _close(a, b, rtol, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, what
    assert np.array_equal(np.isnan(a), np.isnan(b)), what
    ok = ~np.isnan(b)
    scale = np.abs(b[ok]).max()
    err = np.abs(a[ok] - b[ok]).max()
    assert err <= rtol * scale, (what, err / scale)


def _phase_close(p, q, amps, what, tol=1e-7):
    ok = ~np.isnan(amps) & (amps > 1e-6 * np.nanmax(amps))
    d = np.abs((np.asarray(p, np.float64) - q + np.pi) % (2 * np.pi) - np.pi)
    assert d[ok].max() < tol, (what, d[ok].max())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_block_amplitude_matches_reference_run(A, map_folders, dt):
    from pydata.analyze import analyze
    for k in range(3):
        mode, blk, zero = A[f"{dt}_amp{k}_args"].tolist()
        harm, amps, phases, f0 = analyze.block_amplitude(map_folders[dt], mode=int(mode), num_blocks=4,
                                                         block_index=int(blk), zero=zero)
        assert f0 == float(A[f"{dt}_amp{k}_f0"]), (dt, k)
        assert np.array_equal(np.array(harm, np.float64), A[f"{dt}_amp{k}_harm"]), (dt, k)
        _close(amps, A[f"{dt}_amp{k}_amps"], 1e-9, (dt, k, "amps"))
        _phase_close(phases, A[f"{dt}_amp{k}_phases"], A[f"{dt}_amp{k}_amps"], (dt, k))
    harm, amps, phases, f0 = analyze.block_amplitude(map_folders[dt], f0=5.0, mode=2, num_blocks=16, block_index=5)
    assert np.array_equal(np.array(harm, np.float64), A[f"{dt}_ampf_harm"])
    _close(amps, A[f"{dt}_ampf_amps"], 1e-9, (dt, "f0 given"))
    _phase_close(phases, A[f"{dt}_ampf_phases"], A[f"{dt}_ampf_amps"], (dt, "f0 given"))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_spectrogram_matches_reference_run(A, map_folders, dt):
    from pydata.analyze import analyze
    tol = 2e-6 if dt == "float32" else 1e-9
    t, f, S_all, S_avg = analyze.spectrogram(map_folder=map_folders[dt], fs=125, nperseg=64, noverlap=32,
                                             num_blocks=4, block_index=0)
    assert np.array_equal(t, A[f"{dt}_spec_t"]) and np.array_equal(f, A[f"{dt}_spec_f"])
    _close(S_all, A[f"{dt}_spec_all"], tol, (dt, "block"))
    _close(S_avg, A[f"{dt}_spec_avg"], tol, (dt, "avg"))
    st = A[f"{dt}_stack"]
    t, f, S = analyze.spectrogram(array=st[:, 5, 7], fs=125, nperseg=50, noverlap=10)
    assert S.dtype == A[f"{dt}_spec1"].dtype
    assert np.array_equal(t, A[f"{dt}_spec1_t"]) and np.array_equal(f, A[f"{dt}_spec1_f"])
    _close(S, A[f"{dt}_spec1"], tol, (dt, "series"))


def _frame_pixels(A, golden, name):
    df = golden("real_df")
    for n, fr in zip(df["names"], df["frames_u16"]):
        if os.path.basename(str(n)) == name:
            return fr
    assert name == str(A["mask_names"][5])
    return A["frame5_u16"]


@pytest.fixture
def fresh_engines():
    from pyfcd import _lib
    _lib._engines.clear()
    yield
    _lib._engines.clear()


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["plain", "masked"])
def test_folder_matches_reference_run(A, golden, tmp_path, fresh_engines, tag):
    from pydata import images
    from pydata.analyze import analyze
    df = golden("real_df")
    d = tmp_path / "frames"
    d.mkdir()
    ref_path = str(d / "reference_df.tif")
    images.write_tiff(ref_path, df["ref_u16"], bits=10)
    for name in A[f"folder_{tag}_frames"]:
        images.write_tiff(str(d / str(name)), _frame_pixels(A, golden, str(name)), bits=10)
    smoothed = 15 if tag == "masked" else None
    analyze.folder(ref_path, str(d), LAYERS, 0.002, smoothed=smoothed)
    maps = d / "maps"
    names = sorted(f for f in os.listdir(maps) if f.endswith("_map.npy"))
    assert names == [str(n) for n in A[f"folder_{tag}_names"]]
    assert np.load(str(maps / "calibration_factor.npy")).tolist() == A[f"folder_{tag}_cf"].tolist()
    for i, n in enumerate(names):
        h = np.load(str(maps / n))
        assert h.dtype == np.float32 and h.shape == (1024, 1024)
        want = A[f"folder_{tag}_h_sub"][i].astype(np.float64)
        got = h[::4, ::4].astype(np.float64)
        assert np.linalg.norm(got - want) / np.linalg.norm(want) < 1e-4, n
        assert int((h == 0).sum()) == int(A[f"folder_{tag}_zero_count"][i]), n
    cp = maps / "centers.txt"
    assert (open(str(cp)).read() if cp.exists() else "") == str(A[f"folder_{tag}_centers_txt"])


@pytest.mark.parametrize("dt", ["float32", "float64"])
def test_temporal_oracle_matches_reference_run(A, dt):
    """oracle/temporal_oracle.py (the checker of tests/test_temporal.py) against the
    reference's own block_amplitude outputs (CPU)."""
    from oracle import temporal_oracle as ora
    st = A[f"{dt}_stack"]
    for k in range(3):
        mode, blk, zero = A[f"{dt}_amp{k}_args"].tolist()
        harm, amps, phases, f0 = ora.block_amplitude(st, tasa=500, mode=int(mode), num_blocks=4,
                                                     block_index=int(blk), zero=zero)
        assert f0 == float(A[f"{dt}_amp{k}_f0"])
        _close(amps, A[f"{dt}_amp{k}_amps"], 1e-12, (dt, k))
