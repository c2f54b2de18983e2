"""CPU checks of the frame ingest and batch-driver host side:
the decoders against scikit-image's decodes of the reference's own example pictures
(tests/golden/ingest.npz, sha256 of the float32 image analyze.load_image returns),
TIFF / packing round trips, rgb2gray, and analyze.mask / analyze.center against the
reference's procedure (analyze.py:86-100, :119-137) on the camera frames.

The example pictures are read from /root/reference when it is present (this
container); those cases skip elsewhere.  Everything else builds its inputs."""
import hashlib
import os

import numpy as np
import pytest

PICS = "/root/reference/examples/Pictures"
have_pics = pytest.mark.skipif(not os.path.isdir(PICS), reason="reference example pictures not present")


@have_pics
def test_load_image_matches_skimage_decodes(golden):
    from pydata.analyze import analyze
    g = golden("ingest")
    for name, sha, shape, total in zip(g["files"], g["dec_sha"], g["dec_shape"], g["dec_sum"]):
        a = analyze.load_image(os.path.join(PICS, str(name)))
        assert a.dtype == np.float32 and a.shape == tuple(shape), name
        assert hashlib.sha256(a.tobytes()).hexdigest() == str(sha), name
        assert float(a.astype(np.float64).sum()) == float(total)


@have_pics
def test_raw_samples_widen_to_load_image(golden):
    """read_raw's bytes (what crosses PCIe) widen to exactly load_image's float32."""
    from pydata import images
    from pyfcd import _lib
    g = golden("ingest")
    for name in g["files"]:
        p = os.path.join(PICS, str(name))
        raw, fmt = images.read_raw(p)
        rows, cols, fmt2 = images.raw_info(p)
        assert fmt == fmt2
        if fmt == _lib.FCD_FMT_P10:
            s = images.unpack10(raw, rows, cols)
        elif fmt == _lib.FCD_FMT_U16:
            s = raw.view(np.uint16).reshape(rows, cols)
        else:
            s = raw.reshape(rows, cols)
        assert np.array_equal(s.astype(np.float32), images.read_gray(p).astype(np.float32)), name


@pytest.mark.parametrize("bits,endian", [(8, "<"), (10, "<"), (10, ">"), (16, "<"), (16, ">")])
def test_tiff_round_trip(tmp_path, bits, endian):
    from pydata import images
    rng = np.random.default_rng(bits)
    a = rng.integers(0, 1 << bits, (48, 64)).astype(np.uint8 if bits == 8 else np.uint16)
    p = str(tmp_path / "f.tif")
    images.write_tiff(p, a, bits=bits, endian=endian, rows_per_strip=5)
    assert np.array_equal(images.read_gray(p), a)
    if bits == 10:
        raw, _ = images.read_raw(p)
        assert np.array_equal(raw, images.pack10(a))
        assert np.array_equal(images.unpack10(raw, 48, 64), a)


def test_pil_formats_follow_skimage_rules(tmp_path):
    """8-bit grey stays integer; RGB / RGBA go through rgb2gray (float64 in [0, 1])."""
    from PIL import Image
    from pydata import images
    rng = np.random.default_rng(3)
    g = rng.integers(0, 256, (32, 40)).astype(np.uint8)
    for ext in ("png", "bmp"):
        Image.fromarray(g).save(str(tmp_path / f"g.{ext}"))
        out = images.read_gray(str(tmp_path / f"g.{ext}"))
        assert out.dtype == np.uint8 and np.array_equal(out, g)
    rgb = rng.integers(0, 256, (32, 40, 3)).astype(np.uint8)
    Image.fromarray(rgb).save(str(tmp_path / "c.png"))
    want = np.multiply(rgb, 1.0 / 255, dtype=np.float64) @ np.array([0.2125, 0.7154, 0.0721])
    assert np.array_equal(images.read_gray(str(tmp_path / "c.png")), want)
    rgba = rng.integers(0, 256, (32, 40, 4)).astype(np.uint8)
    Image.fromarray(rgba).save(str(tmp_path / "a.png"))
    out = images.read_gray(str(tmp_path / "a.png"))
    assert out.dtype == np.float64 and out.min() >= 0 and out.max() <= 1
    with pytest.raises(ValueError):
        images.read_raw(str(tmp_path / "c.png"))


@have_pics
def test_mask_and_center_match_reference(golden):
    from pydata.analyze import analyze
    g = golden("ingest")
    names = [str(n) for n in g["mask_names"]]
    for k, (idx, _) in enumerate(g["folder_which"][::2]):
        img = analyze.load_image(os.path.join(PICS, "mask", names[idx]))
        m, c = analyze.mask(img, smoothed=int(g["mask_smoothed"][k]), find_center=True)
        want = np.unpackbits(g["mask_bits"][k])[: m.size].reshape(m.shape).astype(bool)
        assert np.array_equal(m, want)
        assert c == tuple(int(v) for v in g["mask_centers"][k])


def test_mask_center_synthetic():
    """A dark ring around a bright disc: the mask is the ring, the centre the disc's."""
    from pydata.analyze import analyze
    n = 128
    y, x = np.mgrid[:n, :n]
    r = np.hypot(y - 70, x - 60)
    img = np.full((n, n), 200.0, np.float32)
    img[(r > 20) & (r < 40)] = 10.0
    m = analyze.mask(img, smoothed=3)
    assert m[70, 60 + 30] and not m[70, 60] and not m[2, 2]
    assert analyze.center(m) == (70, 60)
    with pytest.raises(UnboundLocalError):
        analyze.center(np.zeros((16, 16), bool))


def test_folder_argument_errors(tmp_path):
    from pydata.analyze import analyze
    with pytest.raises(NotImplementedError):
        analyze.folder("ref.tif", str(tmp_path), None, 0.002, polar=True)
    with pytest.raises(ValueError):
        analyze.folder("ref.tif", str(tmp_path), None, 0.002, show_mask=True)
