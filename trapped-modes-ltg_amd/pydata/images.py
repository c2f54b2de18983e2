"""Frame decoders for the reference's image files.

`read_gray(path)` reproduces `skimage.io.imread(path, as_gray=True)` (scikit-image
0.18.3, the call inside analyze.load_image, /root/reference/pydata/analyze.py:25-40)
for the formats the reference's data use:

* uncompressed TIFF, one sample per pixel, 8 / 16 bits, or 10 bits packed MSB-first
  (the high-speed camera's files: reference_df.tif, prueba1_*.tif, mask/*.tif;
  BitsPerSample=10, RowsPerStrip=6) -> uint8 / uint16 samples;
* PNG / BMP / anything else Pillow opens: 8-bit grey -> uint8, 16-bit grey ->
  uint16, RGB / RGBA / palette -> skimage's rgb2gray (rgba2rgb over a white
  background first), float64 in [0, 1].

`read_raw(path)` returns the samples in the form the engine ingests without host-side
conversion (fcd_process_raw): (bytes ndarray, format) with FCD_FMT_U8 for 8-bit grey,
FCD_FMT_U16 for 16-bit, FCD_FMT_P10 for the packed 10-bit TIFF rows as stored on disk
(the strips are read straight into the caller's buffer, no unpacking on the host).
"""
import struct

import numpy as np

from pyfcd._lib import FCD_FMT_P10, FCD_FMT_U8, FCD_FMT_U16

_TIFF_TYPES = {1: "B", 3: "H", 4: "I", 16: "Q"}


class TiffInfo:
    __slots__ = ("rows", "cols", "bits", "offsets", "counts", "endian")


def _tiff_info(buf):
    if buf[:4] not in (b"II*\x00", b"MM\x00*"):
        return None
    e = "<" if buf[:2] == b"II" else ">"
    (ifd,) = struct.unpack_from(e + "I", buf, 4)
    (n,) = struct.unpack_from(e + "H", buf, ifd)
    tags = {}
    for i in range(n):
        tag, typ, cnt, val = struct.unpack_from(e + "HHI4s", buf, ifd + 2 + 12 * i)
        code = _TIFF_TYPES.get(typ)
        if code is None:
            continue
        size = struct.calcsize(code) * cnt
        raw = val if size <= 4 else buf[struct.unpack(e + "I", val)[0]:][:size]
        tags[tag] = struct.unpack_from(e + code * cnt, raw)
    compression = tags.get(259, (1,))[0]
    spp = tags.get(277, (1,))[0]
    planar = tags.get(284, (1,))[0]
    fill = tags.get(266, (1,))[0]
    if compression != 1 or spp != 1 or planar != 1 or fill != 1:
        raise ValueError(f"unsupported TIFF (compression {compression}, samples/pixel {spp}, planar {planar}, "
                         f"fill order {fill}): only uncompressed single-channel images are decoded")
    t = TiffInfo()
    t.cols, t.rows = tags[256][0], tags[257][0]
    t.bits = tags.get(258, (1,))[0]
    t.offsets, t.counts = tags[273], tags[279]
    t.endian = e
    if t.bits not in (8, 10, 16):
        raise ValueError(f"unsupported TIFF BitsPerSample {t.bits}")
    return t


def _tiff_rows_bytes(buf, t, out=None):
    """The image's row bytes (strips concatenated), rows * ceil(cols * bits / 8)."""
    pitch = (t.cols * t.bits + 7) // 8
    total = pitch * t.rows
    dst = np.empty(total, np.uint8) if out is None else out
    pos = 0
    for off, cnt in zip(t.offsets, t.counts):
        cnt = min(cnt, total - pos)
        dst[pos:pos + cnt] = np.frombuffer(buf, np.uint8, cnt, off)
        pos += cnt
        if pos >= total:
            break
    if pos != total:
        raise ValueError("truncated TIFF strips")
    return dst


def unpack10(rows_bytes, rows, cols):
    """10-bit MSB-first packed rows -> uint16 [rows, cols] (cols % 4 == 0)."""
    b = rows_bytes.reshape(rows, cols // 4, 5).astype(np.uint16)
    out = np.empty((rows, cols // 4, 4), np.uint16)
    out[..., 0] = (b[..., 0] << 2) | (b[..., 1] >> 6)
    out[..., 1] = ((b[..., 1] & 63) << 4) | (b[..., 2] >> 4)
    out[..., 2] = ((b[..., 2] & 15) << 6) | (b[..., 3] >> 2)
    out[..., 3] = ((b[..., 3] & 3) << 8) | b[..., 4]
    return out.reshape(rows, cols)


def pack10(samples):
    """uint16 [rows, cols] (values < 1024, cols % 4 == 0) -> 10-bit MSB-first packed
    row bytes [rows * cols * 10 / 8] (the inverse of unpack10; FCD_FMT_P10)."""
    s = np.asarray(samples, np.uint16)
    rows, cols = s.shape
    q = s.reshape(rows, cols // 4, 4).astype(np.uint16)
    b = np.empty((rows, cols // 4, 5), np.uint8)
    b[..., 0] = q[..., 0] >> 2
    b[..., 1] = ((q[..., 0] & 3) << 6) | (q[..., 1] >> 4)
    b[..., 2] = ((q[..., 1] & 15) << 4) | (q[..., 2] >> 6)
    b[..., 3] = ((q[..., 2] & 63) << 2) | (q[..., 3] >> 8)
    b[..., 4] = q[..., 3] & 255
    return b.reshape(-1)


def write_tiff(path, samples, bits=None, rows_per_strip=6, endian="<"):
    """Minimal uncompressed single-channel TIFF writer (8, 10-packed or 16 bits), the
    layout of the camera files the reference reads (used to build test inputs)."""
    s = np.asarray(samples)
    rows, cols = s.shape
    bits = bits or (8 if s.dtype == np.uint8 else 16)
    if bits == 10:
        data = pack10(s).tobytes()
    elif bits == 16:
        data = s.astype(np.dtype(np.uint16).newbyteorder(endian)).tobytes()
    else:
        data = s.astype(np.uint8).tobytes()
    pitch = (cols * bits + 7) // 8
    nstrips = (rows + rows_per_strip - 1) // rows_per_strip
    offs = [8 + i * rows_per_strip * pitch for i in range(nstrips)]
    cnts = [min(rows_per_strip, rows - i * rows_per_strip) * pitch for i in range(nstrips)]
    ifd = 8 + len(data)
    tags = [(256, 3, 1, cols), (257, 3, 1, rows), (258, 3, 1, bits), (259, 3, 1, 1), (262, 3, 1, 1),
            (273, 4, nstrips, None), (277, 3, 1, 1), (278, 3, 1, rows_per_strip), (279, 4, nstrips, None),
            (284, 3, 1, 1)]
    extra_at = ifd + 2 + 12 * len(tags) + 4
    out = bytearray((b"II*\x00" if endian == "<" else b"MM\x00*") + struct.pack(endian + "I", ifd))
    out += data
    out += struct.pack(endian + "H", len(tags))
    extra = bytearray()
    for tag, typ, cnt, val in tags:
        if val is None:
            arr = offs if tag == 273 else cnts
            if cnt == 1:
                out += struct.pack(endian + "HHII", tag, typ, 1, arr[0])
            else:
                out += struct.pack(endian + "HHII", tag, typ, cnt, extra_at + len(extra))
                extra += struct.pack(endian + "I" * cnt, *arr)
        elif typ == 3:
            out += struct.pack(endian + "HHIHH", tag, typ, cnt, val, 0)
        else:
            out += struct.pack(endian + "HHII", tag, typ, cnt, val)
    out += struct.pack(endian + "I", 0) + extra
    with open(path, "wb") as f:
        f.write(out)


def _tiff_samples(buf, t):
    rb = _tiff_rows_bytes(buf, t)
    if t.bits == 8:
        return rb.reshape(t.rows, t.cols)
    if t.bits == 16:
        return rb.view(np.dtype(np.uint16).newbyteorder(t.endian)).reshape(t.rows, t.cols).astype(np.uint16)
    if t.cols % 4:
        raise ValueError("10-bit TIFF width must be a multiple of 4")
    return unpack10(rb, t.rows, t.cols)


def _rgb2gray(rgb):
    """skimage.color.rgb2gray (0.18.3): img_as_float, then 0.2125 R + 0.7154 G + 0.0721 B."""
    a = rgb[..., :3]
    if a.dtype == np.uint8:
        a = np.multiply(a, 1.0 / 255, dtype=np.float64)  # skimage img_as_float (dtype.py _convert)
    elif a.dtype == np.uint16:
        a = np.multiply(a, 1.0 / 65535, dtype=np.float64)
    coeffs = np.array([0.2125, 0.7154, 0.0721], dtype=a.dtype)
    return a @ coeffs


def _rgba2rgb(rgba):
    """skimage.color.rgba2rgb over the default white background."""
    a = np.multiply(rgba, 1.0 / (255 if rgba.dtype == np.uint8 else 65535), dtype=np.float64)
    alpha = a[..., -1:]
    return np.clip((1 - alpha) + alpha * a[..., :3], 0, 1)


def _pil_gray(path):
    from PIL import Image
    with Image.open(path) as im:
        mode = im.mode
        if mode == "P":
            im = im.convert("RGBA" if "transparency" in im.info else "RGB")
            mode = im.mode
        a = np.asarray(im)
    if mode in ("L", "I;16", "I;16B", "I;16L"):
        return a.astype(np.uint16) if mode.startswith("I;16") else a
    if mode == "RGB":
        return _rgb2gray(a)
    if mode == "RGBA":
        return _rgb2gray(_rgba2rgb(a))
    if mode in ("I", "F"):
        return a
    raise ValueError(f"unsupported image mode {mode!r} in {path}")


def read_gray(path):
    """skimage.io.imread(path, as_gray=True) for the supported formats."""
    with open(path, "rb") as f:
        buf = f.read()
    t = _tiff_info(buf)
    if t is not None:
        return _tiff_samples(buf, t)
    return _pil_gray(path)


def raw_info(path):
    """(rows, cols, format) of the raw samples read_raw returns."""
    with open(path, "rb") as f:
        head = f.read(1 << 16)
    t = None
    if head[:4] in (b"II*\x00", b"MM\x00*"):
        with open(path, "rb") as f:
            t = _tiff_info(f.read())
    if t is not None:
        fmt = {8: FCD_FMT_U8, 10: FCD_FMT_P10, 16: FCD_FMT_U16}[t.bits]
        return t.rows, t.cols, fmt
    g = _pil_gray(path)
    fmt = {np.dtype(np.uint8): FCD_FMT_U8, np.dtype(np.uint16): FCD_FMT_U16}.get(g.dtype)
    if fmt is None:
        raise ValueError(f"{path}: colour images have no raw single-channel form")
    return g.shape[0], g.shape[1], fmt


def read_raw(path, out=None):
    """Raw samples as stored, for fcd_process_raw: returns (uint8 byte array, format).
    `out` (optional, e.g. a slice of a pinned buffer) receives the bytes."""
    with open(path, "rb") as f:
        buf = f.read()
    t = _tiff_info(buf)
    if t is not None:
        if t.bits == 10:
            if t.cols % 4:
                raise ValueError("10-bit TIFF width must be a multiple of 4")
            return _tiff_rows_bytes(buf, t, out), FCD_FMT_P10
        s = _tiff_samples(buf, t)
    else:
        s = _pil_gray(path)
    fmt = {np.dtype(np.uint8): FCD_FMT_U8, np.dtype(np.uint16): FCD_FMT_U16}.get(s.dtype)
    if fmt is None:
        raise ValueError(f"{path}: colour images have no raw single-channel form")
    b = np.ascontiguousarray(s).view(np.uint8).reshape(-1)
    if out is not None:
        out[:b.size] = b
        b = out[:b.size]
    return b, fmt
