"""Generate the committed golden fixtures from the reference itself.

Run ONLY in the survey/build container (never on the GPU box), with the
interpreter that can import the reference:

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -B tests/golden/make_golden.py

Versions pinned by that interpreter: numpy 1.26.4, scipy 1.7.1,
scikit-image 0.18.3 (recorded in every fixture as `versions`).  The reference
is imported read-only from /root/reference; nothing from it is copied: only
inputs and the reference's OUTPUTS are written, as small .npz files.

Fixtures (all under tests/golden/):
  real_pair.npz      reference_2.png + 202406_1457001661.bmp (examples/fcd_example.py:10-23)
  real_df.npz        reference_df.tif + three 10-bit frames (analyze.folder inputs)
  unwrap_crops.npz   stage-isolated unwrap: reference wrapped phases (crops + one
                     full 1024^2 map) and skimage's unwrap of exactly those inputs
  synthetic.npz      seeded synthetic checkerboards 64/128/256 (rotated sinusoid and
                     pattern.py-style binary), full outputs of compute_height_map
  integrate.npz      fourier.integrate_in_fourier on seeded gradient fields
  val.npz            pyval.val(0, gauss_sin) accuracy (README.md:5-7 "< 0.52 %")
  ingest.npz         analyze.load_image decodes of every example picture (sha256 of the
                     float32 image), analyze.mask / center of camera frames, and the
                     analyze.folder loop body's height maps with and without the mask
"""
import os
import sys
import warnings

import numpy as np

warnings.filterwarnings("ignore")
sys.dont_write_bytecode = True
REF = "/root/reference"
sys.path.insert(0, REF)

import scipy  # noqa: E402
import skimage  # noqa: E402
from scipy.fft import fft2, ifft2  # noqa: E402
from skimage import io  # noqa: E402
from skimage.restoration import unwrap_phase  # noqa: E402

from pyfcd.fcd import fcd, fourier  # noqa: E402  (reference, read-only)

OUT = os.path.dirname(os.path.abspath(__file__))
PICS = os.path.join(REF, "examples", "Pictures")
VERSIONS = f"numpy {np.__version__}; scipy {scipy.__version__}; scikit-image {skimage.__version__}"
LAYERS = [[5.7e-2, 1.0003], [1.2e-2, 1.48899], [4.3e-2, 1.34], [80e-2, 1.0003]]  # fcd_example.py:17


def load_raw(name):
    """Raw integer pixels; analyze.load_image (analyze.py:40) is exactly .astype(float32) of these."""
    a = io.imread(os.path.join(PICS, name), as_gray=True)
    assert a.ndim == 2 and a.dtype in (np.uint8, np.uint16), (name, a.dtype)
    return a


def kfield(wrapped, unwrapped):
    return np.rint((unwrapped - wrapped.astype(np.float64)) / (2 * np.pi)).astype(np.int16)


def peak_locations(reference):
    """The 4 blob peaks find_peaks picks from (fourier.py:18-37), for debugging fixtures."""
    image_fft = np.fft.fftshift(np.abs(fft2(reference - np.mean(reference))))
    kr, kc = fourier.wavenumber_meshgrid(image_fft.shape, shifted=True)
    kmin = 4 * np.pi / min(reference.shape)
    image_fft *= (kr ** 2 + kc ** 2) > kmin ** 2
    thr = 0.5 * np.max(image_fft)
    locs = fourier.find_peak_locations(image_fft, thr, 4)
    return np.array([np.asarray(p) for p in locs], np.int64), float(thr)


def run_pair(ref_f32, disp_f32, sq, layers=None, height=None):
    """Reference compute_height_map plus its intermediates (fcd.py:13-35, 103-120)."""
    hmap, phases, cf = fcd.compute_height_map(ref_f32, disp_f32, sq, layers=layers, height=height)
    carriers, cf2 = fcd.compute_carriers(ref_f32, sq)
    assert cf2 == cf
    D = fft2(disp_f32)
    wrapped = np.stack([(-np.angle(ifft2(D * c.mask) * c.ccsgn)).astype(np.float32) for c in carriers])
    return dict(
        height=hmap, phases=phases, cf=cf, wrapped=wrapped,
        peaks=np.array([np.asarray(c.pixels) for c in carriers], np.int64),
        radius=float(carriers[0].radius),
        freqs=np.array([c.frequencies for c in carriers], np.float64),
        mask_count=np.array([int(c.mask.sum()) for c in carriers], np.int64),
    )


def stats(a):
    a = np.asarray(a, np.float64)
    return np.array([a.sum(), np.sqrt((a * a).sum()), np.abs(a).max()], np.float64)


def make_real_pair():
    ref_u8 = load_raw("reference_2.png")
    disp_u8 = load_raw("202406_1457001661.bmp")
    ref, disp = ref_u8.astype(np.float32), disp_u8.astype(np.float32)
    sq = 0.0022
    r = run_pair(ref, disp, sq, layers=LAYERS)
    cf_plain, peaks_plain = fcd.compute_calibration_factor(sq, ref)
    locs, thr = peak_locations(ref)
    np.savez_compressed(
        os.path.join(OUT, "real_pair.npz"), versions=VERSIONS,
        ref_u8=ref_u8, disp_u8=disp_u8, square_size=sq, layers=np.array(LAYERS),
        eff_height=fcd.height_from_layers(LAYERS),
        peaks=r["peaks"], radius=r["radius"], cf=r["cf"], freqs=r["freqs"], mask_count=r["mask_count"],
        blob_peaks=locs, threshold=thr, cf_plain=cf_plain,
        wrapped_sub=r["wrapped"][:, ::8, ::8], wrapped_stats=np.stack([stats(w) for w in r["wrapped"]]),
        k=np.stack([kfield(w, p) for w, p in zip(r["wrapped"], r["phases"])]),
        height_sub=r["height"][::4, ::4].astype(np.float32), height_stats=stats(r["height"]),
    )
    print("real_pair", r["peaks"].tolist(), r["cf"], r["radius"])


def make_real_df():
    ref_u16 = load_raw("reference_df.tif")
    names = ["prueba1_20250317_122608_C1S0001000001.tif",
             "mask/0_5mm_circular_100ms_20250529_141304_C1S0001000005.tif",
             "ellipse_10.tif"]
    frames = np.stack([load_raw(n) for n in names])
    ref = ref_u16.astype(np.float32)
    sq = 0.002
    ks, hsub, hst, wsub, res = [], [], [], [], []
    for f in frames:
        r = run_pair(ref, f.astype(np.float32), sq, layers=LAYERS)
        ks.append(np.stack([kfield(w, p) for w, p in zip(r["wrapped"], r["phases"])]))
        hsub.append(r["height"][::4, ::4].astype(np.float32))
        hst.append(stats(r["height"]))
        wsub.append(r["wrapped"][:, ::8, ::8])
    committed_cf = np.load(os.path.join(PICS, "mask", "maps", "calibration_factor.npy"))
    locs, thr = peak_locations(ref)
    np.savez_compressed(
        os.path.join(OUT, "real_df.npz"), versions=VERSIONS, names=np.array(names),
        ref_u16=ref_u16, frames_u16=frames, square_size=sq,
        peaks=r["peaks"], radius=r["radius"], cf=r["cf"], freqs=r["freqs"], mask_count=r["mask_count"],
        committed_cf=committed_cf, blob_peaks=locs, threshold=thr,
        k=np.stack(ks), height_sub=np.stack(hsub), height_stats=np.stack(hst), wrapped_sub=np.stack(wsub),
    )
    print("real_df", r["peaks"].tolist(), r["cf"], committed_cf)


def make_unwrap_crops():
    """Stage-isolated unwrap vectors: the reference's own wrapped phases -> skimage unwrap."""
    ref = load_raw("reference_df.tif").astype(np.float32)
    disp = load_raw("ellipse_10.tif").astype(np.float32)
    carriers, _ = fcd.compute_carriers(ref, 0.002)
    D = fft2(disp)
    full = (-np.angle(ifft2(D * carriers[0].mask) * carriers[0].ccsgn)).astype(np.float32)
    ref2 = load_raw("reference_2.png").astype(np.float32)
    disp2 = load_raw("202406_1457001661.bmp").astype(np.float32)
    c2, _ = fcd.compute_carriers(ref2, 0.0022)
    full2 = (-np.angle(ifft2(fft2(disp2) * c2[1].mask) * c2[1].ccsgn)).astype(np.float32)
    crops = np.stack([full[384:640, 384:640], full[0:256, 512:768], full2[300:556, 600:856],
                      full2[700:956, 100:356]])
    ks = np.stack([kfield(c, unwrap_phase(c)) for c in crops])
    # rectangular crop too (H != W)
    rect = np.ascontiguousarray(full2[100:228, 200:456])
    np.savez_compressed(
        os.path.join(OUT, "unwrap_crops.npz"), versions=VERSIONS,
        crops=crops, k_crops=ks, rect=rect, k_rect=kfield(rect, unwrap_phase(rect)),
        full=full, k_full=kfield(full, unwrap_phase(full)),
    )
    print("unwrap_crops", crops.shape)


def synth_frame(n, kind, seed, rotate_deg=5.0, amp=None):
    """Seeded synthetic pair: checkerboard I0 and I0 warped by grad of a Gaussian-bump surface."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:n, 0:n].astype(np.float64)
    period = max(8.0, n / 12.0)  # pixels per checker period
    th = np.deg2rad(rotate_deg)

    def board(yy, xx):
        u = (xx * np.cos(th) + yy * np.sin(th)) * 2 * np.pi / period
        v = (-xx * np.sin(th) + yy * np.cos(th)) * 2 * np.pi / period
        s = np.sin(u) * np.sin(v)
        if kind == "binary":
            return np.where(s >= 0, 65535.0, 0.0)
        return 0.5 + 0.5 * s

    h = np.zeros((n, n))
    c = 0.3 if amp is None else amp  # peak strain ~ c: keeps the warp fold-free
    for _ in range(4):
        cy, cx = rng.uniform(0.25 * n, 0.75 * n, 2)
        sg = rng.uniform(0.08 * n, 0.15 * n)
        h += rng.choice([-1.0, 1.0]) * c * sg * sg * np.exp(-((y - cy) ** 2 + (x - cx) ** 2) / (2 * sg * sg))
    gy, gx = np.gradient(h)
    I0 = board(y, x).astype(np.float32)
    I = board(np.clip(y + gy, 0, n - 1), np.clip(x + gx, 0, n - 1)).astype(np.float32)
    return I0, I, period


def make_synthetic():
    out = {"versions": VERSIONS}
    cases = []
    for n in (64, 128, 256):
        for kind in ("sine", "binary"):
            seed = 1000 + n + (kind == "binary")
            I0, I, period = synth_frame(n, kind, seed)
            sq = period / 2.0  # => calibration factor ~ 1
            r = run_pair(I0, I, sq, height=1.0)
            tag = f"{kind}{n}"
            cases.append(tag)
            out[f"{tag}_ref"] = I0
            out[f"{tag}_disp"] = I
            out[f"{tag}_sq"] = sq
            for key in ("height", "phases", "wrapped", "peaks", "freqs", "mask_count"):
                out[f"{tag}_{key}"] = r[key]
            out[f"{tag}_cf"] = r["cf"]
            out[f"{tag}_radius"] = r["radius"]
            unw = np.stack([unwrap_phase(w) for w in r["wrapped"]])
            assert np.array_equal(unw, r["phases"])
            print(tag, r["peaks"].tolist(), r["cf"])
    # one rectangular case (H != W)
    I0, I, period = synth_frame(128, "sine", 77)
    I0, I = np.ascontiguousarray(I0[:64]), np.ascontiguousarray(I[:64])
    r = run_pair(I0, I, period / 2.0, height=1.0)
    for key in ("height", "phases", "wrapped", "peaks", "freqs", "mask_count"):
        out[f"rect_{key}"] = r[key]
    out.update(rect_ref=I0, rect_disp=I, rect_sq=period / 2.0, rect_cf=r["cf"], rect_radius=r["radius"])
    cases.append("rect")
    out["cases"] = np.array(cases)
    np.savez_compressed(os.path.join(OUT, "synthetic.npz"), **out)


def make_integrate():
    rng = np.random.default_rng(7)
    out = {"versions": VERSIONS}
    for (h, w) in ((64, 64), (128, 64), (256, 256)):
        gx = rng.standard_normal((h, w))
        gy = rng.standard_normal((h, w))
        cf = 0.37
        out[f"gx_{h}x{w}"] = gx
        out[f"gy_{h}x{w}"] = gy
        out[f"h_{h}x{w}"] = fourier.integrate_in_fourier(gx, gy, cf)
        out[f"cf_{h}x{w}"] = cf
        kr, kc = fourier.wavenumber_meshgrid((h, w), cf)
        out[f"krow_{h}x{w}"] = kr[:, 0].copy()
        out[f"kcol_{h}x{w}"] = kc[0, :].copy()
    np.savez_compressed(os.path.join(OUT, "integrate.npz"), **out)


def make_val():
    from pyval.val import val  # reference harness, read-only

    def step(X, a=0.02, w=400):  # examples/val_example.py:16-18
        x0 = len(X) // 2
        return 1 / (1 + np.exp(-a * (X - x0 + w / 2))) * 1 / (1 + np.exp(a * (X - x0 - w / 2)))

    def gauss_sin(X, Y, A=100, w=0.05):  # examples/val_example.py:19-20
        return step(X) * step(Y) * A * np.sin(w * (X + Y))

    X, Y, h, I, hmap, I0, cf = val(0, func=gauss_sin, centrado_si=False)
    err = np.max(np.abs(hmap - h)) * 100 / np.max(np.abs(hmap))
    np.savez_compressed(os.path.join(OUT, "val.npz"), versions=VERSIONS, err_percent=err, cf=cf,
                        height_sub=hmap[::8, ::8].astype(np.float32))
    print("val err %", err, "cf", cf)


def make_ingest():
    """Decoder, mask and folder-loop fixtures (analyze.py:25-40, 42-139, 216-246).

    analyze.py itself cannot be imported here (its module imports cv2, absent), so the
    mask / center steps call the same scikit-image / scipy functions with the same
    arguments as analyze.py:86-100 and :119-137, and the folder loop body is
    load_image -> [mask blend] -> fcd.compute_height_map -> [height *= ~mask] ->
    float32, as analyze.py:216-246."""
    import hashlib
    from scipy.ndimage import uniform_filter
    from skimage.measure import label, regionprops

    out = {"versions": VERSIONS}
    names = sorted(f for f in os.listdir(PICS) if os.path.isfile(os.path.join(PICS, f)))
    mask_dir = os.path.join(PICS, "mask")
    mask_names = sorted(f for f in os.listdir(mask_dir) if f.endswith(".tif"))
    files = [n for n in names] + ["mask/" + n for n in mask_names]
    dec_sha, dec_shape, dec_sum = [], [], []
    for n in files:
        a = io.imread(os.path.join(PICS, n), as_gray=True).astype(np.float32)  # analyze.py:40
        dec_sha.append(hashlib.sha256(a.tobytes()).hexdigest())
        dec_shape.append(a.shape)
        dec_sum.append(float(a.astype(np.float64).sum()))
    out.update(files=np.array(files), dec_sha=np.array(dec_sha), dec_shape=np.array(dec_shape),
               dec_sum=np.array(dec_sum))

    def mask_of(image, smoothed):  # analyze.py:86-94
        smooth = uniform_filter(image, size=smoothed)
        Mask = smooth < np.mean(smooth)
        labels = label(Mask)
        r = sorted(regionprops(labels), key=lambda r: r.area, reverse=True)[0]
        return labels == r.label

    def center_of(mask):  # analyze.py:119-137
        props = regionprops(label(~mask))
        n_rows, n_cols = mask.shape
        holes = [r for r in props if r.bbox[0] > 0 and r.bbox[1] > 0 and r.bbox[2] < n_rows and r.bbox[3] < n_cols]
        cy, cx = max(holes, key=lambda r: r.area).centroid
        return int(cy), int(cx)

    ref = io.imread(os.path.join(PICS, "reference_df.tif"), as_gray=True).astype(np.float32)
    sq = 0.002
    masks, centers, smooths, heights, hsum, hnorm, which = [], [], [], [], [], [], []
    for idx, smoothed in ((4, 15), (5, 14), (8, 15)):
        disp = io.imread(os.path.join(mask_dir, mask_names[idx]), as_gray=True).astype(np.float32)
        m = mask_of(disp, smoothed)
        masks.append(np.packbits(m))
        centers.append(center_of(m))
        smooths.append(smoothed)
        for masked in (False, True):
            img = np.where(m == 1, ref, disp) if masked else disp  # analyze.py:219
            h, _, cf = fcd.compute_height_map(ref, img, sq, LAYERS)  # analyze.py:233-238
            if masked:
                h *= ~m  # analyze.py:241
            h = h.astype(np.float32)  # analyze.py:248
            heights.append(h[::4, ::4])
            hsum.append(float(h.astype(np.float64).sum()))
            hnorm.append(float(np.linalg.norm(h.astype(np.float64))))
            which.append((idx, int(masked)))
    out.update(mask_names=np.array(mask_names), mask_bits=np.stack(masks), mask_centers=np.array(centers),
               mask_smoothed=np.array(smooths), folder_which=np.array(which), folder_h_sub=np.stack(heights),
               folder_h_sum=np.array(hsum), folder_h_norm=np.array(hnorm), folder_sq=sq, folder_cf=cf)
    np.savez_compressed(os.path.join(OUT, "ingest.npz"), **out)
    print("ingest", len(files), "files; centers", centers, "cf", cf)


if __name__ == "__main__":
    which = sys.argv[1:] or ["real_pair", "real_df", "unwrap", "synthetic", "integrate", "val", "ingest"]
    if "real_pair" in which:
        make_real_pair()
    if "real_df" in which:
        make_real_df()
    if "unwrap" in which:
        make_unwrap_crops()
    if "synthetic" in which:
        make_synthetic()
    if "integrate" in which:
        make_integrate()
    if "val" in which:
        make_val()
    if "ingest" in which:
        make_ingest()
