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
  spectrum.npz       sha256 digests of scipy.fft.fft2, np.mean and the find_peaks spectrum
                     |fftshift(fft2(image - mean))| (fourier.py:18) for float32 images of
                     several shapes (the bit-exact restatement in oracle/pocketfft.py and
                     the engine's fcd_fft2 are checked against them)
  bench_board.npz    the benchmarked c2 board (bench_data.py: pattern.py geometry, 1024^2,
                     unrotated and rotated 5 degrees): the reference's find_peaks picks,
                     blobs, cf, radius, and compute_height_map of two warped frames
  large.npz          the c3 / c5 frame sizes (2048^2, 4096^2): per size one residue-free
                     rotated-board frame and one with residues (bump field + edge-dislocation
                     pairs), the reference's carrier picks, heights, wrapped phases and FULL
                     unwrap k-fields (bench_data.make_residue_frame, frame digests stored)
  mixed.npz          frame sides that are not powers of two (1024 x 1280, 1536 x 2048, a
                     960-row camera crop): as large.npz, plus fft2 digests of 5-smooth shapes
  anyshape.npz       frame sides of any size (1080 x 1920, 1000 x 1000, prime / Bluestein
                     sides 1023 x 1021 / 1021 x 1023, a 1000 x 1000 camera crop): as mixed.npz
  shapes.npz         any frame shape and float64 images: fft2 / mean / spectrum digests of
                     hashed integer images (bench_data.hash_image) at odd, prime, Bluestein
                     and camera shapes in float32 and float64, and the reference's carrier
                     picks for float64 references (pyval's tie-prone sine board I0 among them)
  intref.npz         integer-typed references (pattern.py's uint16 board, raw uint8 / uint16
                     example pictures): the reference's complex128 picks, blobs, threshold,
                     cf and fft2 digests, and heights with the uint16 board as reference
  analyze_ref.npz    pydata/analyze.py ITSELF (imported with a placeholder `cv2` module
                     whose every attribute access raises: cv2 is only used on the polar
                     paths, analyze.py:237-241, 674-676, which are not run): analyze.mask /
                     center on camera frames, analyze.folder on a directory of frames
                     (with and without the mask), block_split / block_amplitude /
                     spectrogram on synthetic float32 and float64 map folders
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


def spectrum_images():
    """name -> float32 image: the c2 board flat / rotated (bench_data.py), the two example
    references, and seeded integer-valued images of other shapes (stored in the fixture)."""
    import hashlib  # noqa: F401
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import checkerboard
    rng = np.random.default_rng(2024)
    imgs = {
        "board_flat": checkerboard(1024),
        "board_rot5": checkerboard(1024, 5.0),
        "reference_2": load_raw("reference_2.png").astype(np.float32),
        "reference_df": load_raw("reference_df.tif").astype(np.float32),
    }
    stored = {}
    for (h, w) in ((64, 64), (128, 256), (256, 128), (2048, 64), (64, 4096)):
        u = rng.integers(0, 1024, (h, w)).astype(np.uint16)
        stored[f"rand_{h}x{w}"] = u
        imgs[f"rand_{h}x{w}"] = u.astype(np.float32) * np.float32(0.37)
    return imgs, stored


def make_spectrum():
    import hashlib
    imgs, stored = spectrum_images()
    out = {"versions": VERSIONS, "names": np.array(list(imgs))}
    for name, img in imgs.items():
        F = fft2(img)
        assert F.dtype == np.complex64
        m = np.mean(img)
        spec = np.fft.fftshift(np.abs(fft2(img - m)))  # fourier.py:18
        out[f"{name}_fft2_sha"] = hashlib.sha256(F.tobytes()).hexdigest()
        out[f"{name}_mean"] = np.float32(m)
        out[f"{name}_spec_sha"] = hashlib.sha256(spec.tobytes()).hexdigest()
        out[f"{name}_fft2_corner"] = F[:4, :4]
    for k, v in stored.items():
        out[k + "_u16"] = v
    np.savez_compressed(os.path.join(OUT, "spectrum.npz"), **out)
    print("spectrum", list(imgs))


def make_bench_board():
    """Carrier picks of the reference on the exact board bench.py runs (configs[1]):
    bench_data.checkerboard(1024) (pattern.py geometry, pattern.py:17-36), and the same
    board rotated 5 degrees (SURVEY.md §8a parity fact 2)."""
    import hashlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))  # the repo root: bench_data.py (numpy only)
    from bench_data import make_frames_numpy
    out = {"versions": VERSIONS}
    for tag, rot in (("flat", 0.0), ("rot5", 5.0)):
        ref, frames = make_frames_numpy(1024, 2, seed=0, rotate_deg=rot)
        sq = 0.001
        locs, thr = peak_locations(ref)
        image_fft = np.fft.fftshift(np.abs(fft2(ref - np.mean(ref))))
        out[f"{tag}_blob_values"] = np.array([image_fft[p[0], p[1]] for p in locs], np.float32)
        out[f"{tag}_blob_peaks"] = locs
        out[f"{tag}_threshold"] = thr
        out[f"{tag}_ref_sha"] = hashlib.sha256(ref.tobytes()).hexdigest()
        out[f"{tag}_frames_sha"] = hashlib.sha256(frames.tobytes()).hexdigest()
        for f in range(2):
            r = run_pair(ref, frames[f], sq, height=1.0)
            out[f"{tag}_height_sub{f}"] = r["height"][::4, ::4].astype(np.float32)
            out[f"{tag}_height_stats{f}"] = stats(r["height"])
            out[f"{tag}_wrapped_sub{f}"] = r["wrapped"][:, ::8, ::8]
        for key in ("peaks", "cf", "radius", "freqs", "mask_count"):
            out[f"{tag}_{key}"] = r[key]
        print("bench_board", tag, r["peaks"].tolist(), locs.tolist(), out[f"{tag}_blob_values"].tolist(), r["cf"])
    np.savez_compressed(os.path.join(OUT, "bench_board.npz"), **out)


# The c3 / c5 frame sizes (BASELINE configs[2], [4]): one residue-free rotated-board frame
# (bench_data.make_frames_numpy) and one frame with residues (bump field + edge-dislocation
# pairs, bench_data.make_residue_frame) per size, each through the reference's
# compute_height_map with its skimage unwrap (fcd.py:13-35, 119).
LARGE_CASES = {
    "s2048": dict(n=2048, seed=11, pairs=[]),
    "r2048": dict(n=2048, seed=21, pairs=[(487.0, 870.4), (1300.3, 1200.7), (1700.6, 400.2)]),
    "s4096": dict(n=4096, seed=2, pairs=[]),
    "r4096": dict(n=4096, seed=23, pairs=[(607.0, 870.4), (2500.3, 3000.1), (3300.6, 1500.2)]),
}


def large_case_frames(spec):
    """(ref, frame) of a LARGE_CASES entry: bench_data.make_residue_frame with the
    displacement rounded to 1/4096 px, so the frame bytes do not depend on the numpy
    build (tests regenerate it and check the digest)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))  # the repo root: bench_data.py (numpy only)
    from bench_data import make_residue_frame
    return make_residue_frame(spec["n"], spec["pairs"], seed=spec["seed"], rotate_deg=5.0, quantum=4096)


def residue_count(w):
    w = np.asarray(w, np.float64)
    wr = lambda d: (d + np.pi) % (2 * np.pi) - np.pi  # noqa: E731
    c = (wr(w[:-1, 1:] - w[:-1, :-1]) + wr(w[1:, 1:] - w[:-1, 1:]) + wr(w[1:, :-1] - w[1:, 1:])
         + wr(w[:-1, :-1] - w[1:, :-1]))
    return int((np.abs(c) > 1).sum())


def make_large():
    """large.npz: per case the frame digests, the reference's carrier picks, its height on a
    256^2 sub-grid (+ sum / norm / max over the full map), wrapped phases on a 128^2
    sub-grid, and the FULL unwrap k-fields of both maps (int8, exact up to one global
    integer per map; they compress to runs), plus the residue count per map."""
    import hashlib
    out = {"versions": VERSIONS, "cases": np.array(list(LARGE_CASES))}
    for tag, spec in LARGE_CASES.items():
        n = spec["n"]
        ref, frame = large_case_frames(spec)
        sq = 0.001
        r = run_pair(ref, frame, sq, height=1.0)
        locs, thr = peak_locations(ref)
        k = np.stack([kfield(w, p) for w, p in zip(r["wrapped"], r["phases"])])
        assert np.abs(k).max() < 127
        out.update({
            f"{tag}_n": n, f"{tag}_seed": spec["seed"], f"{tag}_pairs": np.array(spec["pairs"], np.float64).reshape(-1, 2),
            f"{tag}_ref_sha": hashlib.sha256(ref.tobytes()).hexdigest(),
            f"{tag}_frame_sha": hashlib.sha256(frame.tobytes()).hexdigest(),
            f"{tag}_peaks": r["peaks"], f"{tag}_cf": r["cf"], f"{tag}_radius": r["radius"],
            f"{tag}_freqs": r["freqs"], f"{tag}_mask_count": r["mask_count"],
            f"{tag}_blob_peaks": locs, f"{tag}_threshold": thr,
            f"{tag}_height_sub": r["height"][::n // 256, ::n // 256].astype(np.float32),
            f"{tag}_height_stats": stats(r["height"]),
            f"{tag}_wrapped_sub": r["wrapped"][:, ::n // 128, ::n // 128],
            f"{tag}_k": k.astype(np.int8),
            f"{tag}_residues": np.array([residue_count(w) for w in r["wrapped"]]),
        })
        print("large", tag, r["peaks"].tolist(), r["cf"], "residues", out[f"{tag}_residues"].tolist(),
              "k range", int(k.min()), int(k.max()), flush=True)
    np.savez_compressed(os.path.join(OUT, "large.npz"), **out)


# Frame sides that are not powers of two (the engine's mixed-radix generic chain): camera
# formats 1280 x 1024 (here 1024 rows x 1280 columns) and 2048 x 1536, a residue frame, and
# a 960-row crop of the 10-bit camera pair (real_df.npz's reference and frame 0, rows
# 32..991: every map carries residues).
MIXED_CASES = {
    "s1024x1280": dict(rows=1024, cols=1280, seed=31, pairs=[]),
    "r1024x1280": dict(rows=1024, cols=1280, seed=32, pairs=[(300.3, 500.4), (700.6, 900.2)]),
    "s1536x2048": dict(rows=1536, cols=2048, seed=33, pairs=[]),
    "c960x1024": dict(crop=(32, 992)),
}


def mixed_case_frames(spec):
    if "crop" in spec:
        r0, r1 = spec["crop"]
        ref = load_raw("reference_df.tif").astype(np.float32)[r0:r1]
        frame = load_raw("prueba1_20250317_122608_C1S0001000001.tif").astype(np.float32)[r0:r1]
        return np.ascontiguousarray(ref), np.ascontiguousarray(frame), 0.002
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import make_residue_frame
    ref, frame = make_residue_frame(spec["rows"], spec["pairs"], seed=spec["seed"], rotate_deg=5.0, quantum=4096,
                                    cols=spec["cols"])
    return ref, frame, 0.001


# Frame sides of any size (the generic chain with its radix-7 / generic odd-prime passes,
# Bluestein sides and frames padded to multiples of 64 for the unwrap): the HD camera format
# 1080 x 1920, 1000 x 1000 with residues, prime / Bluestein sides 1023 x 1021 and
# 1021 x 1023 (with residues), and a 1000 x 1000 crop of the 10-bit camera pair.
ANY_CASES = {
    "s1080x1920": dict(rows=1080, cols=1920, seed=41, pairs=[]),
    "r1000x1000": dict(rows=1000, cols=1000, seed=42, pairs=[(300.3, 400.6), (650.2, 700.7)]),
    "s1023x1021": dict(rows=1023, cols=1021, seed=43, pairs=[]),
    "r1021x1023": dict(rows=1021, cols=1023, seed=44, pairs=[(410.3, 520.4)]),
    "c1000x1000": dict(crop=(12, 1012), ccrop=(20, 1020)),
}


def mixed_case_frames_any(spec):
    if "ccrop" in spec:
        (r0, r1), (c0, c1) = spec["crop"], spec["ccrop"]
        ref = load_raw("reference_df.tif").astype(np.float32)[r0:r1, c0:c1]
        frame = load_raw("prueba1_20250317_122608_C1S0001000001.tif").astype(np.float32)[r0:r1, c0:c1]
        return np.ascontiguousarray(ref), np.ascontiguousarray(frame), 0.002
    return mixed_case_frames(spec)


def make_mixed(cases=None, name="mixed"):
    """mixed.npz: as large.npz for MIXED_CASES (heights on a ~256-wide sub-grid, wrapped
    phases on a ~128-wide one, the full k-fields), plus sha256 digests of scipy's fft2 of
    each reference and of seeded integer-valued images of other 5-smooth shapes (the
    restated radix-3 / radix-5 pocketfft passes).  anyshape.npz: the same for ANY_CASES."""
    import hashlib
    cases = MIXED_CASES if cases is None else cases
    out = {"versions": VERSIONS, "cases": np.array(list(cases))}
    for tag, spec in cases.items():
        ref, frame, sq = mixed_case_frames_any(spec)
        rows, cols = ref.shape
        r = run_pair(ref, frame, sq, height=1.0)
        locs, thr = peak_locations(ref)
        k = np.stack([kfield(w, p) for w, p in zip(r["wrapped"], r["phases"])])
        assert np.abs(k).max() < 127
        hs, ws = max(1, cols // 256), max(1, cols // 128)
        out.update({
            f"{tag}_shape": np.array([rows, cols]), f"{tag}_sq": sq,
            f"{tag}_seed": spec.get("seed", -1),
            f"{tag}_pairs": np.array(spec.get("pairs", []), np.float64).reshape(-1, 2),
            f"{tag}_ref_sha": hashlib.sha256(ref.tobytes()).hexdigest(),
            f"{tag}_frame_sha": hashlib.sha256(frame.tobytes()).hexdigest(),
            f"{tag}_ref_fft2_sha": hashlib.sha256(fft2(ref).tobytes()).hexdigest(),
            f"{tag}_peaks": r["peaks"], f"{tag}_cf": r["cf"], f"{tag}_radius": r["radius"],
            f"{tag}_freqs": r["freqs"], f"{tag}_mask_count": r["mask_count"],
            f"{tag}_blob_peaks": locs, f"{tag}_threshold": thr,
            f"{tag}_height_step": hs, f"{tag}_wrapped_step": ws,
            f"{tag}_height_sub": r["height"][::hs, ::hs].astype(np.float32),
            f"{tag}_height_stats": stats(r["height"]),
            f"{tag}_wrapped_sub": r["wrapped"][:, ::ws, ::ws],
            f"{tag}_k": k.astype(np.int8),
            f"{tag}_residues": np.array([residue_count(w) for w in r["wrapped"]]),
        })
        print("mixed", tag, ref.shape, r["peaks"].tolist(), r["cf"], "residues", out[f"{tag}_residues"].tolist(),
              flush=True)
    if name != "mixed":
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
        return
    rng = np.random.default_rng(4242)
    shapes = [(192, 320), (320, 192), (576, 960), (128, 384)]
    for (h, w) in shapes:
        u = rng.integers(0, 1024, (h, w)).astype(np.uint16)
        img = u.astype(np.float32) * np.float32(0.37)
        out[f"rand_{h}x{w}_u16"] = u
        out[f"rand_{h}x{w}_fft2_sha"] = hashlib.sha256(fft2(img).tobytes()).hexdigest()
        out[f"rand_{h}x{w}_mean"] = np.float32(np.mean(img))
        out[f"rand_{h}x{w}_spec_sha"] = hashlib.sha256(np.fft.fftshift(np.abs(fft2(img - np.mean(img)))).tobytes()).hexdigest()
    out["rand_shapes"] = np.array(shapes)
    np.savez_compressed(os.path.join(OUT, "mixed.npz"), **out)


# Frame shapes for the exact reference spectrum (scipy's fft2 in the image's precision):
# powers of two, 5-smooth, 7 / 11 / larger primes (rfftp radfg, cfftp pass7 / pass11 /
# passg), Bluestein sides (1021, 4099, 257 ...), odd sides and camera formats.
SHAPES_FFT = [(64, 64), (63, 64), (64, 63), (93, 186), (100, 75), (189, 256), (257, 251), (343, 121), (17, 2),
              (1, 64), (1023, 1021), (1021, 1023), (1080, 1920), (1000, 1000), (600, 2448), (4099, 40), (50, 4097)]
# float64 references (the reference computes find_peaks' spectrum in complex128 for them,
# fourier.py:18; pyval/val.py:98 hands compute_height_map a float64 I0): pyval's own
# unrotated sine board (tie-prone: its four blobs tie in exact arithmetic), the pattern.py
# board as float64, and sine boards of other shapes.
F64_REFS = {
    "val1024": dict(kind="sine", rows=1024, cols=1024, n=60),
    "val512": dict(kind="sine", rows=512, cols=512, n=30),
    "val600x800": dict(kind="sine", rows=600, cols=800, n=37, n_cols=49),
    "val1021x1023": dict(kind="sine", rows=1021, cols=1023, n=57, n_cols=61),
    "flat1024": dict(kind="board", rows=1024, rot=0.0),
    "rot768x1280": dict(kind="board", rows=768, cols=1280, rot=5.0),
}


def f64_reference(spec):
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import checkerboard, sine_board
    if spec["kind"] == "sine":
        img, sx, sy = sine_board(spec["rows"], spec["cols"], spec["n"], spec.get("n_cols"))
        return img, {"sx": sx, "sy": sy}
    return checkerboard(spec["rows"], spec["rot"], cols=spec.get("cols")).astype(np.float64), {}


def make_shapes():
    """shapes.npz: digests of scipy's fft2, np.mean and the find_peaks spectrum for hashed
    integer images (bench_data.hash_image) of SHAPES_FFT in float32 and float64, and the
    reference's carrier picks (find_peaks, compute_calibration_factor) for the float64
    references of F64_REFS."""
    import hashlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import hash_image
    out = {"versions": VERSIONS, "fft_shapes": np.array(SHAPES_FFT), "f64_refs": np.array(list(F64_REFS))}
    for k, (h, w) in enumerate(SHAPES_FFT):
        u = hash_image(h, w, seed=k)
        out[f"{h}x{w}_u16_sha"] = hashlib.sha256(u.tobytes()).hexdigest()
        for T, tag in ((np.float32, "f32"), (np.float64, "f64")):
            img = u.astype(T) * T(0.37)
            F = fft2(img)
            assert F.dtype == (np.complex64 if T == np.float32 else np.complex128)
            m = np.mean(img)
            out[f"{h}x{w}_{tag}_fft2_sha"] = hashlib.sha256(F.tobytes()).hexdigest()
            out[f"{h}x{w}_{tag}_mean"] = np.asarray(m, T)
            out[f"{h}x{w}_{tag}_spec_sha"] = hashlib.sha256(np.fft.fftshift(np.abs(fft2(img - m))).tobytes()).hexdigest()
    for tag, spec in F64_REFS.items():
        img, tables = f64_reference(spec)
        assert img.dtype == np.float64
        sq = 0.001
        cf, (p0, p1) = fcd.compute_calibration_factor(sq, img)
        locs, thr = peak_locations(img)
        out[f"{tag}_sha"] = hashlib.sha256(img.tobytes()).hexdigest()
        out[f"{tag}_peaks"] = np.array([np.asarray(p0), np.asarray(p1)], np.int64)
        out[f"{tag}_cf"] = cf
        out[f"{tag}_blob_peaks"] = locs
        out[f"{tag}_threshold"] = thr
        # the picks of the same image rounded to float32 (what an engine demodulating the
        # float32 rounding would have picked)
        c32, (q0, q1) = fcd.compute_calibration_factor(sq, img.astype(np.float32))
        out[f"{tag}_peaks_f32"] = np.array([np.asarray(q0), np.asarray(q1)], np.int64)
        for k, v in tables.items():
            out[f"{tag}_{k}"] = v
        print("shapes f64 ref", tag, img.shape, out[f"{tag}_peaks"].tolist(), "f32 picks", out[f"{tag}_peaks_f32"].tolist(),
              locs.tolist(), thr, flush=True)
    np.savez_compressed(os.path.join(OUT, "shapes.npz"), **out)


# Integer-typed references: scipy's fft2 promotes every non-float
# image to float64 (scipy/fft/_pocketfft/helper.py:91-92) and `image - np.mean(image)` of
# an integer image is float64, so the reference picks carriers from a complex128 spectrum
# for them (fourier.py:18).  pattern.py:17-36 writes its board as uint16; the example
# pictures decode to uint8 / uint16 before analyze.load_image's float32 cast.
INT_REFS = {
    "board_u16": dict(kind="board", rows=1024, rot=0.0, dtype="uint16"),
    "board_rot5_u16": dict(kind="board", rows=1024, rot=5.0, dtype="uint16"),
    "board_i32": dict(kind="board", rows=512, rot=0.0, dtype="int32"),
    "ref2_u8": dict(kind="picture", name="reference_2.png"),
    "refdf_u16": dict(kind="picture", name="reference_df.tif"),
}


def int_reference(spec):
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import checkerboard
    if spec["kind"] == "picture":
        return load_raw(spec["name"])
    return checkerboard(spec["rows"], spec["rot"], dtype=np.dtype(spec["dtype"]))


def make_intref():
    """intref.npz: find_peaks / compute_calibration_factor of integer-typed references as
    the reference computes them (complex128 spectrum), the picks of the same images as
    float32 (what a float32 engine would pick), scipy's fft2 digest of each integer image,
    and compute_height_map heights with the uint16 board as the reference."""
    import hashlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from bench_data import make_frames_numpy
    out = {"versions": VERSIONS, "tags": np.array(list(INT_REFS))}
    for tag, spec in INT_REFS.items():
        img = int_reference(spec)
        assert img.dtype.kind in "iu", (tag, img.dtype)
        sq = 0.001
        cf, (p0, p1) = fcd.compute_calibration_factor(sq, img)
        locs, thr = peak_locations(img)
        F = fft2(img)
        assert F.dtype == np.complex128
        out[f"{tag}_dtype"] = str(img.dtype)
        out[f"{tag}_sha"] = hashlib.sha256(img.tobytes()).hexdigest()
        out[f"{tag}_fft2_sha"] = hashlib.sha256(F.tobytes()).hexdigest()
        out[f"{tag}_peaks"] = np.array([np.asarray(p0), np.asarray(p1)], np.int64)
        out[f"{tag}_cf"] = cf
        out[f"{tag}_blob_peaks"] = locs
        out[f"{tag}_threshold"] = thr
        c32, (q0, q1) = fcd.compute_calibration_factor(sq, img.astype(np.float32))
        out[f"{tag}_peaks_f32"] = np.array([np.asarray(q0), np.asarray(q1)], np.int64)
        print("intref", tag, img.dtype, img.shape, out[f"{tag}_peaks"].tolist(), "f32 picks",
              out[f"{tag}_peaks_f32"].tolist(), locs.tolist(), thr, cf, flush=True)
    # the uint16 board as the reference of compute_height_map (fcd.py:13-35): carriers from
    # the complex128 spectrum, displaced frames as float32 (analyze.load_image's type)
    ref = int_reference(INT_REFS["board_u16"])
    _, frames = make_frames_numpy(1024, 2, seed=0, rotate_deg=0.0)
    out["board_u16_frames_sha"] = hashlib.sha256(frames.tobytes()).hexdigest()
    for f in range(2):
        hmap, phases, cf = fcd.compute_height_map(ref, frames[f], 0.001, height=1.0)
        out[f"board_u16_height_sub{f}"] = hmap[::4, ::4].astype(np.float32)
        out[f"board_u16_height_stats{f}"] = stats(hmap)
        out[f"board_u16_hcf{f}"] = cf
    np.savez_compressed(os.path.join(OUT, "intref.npz"), **out)


def import_reference_analyze():
    """/root/reference/pydata/analyze.py, imported as the reference ships it.  Its module
    top level does `import cv2` (analyze.py:21), absent here; cv2 is used only by the
    polar paths (analyze.py:237-241, 674-676), which no fixture runs.  A placeholder
    module stands in for the import and raises on any attribute access, so a fixture that
    reached cv2 would fail instead of silently using a stand-in."""
    import types

    class _NoCv2(types.ModuleType):
        def __getattr__(self, name):
            raise RuntimeError(f"cv2.{name} used: the fixture reached a cv2 path of analyze.py")

    sys.modules.setdefault("cv2", _NoCv2("cv2"))
    import matplotlib
    matplotlib.use("Agg")
    from pydata.analyze import analyze  # reference, read-only
    return analyze


def synthetic_maps(T, n, dtype, seed):
    """A map stack like analyze.folder's output: a standing oscillation at 5.2 Hz (500 Hz
    sampling, block_amplitude's default `tasa`) and its second harmonic, plus noise;
    some pixels are exactly 0 in the first map (the reference NaN-masks those)."""
    rng = np.random.default_rng(seed)
    t = np.arange(T) / 500.0
    y, x = np.mgrid[0:n, 0:n] / n
    a1 = 1e-3 * (1 + np.sin(2 * np.pi * x) * np.cos(np.pi * y))
    a2 = 2e-4 * np.cos(3 * np.pi * x * y)
    ph = 2 * np.pi * (x + 0.5 * y)
    st = (a1[None] * np.cos(2 * np.pi * 5.2 * t[:, None, None] + ph[None])
          + a2[None] * np.cos(2 * np.pi * 10.4 * t[:, None, None] - ph[None])
          + 5e-5 * rng.standard_normal((T, n, n)))
    st = st.astype(dtype)
    holes = rng.random((n, n)) < 0.03
    st[0][holes] = 0
    return st


def make_analyze_ref():
    import shutil
    import tempfile
    analyze = import_reference_analyze()
    out = {"versions": VERSIONS}
    mask_dir = os.path.join(PICS, "mask")
    mask_names = sorted(f for f in os.listdir(mask_dir) if f.endswith(".tif"))
    # analyze.mask / center (analyze.py:43-140): full camera frames 4 and 5 (frame 4 is
    # real_df.npz's frame 1; frame 5 is stored here), and 512^2 crops around the floater of
    # frames 2, 5, 8 (stored), each with its own smoothing size
    crop = (slice(150, 662), slice(380, 892))
    out["frame5_u16"] = load_raw("mask/" + mask_names[5])
    cases = [("full", 4, 15), ("full", 5, 14), ("crop", 2, 20), ("crop", 5, 15), ("crop", 8, 15)]
    crops, mbits, cents = {}, [], []
    for kind, idx, smoothed in cases:
        raw = load_raw("mask/" + mask_names[idx])
        if kind == "crop":
            raw = np.ascontiguousarray(raw[crop])
            crops[idx] = raw
        m, c = analyze.mask(raw.astype(np.float32), smoothed=smoothed, find_center=True)
        mbits.append(np.packbits(m))
        cents.append(c)
    out.update(mask_names=np.array(mask_names), mask_cases=np.array([(k, i, s) for k, i, s in cases]),
               mask_bits=np.concatenate(mbits),
               mask_bits_len=np.array([len(b) for b in mbits]), mask_centers=np.array(cents),
               crop_rows=np.array([crop[0].start, crop[0].stop]), crop_cols=np.array([crop[1].start, crop[1].stop]))
    for idx, raw in crops.items():
        out[f"crop{idx}_u16"] = raw
    # analyze.folder (analyze.py:143-286): real_df.npz's three frames plain, frames 4 + 5 masked
    tmp = tempfile.mkdtemp(prefix="fcd_golden_")
    try:
        refp = os.path.join(PICS, "reference_df.tif")
        runs = (("plain", None, ["prueba1_20250317_122608_C1S0001000001.tif", "mask/" + mask_names[4], "ellipse_10.tif"]),
                ("masked", 15, ["mask/" + mask_names[4], "mask/" + mask_names[5]]))
        for tag, smoothed, frames in runs:
            ddir = os.path.join(tmp, "frames_" + tag)
            os.makedirs(ddir)
            for f in frames:
                shutil.copy(os.path.join(PICS, f), os.path.join(ddir, os.path.basename(f)))
            analyze.folder(refp, ddir, LAYERS, 0.002, smoothed=smoothed)
            mdir = os.path.join(ddir, "maps")
            names = sorted(f for f in os.listdir(mdir) if f.endswith("_map.npy"))
            maps = [np.load(os.path.join(mdir, f)) for f in names]
            out[f"folder_{tag}_frames"] = np.array([os.path.basename(f) for f in frames])
            out[f"folder_{tag}_names"] = np.array(names)
            out[f"folder_{tag}_h_sub"] = np.stack([m[::4, ::4] for m in maps])
            out[f"folder_{tag}_h_stats"] = np.stack([stats(m) for m in maps])
            out[f"folder_{tag}_zero_count"] = np.array([int((m == 0).sum()) for m in maps])
            out[f"folder_{tag}_cf"] = np.load(os.path.join(mdir, "calibration_factor.npy"))
            cp = os.path.join(mdir, "centers.txt")
            out[f"folder_{tag}_centers_txt"] = open(cp).read() if os.path.exists(cp) else ""
        # temporal post-analysis (analyze.py:365-641) on synthetic map folders
        for dt in ("float32", "float64"):
            T, n = (240, 32) if dt == "float32" else (150, 32)
            st = synthetic_maps(T, n, np.dtype(dt), seed=11 if dt == "float32" else 12)
            mdir = os.path.join(tmp, "maps_" + dt)
            os.makedirs(mdir)
            for t in range(T):
                np.save(os.path.join(mdir, f"f{t:05d}_map.npy"), st[t])
            np.save(os.path.join(mdir, "calibration_factor.npy"), np.array([0.001]))
            out[f"{dt}_stack"] = st
            bs = analyze.block_split(mdir, t_limit=T - 7, num_blocks=4, block_index=1)
            out[f"{dt}_split"] = bs
            for k, (mode, blk, zero) in enumerate(((3, 0, 0), (2, 3, 0), (1, 2, 1e-4))):
                res = analyze.block_amplitude(mdir, mode=mode, num_blocks=4, block_index=blk, zero=zero)
                harm, amps, phases, f0 = res
                out[f"{dt}_amp{k}_args"] = np.array([mode, blk, zero])
                out[f"{dt}_amp{k}_harm"] = np.array(harm, np.float64)
                out[f"{dt}_amp{k}_amps"] = amps
                out[f"{dt}_amp{k}_phases"] = phases
                out[f"{dt}_amp{k}_f0"] = f0
            f0_given = 5.0
            harm, amps, phases, f0 = analyze.block_amplitude(mdir, f0=f0_given, mode=2, num_blocks=16, block_index=5)
            out[f"{dt}_ampf_harm"] = np.array(harm, np.float64)
            out[f"{dt}_ampf_amps"] = amps
            out[f"{dt}_ampf_phases"] = phases
            t_, f_, S_all, S_avg = analyze.spectrogram(map_folder=mdir, fs=125, nperseg=64, noverlap=32,
                                                      num_blocks=4, block_index=0)
            out[f"{dt}_spec_t"], out[f"{dt}_spec_f"] = t_, f_
            out[f"{dt}_spec_all"], out[f"{dt}_spec_avg"] = S_all, S_avg
            t_, f_, S = analyze.spectrogram(array=st[:, 5, 7], fs=125, nperseg=50, noverlap=10)
            out[f"{dt}_spec1_t"], out[f"{dt}_spec1_f"], out[f"{dt}_spec1"] = t_, f_, S
            print("analyze temporal", dt, [out[f"{dt}_amp{k}_f0"] for k in range(3)], S_all.shape)
    finally:
        shutil.rmtree(tmp)
    np.savez_compressed(os.path.join(OUT, "analyze_ref.npz"), **out)
    print("analyze_ref: centers", cents, "folder centers", repr(out["folder_masked_centers_txt"]))


if __name__ == "__main__":
    which = sys.argv[1:] or ["real_pair", "real_df", "unwrap", "synthetic", "integrate", "val", "ingest",
                             "bench_board", "analyze_ref", "spectrum", "large", "mixed", "shapes", "anyshape", "intref"]
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
    if "bench_board" in which:
        make_bench_board()
    if "analyze_ref" in which:
        make_analyze_ref()
    if "spectrum" in which:
        make_spectrum()
    if "large" in which:
        make_large()
    if "mixed" in which:
        make_mixed()
    if "shapes" in which:
        make_shapes()
    if "anyshape" in which:
        make_mixed(ANY_CASES, "anyshape")
    if "intref" in which:
        make_intref()
