"""GPU checks of frame ingest and the batch driver:

* fcd_process_raw on 8-bit, 16-bit and 10-bit-packed samples gives bit-identical
  heights to fcd_process on the same samples widened to float32 on the host, through
  every host path (pageable staging, page-locked buffers, the multi-chunk pipeline)
  and with device pointers;
* analyze.folder (the reference's analyze.py:142-286 contract) on 10-bit camera TIFFs
  written from the golden frames: maps equal the reference's compute_height_map
  outputs (real_df.npz), calibration_factor.npy equals the committed file's value, the
  mask path equals the reference's masked loop body (ingest.npz), resume skips done
  frames;
* the examples/fcd_example.py chain (PNG / BMP through analyze.load_image) against the
  real-pair golden.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LAYERS = [[5.7e-2, 1.0003], [1.2e-2, 1.48899], [4.3e-2, 1.34], [80e-2, 1.0003]]  # fcd_example.py:17


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.fixture(scope="module")
def df(golden):
    return golden("real_df")


@pytest.fixture
def fresh_engines():
    from pyfcd import _lib
    _lib._engines.clear()
    yield
    _lib._engines.clear()


def _engine(ref, sq):
    from pyfcd import _lib
    eng = _lib.Engine(ref.shape)
    eng.set_reference(ref, sq)
    return eng


@pytest.mark.parametrize("fmt_name", ["U8", "U16", "P10"])
def test_raw_formats_equal_float32(df, fmt_name):
    from pyfcd import _lib
    from pydata import images
    fmt = getattr(_lib, "FCD_FMT_" + fmt_name)
    ref = df["ref_u16"].astype(np.float32)
    samples = df["frames_u16"]
    if fmt_name == "U8":
        samples = (samples >> 2).astype(np.uint8)
        raw = samples.reshape(len(samples), -1)
    elif fmt_name == "U16":
        raw = samples.view(np.uint8).reshape(len(samples), -1)
    else:
        raw = np.stack([images.pack10(s) for s in samples])
    eng = _engine(ref, float(df["square_size"]))
    assert raw.shape[1] == eng.frame_bytes(fmt)
    want, _, _ = eng.process(samples.astype(np.float32), 1.0, unwrap=True, want_phases=False)
    got = eng.process_raw(raw, fmt, len(samples), 1.0)
    assert np.array_equal(got, want)
    # page-locked input and output buffers (DMA straight from / to the caller's pages)
    pin_in = _lib.PinnedBuffer(raw.shape, np.uint8)
    pin_out = _lib.PinnedBuffer((len(samples),) + ref.shape, np.float32)
    pin_in.array[:] = raw
    eng.process_raw(pin_in.array, fmt, len(samples), 1.0, out=pin_out.array)
    assert np.array_equal(pin_out.array, want)
    pin_in.free()
    pin_out.free()


def test_host_pipeline_many_chunks(monkeypatch, fresh_engines):
    """More frames than one pipeline slot (FCD_PIPE_MB=1 -> 1 frame per slot at 512^2):
    every chunk boundary of the two-slot, three-stream pipeline, against the
    device-pointer path on the same frames (bit-identical)."""
    import torch
    from pyfcd import _lib
    from bench_data import make_frames_numpy
    monkeypatch.setenv("FCD_PIPE_MB", "1")
    ref, frames = make_frames_numpy(512, 7, seed=4, rotate_deg=5.0)
    eng = _engine(ref, 0.001)
    got, _, _ = eng.process(frames, 1.0, unwrap=True, want_phases=False)
    u16 = np.clip(frames / frames.max() * 1023, 0, 1023).astype(np.uint16)
    raw = np.stack([__import__("pydata.images", fromlist=["pack10"]).pack10(f) for f in u16])
    got10 = eng.process_raw(raw, _lib.FCD_FMT_P10, len(u16), 1.0)
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(frames).to(dev)
    hd = torch.empty_like(fd)
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(got, hd.cpu().numpy())
    fd = torch.from_numpy(u16.astype(np.float32)).to(dev)
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(got10, hd.cpu().numpy())


def test_device_raw_pointer_path(df):
    import ctypes
    import torch
    from pyfcd import _lib
    from pydata import images
    ref = df["ref_u16"].astype(np.float32)
    eng = _engine(ref, float(df["square_size"]))
    raw = np.stack([images.pack10(s) for s in df["frames_u16"]])
    want, _, _ = eng.process(df["frames_u16"].astype(np.float32), 1.0, unwrap=True, want_phases=False)
    dev = torch.device("cuda", 0)
    rd = torch.from_numpy(raw).to(dev)
    hd = torch.empty((len(raw),) + ref.shape, dtype=torch.float32, device=dev)
    lib = _lib.load_library()
    _lib._check(lib.fcd_process_raw(eng.handle, ctypes.c_void_p(rd.data_ptr()), _lib.FCD_FMT_P10, len(raw),
                                    _lib.FCD_DEVICE_PTRS, 1.0, 1, ctypes.c_void_p(hd.data_ptr()), None, None, None))
    lib.fcd_synchronize(eng.handle)
    torch.cuda.synchronize()
    assert np.array_equal(hd.cpu().numpy(), want)


def _write_folder(tmp_path, df, idx=None):
    from pydata import images
    d = tmp_path / "frames"
    d.mkdir()
    ref_path = str(d / "reference_df.tif")
    images.write_tiff(ref_path, df["ref_u16"], bits=10)
    names = [os.path.basename(str(n)) for n in df["names"]]
    for i, (n, f) in enumerate(zip(names, df["frames_u16"])):
        if idx is None or i in idx:
            images.write_tiff(str(d / n), f, bits=10)
    return ref_path, str(d), names


def test_folder_matches_reference_maps(tmp_path, df, fresh_engines):
    from pydata.analyze import analyze
    ref_path, d, names = _write_folder(tmp_path, df)
    analyze.folder(ref_path, d, LAYERS, float(df["square_size"]), batch=2)
    maps = os.path.join(d, "maps")
    assert np.load(os.path.join(maps, "calibration_factor.npy")).tolist() == df["committed_cf"].tolist()
    order = sorted(range(3), key=lambda i: names[i])
    for i in order:
        h = np.load(os.path.join(maps, names[i].replace(".tif", "") + "_map.npy"))
        assert h.dtype == np.float32 and h.shape == (1024, 1024)
        # maps with 7..1611 residues; the reference seeds border reliabilities from rand()
        assert rel_l2(h[::4, ::4], df["height_sub"][i]) < 1e-4, names[i]
    # resume: nothing to do when every map exists; the last one is redone when removed
    last = os.path.join(maps, sorted(names)[-1].replace(".tif", "") + "_map.npy")
    before = np.load(last)
    os.remove(last)
    t0 = {n: os.path.getmtime(os.path.join(maps, n)) for n in os.listdir(maps) if n.endswith("_map.npy")}
    analyze.folder(ref_path, d, LAYERS, float(df["square_size"]))
    assert np.array_equal(np.load(last), before)
    assert all(os.path.getmtime(os.path.join(maps, n)) == t for n, t in t0.items())


def test_folder_mask_path_matches_reference(tmp_path, df, golden, fresh_engines):
    """The camera frame mask/*0005.tif (real_df frame 1 = ingest fixture's mask frame 4),
    smoothed=15: mask blend + height *= ~mask + centers.txt, against the reference's
    loop body outputs."""
    from pydata.analyze import analyze
    g = golden("ingest")
    assert str(g["mask_names"][4]).endswith("0005.tif") and os.path.basename(str(df["names"][1])) == str(
        g["mask_names"][4])
    ref_path, d, names = _write_folder(tmp_path, df, idx={1})
    analyze.folder(ref_path, d, LAYERS, float(g["folder_sq"]), smoothed=int(g["mask_smoothed"][0]))
    maps = os.path.join(d, "maps")
    h = np.load(os.path.join(maps, names[1].replace(".tif", "") + "_map.npy"))
    k = [tuple(w) for w in g["folder_which"].tolist()].index((4, 1))
    assert rel_l2(h[::4, ::4], g["folder_h_sub"][k]) < 1e-4
    want_mask = np.unpackbits(g["mask_bits"][0])[: h.size].reshape(h.shape).astype(bool)
    assert np.all(h[want_mask] == 0)
    lines = open(os.path.join(maps, "centers.txt")).read().splitlines()
    assert lines == [f"0\t{tuple(int(v) for v in g['mask_centers'][0])}"]


def test_fcd_example_chain_png_bmp(tmp_path, golden, fresh_engines):
    """examples/fcd_example.py:10-23 with our pydata/pyfcd: PNG reference + BMP frame."""
    from PIL import Image
    from pydata.analyze import analyze
    from pyfcd.fcd import fcd
    r = golden("real_pair")
    Image.fromarray(r["ref_u8"]).save(str(tmp_path / "reference_2.png"))
    Image.fromarray(r["disp_u8"]).save(str(tmp_path / "frame.bmp"))
    reference = analyze.load_image(str(tmp_path / "reference_2.png"))
    displaced = analyze.load_image(str(tmp_path / "frame.bmp"))
    assert np.array_equal(reference, r["ref_u8"].astype(np.float32))
    values = fcd.compute_height_map(reference, displaced, float(r["square_size"]), LAYERS)
    assert values[2] == float(r["cf"])
    assert rel_l2(values[0][::4, ::4], r["height_sub"]) < 1e-4


def test_host_pipeline_follows_reference_change(df):
    """The pipelined host path sizes its slots from the CURRENT reference's chunk
    workspace: switching references between calls (different carrier bands, different
    chunk sizes) keeps the host-path heights equal to the synchronous path's."""
    from bench_data import make_frames_numpy
    from pyfcd import _lib
    ref_s, frames = make_frames_numpy(1024, 5, seed=21, rotate_deg=5.0)
    eng = _engine(df["ref_u16"].astype(np.float32), float(df["square_size"]))
    a = eng.process_raw(df["frames_u16"].astype(np.float32).reshape(3, -1).view(np.uint8), _lib.FCD_FMT_F32, 3, 1.0)
    want_a, _, _ = eng.process(df["frames_u16"].astype(np.float32), 1.0, want_phases=True)
    assert np.array_equal(a, want_a)
    eng.set_reference(ref_s, 0.001)
    b = eng.process_raw(frames.reshape(5, -1).view(np.uint8), _lib.FCD_FMT_F32, 5, 1.0)
    want_b, _, _ = eng.process(frames, 1.0, want_phases=True)
    assert rel_l2(b, want_b) < 1e-6


@pytest.mark.parametrize("case", ["real_1024_fused", "synthetic_512_unfused"])
def test_two_stream_split_equals_one_stream(df, monkeypatch, case):
    """Device-pointer chunks run as two halves on two streams (FCD_STREAMS=2, the
    default): heights bit-identical to the one-stream chain and to the host path, for
    the fused 1024-wide chain (real frames, 7..1611 residues: the exact MST pass runs
    after the join), with an odd frame count; the unfused chain (512^2) is not split
    and must give the same heights under either setting."""
    import torch
    from bench_data import make_frames_numpy
    if case.startswith("real"):
        ref, sq = df["ref_u16"].astype(np.float32), float(df["square_size"])
        frames = np.concatenate([df["frames_u16"], df["frames_u16"][:2]]).astype(np.float32)  # 5 frames
    else:
        ref, frames = make_frames_numpy(512, 5, seed=8, rotate_deg=5.0)
        sq = 0.001
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(frames).to(dev)
    out = {}
    for ns in ("1", "2"):
        monkeypatch.setenv("FCD_STREAMS", ns)
        eng = _engine(ref, sq)
        hd = torch.empty_like(fd)
        eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
        torch.cuda.synchronize()
        out[ns] = hd.cpu().numpy()
    assert np.array_equal(out["1"], out["2"])
    want, _, _ = _engine(ref, sq).process(frames, 1.0, unwrap=True, want_phases=False)
    assert np.array_equal(out["2"], want)


def test_exact_first_mode_for_residue_heavy_batches(df, monkeypatch):
    """After a device call whose frames mostly carried residues, the next call skips the
    fused first pass and runs the exact chain at once (demod, residue count, scan unwrap
    for residue-free maps and the MST for the rest, integration): heights bit-identical
    to the two-pass form for the residue frames (same kernels and k-fields), and for a
    residue-free frame of the same batch (the reference itself) too: it is redone by the
    first pass's chain, so no frame's heights depend on what earlier calls held; a mostly
    residue-free call switches back."""
    import torch
    ref, sq = df["ref_u16"].astype(np.float32), float(df["square_size"])
    real = df["frames_u16"].astype(np.float32)  # 3 frames, 7..1611 residues per map
    frames = np.stack([real[0], ref, real[1], real[2]])
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(frames).to(dev)
    out = {}
    for ef in ("0", "1"):
        monkeypatch.setenv("FCD_EXACT_FIRST", ef)
        eng = _engine(ref, sq)
        hd = torch.empty_like(fd)
        eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
        torch.cuda.synchronize()
        out[ef] = hd.cpu().numpy()
    real_idx = [0, 2, 3]
    assert np.array_equal(out["0"], out["1"])
    monkeypatch.delenv("FCD_EXACT_FIRST")
    # auto: the first call (3 of 4 frames with residues) switches the mode for the next
    eng = _engine(ref, sq)
    eng.profile(True)
    hd = torch.empty_like(fd)
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
    torch.cuda.synchronize()
    st, _ = eng.stage_times()
    assert st["launches"] >= 1 and int(st["fixup_frames"]) == 3
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr())
    torch.cuda.synchronize()
    st, _ = eng.stage_times()
    # no fused first pass over the batch: only the residue-free frame's (one launch group)
    assert st["launches"] == 1 and int(st["fixup_frames"]) == 3
    assert np.array_equal(hd.cpu().numpy(), out["0"])
    # with the k-fields requested the exact chain writes them (k_cg_finalize) instead of
    # reading the MST labels inside k_int_rows2: a fresh engine's first call (two passes)
    # and its second (exact chain) give the same heights and k-fields
    e2 = _engine(ref, sq)
    e2.profile(True)
    ks, hs = [], []
    for call in range(2):
        hk = torch.empty_like(fd)
        kk = torch.empty((len(frames), 2) + ref.shape, dtype=torch.int32, device=dev)
        e2.process_device(fd.data_ptr(), len(frames), 1.0, True, hk.data_ptr(), k_ptr=kk.data_ptr())
        torch.cuda.synchronize()
        st, _ = e2.stage_times()
        # the second call: the exact chain (its one first-pass launch group is the
        # residue-free frame's); the first: the first pass over the whole batch
        assert st["launches"] == 1 and (call == 1 or st["demod"] > 0), (call, st)
        hs.append(hk.cpu().numpy())
        ks.append(kk.cpu().numpy())
    assert np.array_equal(hs[0][real_idx], hs[1][real_idx])
    for f in real_idx:
        for m in range(2):
            d = ks[1][f, m].astype(np.int64) - ks[0][f, m]
            assert np.all(d == d.flat[0]), (f, m)
    # a residue-free call (the reference repeated) switches back after it
    fr = torch.from_numpy(np.stack([ref] * 4)).to(dev)
    eng.process_device(fr.data_ptr(), 4, 1.0, True, hd.data_ptr())
    eng.process_device(fr.data_ptr(), 4, 1.0, True, hd.data_ptr())
    torch.cuda.synchronize()
    st, _ = eng.stage_times()
    assert st["launches"] >= 1 and int(st["fixup_frames"]) == 0
    eng.profile(False)
    # host-pointer calls switch the same way
    eng = _engine(ref, sq)
    ha, _, _ = eng.process(frames, 1.0, unwrap=True, want_phases=False)
    hb, _, _ = eng.process(frames, 1.0, unwrap=True, want_phases=False)
    assert np.array_equal(ha, out["0"]) and np.array_equal(hb, ha)


def test_early_census_device_calls(df, monkeypatch):
    """Device-pointer calls read the residue census back before their integration kernels
    and return with those still queued (FCD_EARLY_CENSUS=1, the default): several chunks
    per call (FCD_CHUNK_MAX=3: the early readback waits only for the last chunk's census,
    the earlier chunks' flags precede it on the same streams), residue frames in the first
    and the last chunk redone by the exact pass, and two calls issued back to back into
    different outputs before one synchronisation -- every height bit-identical to the
    census read back after the whole chain (=0)."""
    import torch
    ref, sq = df["ref_u16"].astype(np.float32), float(df["square_size"])
    real = df["frames_u16"].astype(np.float32)  # 7..1611 residues per map
    from bench_data import displacement_numpy, warp_numpy
    smooth = [warp_numpy(ref, *displacement_numpy(ref.shape[0], 3 + i)) for i in range(5)]
    frames = np.stack([real[0], smooth[0], smooth[1], smooth[2], smooth[3], ref, smooth[4], real[1]])
    other = np.stack([ref, real[2], smooth[1]])
    dev = torch.device("cuda", 0)
    fd, od = torch.from_numpy(frames).to(dev), torch.from_numpy(other).to(dev)
    monkeypatch.setenv("FCD_CHUNK_MAX", "3")
    work = torch.cuda.Stream(dev)  # a caller stream: the calls stay asynchronous
    out = {}
    for early in ("0", "1"):
        monkeypatch.setenv("FCD_EARLY_CENSUS", early)
        eng = _engine(ref, sq)
        hd, ho = torch.empty_like(fd), torch.empty_like(od)
        torch.cuda.synchronize()
        eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr(), stream=work.cuda_stream)
        eng.process_device(od.data_ptr(), len(other), 1.0, True, ho.data_ptr(), stream=work.cuda_stream)
        torch.cuda.synchronize()
        out[early] = (hd.cpu().numpy(), ho.cpu().numpy())
        del eng
    assert np.array_equal(out["0"][0], out["1"][0])
    assert np.array_equal(out["0"][1], out["1"][1])
    assert np.isfinite(out["1"][0]).all() and np.abs(out["1"][0][0]).max() > 0


def test_pending_device_call_orders_later_calls(df):
    """A device call returns with its integration queued on its stream; a following call
    on another stream, or a new reference (which rewrites the tables those kernels read),
    must not overtake it: heights equal to the same call run on its own.  Residue-free
    frames (warps of the reference), so no exact pass synchronises the calls."""
    import torch
    from bench_data import checkerboard, displacement_numpy, warp_numpy
    ref, sq = df["ref_u16"].astype(np.float32), float(df["square_size"])
    board = checkerboard(ref.shape[0])
    frames = np.stack([warp_numpy(ref, *displacement_numpy(ref.shape[0], 11 + i)) for i in range(6)])
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(frames).to(dev)
    fflip = fd.flip(0).contiguous()
    eng = _engine(ref, sq)
    want = torch.empty_like(fd)
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, want.data_ptr())
    torch.cuda.synchronize()
    main = torch.cuda.Stream(dev)  # a caller stream: the calls return with work queued
    # (1) a new reference right after the call
    got = torch.empty_like(fd)
    torch.cuda.synchronize()
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, got.data_ptr(), stream=main.cuda_stream)
    eng.set_reference(board, 0.001)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    # (2) a call on another stream, into the same workspace, right after the call
    eng.set_reference(ref, sq)
    side = torch.cuda.Stream(dev)
    got2, other = torch.empty_like(fd), torch.empty_like(fd)
    torch.cuda.synchronize()
    eng.process_device(fd.data_ptr(), len(frames), 1.0, True, got2.data_ptr(), stream=main.cuda_stream)
    eng.process_device(fflip.data_ptr(), len(frames), 1.0, True, other.data_ptr(), stream=side.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(got2, want)
    assert torch.equal(other.flip(0), want)


def test_null_stream_call_returns_finished_heights(df):
    """A device call without a caller stream (torch's default stream has cuda_stream == 0,
    which arrives as NULL) runs on the context's own non-blocking stream, which no torch
    stream is ordered with: the call must wait for its work, so torch ops on the default
    stream right after it read finished heights (the early-census return used
    to leave the integration queued there).  Back-to-back calls into fresh tensors, each
    read on the default stream after only that stream's own synchronisation."""
    import torch
    from bench_data import displacement_numpy, warp_numpy
    ref, sq = df["ref_u16"].astype(np.float32), float(df["square_size"])
    frames = np.stack([warp_numpy(ref, *displacement_numpy(ref.shape[0], 21 + i)) for i in range(8)])
    dev = torch.device("cuda", 0)
    fd = torch.from_numpy(frames).to(dev)
    eng = _engine(ref, sq)
    want, _, _ = eng.process(frames, 1.0, unwrap=True, want_phases=False)
    torch.cuda.synchronize()
    for _ in range(3):
        hd = torch.full_like(fd, float("nan"))
        torch.cuda.current_stream(dev).synchronize()
        eng.process_device(fd.data_ptr(), len(frames), 1.0, True, hd.data_ptr(),
                           stream=torch.cuda.current_stream(dev).cuda_stream)
        got = (hd * 1.0).cpu().numpy()  # a torch kernel + copy on the default stream
        assert np.array_equal(got, want)
