"""Headline benchmark: frames/s of the full FCD height-map pipeline
(fcd.compute_height_map: FFT, disk band-pass, inverse FFTs, phase, unwrap,
displacement solve, spectral integration) on 1024x1024 checkerboard frames,
with the HBM roofline of the demodulation stage and the CPU oracle timed on
the same host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 1024] [--batch 256]

For N > 1 there is one process per GPU: either the caller launches the ranks
(torch.distributed.run sets WORLD_SIZE), or a plain `python bench.py --gpus N`
launches them itself through torch.distributed.run before anything touches the
GPU (pyfcd/dist.py:spawn_ranks) and exits with the ranks' exit code.  Each rank
checks WORLD_SIZE == N, processes its own `--batch` frames (weak scaling,
SURVEY.md §8e: frames are independent, no collective in the compute), the step
time is the max over ranks, and rank 0 prints one JSON line.  `--gather` then
times a grouped send/recv gather of every rank's heights to rank 0, reported as
`gather` beside (never inside) the frames/s.  `--dry-run` stops after the
rendezvous (no GPU): rank 0 prints the world it saw (CPU test of the launcher).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "frames/sec @1024×1024 checkerboard batch + HBM GB/s vs peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def load_traffic(n, chunk):
    """HBM bytes per demod launch group from the committed PMC summary of this frame
    size (profiles/traffic_<n>.json, written by tools/traffic_summary.py from two
    rocprofv3 --pmc passes, FETCH_SIZE and WRITE_SIZE, over this bench command at that
    size), if one was measured."""
    p = os.path.join(ROOT, "profiles", f"traffic_{n}.json")
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("frame") != n:
        return None
    return t


def log(msg):
    """Progress on stderr (keeps long profiled runs visibly alive; stdout holds only the JSON line)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(size, frames, seconds_cap=25.0):
    """The CPU oracle (numpy/scipy FFTs + C Herraez unwrap), 1 core, bounded sample."""
    import numpy as np
    from bench_data import make_frames_numpy
    from oracle import fcd_oracle as O
    ref, fr = make_frames_numpy(size, frames, seed=0)
    carriers = O.compute_carriers(ref, 0.001)  # once per reference, like the GPU run
    t0 = time.perf_counter()
    done = 0
    for f in fr:
        O.compute_height_map(ref, f, 0.001, height=1.0, carriers=carriers)
        done += 1
        if time.perf_counter() - t0 > seconds_cap:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} frames of {size}x{size} (same synthetic recipe), oracle/fcd_oracle.compute_height_map "
                      f"with carriers cached, scipy.fft workers=1, {dt:.1f} s"}


def _cpu_worker(args):
    """One process of the all-cores CPU baseline: its own seeded frames, carriers once,
    then `count` frames through the oracle; returns (frames, seconds)."""
    size, count, seed = args
    for p in (ROOT, os.path.join(ROOT, "trapped-modes-ltg_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from bench_data import make_frames_numpy
    from oracle import fcd_oracle as O
    ref, fr = make_frames_numpy(size, count, seed=seed)
    carriers = O.compute_carriers(ref, 0.001)
    t0 = time.perf_counter()
    for f in fr:
        O.compute_height_map(ref, f, 0.001, height=1.0, carriers=carriers)
    return len(fr), time.perf_counter() - t0


def cpu_baseline_all_cores(size, workers=16, per_worker=6):
    """The same oracle on `workers` host cores (one process per core, frames split
    between them): total frames / slowest worker's time.  16 workers =
    the GPU box's CPU share per GPU."""
    import multiprocessing as mp
    env = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in env:
        os.environ[k] = "1"
    try:
        with mp.get_context("spawn").Pool(workers) as pool:
            res = pool.map(_cpu_worker, [(size, per_worker, 1000 + w) for w in range(workers)])
    finally:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    frames = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": frames / wall, "unit": "frames/s", "cores": workers, "kind": "port",
            "sample": f"{frames} frames of {size}x{size} ({per_worker} per process, {workers} processes, one core "
                      f"each), oracle/fcd_oracle.compute_height_map with carriers cached, slowest process {wall:.1f} s"}


def real_frames_rate(dev, stream, batch=96, reps=3):
    """Side measurement, never `value`: the three real 10-bit camera frames of
    tests/golden/real_df.npz (7..1611 residues per map, so every frame takes the exact MST
    unwrap) tiled to `batch` device-resident frames, frames/s over `reps` calls after a
    warm-up call."""
    import numpy as np
    import torch
    from pyfcd import _lib
    d = np.load(os.path.join(ROOT, "tests", "golden", "real_df.npz"))
    frames = np.concatenate([d["frames_u16"].astype(np.float32)] * (batch // 3))
    fr = torch.from_numpy(frames).to(dev)
    h = torch.empty_like(fr)
    eng = _lib.Engine(frames.shape[1:], device=dev.index)
    eng.set_reference(d["ref_u16"].astype(np.float32), float(d["square_size"]))
    eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.process_device(fr.data_ptr(), len(frames), 1.0, True, h.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(len(frames) / dt, 1), "unit": "frames/s",
            "sample": f"{len(frames)} real 1024x1024 camera frames (3 frames of tests/golden/real_df.npz, "
                      "7..1611 residues per map) per call, device-resident, exact MST unwrap for every frame",
            "ms_per_frame": round(dt / len(frames) * 1e3, 4)}


def generic_shape_rate(dev, stream, rows=1080, cols=1920, batch=64, reps=3):
    """Side measurement, never `value`: the generic chain (kernels_mr.hip, frame sides that
    are not powers of two) at the HD camera format, residue-free synthetic boards (the
    pattern.py board warped by the bump field of bench_data.py, generated on the host),
    `batch` device-resident frames per call, frames/s over `reps` calls after a warm-up."""
    import numpy as np
    import torch
    from bench_data import checkerboard, displacement_numpy, warp_numpy
    from pyfcd import _lib
    ref = checkerboard(rows, cols=cols)
    base = [warp_numpy(ref, *displacement_numpy(rows, s, cols=cols)) for s in range(4)]
    fr = torch.from_numpy(np.stack([base[i % 4] for i in range(batch)])).to(dev)
    h = torch.empty_like(fr)
    eng = _lib.Engine((rows, cols), device=dev.index)
    eng.set_reference(ref, 0.001)
    eng.process_device(fr.data_ptr(), batch, 1.0, True, h.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.process_device(fr.data_ptr(), batch, 1.0, True, h.data_ptr(), stream=stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    eng.close()
    return {"value": round(batch / dt, 1), "unit": "frames/s", "shape": [rows, cols],
            "us_per_megapixel": round(dt / batch * 1e6 / (rows * cols / 1e6), 2),
            "sample": f"{batch} synthetic {rows}x{cols} boards per call (residue-free), device-resident, "
                      "the generic mixed-radix chain"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=12)
    ap.add_argument("--cpu-workers", type=int, default=16, help="processes of the all-cores CPU baseline")
    ap.add_argument("--gather", action="store_true", help="also time an RCCL gather of the heights to rank 0")
    ap.add_argument("--dry-run", action="store_true", help="rendezvous only, no GPU (launcher test)")
    ap.add_argument("--no-real-frames", action="store_true",
                    help="skip the side measurement on real camera frames with residues (1 GPU, 1024^2)")
    args = ap.parse_args()

    from pyfcd.dist import dist_env, spawn_ranks
    rank, world, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start one rank per GPU as child processes (nothing
        # has touched the GPU in this process) and report their exit status
        sys.exit(spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist
    if world > 1:
        # "nccl" is RCCL on ROCm (one process per GPU, xGMI); FCD_BENCH_BACKEND=gloo only
        # to rehearse N ranks sharing the GPUs of a smaller box (and for --dry-run)
        backend = "gloo" if args.dry_run else os.environ.get("FCD_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, init_method="env://")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    if args.dry_run:
        seen = torch.zeros(world, dtype=torch.int64)
        seen[rank] = rank + 1
        if world > 1:
            dist.all_reduce(seen)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": seen.tolist()}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    from pyfcd import _lib
    from pyfcd.dist import gather_stack, max_over_ranks
    from bench_data import make_frames_torch, SQUARE_SIZE
    ndev = torch.cuda.device_count()
    if world > 1 and ndev < world and os.environ.get("FCD_BENCH_BACKEND", "nccl") == "nccl":
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible")
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n, B = args.size, args.batch

    # synthetic batch, generated in HBM; rank r owns frames [r*B, (r+1)*B)
    ref_t, frames = make_frames_torch(n, B, seed=rank * B, device=dev)
    log(f"rank {rank}: {B} frames of {n}x{n} generated on {dev}")
    heights = torch.empty((B, n, n), dtype=torch.float32, device=dev)
    eng = _lib.Engine((n, n), device=local)
    eng.set_reference(ref_t.cpu().numpy(), SQUARE_SIZE)
    # a dedicated (non-default) stream: the engine keeps a call on a caller stream
    # asynchronous (the integration stays queued behind the census read-back), while a
    # null stream (torch's default stream has cuda_stream == 0) makes it wait before
    # returning; the HIP events below record on it too (torch.cuda.stream context)
    torch.cuda.synchronize(dev)  # the frames were generated on the default stream
    work = torch.cuda.Stream(dev)
    torch.cuda.set_stream(work)
    stream = work.cuda_stream

    def step():
        eng.process_device(frames.data_ptr(), B, 1.0, True, heights.data_ptr(), stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    log(f"rank {rank}: warmup done")
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    log(f"rank {rank}: timed steps done ({wall:.3f} s)")
    # per-stage device time from the engine's own HIP events (separate, profiled
    # passes, so the headline timing above carries no event overhead):
    #  (1) the headline path itself (heights only: fused band transform + unwrap + row
    #      FFT, kernels_phase_rows.hip), for the stage breakdown;
    #  (2) the demodulation unit of SURVEY.md §8d as its own launch group: the same
    #      frames with the wrapped phases written to HBM (k_demod_rows + k_demod_cols
    #      + k_band_phase_res), for the roofline.
    prof_steps = max(2, min(args.steps, 4))
    eng.profile(True)
    for _ in range(prof_steps):
        step()
    path_stages, path_frames = eng.stage_times()
    wrapped = torch.empty((B, 2, n, n), dtype=torch.float32, device=dev)
    for _ in range(prof_steps):
        eng.process_device(frames.data_ptr(), B, 1.0, True, heights.data_ptr(), wrapped_ptr=wrapped.data_ptr(),
                           stream=stream)
    stages, nframes = eng.stage_times()
    eng.profile(False)
    del wrapped
    wall_max = max_over_ranks(wall, device=dev)
    ms_per_step = wall_max / args.steps * 1e3
    total_frames = B * world * args.steps
    value = total_frames / wall_max

    gather_ms = None
    if args.gather and world > 1:
        # heights of every rank's last step to rank 0 (one grouped send/recv batch);
        # a first untimed gather sets up the point-to-point channels
        stacked = gather_stack(heights, B * world)
        del stacked
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        stacked = gather_stack(heights, B * world)
        torch.cuda.synchronize(dev)
        gather_ms = max_over_ranks((time.perf_counter() - g0) * 1e3, device=dev)
        if rank == 0:  # rank 0's own shard sits first in the stack
            assert torch.equal(stacked[:B], heights)
        del stacked

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # Roofline of the demodulation launch group (SURVEY.md §8d unit: frame f32 in ->
    # two wrapped phase planes f32 out, B_demod = 12 N^2 bytes per frame): one group =
    # k_demod_rows + k_demod_cols + k_band_phase_res over one chunk of `chunk` frames,
    # timed by HIP events the engine records on the launch stream around the group.
    chunk = int(stages.pop("chunk"))
    launches = int(stages.pop("launches"))
    demod_bytes = 12.0 * n * n
    demod_us_per_launch = stages["demod"] * 1e3 / max(launches, 1)
    demod_frames_per_launch = nframes / max(launches, 1)
    achieved = demod_bytes * demod_frames_per_launch / (demod_us_per_launch * 1e-6) / 1e9
    fix_frames = int(path_stages.pop("fixup_frames"))
    path_names = {"demod": "demod_rows+demod_cols", "unwrap": "phase_rows+colk+seam (fused)",
                  "integrate": "int_cols+int_c2r", "total": "total", "fixup": "exact_fixup"}
    per_frame = {path_names[k]: round(v / max(path_frames, 1) * 1e3, 3) for k, v in path_stages.items()
                 if k in path_names}  # us per frame
    per_frame["fixup_frames_per_step"] = fix_frames / prof_steps
    traffic = load_traffic(n, chunk)
    traffic_launch = None
    if traffic:  # measured per frame at traffic["chunk"] frames per launch; scaled to this launch size
        traffic_launch = int(round(traffic["demod_group_bytes_per_frame"] * demod_frames_per_launch))
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: pattern.py geometry (10-px binary checkerboard, 0/65535) warped by seeded Gaussian bumps, "
                "generated on device (bench_data.py)",
        "config": {"workload": f"{ {1024: 'c2', 2048: 'c3', 4096: 'c5'}.get(n, 'custom')}: {n}x{n} frames, {B} per GPU per step, full compute_height_map pipeline "
                               f"(demod + unwrap + integration), reference state cached",
                   "frame": n, "batch_per_gpu": B, "global_batch": B * world,
                   "parallelism": f"frame-sharded x{world}, no collective in the compute",
                   # each step's chunk runs as this many concurrent parts (engine FCD_STREAMS;
                   # default two up to 1024-wide rows, one above)
                   "streams_per_chunk": (2 if int(os.environ["FCD_STREAMS"]) >= 2 else 1) if os.environ.get("FCD_STREAMS")
                   else (2 if n <= 1024 else 1)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_launch,
                     "kernel": "demod launch group k_demod_rows + k_demod_cols + k_band_phase_res "
                               "(theta-resident band-pruned inverse + phase; 512-bin window at 4096) "
                               "(frame f32 in -> 2 wrapped phases f32 out), 12*N^2 B/frame",
                     "frames_per_launch": round(demod_frames_per_launch, 2),
                     "us_per_launch": round(demod_us_per_launch, 2),
                     "algorithmic_bytes_per_launch": int(demod_bytes * demod_frames_per_launch),
                     "traffic_source": (traffic["source"] + f"; measured at {traffic['chunk']} frames per launch, "
                                        "per-frame bytes x frames per launch") if traffic else None,
                     "measured_as": "separate profiled pass of the same frames with the wrapped phases written "
                                    "(the headline path fuses the band transform with the unwrap)"},
        # the heights-only headline path against the same 8 TB/s: its own compulsory bytes
        # (frame f32 in + height f32 out, 8 N^2) and the BASELINE.md unit (12 N^2) at the
        # headline rate; traffic: PMC bytes per frame summed over the headline's kernels
        "headline_roofline": {
            "per_gpu": True, "bytes_per_frame": 8 * n * n,
            "achieved_GBps": round(8.0 * n * n * value / world / 1e9, 1),
            "frac": round(8.0 * n * n * value / world / 1e9 / HBM_PEAK_GBS, 4),
            "demod_unit_frac_at_headline_rate": round(12.0 * n * n * value / world / 1e9 / HBM_PEAK_GBS, 4),
            "traffic_bytes_per_frame": traffic.get("headline_bytes_per_frame") if traffic else None},
        "stage_us_per_frame": per_frame,
        "event_ms_per_step": round(ev0.elapsed_time(ev1) / args.steps, 3),
    }
    if gather_ms is not None:
        gb = 4.0 * n * n * B * (world - 1) / 1e9
        out["gather"] = {"ms": round(gather_ms, 3), "bytes_to_root_GB": round(gb, 3),
                         "GB_per_s_into_root": round(gb / (gather_ms * 1e-3), 1),
                         "how": "dist.batch_isend_irecv: every rank's last-step heights to rank 0, all links at once; "
                                "not inside the frames/s"}
    if world == 1 and n == 1024 and not args.no_real_frames:
        out["residue_frames"] = real_frames_rate(dev, stream)
        out["generic_hd_frames"] = generic_shape_rate(dev, stream)
    if world == 1 and not args.no_cpu_baseline:
        log("CPU baseline (oracle, 1 core, then all cores)")
        single = cpu_baseline(n, args.cpu_frames)
        out["cpu_baseline"] = cpu_baseline_all_cores(n, workers=args.cpu_workers)
        out["cpu_baseline"]["single_core"] = single
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
