"""The frame-sharded multi-rank path driving the engine: two rank
processes share the box's one GPU (gloo for the process group, as the CPU tests;
RCCL refuses two ranks on one device, and on an 8-GPU node the same code runs one rank
per GPU over RCCL), each demodulates its contiguous shard of the batch, the heights are
gathered to rank 0 with the grouped send/recv of pyfcd.dist.gather_stack, and rank 0
checks the stack bit-for-bit against one process running the whole batch (frames are
independent, the reference state is deterministic).  Two shapes: a small host-pointer
batch, and c4's per-rank shape (1024^2 frames, 16 per rank, generated and demodulated
device-resident on a caller stream, as bench.py does)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rank(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "trapped-modes-ltg_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch  # noqa: F401  (torch's HIP runtime first, conftest.py)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bench_data import make_frames_numpy
        from pyfcd import _lib
        from pyfcd.dist import gather_stack, shard_range
        ref, frames = make_frames_numpy(256, 7, seed=2, rotate_deg=5.0)
        a, b = shard_range(len(frames), rank, world)
        eng = _lib.Engine(ref.shape, device=0)
        eng.set_reference(ref, 0.001)
        h, _, _ = eng.process(frames[a:b], 1.0, unwrap=True, want_phases=False)
        out = gather_stack(torch.from_numpy(h), len(frames))
        if rank == 0:
            full, _, _ = eng.process(frames, 1.0, unwrap=True, want_phases=False)
            q.put(bool(np.array_equal(out.numpy(), full)))
        eng.close()
    finally:
        dist.destroy_process_group()


def _rank_c4(rank, world, port, q, per_rank=16):
    """c4 per-rank shape: rank r generates frames [r * per_rank, (r + 1) * per_rank) of the
    bench recipe on the device (make_frames_torch seeds frame b with b), demodulates them
    from device pointers on its own stream, and the heights go through gather_stack."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "trapped-modes-ltg_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bench_data import make_frames_torch, SQUARE_SIZE
        from pyfcd import _lib
        from pyfcd.dist import gather_stack, shard_range
        n, total = 1024, per_rank * world
        dev = torch.device("cuda", 0)
        a, b = shard_range(total, rank, world)
        ref, frames = make_frames_torch(n, b - a, seed=a, device=dev)
        eng = _lib.Engine((n, n), device=0)
        eng.set_reference(ref.cpu().numpy(), SQUARE_SIZE)
        work = torch.cuda.Stream(dev)
        torch.cuda.synchronize(dev)
        h = torch.empty_like(frames)
        eng.process_device(frames.data_ptr(), b - a, 1.0, True, h.data_ptr(), stream=work.cuda_stream)
        torch.cuda.synchronize(dev)
        out = gather_stack(h.cpu(), total)  # gloo moves host tensors
        if rank == 0:
            _, full_frames = make_frames_torch(n, total, seed=0, device=dev)
            full = torch.empty_like(full_frames)
            eng.process_device(full_frames.data_ptr(), total, 1.0, True, full.data_ptr(), stream=work.cuda_stream)
            torch.cuda.synchronize(dev)
            same_frames = bool(torch.equal(full_frames[a:b], frames))
            q.put(same_frames and bool(torch.equal(out, full.cpu())) and bool(torch.isfinite(out).all()))
        eng.close()
    finally:
        dist.destroy_process_group()


def _run_ranks(target, world=2):
    import multiprocessing as mp
    from pyfcd.dist import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return ok


def test_c4_shape_two_ranks_device_resident():
    assert _run_ranks(_rank_c4)


def test_two_ranks_shard_and_gather_equal_one_process():
    import multiprocessing as mp
    from pyfcd.dist import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


def _rank_rccl_one(rank, world, port, q):
    """A one-rank RCCL group on the box's GPU: the device-tensor collectives bench.py's
    ranks use (the step-time max, a sum) and gather_stack's one-rank pass-through. Two
    ranks cannot share one device under RCCL; the N-rank exchange runs on the driver's
    8-GPU node (bench.py --gpus N --gather)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "trapped-modes-ltg_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        from pyfcd.dist import gather_stack, max_over_ranks, sum_over_ranks
        ok = dist.get_backend() == "nccl"
        ok = ok and max_over_ranks(2.5, device=dev) == 2.5 and sum_over_ranks(3.0, device=dev) == 3.0
        t = torch.arange(24, dtype=torch.float32, device=dev).reshape(2, 3, 4)
        dist.all_reduce(t)  # one rank: unchanged, but through RCCL on the device
        torch.cuda.synchronize(dev)
        ok = ok and bool(torch.equal(t.cpu(), torch.arange(24, dtype=torch.float32).reshape(2, 3, 4)))
        ok = ok and gather_stack(t, 2) is t
        q.put(ok)
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_group():
    assert _run_ranks(_rank_rccl_one, world=1)

