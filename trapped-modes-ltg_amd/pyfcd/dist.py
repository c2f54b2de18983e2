"""Multi-GPU sharding of a frame batch.

Frames are independent and the reference-derived state is deterministic, so
the batch is split contiguously over ranks (rank r gets frames
[r*B/N, (r+1)*B/N)), every rank builds its own reference state from the same
reference image (no broadcast), and there is no exchange in the compute.  The
only collective is an optional gather of the height stack to rank 0 over RCCL
(torch.distributed "nccl" backend on ROCm = RCCL over xGMI), timed apart from
the compute, plus the scalar max-over-ranks of the step time.
"""
import os


def dist_env():
    """(rank, world_size, local_rank) from torchrun's environment (1 process per GPU)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def shard_range(total, rank, world):
    """Contiguous, balanced [start, stop) of `total` frames for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (identity without an initialised process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def free_port():
    """An unused TCP port on 127.0.0.1 for the rendezvous."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nproc, script, argv, env=None):
    """Run `script argv` as `nproc` rank processes (one per GPU) under
    torch.distributed.run on this node, rendezvous on 127.0.0.1, and return the
    launcher's exit code.

    Called by a parent that has not touched the GPU (no HIP call, no
    torch.cuda.is_available()): the ranks are child processes, the parent only
    waits for them, so nothing is exec'd over a process holding a GPU context."""
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script] + list(argv)
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.call(cmd, env=e)


def gather_stack(local, total_frames):
    """Gather every rank's [b_r, H, W] shard into rank 0's [total, H, W] tensor.

    One batch of point-to-point operations (dist.batch_isend_irecv: a grouped
    ncclSend/ncclRecv on RCCL): every non-root rank posts its
    send and the root posts all its receives at once, so on xGMI the shards
    arrive over the root's links in parallel instead of one sender at a time.
    Returns the stacked tensor on rank 0, None elsewhere.
    """
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    if world > 1 and total_frames < world:
        # an empty shard would leave its rank out of the grouped send/recv; on RCCL every
        # rank must enter a group's first point-to-point batch
        raise ValueError(f"gather_stack: {total_frames} frames over {world} ranks leaves a rank without frames")
    a0, b0 = shard_range(total_frames, rank, world)
    if local.shape[0] != b0 - a0:
        raise ValueError(f"rank {rank}: shard of {local.shape[0]} frames, expected {b0 - a0}")
    if world == 1:  # no peers: an empty point-to-point batch is an error in torch.distributed
        return local
    if rank != 0:
        ops = [dist.P2POp(dist.isend, local.contiguous(), 0)]
        out = None
    else:
        out = torch.empty((total_frames,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        out[a0:b0].copy_(local)
        ops = []
        for r in range(1, world):
            a, b = shard_range(total_frames, r, world)
            ops.append(dist.P2POp(dist.irecv, out[a:b], r))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return out
