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


def gather_stack(local, total_frames):
    """Gather every rank's [b_r, H, W] shard into rank 0's [total, H, W] tensor.

    Uses point-to-point send/recv (RCCL on GPU tensors, gloo on CPU tensors):
    each non-root rank sends its shard once, the root receives the shards in
    rank order; on xGMI every sender has its own link to the root.
    Returns the stacked tensor on rank 0, None elsewhere.
    """
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank != 0:
        dist.send(local.contiguous(), dst=0)
        return None
    out = torch.empty((total_frames,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        a, b = shard_range(total_frames, r, world)
        if r == 0:
            out[a:b].copy_(local)
        elif b > a:
            dist.recv(out[a:b], src=r)
    return out
