"""Batch split across GPUs: one process per GPU, independent frames (problems) per rank.

PICP problems are independent, so the split needs no data-path collective:
each rank owns a contiguous range of problem ids (inputs generated/loaded locally), solves
them on its own device, and the poses are gathered once at the end (RCCL all-gather over xGMI
when the process group is "nccl"; gloo for CPU tests).
"""
import numpy as np


def shard_range(n_items, world, rank):
    """Contiguous, balanced split of range(n_items): sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local, n_total, dist, device=None):
    """All-gather a (n_local, k) float32 array from every rank into (n_total, k), in rank
    order (ranks own contiguous ranges, see shard_range).  `dist` is torch.distributed with
    an initialised process group; device = torch device of the backend's tensors."""
    import torch
    world = dist.get_world_size()
    local = np.ascontiguousarray(local, np.float32)
    k = local.shape[1]
    counts = [shard_range(n_total, world, r) for r in range(world)]
    maxn = max(e - s for s, e in counts)
    buf = torch.zeros((maxn, k), dtype=torch.float32, device=device)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(local).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = [p[: e - s].cpu().numpy() for p, (s, e) in zip(parts, counts)]
    return np.concatenate(out, 0)
