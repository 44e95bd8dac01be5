"""Batch split across GPUs: one process per GPU, independent frames (problems) per rank.

PICP problems are independent, so the split needs no data-path collective: each
rank owns a contiguous range of problem ids (picp_shard_range), solves them on its own device,
and the results are all-gathered once at the end.  The product path is the C++ library's:
picp_batch_allgather pads every rank's shard to picp_shard_pad(n, world) states, runs one RCCL
all-gather over xGMI and unpacks the padded buffer with picp_shard_unpack (include/picp_c.h).

gather_rows is the same layout over a torch.distributed process group (gloo): the CPU tests and
bench.py --plan-only move rows through it, so the pad/unpack the RCCL path uses is exercised on
ragged shards without a GPU.
"""
import numpy as np


def shard_range(n_items, world, rank):
    """Contiguous, balanced split of range(n_items): sizes differ by at most one (the same rule as
    picp_shard_range; test_dist checks both agree)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local, n_total, dist, device=None):
    """All-gather a (n_local, k) float32 array from every rank into (n_total, k), problem order:
    each rank's shard padded to picp_shard_pad rows, one all_gather, then the library's
    picp_shard_unpack (host code, no device).  `dist` is torch.distributed with an initialised
    process group; device = torch device of the backend's tensors."""
    import torch

    import picp_amd
    world = dist.get_world_size()
    local = np.ascontiguousarray(local, np.float32)
    k = local.shape[1]
    pad = max(picp_amd.shard_pad(n_total, world), 1)
    buf = torch.zeros((pad, k), dtype=torch.float32, device=device)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(local).to(buf.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    padded = np.ascontiguousarray(torch.cat(parts, 0).cpu().numpy())
    return picp_amd.shard_unpack(padded, n_total, world)
