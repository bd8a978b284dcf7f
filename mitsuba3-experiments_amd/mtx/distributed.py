"""Multi-GPU film sharding over torch.distributed (RCCL on ROCm, gloo on CPU).

The reference has no distributed code; the path shards
naturally (§8e):
  * sample shards (weak scaling, bench.py): every rank traces the global
    sample range [r*spp, (r+1)*spp) of every pixel; films are gathered to
    rank 0 and summed in rank order (deterministic).
  * row bands (strong scaling): rank r traces film rows [y0_r, y1_r); each
    band carries its 1-row tent halo above and below, stitched on rank 0 by
    adding the overlapping halo rows in rank order.
One collective per render (an all_gather of ~15 MB films for 1280x720);
no data-path exchange during tracing.
"""
from __future__ import annotations

import numpy as np


def row_bands(height: int, world: int):
    """Balanced contiguous row ranges [y0, y1) per rank."""
    edges = [round(r * height / world) for r in range(world + 1)]
    return [(edges[r], edges[r + 1]) for r in range(world)]


def _to_tensor(film, like_device=None):
    import torch

    if isinstance(film, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(film))
    return film


def gather_sum(film, group=None):
    """Sum of every rank's film in rank order, returned on rank 0 (None elsewhere).
    `film` is a torch tensor (device for nccl, cpu for gloo) or numpy array."""
    import torch
    import torch.distributed as dist

    t = _to_tensor(film)
    world = dist.get_world_size(group)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    if dist.get_rank(group) != 0:
        return None
    total = torch.zeros_like(t)
    for p in parts:
        total.add_(p)
    return total


def gather_bands(band, y0: int, y1: int, height: int, group=None):
    """Stitch row-band films (with halos) into the full film on rank 0."""
    import torch
    import torch.distributed as dist

    t = _to_tensor(band)
    world = dist.get_world_size(group)
    W2 = t.shape[1]
    maxrows = max(b1 - b0 for b0, b1 in row_bands(height, world)) + 2
    buf = torch.zeros((maxrows, W2, t.shape[2]), dtype=t.dtype, device=t.device)
    buf[: t.shape[0]] = t
    meta = torch.tensor([y0, y1], dtype=torch.int64, device=t.device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    dist.all_gather(metas, meta, group=group)
    if dist.get_rank(group) != 0:
        return None
    full = torch.zeros((height + 2, W2, t.shape[2]), dtype=t.dtype, device=t.device)
    for p, m in zip(parts, metas):
        a, b = int(m[0]), int(m[1])
        full[a: b + 2] += p[: b - a + 2]
    return full


def render_sharded(render, height: int, spp: int, mode: str = "samples", group=None):
    """Run `render(spp, spp_total, sample_offset, y0, y1)` for this rank's shard
    and combine on rank 0. `render` returns a film (numpy or tensor)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if mode == "samples":
        film = render(spp, spp * world, spp * rank, 0, height)
        return gather_sum(film, group)
    if mode == "rows":
        y0, y1 = row_bands(height, world)[rank]
        film = render(spp, spp, 0, y0, y1)
        return gather_bands(film, y0, y1, height, group)
    raise ValueError(mode)
