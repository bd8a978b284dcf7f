"""Multi-GPU film sharding over torch.distributed (RCCL on ROCm, gloo on CPU).

The reference has no distributed code; the path shards
naturally (§8e):
  * sample shards (strong scaling, bench.py): rank r traces the global
    sample range [r*spp/N, (r+1)*spp/N) of every pixel of one fixed-spp
    render; films are combined on rank 0 by a pairwise tree over the ranks
    (deterministic; at N = 2, 4, 8 the top of the film's 8-slot tree, so the
    combined film equals the one-GPU film bit for bit).
  * row bands (strong scaling): rank r traces film rows [y0_r, y1_r); each
    band carries its 1-row tent halo above and below, stitched on rank 0 by
    adding the overlapping halo rows in rank order.
One collective per render (a gather of ~15 MB films to rank 0 for 1280x720);
no data-path exchange during tracing.

prefix_sum (prefix_sum.py:9-36) on a u32 array split into contiguous
per-rank slices shards with one exchange: a local scan on
each rank's GPU, an all_gather of the slice totals, then the lower ranks'
total added (mod 2^32, exact). hashgrid / scatter_reduce build small global
tables and run as replicas (each rank builds its own).

ReSTIR GI (restirgi.py) is the one path with an exchange step: its spatial
reuse reads samples and temporal reservoirs up to `initial_search_radius`
rows away (:301-313) and its temporal reuse reprojects into the previous
frame. A row-banded frame runs stage A (initial sample + temporal) on the
band, swaps a halo of ceil(radius) rows of samples and temporal reservoirs
with the neighbouring bands (point-to-point), then stage B (spatial + final).
"""
from __future__ import annotations

import numpy as np


def row_bands(height: int, world: int):
    """Balanced contiguous row ranges [y0, y1) per rank."""
    edges = [round(r * height / world) for r in range(world + 1)]
    return [(edges[r], edges[r + 1]) for r in range(world)]


def sample_range(spp: int, world: int, rank: int):
    """Strong-scaling sample shard: rank r traces the global samples
    [r*spp//N, (r+1)*spp//N) of every pixel (global-lane seeding keeps each
    path identical to the single-GPU render, path.py:156-161).

    Every rank needs at least one sample (mtx_render rejects spp = 0): with
    spp < world this raises on every rank alike, before any collective, so no
    rank is left waiting in a gather."""
    if spp < world:
        raise ValueError(f"sample shards: spp={spp} < world size {world} (every rank needs >= 1 sample per pixel)")
    return rank * spp // world, (rank + 1) * spp // world


def _to_tensor(film, like_device=None):
    import torch

    if isinstance(film, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(film))
    return film


def _host_staged(group=None) -> bool:
    """gloo moves host memory only: device tensors are staged through the
    host (used when several ranks share one GPU, e.g. a 1-GPU rehearsal of
    the N>1 path). RCCL (backend "nccl") sends device memory directly."""
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def _comm(t, group=None):
    """The tensor handed to the collective: `t` itself, or its host copy."""
    return t.cpu() if (t.is_cuda and _host_staged(group)) else t


def _tree_sum(parts):
    """Sum of `parts` (rank order) by adjacent pairs, level by level (an odd
    last part moves up unchanged): for 2, 4 and 8 ranks the top of the film's
    8-slot tree (mtx_core/common.h film_tree8), so sample-range shards of
    whole slots combine to the one-device film bit for bit."""
    import torch

    level = list(parts)
    if len(level) == 1:
        return torch.zeros_like(level[0]) + level[0]
    while len(level) > 1:
        nxt = [level[i] + level[i + 1] for i in range(0, len(level) - 1, 2)]
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def gather_sum(film, group=None):
    """Sum of every rank's film in rank order, returned on rank 0 (None elsewhere).
    `film` is a torch tensor (device for nccl, cpu for gloo) or numpy array.
    One gather to rank 0 (point-to-point receives over xGMI with RCCL), then
    a fixed pairwise tree over the ranks (_tree_sum): deterministic.""" 
    import torch
    import torch.distributed as dist

    t = _to_tensor(film)
    c = _comm(t, group)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [torch.empty_like(c) for _ in range(world)] if rank == 0 else None
    dist.gather(c, parts, dst=0, group=group)
    if rank != 0:
        return None
    return _tree_sum(parts).to(t.device)


_ALL_TO_ALL_BACKENDS = ("nccl", "gloo")  # backends with all_to_all_single (RCCL, gloo)


def reduce_sum(film, group=None):
    """`gather_sum` with the sum spread over the ranks: an all_to_all hands
    every rank one 1/N slice of every film, each rank sums its slice by the
    same rank tree, and rank 0 gathers the N summed slices (None on other ranks).
    Bit-identical to `gather_sum` (the same additions, elementwise, in the
    same order); rank 0 receives (N-1)/N of one film instead of N-1 films
    and adds 1/N of them, and every xGMI link carries 2/N of a film."""
    import torch
    import torch.distributed as dist

    t = _to_tensor(film)
    world = dist.get_world_size(group)
    # decided from the backend, identically on every rank (a communication
    # error is raised, never turned into a different collective sequence)
    if world > 1 and dist.get_backend(group) not in _ALL_TO_ALL_BACKENDS:
        return gather_sum(film, group)
    c = _comm(t, group)
    rank = dist.get_rank(group)
    if world == 1:
        return (torch.zeros_like(c) + c).to(t.device)
    flat = c.reshape(-1)
    n = flat.numel()
    chunk = -(-n // world)
    send = flat if chunk * world == n else torch.cat([flat, flat.new_zeros(chunk * world - n)])
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    part = _tree_sum([recv[r * chunk:(r + 1) * chunk] for r in range(world)])
    parts = [torch.empty_like(part) for _ in range(world)] if rank == 0 else None
    dist.gather(part, parts, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat(parts)[:n].reshape(c.shape).to(t.device)


def gather_bands(band, y0: int, y1: int, height: int, group=None):
    """Stitch row-band films (with halos) into the full film on rank 0."""
    import torch
    import torch.distributed as dist

    t = _to_tensor(band)
    world = dist.get_world_size(group)
    W2 = t.shape[1]
    maxrows = max(b1 - b0 for b0, b1 in row_bands(height, world)) + 2
    dev = t.device
    t = _comm(t, group)
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
    return full.to(dev)


def render_sharded(render, height: int, spp: int, mode: str = "samples", group=None):
    """Run `render(spp, spp_total, sample_offset, y0, y1)` for this rank's shard
    of ONE render at `spp` global samples per pixel (strong scaling) and
    combine on rank 0. `render` returns a film (numpy or tensor)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if mode == "samples":
        s0, s1 = sample_range(spp, world, rank)
        film = render(s1 - s0, spp, s0, 0, height)
        return reduce_sum(film, group)
    if mode == "rows":
        y0, y1 = row_bands(height, world)[rank]
        film = render(spp, spp, 0, y0, y1)
        return gather_bands(film, y0, y1, height, group)
    raise ValueError(mode)


# ------------------------------------------------------------ ReSTIR bands --
def restir_halo(integ) -> int:
    """Halo rows a band needs from each neighbour: the spatial taps reach
    trunc(radius) <= initial_search_radius rows (the radius only shrinks), the
    temporal reprojection of a static camera one row. A camera that moved
    since the previous frame reprojects arbitrarily far: render_restir_sharded
    then gathers the whole previous-sample buffer (gather_prev_samples)."""
    import math

    return max(1, int(math.ceil(float(integ.initial_search_radius))))


def halo_plan(y0: int, y1: int, height: int, halo: int):
    """(send_up, send_down, recv_up, recv_down) row ranges (row0, nrows) for
    band [y0, y1): the previous band needs rows [y0, y0 + min(halo, H - y0)),
    the next band rows [y1 - min(halo, y1), y1); this band receives the
    min(halo, y0) rows above it and the min(halo, H - y1) rows below it."""
    send_up = (y0, min(halo, height - y0))
    send_down = (y1 - min(halo, y1), min(halo, y1))
    recv_up = (y0 - min(halo, y0), min(halo, y0))
    recv_down = (y1, min(halo, height - y1))
    return send_up, send_down, recv_up, recv_down


def exchange_halos(export_rows, import_rows, y0: int, y1: int, height: int, halo: int, group=None):
    """Swap halo rows with the neighbouring ranks (torch.distributed P2P).

    export_rows(which, row0, nrows) -> contiguous tensor; import_rows(which,
    row0, tensor). which in ('sample', 'temporal'). Bands must be at least
    `halo` rows tall so the neighbours own every halo row."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    send_up, send_down, recv_up, recv_down = halo_plan(y0, y1, height, halo)
    if (rank > 0 and send_up[1] > y1 - y0) or (rank < world - 1 and send_down[1] > y1 - y0):
        raise ValueError(f"band [{y0}, {y1}) is shorter than the {halo}-row halo")
    for which in ("sample", "temporal"):
        ops, recvs = [], []
        if rank > 0 and send_up[1]:
            ops.append(dist.P2POp(dist.isend, _comm(export_rows(which, *send_up), group), rank - 1, group))
        if rank < world - 1 and send_down[1]:
            ops.append(dist.P2POp(dist.isend, _comm(export_rows(which, *send_down), group), rank + 1, group))
        for peer, (row0, nrows) in ((rank - 1, recv_up), (rank + 1, recv_down)):
            if 0 <= peer < world and nrows:
                tmpl = export_rows(which, row0, nrows)  # shape / dtype / device template
                t = torch.empty_like(_comm(tmpl, group))
                ops.append(dist.P2POp(dist.irecv, t, peer, group))
                recvs.append((row0, t, tmpl.device))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for row0, t, dev in recvs:
            import_rows(which, row0, t.to(dev))


def restir_band_frame(integ, scene, seed: int, y0: int, y1: int, exchange, spp: int = 1, out=None, ctx=None):
    """One ReSTIR GI frame for rows [y0, y1): stage A, exchange(), stage B.
    Returns the band film (rows y0-1 .. y1)."""
    integ.render_film(scene, seed=seed, spp=spp, y0=y0, y1=y1, stage="A", ctx=ctx)
    exchange()
    return integ.render_film(scene, seed=seed, spp=spp, y0=y0, y1=y1, stage="B", out=out, ctx=ctx)


def device_row_io(integ, scene, spp: int = 1, ctx=None):
    """export_rows / import_rows over mtx_restir_rows with device tensors."""
    import torch

    lanes_per_row = scene.width * spp
    dev = torch.device("cuda", (ctx.device if ctx is not None else torch.cuda.current_device()))

    def export_rows(which, row0, nrows):
        planes = 6 if which == "temporal" else 5
        t = torch.empty((planes, nrows, lanes_per_row, 4), dtype=torch.float32, device=dev)
        integ.rows(which, row0, nrows, t, to_state=False, ctx=ctx)
        return t

    def import_rows(which, row0, t):
        integ.rows(which, row0, t.shape[1], t.contiguous(), to_state=True, ctx=ctx)

    return export_rows, import_rows


def gather_prev_samples(export_rows, import_rows, y0: int, y1: int, height: int, group=None):
    """Give every rank the previous frame's samples of the whole film: each
    rank contributes its band rows [y0, y1) (what its last stage A wrote), one
    all_gather (bands padded to the tallest), then the other ranks' rows are
    imported. Temporal resampling (restirgi.py:374-383) gathers prev_sample at
    the pixel the current hit reprojects to through the previous camera; with
    a moving camera that pixel can lie in any band. Costs 80 B per lane."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    bands = row_bands(height, world)
    maxrows = max(b1 - b0 for b0, b1 in bands)
    mine = export_rows("prev_sample", y0, y1 - y0)
    dev = mine.device
    mine = _comm(mine, group)
    buf = torch.zeros((mine.shape[0], maxrows) + tuple(mine.shape[2:]), dtype=mine.dtype, device=mine.device)
    buf[:, : y1 - y0] = mine
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    for r, (b0, b1) in enumerate(bands):
        if r != rank and b1 > b0:
            import_rows("prev_sample", b0, parts[r][:, : b1 - b0].contiguous().to(dev))


def render_restir_sharded(integ, scene, seed: int, spp: int = 1, group=None):
    """Row-banded ReSTIR GI frame over torch.distributed (one rank per GPU):
    returns the stitched film on rank 0 (None elsewhere).

    Static camera: one halo exchange of ceil(initial_search_radius) rows of
    samples and temporal reservoirs between stage A and stage B. When the
    camera moved since the previous frame (test-restir-dynamic.py:25-32), the
    previous frame's samples of the whole film are gathered first
    (gather_prev_samples), so the reprojection reads the same samples as a
    single-GPU frame wherever it lands."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    y0, y1 = row_bands(scene.height, world)[rank]
    halo = restir_halo(integ)
    ex, im = device_row_io(integ, scene, spp)
    cam = bytes(scene.camera)
    if integ.n > 0 and getattr(integ, "_shard_prev_cam", cam) != cam:
        gather_prev_samples(ex, im, y0, y1, scene.height, group)
    film = restir_band_frame(integ, scene, seed, y0, y1,
                             lambda: exchange_halos(ex, im, y0, y1, scene.height, halo, group), spp)
    integ._shard_prev_cam = cam
    return gather_bands(film, y0, y1, scene.height, group)


def prefix_sum_sharded(x, inclusive: bool = True, group=None, scan=None):
    """prefix_sum.py:9-36 over a u32 array whose contiguous slices live on the
    ranks in rank order (`x` is this rank's slice, possibly empty). The local
    scan runs on this rank's GPU (`scan`, default mtx.primitives.prefix_sum);
    one all_gather of the per-rank totals gives the offset, the sum of the
    lower ranks' totals, added mod 2^32. Bit-identical to the scan of the
    concatenated array: u32 addition is associative mod 2^32. (The f32
    Hillis-Steele order is not shard-invariant and has no sharded form.)"""
    import torch
    import torch.distributed as dist

    x = np.ascontiguousarray(x, dtype=np.uint32)
    if scan is None:
        from . import primitives

        scan = primitives.prefix_sum
    local = scan(x, inclusive=inclusive) if x.size else np.zeros(0, np.uint32)
    total = 0
    if x.size:
        total = int(local[-1]) if inclusive else (int(local[-1]) + int(x[-1])) & 0xFFFFFFFF
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([total], dtype=torch.int64, device=dev)
    world = dist.get_world_size(group)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    rank = dist.get_rank(group)
    offset = sum(int(p.item()) for p in parts[:rank]) & 0xFFFFFFFF
    return (local + np.uint32(offset)).astype(np.uint32)
