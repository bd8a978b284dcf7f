"""GPU primitives with the reference's function names (prefix_sum.py,
hashgrid.py, reductions.py), backed by libmtx."""
from __future__ import annotations

import numpy as np

from ._lib import check, context, lib

ADD, MIN, MAX, MUL = 0, 1, 2, 3
_OPS = {"add": ADD, "min": MIN, "max": MAX, "mul": MUL}


def _dev_ctx(t):
    """The context of a torch CUDA tensor's device, after the tensor's
    producers on torch's stream have finished (libmtx runs on its own
    stream; its *_dev calls return with their results complete)."""
    import torch

    dev = t.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    torch.cuda.current_stream(dev).synchronize()
    return context(idx)


def prefix_sum(x, inclusive: bool = True, device: int | None = None):
    """prefix_sum.py:9-36. u32 input: single-pass decoupled look-back scan.
    f32 input: Hillis-Steele passes in the reference's exact summation order.
    A torch CUDA tensor stays in HBM (mtx_prefix_sum_*_dev: no host copy;
    u32 data as torch.int32 / torch.uint32 bits) and the result is one."""
    if _torch_cuda(x):
        import torch

        t = x.contiguous()
        out = torch.empty_like(t)
        if len(t) == 0:
            return out
        ctx = _dev_ctx(t)
        if t.dtype in (torch.int32, getattr(torch, "uint32", torch.int32)):
            check(lib().mtx_prefix_sum_u32_dev(ctx.handle, t.data_ptr(), out.data_ptr(), len(t), int(inclusive)),
                  "mtx_prefix_sum_u32_dev")
        elif t.dtype == torch.float32:
            if not inclusive:
                raise ValueError("the Hillis-Steele f32 scan is inclusive (prefix_sum.py:25-32)")
            check(lib().mtx_prefix_sum_f32_hs_dev(ctx.handle, t.data_ptr(), out.data_ptr(), len(t)),
                  "mtx_prefix_sum_f32_hs_dev")
        else:
            raise TypeError("prefix_sum supports uint32 (int32 bits) and float32 tensors")
        return out
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    ctx = context(device)
    if x.dtype == np.uint32:
        check(lib().mtx_prefix_sum_u32(ctx.handle, x.ctypes.data, out.ctypes.data, len(x), int(inclusive)),
              "mtx_prefix_sum_u32")
    elif x.dtype == np.float32:
        if not inclusive:
            raise ValueError("the Hillis-Steele f32 scan is inclusive (prefix_sum.py:25-32)")
        check(lib().mtx_prefix_sum_f32_hs(ctx.handle, x.ctypes.data, out.ctypes.data, len(x)), "mtx_prefix_sum_f32_hs")
    else:
        raise TypeError("prefix_sum supports uint32 and float32")
    return out


def hash_cells(p, resolution: int, n_cells: int):
    """hashgrid.py:8-12 + 86-90 on the host (small inputs / documentation)."""
    p = np.asarray(p, np.float32).reshape(3, -1)
    bbmin = np.float32(min(p[0].min(), p[1].min(), p[2].min()))
    bbmax = np.float32(max(p[0].max(), p[1].max(), p[2].max()))
    q = ((p - bbmin) / (bbmax - bbmin) * np.float32(resolution)).astype(np.uint32)
    with np.errstate(over="ignore"):
        h = (q[0] * np.uint32(73856093)) ^ (q[1] * np.uint32(19349663)) ^ (q[2] * np.uint32(83492791))
    return h % np.uint32(n_cells)


class HashGrid:
    """hashgrid.py:15-90: build a 3-D spatial hash grid over `sample` points
    (Point3f as a [3, n] array). Attributes: cell_size, cell_offset (exclusive
    scan), sample_idx (samples grouped by cell, ascending sample index within
    a cell: one of the orders the reference's race-defined election can
    produce, and a deterministic one), cell (per-sample cell index)."""

    def __init__(self, sample, resolution: int, n_cells: int | None = None, device: int | None = None):
        if _torch_cuda(sample):  # a [3, n] float32 tensor in HBM: mtx_hashgrid_build_dev, int32 results there
            import torch

            p = sample.to(torch.float32).reshape(3, -1).contiguous()
            n = p.shape[1]
            self.n_samples, self.resolution = n, int(resolution)
            self.n_cells = int(n_cells if n_cells is not None else n)
            kw = {"dtype": torch.int32, "device": p.device}
            self.cell, self.sample_idx = torch.empty(n, **kw), torch.empty(n, **kw)
            self.cell_size, self.cell_offset = torch.empty(self.n_cells, **kw), torch.empty(self.n_cells, **kw)
            ctx = _dev_ctx(p)
            check(lib().mtx_hashgrid_build_dev(ctx.handle, p.data_ptr(), n, self.resolution, self.n_cells,
                                               self.cell.data_ptr(), self.cell_size.data_ptr(),
                                               self.cell_offset.data_ptr(), self.sample_idx.data_ptr()),
                  "mtx_hashgrid_build_dev")
            return
        p = np.ascontiguousarray(np.asarray(sample, np.float32).reshape(3, -1))
        n = p.shape[1]
        self.n_samples = n
        self.n_cells = int(n_cells if n_cells is not None else n)
        self.resolution = int(resolution)
        self.cell = np.zeros(n, np.uint32)
        self.cell_size = np.zeros(self.n_cells, np.uint32)
        self.cell_offset = np.zeros(self.n_cells, np.uint32)
        self.sample_idx = np.zeros(n, np.uint32)
        ctx = context(device)
        check(lib().mtx_hashgrid_build(ctx.handle, p.ctypes.data, n, self.resolution, self.n_cells,
                                       self.cell.ctypes.data, self.cell_size.ctypes.data,
                                       self.cell_offset.ctypes.data, self.sample_idx.ctypes.data),
              "mtx_hashgrid_build")


def group_by(keys, n_keys: int, device: int | None = None):
    """The stable device group-by behind HashGrid and scatter_reduce_with:
    (key_size, key_offset exclusive, order) with order[key_offset[k] + j] the
    j-th element of key k in ascending element index (mtx_group_by_u32)."""
    k = np.ascontiguousarray(keys, np.uint32)
    n_keys = int(n_keys)
    size = np.zeros(n_keys, np.uint32)
    offset = np.zeros(n_keys, np.uint32)
    order = np.zeros(len(k), np.uint32)
    if len(k):
        ctx = context(device)
        check(lib().mtx_group_by_u32(ctx.handle, k.ctypes.data, len(k), n_keys, size.ctypes.data, offset.ctypes.data,
                                     order.ctypes.data), "mtx_group_by_u32")
    return size, offset, order


def fold_rounds(func, target, value, size, offset, order):
    """reductions.py:21-54's loop with a deterministic election: round r
    applies `func(a, b)` once, vectorised, to every target that has more
    than r values, with a = its current value and b = its r-th value in
    ascending index (the reference elects an arbitrary one per round). Works
    on numpy arrays; func sees arrays, as the reference's sees Dr.Jit ones.
    Host cost: one vectorised numpy round per value of the largest group (a
    skewed index costs that many rounds, as the reference's loop does)."""
    t = np.array(target, copy=True)
    v = np.asarray(value)
    size = np.asarray(size, np.int64)
    offset = np.asarray(offset, np.int64)
    order = np.asarray(order, np.int64)
    rounds = int(size.max()) if len(size) else 0
    for r in range(rounds):
        sel = np.nonzero(size > r)[0]
        res = np.asarray(func(t[sel], v[order[offset[sel] + r]]))
        t[sel] = res
    return t


def _torch_cuda(x) -> bool:
    import sys

    torch = sys.modules.get("torch")
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def group_by_device(keys, n_keys: int):
    """group_by on a torch tensor in HBM (mtx_group_by_u32_dev): returns
    (key_size, key_offset, order) as int32 tensors on the keys' device, with
    no host copy of the data (keys < 2^31)."""
    import torch

    k = keys.to(torch.int32).contiguous()
    dev = k.device
    n_keys = int(n_keys)
    size = torch.empty(n_keys, dtype=torch.int32, device=dev)
    offset = torch.empty(n_keys, dtype=torch.int32, device=dev)
    order = torch.empty(len(k), dtype=torch.int32, device=dev)
    if len(k):
        ctx = context(dev.index if dev.index is not None else torch.cuda.current_device())
        torch.cuda.synchronize(dev)  # libmtx runs on its own stream: the keys must be complete
        check(lib().mtx_group_by_u32_dev(ctx.handle, k.data_ptr(), len(k), n_keys, size.data_ptr(),
                                         offset.data_ptr(), order.data_ptr()), "mtx_group_by_u32_dev")
    else:
        size.zero_()
        offset.zero_()
    return size, offset, order


def fold_rounds_device(func, target, value, size, offset, order):
    """fold_rounds with torch tensors on the device: func(a, b) runs on HBM
    arrays (torch ops) as the reference's runs inside its Dr.Jit loop
    (reductions.py:23-54). Targets are ordered by their value count, largest
    first, so round r updates the first cnt[r] of them; the only host reads
    are the round count and the per-round counts (one small copy)."""
    import torch

    t = target.clone()
    sz = size.to(torch.int64)
    rounds = int(sz.max().item()) if len(sz) else 0
    if rounds == 0:
        return t
    _, tid = torch.sort(sz, descending=True, stable=True)
    hist = torch.bincount(sz, minlength=rounds + 1)
    at_least = hist.flip(0).cumsum(0).flip(0)  # at_least[k] = #targets with >= k values
    cnt = at_least[1:rounds + 1].cpu().tolist()
    off = offset.to(torch.int64)[tid]
    ordr = order.to(torch.int64)
    for r in range(rounds):
        m = int(cnt[r])
        sel = tid[:m]
        t[sel] = func(t[sel], value[ordr[off[:m] + r]])
    return t


def scatter_reduce_with(op, target, value, index, device: int | None = None):
    """reductions.py:12-54. func in {'add', 'min', 'max', 'mul'} (or ADD, MIN,
    MAX, MUL): one device pass, each target receiving its values in ascending
    index order (f32). Any other callable `func(a, b)` (the reference accepts
    any, :12, :53): the device groups the values by target (group_by) and the
    callable is folded round by round, the reference's structure with one
    deterministic election per round -- on the device when target / value /
    index are torch tensors in HBM (group_by_device + fold_rounds_device:
    func sees device tensors, nothing goes through the host), else on the host
    over numpy arrays of any dtype func handles."""
    if len(value) != len(index):
        raise ValueError(f"scatter_reduce_with: {len(value)} values for {len(index)} indices")
    on_device = any(_torch_cuda(x) for x in (target, value, index))
    if isinstance(op, str):
        if op not in _OPS:
            raise TypeError(f"scatter_reduce_with: unknown func {op!r} (device ops: add, min, max, mul)")
        op = _OPS[op]
    elif callable(op):
        if on_device:
            import torch

            dev = next(x.device for x in (target, value, index) if _torch_cuda(x))
            tgt = torch.as_tensor(target, device=dev)
            val = torch.as_tensor(value, device=dev)
            idx = torch.as_tensor(index, device=dev).to(torch.int64)
            if len(idx) and (int(idx.min().item()) < 0 or int(idx.max().item()) >= len(tgt)):
                raise ValueError("scatter_reduce_with: index out of range")
            size, offset, order = group_by_device(idx, len(tgt))
            return fold_rounds_device(op, tgt, val, size, offset, order)
        idx = np.ascontiguousarray(index, np.uint32)
        tgt = np.asarray(target)
        if len(idx) and int(idx.max()) >= len(tgt):
            raise ValueError("scatter_reduce_with: index out of range")
        size, offset, order = group_by(idx, len(tgt), device)
        return fold_rounds(op, tgt, value, size, offset, order)
    if on_device:
        # the fixed ops on HBM tensors (mtx_scatter_reduce_f32_dev): no host copy
        import torch

        dev = next(x.device for x in (target, value, index) if _torch_cuda(x))
        t = torch.as_tensor(target, device=dev).to(torch.float32).clone().contiguous()
        v = torch.as_tensor(value, device=dev).to(torch.float32).contiguous()
        i = torch.as_tensor(index, device=dev)
        if i.dtype not in (torch.int32, getattr(torch, "uint32", torch.int32)):
            if len(i) and int(i.min().item()) < 0:
                raise ValueError("scatter_reduce_with: index out of range")
            i = i.to(torch.int32)
        i = i.contiguous()
        if len(v) and len(t):
            ctx = _dev_ctx(t)
            check(lib().mtx_scatter_reduce_f32_dev(ctx.handle, int(op), t.data_ptr(), len(t), v.data_ptr(),
                                                   i.data_ptr(), len(v)), "mtx_scatter_reduce_f32_dev")
        return t
    t = np.array(target, np.float32)
    v = np.ascontiguousarray(value, np.float32)
    i = np.ascontiguousarray(index, np.uint32)
    ctx = context(device)
    check(lib().mtx_scatter_reduce_f32(ctx.handle, int(op), t.ctypes.data, len(t), v.ctypes.data, i.ctypes.data,
                                       len(v)), "mtx_scatter_reduce_f32")
    return t
