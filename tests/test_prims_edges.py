"""Edge cases of the GPU primitives (prefix_sum.py, hashgrid.py,
reductions.py): empty inputs, sizes one past a power of two, a single hot
target / cell, hash collisions, points on the bounding-box maximum, invalid
arguments. HIP results are compared with the oracle or exact numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_prefix_sum_empty_and_sizes():
    from mtx import primitives

    assert primitives.prefix_sum(np.zeros(0, np.uint32)).size == 0
    assert primitives.prefix_sum(np.zeros(0, np.float32)).size == 0
    for n in (2, 63, 64, 65, (1 << 20) + 1):
        x = np.arange(n, dtype=np.uint32) % 7
        assert np.array_equal(primitives.prefix_sum(x), np.cumsum(x, dtype=np.uint64).astype(np.uint32))


def test_prefix_sum_f32_power_of_two_boundaries(oracle):
    from mtx import primitives

    for n in (2047, 2048, 2049, (1 << 20) + 1):
        x = oracle.rng_stream(3, 0, n, 1)[:, 0].copy()
        assert np.array_equal(primitives.prefix_sum(x), oracle.prefix_sum_f32_hs(x))


def test_prefix_sum_rejects_exclusive_f32_and_other_dtypes():
    from mtx import primitives

    with pytest.raises(ValueError):
        primitives.prefix_sum(np.ones(4, np.float32), inclusive=False)
    with pytest.raises(TypeError):
        primitives.prefix_sum(np.ones(4, np.int64))


def _grid_vs_oracle(oracle, p, res, n_cells):
    from mtx import primitives

    n = p.shape[1]
    g = primitives.HashGrid(p, res, n_cells)
    cell, size, off, idx = oracle.hashgrid(p, res, n_cells)
    assert np.array_equal(g.cell, cell)
    assert np.array_equal(g.cell_size, size)
    assert np.array_equal(g.cell_offset, off)
    order = np.lexsort((g.sample_idx, np.repeat(np.arange(n_cells), size)))
    assert np.array_equal(g.sample_idx[order], idx)
    assert int(size.sum()) == n
    return g


def test_hashgrid_single_cell_collisions_and_bbox_max(oracle):
    rng = np.random.default_rng(11)
    p = rng.random((3, 5000), dtype=np.float32)
    # every sample in one cell (maximal contention on one counter)
    g = _grid_vs_oracle(oracle, p, 100, 1)
    assert g.cell_size.tolist() == [5000]
    # fewer cells than occupied grid cells: hash collisions
    _grid_vs_oracle(oracle, p, 100, 97)
    # samples exactly on the bounding-box maximum (q = resolution)
    p[:, :100] = p.max()
    _grid_vs_oracle(oracle, p, 16, 4096)


def test_hashgrid_rejects_empty():
    from mtx import MtxError, primitives

    with pytest.raises(MtxError):
        primitives.HashGrid(np.zeros((3, 0), np.float32), 10, 4)
    with pytest.raises(MtxError):
        primitives.HashGrid(np.random.default_rng(0).random((3, 10), dtype=np.float32), 10, 0)


@pytest.mark.parametrize("op", ["add", "min", "max"])
def test_scatter_reduce_one_hot_target(oracle, op):
    """Every value into target 0: one long ordered fold (ascending index)."""
    from mtx import primitives

    rng = np.random.default_rng(12)
    nv = 1 << 16
    val = rng.random(nv, dtype=np.float32) - 0.5
    idx = np.zeros(nv, np.uint32)
    tgt = rng.random(8, dtype=np.float32)
    o = {"add": 0, "min": 1, "max": 2}[op]
    g = primitives.scatter_reduce_with(op, tgt, val, idx)
    assert np.array_equal(g, oracle.scatter_reduce(o, tgt, val, idx))
    assert np.array_equal(g[1:], tgt[1:])
    if op == "add":  # left fold in ascending index order, as the oracle
        acc = np.float32(tgt[0])
        for v in val:
            acc = np.float32(acc + v)
        assert g[0] == acc


def test_scatter_reduce_empty_and_invalid():
    from mtx import MtxError, primitives

    t = np.arange(5, dtype=np.float32)
    assert np.array_equal(primitives.scatter_reduce_with("add", t, np.zeros(0, np.float32),
                                                         np.zeros(0, np.uint32)), t)
    with pytest.raises(MtxError):
        primitives.scatter_reduce_with("add", t, np.ones(3, np.float32), np.array([0, 5, 1], np.uint32))


def test_hashgrid_wide_keys_lsd_path(oracle):
    """n_cells >= 2^25: the LSD passes of the multisplit (12-bit digits) and
    the run-bounds kernels (dense: k_hash_ranges; sparse: lower bounds)."""
    rng = np.random.default_rng(13)
    p = rng.random((3, 1 << 23), dtype=np.float32)
    _grid_vs_oracle(oracle, p, 400, (1 << 25) + 3)  # n_cells <= 4 n: run bounds
    _grid_vs_oracle(oracle, np.ascontiguousarray(p[:, :1 << 16]), 100, (1 << 25) + 3)  # sparse


@pytest.mark.parametrize("n_cells", [1 << 12, (1 << 12) + 1, 5000, 1 << 20])
def test_hashgrid_digit_splits_clustered(oracle, n_cells):
    """Every top/local digit split of the two-level path (local bits 0, 1, 1,
    8) with clustered points: a few cells hold most samples, so single
    buckets span many tiles and one workgroup's waves split a long run."""
    rng = np.random.default_rng(14)
    n = (1 << 20) + 77
    q = (rng.integers(0, 6, (3, n)) / 6.0).astype(np.float32)
    q[:, : n // 3] = rng.random((3, n // 3), dtype=np.float32)
    _grid_vs_oracle(oracle, q, 64, n_cells)


@pytest.mark.parametrize("nt", [1, 3000, 1 << 16, (1 << 25) + 1])
def test_scatter_reduce_paths_and_mul(oracle, nt):
    """Targets below 2^12 (one key per bucket), the two-level path and the
    LSD path (2^25 + 1 targets); add / min / max / mul folded in ascending
    index order, bit-exact vs the oracle."""
    from mtx import primitives

    rng = np.random.default_rng(15)
    nv = (1 << 20) + 5
    idx = (rng.integers(0, nt, nv) if nt > 1 else np.zeros(nv)).astype(np.uint32)
    idx[: nv // 4] = idx[0]  # one hot target
    for op in ("add", "min", "max", "mul"):
        val = (rng.random(nv, dtype=np.float32) * (0.02 if op == "mul" else 1.0)
               + (0.99 if op == "mul" else -0.5)).astype(np.float32)
        tgt = rng.random(nt, dtype=np.float32)
        o = {"add": 0, "min": 1, "max": 2, "mul": 3}[op]
        assert np.array_equal(primitives.scatter_reduce_with(op, tgt, val, idx),
                              oracle.scatter_reduce(o, tgt, val, idx)), op


def test_groupby_ballot_fallback_matches(tmp_path):
    """The ballot-match kernels (MTX_LDS_RANK=0: used when the one-time check
    of lane-ordered LDS atomic returns fails) give the same bits as the
    default kernels; run in a fresh process so the per-device choice is new."""
    import subprocess
    import sys

    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from mtx import primitives
rng = np.random.default_rng(31)
p = rng.random((3, (1 << 20) + 3), dtype=np.float32)
g = primitives.HashGrid(p, 100, 1 << 20)
idx = rng.integers(0, 1 << 12, 1 << 20).astype(np.uint32)
val = rng.random(1 << 20, dtype=np.float32)
t = primitives.scatter_reduce_with("add", np.zeros(1 << 12, np.float32), val, idx)
np.savez(sys.argv[2], cell=g.cell, size=g.cell_size, off=g.cell_offset, idx=g.sample_idx, t=t)
'''
    import os

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mitsuba3-experiments_amd")
    outs = []
    for flag in ("1", "0"):
        f = tmp_path / f"r{flag}.npz"
        env = dict(os.environ, MTX_LDS_RANK=flag)
        subprocess.run([sys.executable, "-c", code, pkg, str(f)], check=True, env=env, timeout=300)
        outs.append(np.load(f))
    for k in ("cell", "size", "off", "idx", "t"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("n,n_keys", [(1, 1), (100003, 97), (1 << 20, 1 << 20), (200000, 1 << 26)])
def test_group_by_matches_stable_sort(n, n_keys):
    """mtx_group_by_u32 (the hash grid's stable group-by on caller keys; the
    LSD multisplit path for n_keys >= 2^25): sizes, exclusive offsets and the
    order equal numpy's stable argsort."""
    from mtx import primitives

    rng = np.random.default_rng(n)
    k = rng.integers(0, n_keys, n, dtype=np.uint64).astype(np.uint32)
    size, offset, order = primitives.group_by(k, n_keys)
    assert np.array_equal(order, np.argsort(k, kind="stable"))
    ref = np.bincount(k, minlength=n_keys)
    assert np.array_equal(size, ref) and np.array_equal(offset, np.cumsum(ref) - ref)


def test_scatter_reduce_with_callable_on_device_grouping():
    """reductions.py:12-54 with a Python func (here order-dependent, integer
    dtype): the device groups by target, the func is folded round by round
    (ascending index per target) -- equal to the sequential loop; the
    reference's KAT (reductions.py:57-63)."""
    from mtx import primitives

    idx = (np.arange(25) % 10).astype(np.uint32)
    t = primitives.scatter_reduce_with(lambda a, b: a + b, np.zeros(10, np.float32), np.ones(25, np.float32), idx)
    assert np.array_equal(t, np.array([3] * 5 + [2] * 5, np.float32))
    rng = np.random.default_rng(9)
    idx = rng.integers(0, 1000, 50000).astype(np.uint32)
    val = rng.integers(-9, 9, 50000).astype(np.int64)
    tgt = rng.integers(-5, 5, 1200).astype(np.int64)
    ref = tgt.copy()
    for i, v in zip(idx, val):
        ref[i] = (3 * ref[i] - v) % 1000003
    got = primitives.scatter_reduce_with(lambda a, b: (3 * a - b) % 1000003, tgt, val, idx)
    assert np.array_equal(got, ref)


def test_scatter_reduce_with_callable_in_hbm():
    """reductions.py:12-54 with a Python func on torch tensors in HBM: the
    grouping is mtx_group_by_u32_dev (device pointers, no host copy of the
    data) and func runs on device tensors round by round, as the reference's
    runs inside its Dr.Jit loop -- equal to the sequential loop, the KAT
    (reductions.py:57-63), a skewed index, and out-of-range keys rejected."""
    import torch

    from mtx import primitives

    dev = torch.device("cuda", 0)
    idx = torch.arange(25, device=dev) % 10
    t = primitives.scatter_reduce_with(lambda a, b: a + b, torch.zeros(10, device=dev), torch.ones(25, device=dev),
                                       idx)
    assert t.is_cuda and torch.equal(t.cpu(), torch.tensor([3.0] * 5 + [2.0] * 5))
    rng = np.random.default_rng(11)
    for n_t, skew in ((1200, False), (300, True)):
        idx_np = rng.integers(0, n_t, 60000).astype(np.int64)
        if skew:
            idx_np[: 20000] = 7  # one target takes a third of the values
        val_np = rng.integers(-9, 9, 60000).astype(np.int64)
        tgt_np = rng.integers(-5, 5, n_t).astype(np.int64)
        ref = tgt_np.copy()
        for i, v in zip(idx_np, val_np):
            ref[i] = (3 * ref[i] - v) % 1000003
        got = primitives.scatter_reduce_with(lambda a, b: (3 * a - b) % 1000003, torch.as_tensor(tgt_np, device=dev),
                                             torch.as_tensor(val_np, device=dev), torch.as_tensor(idx_np, device=dev))
        assert got.is_cuda and np.array_equal(got.cpu().numpy(), ref)
    # the device group-by itself equals numpy's stable argsort
    k = torch.as_tensor(rng.integers(0, 5000, 1 << 20), device=dev)
    size, offset, order = primitives.group_by_device(k, 5000)
    kn = k.cpu().numpy()
    assert np.array_equal(order.cpu().numpy(), np.argsort(kn, kind="stable"))
    assert np.array_equal(size.cpu().numpy(), np.bincount(kn, minlength=5000))
    with pytest.raises(Exception):
        primitives.group_by_device(torch.tensor([1, 2, 5000], device=dev), 5000)
