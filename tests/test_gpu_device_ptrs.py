"""Device-pointer boundary (SURVEY §8b mtx_device_ptrs): the reference calls
sample(), Scene.ray_intersect / ray_test and its primitives on wavefront-wide
Dr.Jit arrays that live on the GPU (path.py:194-202, path-mis.py:69-71,
prefix_sum.py:9-36, hashgrid.py:16-84, reductions.py:12-54). Torch CUDA
tensors go through the *_dev entry points of include/mtx.h and stay in HBM;
every result is compared bit for bit with the CPU oracle. While the device
calls run, Tensor.cpu / Tensor.numpy are made to raise: nothing goes through
the host in between."""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def no_host_copies():
    import torch

    saved = torch.Tensor.cpu, torch.Tensor.numpy

    def boom(*a, **k):
        raise AssertionError("host copy inside a device-pointer call")

    torch.Tensor.cpu = boom
    torch.Tensor.numpy = boom
    try:
        yield
    finally:
        torch.Tensor.cpu, torch.Tensor.numpy = saved


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("n", [1, 1000, (1 << 20) + 3])
def test_prefix_sum_dev(oracle, n):
    import torch

    from mtx import primitives

    rng = np.random.default_rng(n)
    x = rng.integers(0, 1 << 31, n, dtype=np.uint32)
    xt = torch.as_tensor(x.view(np.int32), device="cuda")
    f = rng.random(n).astype(np.float32)
    ft = torch.as_tensor(f, device="cuda")
    with no_host_copies():
        inc = primitives.prefix_sum(xt, inclusive=True)
        exc = primitives.prefix_sum(xt, inclusive=False)
        hs = primitives.prefix_sum(ft)
    assert inc.is_cuda and hs.is_cuda
    np.testing.assert_array_equal(_np(inc).view(np.uint32), oracle.prefix_sum_u32(x, True))
    np.testing.assert_array_equal(_np(exc).view(np.uint32), oracle.prefix_sum_u32(x, False))
    np.testing.assert_array_equal(_np(hs), oracle.prefix_sum_f32_hs(f))
    np.testing.assert_array_equal(_np(ft), f)  # the input is not clobbered


@pytest.mark.parametrize("n,res,cells", [(1000, 8, 1000), (1 << 20, 64, 1 << 18)])
def test_hashgrid_dev(oracle, n, res, cells):
    import torch

    from mtx import primitives

    p = np.random.default_rng(7).random((3, n)).astype(np.float32)
    with no_host_copies():
        g = primitives.HashGrid(torch.as_tensor(p, device="cuda"), res, cells)
    c_cell, c_size, c_off, c_idx = oracle.hashgrid(p, res, cells)
    for got, ref in ((g.cell, c_cell), (g.cell_size, c_size), (g.cell_offset, c_off), (g.sample_idx, c_idx)):
        assert got.is_cuda
        np.testing.assert_array_equal(_np(got).view(np.uint32), ref)


@pytest.mark.parametrize("op", ["add", "min", "max", "mul"])
def test_scatter_reduce_dev(oracle, op):
    import torch

    from mtx import MtxError, primitives

    rng = np.random.default_rng(3)
    n_t, n_v = 5000, 200000
    target = rng.random(n_t).astype(np.float32)
    value = (rng.random(n_v) * 2).astype(np.float32)
    index = rng.integers(0, n_t, n_v).astype(np.uint32)
    t, v, i = (torch.as_tensor(a, device="cuda") for a in (target, value, index.view(np.int32)))
    with no_host_copies():
        out = primitives.scatter_reduce_with(op, t, v, i)
    assert out.is_cuda
    np.testing.assert_array_equal(_np(out), oracle.scatter_reduce(primitives._OPS[op], target, value, index))
    np.testing.assert_array_equal(_np(t), target)  # the caller's target is not modified
    bad = i.clone()
    bad[17] = n_t
    with pytest.raises(MtxError, match="index"):
        primitives.scatter_reduce_with(op, t, v, bad)


def test_trace_dev(small_scene, oracle):
    import torch

    from mtx import trace_rays

    rng = np.random.default_rng(5)
    n = 40000
    v = np.asarray(small_scene.vpos).reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    o = lo + (hi - lo) * rng.random((n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, :3], rays[:, 4:7] = o, d
    rays[:, 3] = np.float32(3.0e38)
    rays[::3, 3] = np.float32(0.5)
    rt = torch.as_tensor(rays, device="cuda")
    with no_host_copies():
        hits, vis = trace_rays(small_scene, rt, visits=True)
        occ, ovis = trace_rays(small_scene, rt, any_hit=True, visits=True)
    c_hits, c_vis = oracle.trace(small_scene, rays, False)
    np.testing.assert_array_equal(_np(hits).view(np.uint32).reshape(-1), c_hits)
    np.testing.assert_array_equal(_np(vis).view(np.uint32), c_vis)
    c_any, c_ovis = oracle.trace(small_scene, rays, True)
    np.testing.assert_array_equal(_np(occ).view(np.uint32), c_any)
    np.testing.assert_array_equal(_np(ovis).view(np.uint32), c_ovis)
    # the numpy route gives the same words
    np.testing.assert_array_equal(trace_rays(small_scene, rays).reshape(-1), c_hits)


@pytest.mark.parametrize("name", ["path_test", "mypath", "nrc"])
def test_sample_dev(small_scene, oracle, name):
    """sample(scene, sampler, ray) with the wavefront in HBM (a ray object
    with Dr.Jit-layout (3, N) fields): L and valid are device tensors equal to
    the oracle's lanes."""
    import types

    import torch

    from mtx import IndependentSampler, load_dict

    integ = load_dict({"type": name})
    rng = np.random.default_rng(11)
    n = 5000
    cam = small_scene.camera
    o = np.tile(np.asarray(cam.origin, np.float32), (n, 1))
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    lanes = np.arange(n, dtype=np.uint32) * 3 + 1
    ray = types.SimpleNamespace(o=torch.as_tensor(o.T.copy(), device="cuda"),
                                d=torch.as_tensor(d.T.copy(), device="cuda"))
    sampler = IndependentSampler(seed=9, lanes=lanes, skip=2)
    with no_host_copies():
        L, valid, aov = integ.sample(small_scene, sampler, ray)
    assert L.is_cuda and valid.is_cuda and aov == []
    cL, cv = oracle.sample_rays(small_scene, integ.render_args(small_scene, 9, 1),
                                np.concatenate([o, d], 1), lanes, rng_skip=2)
    np.testing.assert_array_equal(_np(L), cL)
    np.testing.assert_array_equal(_np(valid), cv.astype(bool))


def test_dev_entry_points_refuse_host_memory(small_scene):
    import ctypes as C

    from mtx import context, lib, trace_rays  # noqa: F401

    ctx = context()
    x = np.arange(10, dtype=np.uint32)
    out = np.zeros_like(x)
    rc = lib().mtx_prefix_sum_u32_dev(ctx.handle, x.ctypes.data, out.ctypes.data, 10, 1)
    assert rc != 0 and b"not device memory" in lib().mtx_last_error()
    trace_rays(small_scene, np.zeros((1, 8), np.float32))  # binds the scene
    r = np.zeros((4, 8), np.float32)
    h = np.zeros(16, np.uint32)
    assert lib().mtx_trace_dev(ctx.handle, 4, r.ctypes.data, 0, h.ctypes.data, C.c_void_p()) != 0
