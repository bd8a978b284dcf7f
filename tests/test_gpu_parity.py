"""HIP path vs the CPU restatement (oracle/) on identical inputs.

Integer / index outputs (hit prim ids, visit counts, hash cells, scan
results) must match exactly. Floating-point outputs of the path tracer are
compared bit for bit as well: both sides evaluate the same IEEE operation
sequence (-ffp-contract=off, correctly rounded division/sqrt, deterministic
transcendentals), so the stated per-pixel tolerance of north_star is 0 for
lane radiance and for the single-device film; only results that change the
floating-point summation order (row bands, rank shards) use a relative
tolerance, written in the test.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INTEGRATORS = ["path_test", "mypath", "nrc", "integrator"]


def _ctx():
    from mtx import context

    return context(0)


def _camera_rays(scene, n, seed=0):
    """Camera rays through random film positions + random rays inside the room."""
    rng = np.random.default_rng(seed)
    cam = scene.camera
    W, H = scene.width, scene.height
    pos = rng.random((n, 2)).astype(np.float32)
    tx, ty = np.float32(cam.tan_x), np.float32(cam.tan_y)
    dl = np.stack([(1 - 2 * pos[:, 0]) * tx, (1 - 2 * pos[:, 1]) * ty, np.ones(n, np.float32)], 1)
    dl /= np.linalg.norm(dl, axis=1, keepdims=True)
    M = np.stack([np.array(cam.axis_x), np.array(cam.axis_y), np.array(cam.axis_z)], 1).astype(np.float32)
    d = dl @ M.T
    o = np.tile(np.array(cam.origin, np.float32), (n, 1))
    # second half: random origins inside the room, random directions
    h = n // 2
    o[h:] = rng.uniform([-3.0, 0.05, -1.2], [3.8, 2.6, 3.6], (n - h, 3)).astype(np.float32)
    v = rng.normal(size=(n - h, 3)).astype(np.float32)
    d[h:] = v / np.linalg.norm(v, axis=1, keepdims=True)
    return o.astype(np.float32), d.astype(np.float32)


def _trace_gpu(scene, rays, any_hit):
    from mtx import integrators
    from mtx._lib import check, lib

    ctx = _ctx()
    integrators._bind_scene(ctx, scene)
    n = len(rays)
    hits = np.zeros(n if int(any_hit) == 1 else 4 * n, np.uint32)  # any_hit 2: closest hit, 8-wide tree
    visits = np.zeros(2 * n, np.uint32)
    r = np.ascontiguousarray(rays, np.float32)
    check(lib().mtx_trace(ctx.handle, n, r.ctypes.data, int(any_hit), hits.ctypes.data, visits.ctypes.data),
          "mtx_trace")
    return hits, visits.reshape(n, 2)


def test_trace_closest_and_any_hit_bit_exact(small_scene, oracle):
    o, d = _camera_rays(small_scene, 4096)
    rays = np.zeros((len(o), 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = o, d
    rays[:, 3] = np.float32(3.0e38)
    rays[::7, 3] = np.float32(1.5)  # some bounded rays
    g_hits, g_vis = _trace_gpu(small_scene, rays, False)
    c_hits, c_vis = oracle.trace(small_scene, rays, False)
    assert np.array_equal(g_hits, c_hits)
    assert np.array_equal(g_vis, c_vis)
    b_hits, _ = oracle.trace(small_scene, rays, False, brute=True)
    # the BVH finds exactly the brute-force closest hit (prim, t, u, v)
    assert np.array_equal(c_hits, b_hits)
    prim = g_hits.reshape(-1, 4)[:, 1]
    assert (prim != 0xFFFFFFFF).mean() > 0.9
    g_any, g_vis2 = _trace_gpu(small_scene, rays, True)
    c_any, c_vis2 = oracle.trace(small_scene, rays, True)
    assert np.array_equal(g_any, c_any)
    assert np.array_equal(g_vis2, c_vis2)


def test_upload_builds_the_occlusion_tree_when_absent(small_scene, oracle):
    """A scene desc without the occlusion BVH (occ_nodes = NULL, the C ABI's
    drop-in case): mtx_scene_upload builds it from tri_geom with the same
    builder, so any-hit answers and visit counts equal the oracle's on the
    Python-built tree."""
    import copy

    sc = copy.copy(small_scene)
    full = sc.desc

    def desc():
        d = full()
        d.occ_nodes, d.occ_tri_geom, d.n_occ_nodes = None, None, 0
        return d

    sc.desc = desc
    o, d = _camera_rays(small_scene, 2048, seed=4)
    rays = np.zeros((len(o), 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = o, d
    rays[:, 3] = np.float32(3.0e38)
    rays[1::3, 3] = np.float32(0.7)
    g_any, g_vis = _trace_gpu(sc, rays, True)
    c_any, c_vis = oracle.trace(small_scene, rays, True)
    assert np.array_equal(g_any, c_any) and np.array_equal(g_vis, c_vis)


@pytest.mark.parametrize("name", INTEGRATORS)
def test_sample_rays_bit_exact(small_scene, oracle, name):
    from mtx import IndependentSampler, load_dict

    integ = load_dict({"type": name})
    o, d = _camera_rays(small_scene, 3000, seed=1)
    lanes = np.arange(len(o), dtype=np.uint32) * 7 + 3
    sampler = IndependentSampler(5, lanes, skip=2)
    L, valid, _ = integ.sample(small_scene, sampler, (o, d))
    a = integ.render_args(small_scene, 5, 1)
    rays = np.concatenate([o, d], 1)
    Lc, vc = oracle.sample_rays(small_scene, a, rays, lanes, 2)
    assert np.array_equal(valid, vc.astype(bool))
    np.testing.assert_array_equal(L, Lc)
    assert np.isfinite(L).all() and (L > 0).any()
    if name == "path_test":
        # the RayDifferential3f form of path-mis.py:24-31 (fields .o / .d in
        # Dr.Jit's (3, N) layout) gives the same lanes
        class Ray:
            pass

        r = Ray()
        r.o, r.d = o.T.copy(), d.T.copy()
        L2, valid2, _ = integ.sample(small_scene, IndependentSampler(5, lanes, skip=2), r)
        assert np.array_equal(L2, L) and np.array_equal(valid2, valid)


@pytest.mark.parametrize("name", INTEGRATORS)
def test_render_film_bit_exact(small_scene, oracle, name):
    from mtx import load_dict

    integ = load_dict({"type": name, "max_depth": 6} if name != "nrc" else {"type": name})
    spp = 4
    # a small wavefront forces several chunks (chunk boundaries inside rows)
    film = integ.render_film(small_scene, seed=3, spp=spp, chunk_paths=1000)
    a = integ.render_args(small_scene, 3, spp)
    ref = oracle.render(small_scene, a)
    np.testing.assert_array_equal(film, ref)
    assert film[..., 3].sum() > 0


@pytest.mark.parametrize("name", ["path_test", "mypath", "nrc"])
def test_two_stream_chunks_bit_exact(small_scene, oracle, name):
    """Renders of >= 2^16 paths alternate their chunks between two wavefronts
    on two HIP streams (api.cpp Wave2): 7 chunks of 5 rows (boundaries inside
    the sample range of no pixel, an odd count, a short last chunk) give the
    oracle's film bit for bit, as does the default two-chunk split."""
    from mtx import load_dict

    integ = load_dict({"type": name, "max_depth": 6} if name != "nrc" else {"type": name})
    spp = 32  # 64 x 36 x 32 = 73,728 paths
    a = integ.render_args(small_scene, 7, spp)
    ref = oracle.render(small_scene, a)
    for chunk in (64 * 5 * spp, 0):
        film = integ.render_film(small_scene, seed=7, spp=spp, chunk_paths=chunk)
        np.testing.assert_array_equal(film, ref, err_msg=f"chunk_paths={chunk}")
    assert ref[..., 3].sum() > 0


def test_rank_shards_and_row_bands(small_scene, oracle):
    """Sample-range shards of whole film slots (2 and 4 ranks at spp 8)
    combine by the rank tree to the single-call film bit for bit (8-slot film,
    mtx_core/common.h film_tree8); row bands up to float summation order of
    the halo rows (rtol 2e-6)."""
    from mtx import load_dict

    integ = load_dict({"type": "path_test"})
    H, spp = small_scene.height, 4
    full = integ.render_film(small_scene, seed=9, spp=2 * spp, spp_total=2 * spp)
    parts = [integ.render_film(small_scene, seed=9, spp=spp, spp_total=2 * spp, sample_offset=r * spp) for r in range(2)]
    np.testing.assert_array_equal(parts[0] + parts[1], full)
    q = [integ.render_film(small_scene, seed=9, spp=2, spp_total=8, sample_offset=2 * r) for r in range(4)]
    np.testing.assert_array_equal((q[0] + q[1]) + (q[2] + q[3]), full)
    top = integ.render_film(small_scene, seed=9, spp=8, y0=0, y1=H // 2)
    bot = integ.render_film(small_scene, seed=9, spp=8, y0=H // 2, y1=H)
    stitched = np.zeros_like(full)
    stitched[: H // 2 + 2] += top
    stitched[H // 2:] += bot
    np.testing.assert_allclose(stitched, full, rtol=2e-6, atol=1e-6)


def test_full_bedroom_deterministic_and_chunk_invariant():
    """Full-size benchmark scene (≈1.83 M triangles, 1280x720): two renders
    and two wavefront sizes give bit-identical films; radiance is finite."""
    from mtx import load_dict, scene

    sc = scene.bedroom()
    assert sc.n_tris > 1_800_000
    integ = load_dict({"type": "path_test"})
    f1 = integ.render_film(sc, seed=0, spp=1)
    f2 = integ.render_film(sc, seed=0, spp=1, chunk_paths=300_000)
    assert np.array_equal(f1, f2)
    assert np.isfinite(f1).all()
    img = f1[1:-1, 1:-1, :3] / f1[1:-1, 1:-1, 3:]
    assert 0.01 < float(img.mean()) < 10.0


# ------------------------------------------------------------- primitives --

@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 1_000_003])
def test_prefix_sum_u32(n):
    from mtx import primitives

    rng = np.random.default_rng(n)
    x = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    inc = primitives.prefix_sum(x, inclusive=True)
    exc = primitives.prefix_sum(x, inclusive=False)
    ref = np.cumsum(x, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(inc, ref)
    assert np.array_equal(exc, np.concatenate([[0], ref[:-1]]).astype(np.uint32))


def test_prefix_sum_u32_wraps_mod_2_32():
    from mtx import primitives

    x = np.full(3 * 4096 + 11, 0xFFFFFFF0, np.uint32)
    ref = np.cumsum(x.astype(np.uint64)).astype(np.uint32)
    assert np.array_equal(primitives.prefix_sum(x), ref)


@pytest.mark.parametrize("n", [1, 2, 1000, 2049, 1_000_000])
def test_prefix_sum_f32_hillis_steele_bit_exact(oracle, n):
    """prefix_sum.py:39-54 (10^6 PCG32 floats, seed 0) in the reference's order."""
    from mtx import primitives

    x = oracle.rng_stream(0, 0, n, 1)[:, 0].copy() if n <= 1_000_000 else None
    g = primitives.prefix_sum(x)
    c = oracle.prefix_sum_f32_hs(x)
    assert np.array_equal(g, c)
    np.testing.assert_allclose(g, np.cumsum(x.astype(np.float64)), rtol=1e-4)


def test_hashgrid_kat_and_random(oracle):
    from mtx import primitives

    # hashgrid.py:93-98: cells [0,0,1,0], sizes [3,1], offsets [0,3]
    p = np.array([[0, 0.1, 0.6, 1]] * 3, np.float32)
    g = primitives.HashGrid(p, 2, 2)
    assert g.cell.tolist() == [0, 0, 1, 0]
    assert g.cell_size.tolist() == [3, 1] and g.cell_offset.tolist() == [0, 3]
    assert g.sample_idx[3] == 2 and sorted(g.sample_idx[:3].tolist()) == [0, 1, 3]
    rng = np.random.default_rng(2)
    n = 1 << 18
    p = rng.random((3, n), dtype=np.float32)
    g = primitives.HashGrid(p, 100, n)
    cell, size, off, idx = oracle.hashgrid(p, 100, n)
    assert np.array_equal(g.cell, cell)
    assert np.array_equal(g.cell_size, size)
    assert np.array_equal(g.cell_offset, off)
    # within a cell the reference's order is race-defined (hashgrid.py:53); both
    # builds give the ascending-index outcome, so the arrays match exactly
    assert np.array_equal(g.sample_idx, idx)
    # sparse grid (n_cells > 4 n: the lower-bound offset kernel) and a dense one
    for nc in (1 << 21, 1 << 9, 1):
        q = np.ascontiguousarray(p[:, :1 << 16])
        g = primitives.HashGrid(q, 100, nc)
        ref = oracle.hashgrid(q, 100, nc)
        for a, b in zip((g.cell, g.cell_size, g.cell_offset, g.sample_idx), ref):
            assert np.array_equal(a, b)


def test_scatter_reduce(oracle):
    from mtx import primitives

    # reductions.py:57-63
    t = primitives.scatter_reduce_with("add", np.zeros(10, np.float32), np.ones(25, np.float32),
                                       np.arange(25, dtype=np.uint32) % 10)
    assert t.tolist() == [3, 3, 3, 3, 3, 2, 2, 2, 2, 2]
    rng = np.random.default_rng(4)
    nt, nv = 1 << 12, 1 << 16
    idx = rng.integers(0, nt, nv, dtype=np.uint32)
    val = rng.random(nv, dtype=np.float32)
    for op in (0, 1, 2):
        tgt = rng.random(nt, dtype=np.float32)
        g = primitives.scatter_reduce_with(op, tgt, val, idx)
        c = oracle.scatter_reduce(op, tgt, val, idx)
        assert np.array_equal(g, c)


@pytest.mark.parametrize("name", ["pssmlt_simple", "pssmlt"])
@pytest.mark.parametrize("iterations", [1, 60])
def test_pssmlt_film_bit_exact(small_scene, oracle, iterations, name):
    """Pssmlt.render: the film after `iterations` Metropolis steps (60 covers a
    large-step reset at 50 and the aggregation window 41-49) is bit-identical
    to the CPU restatement; chunks of 700 chains exercise the chunking.
    "pssmlt" is pssmltpath.py (NEE + MIS proposals, mutated emitter samples)."""
    from mtx import load_dict

    integ = load_dict({"type": name, "iterations": iterations})
    sc = small_scene.with_film(32, 18)
    film = integ.render_film(sc, seed=2, spp=2, chunk_paths=700)
    ref = oracle.pssmlt_render(sc, integ.render_args(sc, 2, 2), iterations)
    np.testing.assert_array_equal(film, ref)
    if iterations > 41:
        assert film[..., 3].sum() > 0


def test_prims_bucket_path_at_benchmark_scale(oracle):
    """The hand-written partition + per-bucket kernels (prims.hip) at the
    SURVEY §8d primitive sizes: hashgrid 2^22 points (res 100, n_cells = n;
    and 2^24 cells: the 13-bit buckets), clustered points (every point in a
    few hundred cells: long election rounds), scatter_reduce 2^22 values into
    2^20 targets for add / min / max -- all bit-exact against the oracle
    (ascending original index within a cell / per target)."""
    from mtx import primitives

    rng = np.random.default_rng(21)
    n = 1 << 22
    p = rng.random((3, n), dtype=np.float32)
    for nc in (n, 1 << 24):
        g = primitives.HashGrid(p, 100, nc)
        for a, b in zip((g.cell, g.cell_size, g.cell_offset, g.sample_idx), oracle.hashgrid(p, 100, nc)):
            assert np.array_equal(a, b), nc
    q = (rng.integers(0, 8, (3, 1 << 18)) / 8.0).astype(np.float32)  # 512 distinct points
    g = primitives.HashGrid(q, 100, 1 << 16)
    for a, b in zip((g.cell, g.cell_size, g.cell_offset, g.sample_idx), oracle.hashgrid(q, 100, 1 << 16)):
        assert np.array_equal(a, b)
    nt, nv = 1 << 20, 1 << 22
    idx = rng.integers(0, nt, nv, dtype=np.uint32)
    val = (rng.random(nv, dtype=np.float32) - 0.5).astype(np.float32)
    for op in (0, 1, 2):
        tgt = rng.random(nt, dtype=np.float32)
        assert np.array_equal(primitives.scatter_reduce_with(op, tgt, val, idx), oracle.scatter_reduce(op, tgt, val, idx))
