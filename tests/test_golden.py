"""The oracle reproduces the committed golden vectors (tests/golden/), and —
on a GPU — so does the HIP path."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.npz")


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(GOLDEN, allow_pickle=False))


def test_golden_scene_unchanged(golden, small_scene):
    import make_golden

    assert make_golden.scene_digest(small_scene) == golden["scene_sha"].tobytes().decode()


def test_golden_rng(golden, oracle):
    assert np.array_equal(oracle.rng_stream(0, 0, 1024, 64), golden["rng_seed0"])
    assert np.array_equal(oracle.rng_stream(7, 0, 1024, 64), golden["rng_seed7"])


def test_golden_trace(golden, oracle, small_scene):
    assert np.array_equal(oracle.trace(small_scene, golden["trace_rays"])[0], golden["trace_hits"])
    assert np.array_equal(oracle.trace(small_scene, golden["any_rays"], any_hit=True)[0], golden["any_hits"])


@pytest.mark.parametrize("name", ["path_test", "mypath", "nrc", "integrator"])
def test_golden_films_oracle(golden, oracle, small_scene, name):
    from mtx import load_dict

    integ = load_dict({"type": name})
    assert np.array_equal(oracle.render(small_scene, integ.render_args(small_scene, 0, 16)), golden[f"film_{name}"])


def test_golden_independent_of_bvh_collapse(golden, oracle, small_scene, monkeypatch):
    """Closest hits do not depend on the tree (inclusive culling; exact-t ties
    go to the smaller leaf-order index): another tree (8 SAH bins, collapse
    node cost 3) gives other nodes and another triangle numbering (the
    builder orders triangles by node), and the same distance for every ray and
    the same triangle (mapped to the input mesh) and barycentrics for all rays
    but exact-t ties (a shared edge, or coplanar overlapping surfaces), which
    may resolve to the other triangle."""
    from mtx import scene

    monkeypatch.setenv("MTX_BVH_BINS", "8")
    monkeypatch.setenv("MTX_BVH_CNODE", "3")
    sc = scene.Scene.bedroom(width=64, height=36, scale=0.02, tex_res=64)
    assert not np.array_equal(sc.tri_perm, small_scene.tri_perm)
    h = oracle.trace(sc, golden["trace_rays"])[0].reshape(-1, 4)
    g = golden["trace_hits"].reshape(-1, 4)
    assert np.array_equal(h[:, 0], g[:, 0])  # t
    miss = g[:, 1] == 0xFFFFFFFF
    assert np.array_equal(h[:, 1] == 0xFFFFFFFF, miss)
    same = sc.tri_perm[h[~miss, 1]] == small_scene.tri_perm[g[~miss, 1]]
    assert same.mean() > 0.995
    assert np.array_equal(h[~miss][same][:, 2:], g[~miss][same][:, 2:])
    # any hit: a different occlusion tree, the same answers
    assert not np.array_equal(sc.occ_perm, small_scene.occ_perm)
    assert np.array_equal(oracle.trace(sc, golden["any_rays"], any_hit=True)[0], golden["any_hits"])
    # the others are exact-t ties: rays through a shared edge, or onto
    # coplanar overlapping surfaces of two shapes (the floor and the carpet
    # at y = 0): the hit point (same t) lies in both triangles' planes
    rays = golden["trace_rays"].reshape(-1, 8)[~miss][~same]
    t = h[~miss][~same][:, 0].view(np.float32).astype(np.float64)
    p = rays[:, 0:3] + t[:, None] * rays[:, 4:7]
    for geom, prim in ((sc.tri_geom, h[~miss][~same][:, 1]), (small_scene.tri_geom, g[~miss][~same][:, 1])):
        x = geom.reshape(-1, 3, 4)[prim].astype(np.float64)
        n = np.cross(x[:, 1, :3], x[:, 2, :3])
        n /= np.linalg.norm(n, axis=1, keepdims=True)
        assert np.abs(np.sum((p - x[:, 0, :3]) * n, 1)).max() < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["path_test", "mypath", "nrc", "integrator"])
def test_golden_films_gpu(golden, small_scene, name):
    from mtx import load_dict

    integ = load_dict({"type": name})
    assert np.array_equal(integ.render_film(small_scene, seed=0, spp=16), golden[f"film_{name}"])


def test_golden_pssmlt_and_restir_oracle(golden, oracle, small_scene):
    import make_golden
    from mtx import load_dict

    sp = small_scene.with_film(32, 18)
    for name in ("pssmlt_simple", "pssmlt"):
        f = oracle.pssmlt_render(sp, load_dict({"type": name}).render_args(sp, 2, 2), 60)
        assert np.array_equal(f, golden[f"film_{name}"])
    for k, f in enumerate(make_golden.restir_frames(small_scene)):
        assert np.array_equal(f, golden[f"film_restirgi_f{k}"])


@pytest.mark.gpu
def test_golden_pssmlt_and_restir_gpu(golden, small_scene):
    from mtx import load_dict
    import make_golden

    sp = small_scene.with_film(32, 18)
    for name in ("pssmlt_simple", "pssmlt"):
        integ = load_dict({"type": name, "iterations": 60})
        assert np.array_equal(integ.render_film(sp, seed=2, spp=2), golden[f"film_{name}"])
    integ = load_dict({"type": "restirgi", **make_golden.RESTIR_PROPS})
    for k in range(3):
        assert np.array_equal(integ.render_film(small_scene, seed=k, spp=1), golden[f"film_restirgi_f{k}"])
