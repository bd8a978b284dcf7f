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


@pytest.mark.parametrize("name", ["path_test", "mypath", "nrc", "integrator"])
def test_golden_films_oracle(golden, oracle, small_scene, name):
    from mtx import load_dict

    integ = load_dict({"type": name})
    assert np.array_equal(oracle.render(small_scene, integ.render_args(small_scene, 0, 16)), golden[f"film_{name}"])


def test_golden_independent_of_bvh_collapse(golden, oracle, monkeypatch):
    """Closest hits do not depend on the tree (inclusive culling + the
    smaller-index tie rule): the greedy collapse (MTX_BVH_COLLAPSE=0) gives
    other nodes, and the same hits and film bit for bit."""
    from mtx import load_dict, scene

    monkeypatch.setenv("MTX_BVH_COLLAPSE", "0")
    sc = scene.Scene.bedroom(width=64, height=36, scale=0.02, tex_res=64)
    assert oracle.trace(sc, golden["trace_rays"])[0].tobytes() == golden["trace_hits"].tobytes()
    integ = load_dict({"type": "path_test"})
    assert np.array_equal(oracle.render(sc, integ.render_args(sc, 0, 16)), golden["film_path_test"])


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
