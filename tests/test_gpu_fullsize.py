"""Parity at the benchmark's full size and on the traversal's rarely taken
branches (VERDICT r1 "next" #4).

* The full bedroom proxy (≈1.83 M triangles, 1280x720): hit records and
  visit counts of 2^16 rays, and the path_test film (path-mis.py:24-155) at
  spp 2, bit-exact against the oracle (the oracle traces the same 1.84 M
  paths on the host cores in about a second).
* The traversal stacks' global spill area (csrc/device_common.h, pushes
  beyond the LDS entries): a fresh process with MTX_LDS_STACK=1 and
  MTX_OCC_LDS_STACK=1 keeps one entry of either tree's stack in LDS, so every
  deeper push and pop goes through global memory; also without the LDS tree
  tops (MTX_LDS_TOP=0, MTX_OCC_LDS_TOP=0) and the non-XCD-claiming
  traversal (MTX_XCD_CLAIM=0). The environment is read when the context is created, so
  each variant runs in its own subprocess before any GPU call.
* max_depth 65, the default of data/bedroom/scene.xml:6 (SURVEY §8d C2
  secondary configuration).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _rays(scene, n, seed):
    from test_gpu_parity import _camera_rays

    o, d = _camera_rays(scene, n, seed=seed)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = o, d
    rays[:, 3] = np.float32(3.0e38)
    rays[::5, 3] = np.float32(0.75)
    return rays


def test_full_bedroom_trace_bit_exact(full_scene, oracle):
    """Modes 0 (closest hit, 4-wide tree) and 1 (any hit, 8-wide occlusion
    tree): hits and visit counts equal the oracle's."""
    from test_gpu_parity import _trace_gpu

    rays = _rays(full_scene, 1 << 16, 21)
    for mode in (0, 1):
        g_hits, g_vis = _trace_gpu(full_scene, rays, mode)
        c_hits, c_vis = oracle.trace(full_scene, rays, mode)
        assert np.array_equal(g_hits, c_hits), f"mode={mode}"
        assert np.array_equal(g_vis, c_vis), f"mode={mode}"


def test_full_bedroom_path_mis_film_bit_exact(full_scene, oracle):
    """The headline configuration's integrator, scene and film size at spp 2."""
    from mtx import load_dict

    integ = load_dict({"type": "path_test"})
    film = integ.render_film(full_scene, seed=7, spp=2)
    ref = oracle.render(full_scene, integ.render_args(full_scene, 7, 2))
    np.testing.assert_array_equal(film, ref)
    assert film[1:-1, 1:-1, 3].min() > 0


@pytest.mark.parametrize("name", ["path_test", "mypath"])
def test_max_depth_65_film_bit_exact(small_scene, oracle, name):
    """scene.xml:6 max_depth 65 (rr_depth stays the integrator's default)."""
    from mtx import load_dict

    integ = load_dict({"type": name, "max_depth": 65})
    film = integ.render_film(small_scene, seed=11, spp=8)
    ref = oracle.render(small_scene, integ.render_args(small_scene, 11, 8))
    np.testing.assert_array_equal(film, ref)


_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [{pkg!r}, {orc!r}, {tests!r}]
import binding as oracle
from mtx import load_dict, scene
from test_gpu_parity import _trace_gpu
from test_gpu_fullsize import _rays
oracle.build()
for sc in (scene.bedroom(width=64, height=36, scale=0.02, tex_res=64), scene.bedroom(width=96, height=54)):
    rays = _rays(sc, 1 << 14, 5)
    for mode in (0, 1):
        g_hits, g_vis = _trace_gpu(sc, rays, mode)
        c_hits, c_vis = oracle.trace(sc, rays, mode)
        assert np.array_equal(g_hits, c_hits), ("hits", sc.n_tris, mode)
        assert np.array_equal(g_vis, c_vis), ("visits", sc.n_tris, mode)
    integ = load_dict({{"type": "path_test"}})
    film = integ.render_film(sc, seed=2, spp=4, chunk_paths=5000)
    ref = oracle.render(sc, integ.render_args(sc, 2, 4))
    assert np.array_equal(film, ref), ("film", sc.n_tris)
print("CHILD OK")
"""


@pytest.mark.parametrize("env", [{"MTX_LDS_STACK": "1", "MTX_OCC_LDS_STACK": "1"},
                                 {"MTX_LDS_STACK": "2", "MTX_LDS_TOP": "0", "MTX_OCC_LDS_STACK": "2",
                                  "MTX_OCC_LDS_TOP": "0"},
                                 {"MTX_XCD_CLAIM": "0", "MTX_TRACE_BATCH": "64"},
                                 {"MTX_OCC_LDS_STACK": "1", "MTX_OCC_LDS_TOP": "0"}],
                         ids=["spill-all", "spill2-notop", "noxcd-batch64", "occ-spill-notop"])
def test_traversal_variants_bit_exact(env):
    """Traversal variants selected at context creation: bit-exact hits,
    visit counts and films on the 2 % scene and on the full-size scene."""
    code = _CHILD.format(pkg=os.path.join(ROOT, "mitsuba3-experiments_amd"), orc=os.path.join(ROOT, "oracle"),
                         tests=os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0 and "CHILD OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
