"""Closest hit on the 8-wide tree (round 5; oracle/oracle.cpp
trace_closest_cw, the restatement of device_common.h
trace_loop_closest_cw): the same hit records as the 4-wide traversal and the
brute-force intersector (Scene.ray_intersect, path-mis.py:69-71), for camera
rays, clipped rays and rays from inside the scene, on the 2 % bedroom; and
fewer node visits than the 4-wide tree. CPU only."""
import numpy as np


def _rays(scene, n, seed):
    from test_gpu_parity import _camera_rays

    o, d = _camera_rays(scene, n, seed=seed)
    rng = np.random.default_rng(seed)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = o, d
    rays[:, 3] = np.float32(3.0e38)
    rays[::5, 3] = np.float32(0.75)
    # a third start inside the room with random directions
    k = n // 3
    lo, hi = scene.vpos.reshape(-1, 3).min(0), scene.vpos.reshape(-1, 3).max(0)
    rays[:k, 0:3] = lo + (hi - lo) * rng.uniform(0.2, 0.8, size=(k, 3))
    v = rng.normal(size=(k, 3))
    rays[:k, 4:7] = v / np.linalg.norm(v, axis=1, keepdims=True)
    return rays


def test_cw_closest_equals_bvh4_and_brute(small_scene, oracle):
    rays = _rays(small_scene, 6000, 3)
    h0, v0 = oracle.trace(small_scene, rays, 0)
    h2, v2 = oracle.trace(small_scene, rays, 2)
    assert np.array_equal(h2, h0)
    hb, _ = oracle.trace(small_scene, rays[:1500], 0, brute=True)
    assert np.array_equal(h2[: 4 * 1500], hb)
    assert (h2.reshape(-1, 4)[:, 1] != 0xFFFFFFFF).mean() > 0.7
    # the sorted 8-wide descent visits fewer nodes
    assert v2[:, 0].mean() < 0.85 * v0[:, 0].mean()


def test_occ_perm_maps_the_records(small_scene):
    g = small_scene.tri_geom.reshape(-1, 12)
    og = small_scene.occ_tri_geom.reshape(-1, 12)
    perm = np.asarray(small_scene.occ_perm)
    assert np.array_equal(np.sort(perm), np.arange(len(perm)))
    assert np.array_equal(og[:, [0, 1, 2, 4, 5, 6, 8, 9, 10]], g[perm][:, [0, 1, 2, 4, 5, 6, 8, 9, 10]])
