"""Bedroom proxy and BVH invariants (host code; no GPU)."""
import hashlib
import json
import math
import os

import numpy as np

from conftest import ROOT


def test_bedroom_spec_matches_reference_xml_facts():
    from mtx import scene

    spec = scene.load_bedroom_spec()
    assert spec["sensor"]["fov"] == 65.0 and spec["sensor"]["film"]["width"] == 1280
    assert spec["sensor"]["film"]["rfilter"] == "tent"
    assert len(spec["bsdfs"]) == 31
    shapes = spec["shapes"]
    assert sum(s["type"] == "obj" for s in shapes) == 70 and sum(s["type"] == "rectangle" for s in shapes) == 2
    em = [s for s in shapes if "emitter" in s]
    assert len(em) == 2 and all(e["emitter"]["radiance"] == [16.4648] * 3 for e in em)
    sizes = sum(s.get("lfs_size") or 0 for s in shapes)
    assert sizes == 175_869_300


def test_proxy_budgets_exact():
    from mtx import proxy, scene

    spec = scene.load_bedroom_spec()
    fam = {}
    total = 0
    for sd in spec["shapes"]:
        if sd["type"] != "obj":
            continue
        f = sd["id"].split("_")[0]
        k = fam.get(f, 0)
        fam[f] = k + 1
        n = proxy.budget_from_lfs(sd["lfs_size"], 0.01)
        P, N, UV, F = proxy.generate_mesh(sd["id"], n, k)
        assert len(F) == n
        assert F.max() < len(P) and np.isfinite(P).all()
        total += math.ceil(sd["lfs_size"] / 96)
    assert total == 1_832_000  # sum of ceil(size / 96 B) per shape (versioned budget)


def test_scene_is_deterministic(small_scene):
    from mtx import scene

    other = scene.Scene.bedroom(width=64, height=36, scale=0.02, tex_res=64)

    def digest(s):
        h = hashlib.sha256()
        for a in (s.vpos, s.vnormal, s.vuv, s.nodes, s.tri_geom, s.tri_vidx, s.tri_shape, s.texels, s.tables):
            h.update(np.ascontiguousarray(a).tobytes())
        for a in (s.shapes, s.materials, s.emitters, s.textures, s.camera):
            h.update(bytes(a))
        return h.hexdigest()

    assert digest(small_scene) == digest(other)


def test_bvh_invariants(small_scene):
    s = small_scene
    nodes = s.nodes.reshape(-1, 16)
    f = nodes.view(np.float32)
    seen = np.zeros(s.n_tris, np.int32)
    geom = s.tri_geom.reshape(-1, 12)
    v0 = geom[:, 0:3]
    v1 = v0 + geom[:, 4:7]
    v2 = v0 + geom[:, 8:11]
    lo = np.minimum(np.minimum(v0, v1), v2)
    hi = np.maximum(np.maximum(v0, v1), v2)
    depth = np.zeros(len(nodes), np.int32)
    stack = [0]
    max_depth = 1
    while stack:
        i = stack.pop()
        for c, bx in ((nodes[i, 12], (0, 1, 2, 3, 8, 9)), (nodes[i, 13], (4, 5, 6, 7, 10, 11))):
            b = f[i, list(bx)]
            blo, bhi = b[[0, 2, 4]], b[[1, 3, 5]]
            if c >= 0:
                depth[c] = depth[i] + 1
                max_depth = max(max_depth, depth[c] + 1)
                stack.append(c)
                continue
            x = ~int(c)
            first, cnt = x >> 3, (x & 7) + 1
            assert cnt <= 8
            seen[first:first + cnt] += 1
            assert (lo[first:first + cnt] >= blo).all() and (hi[first:first + cnt] <= bhi).all()
    assert (seen >= 1).all()
    assert max_depth <= 40 and max_depth == s.bvh_depth


def test_bvh_closest_hit_equals_brute_force(small_scene, oracle):
    rng = np.random.default_rng(11)
    n = 6000
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform([-3.0, 0.05, -1.2], [3.8, 2.6, 3.6], (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 3] = 3e38
    h, _ = oracle.trace(small_scene, rays)
    b, _ = oracle.trace(small_scene, rays, brute=True)
    assert np.array_equal(h, b)


def test_scene_save_load_roundtrip(small_scene, tmp_path):
    from mtx import scene

    p = os.path.join(tmp_path, "s.npz")
    small_scene.save(p)
    t = scene.Scene.load(p)
    assert np.array_equal(t.nodes, small_scene.nodes) and bytes(t.materials) == bytes(small_scene.materials)
    assert bytes(t.camera) == bytes(small_scene.camera)
    assert json.dumps(t.meta, sort_keys=True) == json.dumps(small_scene.meta, sort_keys=True)
