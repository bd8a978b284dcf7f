"""Bedroom proxy and BVH invariants (host code; no GPU)."""
import hashlib
import json
import math
import os

import numpy as np
import pytest

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


def _decode(org, e, q):
    """Child bound = origin + q * 2^e in fp32 (mtx.h / geometry.h wide_decode)."""
    sc = np.float32(2.0) ** np.float32(e)
    return np.float32(org) + np.float32(q) * sc


def test_bvh_invariants(small_scene):
    """4-wide quantised nodes (mtx.h): every triangle in exactly one leaf of
    at most 8, children's decoded boxes contain their triangles / subtrees,
    depth as reported."""
    s = small_scene
    _check_bvh(s.nodes, s.tri_geom, s.n_tris, s.bvh_depth)


def _check_bvh(nodes, tri_geom, n_tris, bvh_depth):
    nodes = nodes.reshape(-1, 16)
    f = nodes.view(np.float32)
    u = nodes.view(np.uint32)
    seen = np.zeros(n_tris, np.int32)
    geom = tri_geom.reshape(-1, 12)
    v0 = geom[:, 0:3]
    v1 = v0 + geom[:, 4:7]
    v2 = v0 + geom[:, 8:11]
    lo = np.minimum(np.minimum(v0, v1), v2)
    hi = np.maximum(np.maximum(v0, v1), v2)

    def subtree_box(ref):
        if ref < 0:
            x = ~int(ref)
            a, c = x >> 3, (x & 7) + 1
            return lo[a:a + c].min(0), hi[a:a + c].max(0)
        return boxes[ref]

    boxes = {}
    order = []
    stack = [(0, 1)]
    max_depth = 0
    while stack:
        i, dep = stack.pop()
        order.append(i)
        max_depth = max(max_depth, dep)
        nch = int(u[i, 3] >> 24)
        assert 1 <= nch <= 4
        for k in range(nch):
            c = int(nodes[i, 4 + k])
            if c >= 0:
                stack.append((c, dep + 1))
            else:
                x = ~c
                first, cnt = x >> 3, (x & 7) + 1
                assert cnt <= 8
                seen[first:first + cnt] += 1
    for i in reversed(order):  # children before parents
        nch = int(u[i, 3] >> 24)
        e = [np.int8(np.uint8((u[i, 3] >> (8 * a)) & 255)) for a in range(3)]
        blo = np.full(3, np.inf, np.float32)
        bhi = np.full(3, -np.inf, np.float32)
        for k in range(nch):
            clo, chi = subtree_box(int(nodes[i, 4 + k]))
            for a in range(3):
                qlo = (u[i, 8 + 2 * a] >> (8 * k)) & 255
                qhi = (u[i, 9 + 2 * a] >> (8 * k)) & 255
                assert _decode(f[i, a], e[a], qlo) <= clo[a] and _decode(f[i, a], e[a], qhi) >= chi[a]
            blo, bhi = np.minimum(blo, clo), np.maximum(bhi, chi)
        boxes[i] = (blo, bhi)
    assert (seen == 1).all() or ((seen >= 1).all() and n_tris == 1)
    assert max_depth <= 40 and max_depth == bvh_depth
    _check_device_nodes(nodes, n_tris)


def _check_device_nodes(nodes, n_tris):
    """The builder's layout (mtx.h) and the 48-B device form decoded here in
    numpy (bvh_build.cpp mtx_bvh_device_nodes; device_common.h wide_dref)
    give every child reference of the 64-B node."""
    import ctypes as C

    from mtx import _lib

    u = nodes.view(np.uint32)
    for i in range(len(nodes)):
        nch = int(u[i, 3] >> 24)
        refs = [int(nodes[i, 4 + k]) for k in range(nch)]
        n_in = sum(r >= 0 for r in refs)
        assert all(r >= 0 for r in refs[:n_in]) and all(r < 0 for r in refs[n_in:])  # inner first
        assert refs[:n_in] == list(range(refs[0], refs[0] + n_in)) if n_in else True
        first = [(~r) >> 3 for r in refs[n_in:]]
        cnt = [((~r) & 7) + 1 for r in refs[n_in:]]
        assert all(first[j + 1] == first[j] + cnt[j] for j in range(len(first) - 1))
        assert all(-32 <= np.int8(np.uint8((u[i, 3] >> (8 * a)) & 255)) <= 31 for a in range(3))
    L = _lib.lib()
    out = np.zeros((len(nodes), 12), np.int32)
    assert L.mtx_bvh_device_nodes(np.ascontiguousarray(nodes).ctypes.data, len(nodes), n_tris, out.ctypes.data) == 0
    w = out.view(np.uint32)
    assert np.array_equal(out[:, 0:3], nodes[:, 0:3]) and np.array_equal(out[:, 6:12], nodes[:, 8:14])
    ends = (w[:, 3] >> 20) | ((w[:, 4] >> 24) << 12) | ((w[:, 5] >> 24) << 20)
    nb, tb = w[:, 4] & 0xFFFFFF, w[:, 5] & 0xFFFFFF
    for i in range(len(nodes)):
        nch = int((w[i, 3] >> 18) & 3) + 1
        assert nch == int(u[i, 3] >> 24)
        for a in range(3):
            e6 = int((w[i, 3] >> (6 * a)) & 63)
            assert (e6 - 64 if e6 >= 32 else e6) == int(np.int8(np.uint8((u[i, 3] >> (8 * a)) & 255)))
        for k in range(nch):
            e1 = int(ends[i] >> (6 * k)) & 63
            e0 = int((int(ends[i]) << 6) >> (6 * k)) & 63
            ref = int(nb[i]) + k if e1 == 0 else ~(((int(tb[i]) + e0) << 3) | (e1 - e0 - 1))
            assert ref == int(nodes[i, 4 + k]), (i, k)
    bad = nodes.copy()
    bad[0, 4], bad[0, 5] = bad[0, 5], bad[0, 4]  # slot order broken
    if int(u[0, 3] >> 24) >= 2 and bad[0, 4] != nodes[0, 4]:
        assert L.mtx_bvh_device_nodes(bad.ctypes.data, len(bad), n_tris, out.ctypes.data) != 0


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


def _tiny_mesh(kind):
    rng = np.random.default_rng(5)
    if kind == "one":
        v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
        return v, np.array([[0, 1, 2]], np.uint32)
    if kind == "identical":  # 20 copies of one triangle: zero-extent splits
        v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
        return v, np.tile(np.array([[0, 1, 2]], np.uint32), (20, 1))
    n = {"two": 2, "nine": 9, "random": 400, "planar": 300}[kind]
    v = rng.uniform(-1, 1, (3 * n, 3)).astype(np.float32)
    if kind == "planar":
        v[:, 2] = 0.5  # every box flat in z
    return v, np.arange(3 * n, dtype=np.uint32).reshape(n, 3)


@pytest.mark.parametrize("collapse", ["0", "1"])
@pytest.mark.parametrize("kind", ["one", "two", "nine", "identical", "planar", "random"])
def test_bvh_build_small_and_degenerate_meshes(kind, collapse, monkeypatch):
    """Greedy (MTX_BVH_COLLAPSE=0) and dynamic-programming collapses keep the
    node invariants on tiny, coplanar and coincident-triangle meshes."""
    import ctypes as C

    from mtx import _lib

    monkeypatch.setenv("MTX_BVH_COLLAPSE", collapse)
    v, idx = _tiny_mesh(kind)
    n = len(idx)
    nodes = np.zeros((2 * n + 2) * 16, np.int32)
    geom = np.zeros(12 * n, np.float32)
    perm = np.zeros(n, np.uint32)
    nn, dep = C.c_uint32(), C.c_uint32()
    L = _lib.lib()
    rc = L.mtx_bvh_build(v.ctypes.data, len(v), np.ascontiguousarray(idx).ctypes.data, n, nodes.ctypes.data,
                         C.byref(nn), geom.ctypes.data, perm.ctypes.data, C.byref(dep))
    assert rc == 0, L.mtx_last_error()
    assert sorted(perm.tolist()) == list(range(n))
    _check_bvh(nodes[: 16 * nn.value], geom, n, dep.value)
