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
    """Closest-hit tree, 4-wide quantised nodes (mtx.h): every triangle in
    exactly one leaf of at most 8, a node's inner children first in slot order
    and at consecutive indices after it (breadth-first), its leaves' triangle
    ranges consecutive, children's decoded boxes contain their triangles /
    subtrees, depth as reported."""
    s = small_scene
    _check_bvh4(s.nodes, s.tri_geom, s.n_tris, s.bvh_depth)


def test_occlusion_bvh_invariants(small_scene):
    """Occlusion tree, 8-wide compressed nodes (mtx.h): every triangle in
    exactly one leaf of at most 3, leaves' triangles consecutive from tri_base
    in slot order, inner children consecutive from child_base in slot order
    (breadth-first: after their parent), meta bytes as documented, empty slots
    never hit (q_lo 255 > q_hi 0), children's decoded boxes contain their
    triangles / subtrees, depth as reported; its records are the scene's
    records bit for bit, permuted."""
    s = small_scene
    _check_occ(s.occ_nodes, s.occ_tri_geom, s.n_tris, s.occ_depth)
    assert sorted(s.occ_perm.tolist()) == list(range(s.n_tris))
    assert np.array_equal(s.occ_tri_geom.reshape(-1, 12).view(np.uint32),
                          s.tri_geom.reshape(-1, 12)[s.occ_perm].view(np.uint32))


def _tri_boxes(tri_geom):
    geom = tri_geom.reshape(-1, 12)
    v0 = geom[:, 0:3]
    v1 = v0 + geom[:, 4:7]
    v2 = v0 + geom[:, 8:11]
    return np.minimum(np.minimum(v0, v1), v2), np.maximum(np.maximum(v0, v1), v2)


def _check_bvh4(nodes, tri_geom, n_tris, bvh_depth):
    nodes = nodes.reshape(-1, 16)
    f = nodes.view(np.float32)
    u = nodes.view(np.uint32)
    seen = np.zeros(n_tris, np.int32)
    lo, hi = _tri_boxes(tri_geom)

    def subtree_box(ref):
        if ref < 0:
            x = ~int(ref)
            a, c = x >> 3, (x & 7) + 1
            return lo[a:a + c].min(0), hi[a:a + c].max(0)
        return boxes[ref]

    boxes, order = {}, []
    stack = [(0, 1)]
    max_depth = 0
    while stack:
        i, dep = stack.pop()
        order.append(i)
        max_depth = max(max_depth, dep)
        nch = int(u[i, 3] >> 24)
        assert 1 <= nch <= 4
        refs = [int(nodes[i, 4 + k]) for k in range(nch)]
        n_in = sum(r >= 0 for r in refs)
        assert all(r >= 0 for r in refs[:n_in])  # inner children first
        assert refs[:n_in] == list(range(refs[0], refs[0] + n_in)) if n_in else True
        assert all(r > i for r in refs[:n_in])  # breadth-first: children after their parent
        firsts = [(~r) >> 3 for r in refs[n_in:]]
        cnts = [((~r) & 7) + 1 for r in refs[n_in:]]
        assert all(firsts[j + 1] == firsts[j] + cnts[j] for j in range(len(firsts) - 1))
        for r in refs[:n_in]:
            stack.append((r, dep + 1))
        for a, c in zip(firsts, cnts):
            assert c <= 8
            seen[a:a + c] += 1
    for i in reversed(order):  # children before parents
        nch = int(u[i, 3] >> 24)
        e = [np.int8(np.uint8((u[i, 3] >> (8 * a)) & 255)) for a in range(3)]
        assert all(-32 <= x <= 31 for x in e)
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
    assert (seen == 1).all()
    assert max_depth <= 40 and max_depth == bvh_depth
    assert len(order) == len(nodes)


def _node_children(u, i):
    """[(slot, 'inner', node) | (slot, 'leaf', first, count)] of occlusion node i."""
    imask, cb, tb = int(u[i, 3] >> 24), int(u[i, 4]), int(u[i, 5])
    out, inner, off = [], 0, 0
    for sl in range(8):
        m = int((u[i, 6 + (sl >> 2)] >> (8 * (sl & 3))) & 255)
        if (imask >> sl) & 1:
            assert m == 0x20 | (24 + sl), (i, sl, m)
            out.append((sl, "inner", cb + inner))
            inner += 1
        elif m:
            cnt = {1: 1, 3: 2, 7: 3}[m >> 5]
            assert (m & 31) == off and off + cnt <= 24, (i, sl, m, off)  # consecutive in slot order
            out.append((sl, "leaf", tb + off, cnt))
            off += cnt
    return out


def _check_occ(nodes, tri_geom, n_tris, depth):
    nodes = nodes.reshape(-1, 20)
    f = nodes.view(np.float32)
    u = nodes.view(np.uint32)
    seen = np.zeros(n_tris, np.int32)
    lo, hi = _tri_boxes(tri_geom)
    boxes, order, kids = {}, [], {}
    stack = [(0, 1)]
    max_depth = 0
    while stack:
        i, dep = stack.pop()
        order.append(i)
        max_depth = max(max_depth, dep)
        kids[i] = _node_children(u, i)
        assert kids[i]
        for c in kids[i]:
            if c[1] == "inner":
                assert c[2] > i  # breadth-first: children after their parent
                stack.append((c[2], dep + 1))
            else:
                seen[c[2]:c[2] + c[3]] += 1
    for i in reversed(order):  # children before parents
        e = [np.int8(np.uint8((u[i, 3] >> (8 * a)) & 255)) for a in range(3)]
        assert all(-32 <= x <= 31 for x in e)
        blo = np.full(3, np.inf, np.float32)
        bhi = np.full(3, -np.inf, np.float32)
        used = {c[0] for c in kids[i]}
        for sl in range(8):
            qb = [(u[i, 8 + 4 * a + (sl >> 2)] >> (8 * (sl & 3))) & 255 for a in range(3)]
            qt = [(u[i, 10 + 4 * a + (sl >> 2)] >> (8 * (sl & 3))) & 255 for a in range(3)]
            if sl not in used:
                assert qb == [255] * 3 and qt == [0] * 3
        for c in kids[i]:
            sl = c[0]
            if c[1] == "inner":
                clo, chi = boxes[c[2]]
            else:
                clo, chi = lo[c[2]:c[2] + c[3]].min(0), hi[c[2]:c[2] + c[3]].max(0)
            for a in range(3):
                qlo = (u[i, 8 + 4 * a + (sl >> 2)] >> (8 * (sl & 3))) & 255
                qhi = (u[i, 10 + 4 * a + (sl >> 2)] >> (8 * (sl & 3))) & 255
                assert _decode(f[i, a], e[a], qlo) <= clo[a] and _decode(f[i, a], e[a], qhi) >= chi[a]
            blo, bhi = np.minimum(blo, clo), np.maximum(bhi, chi)
        boxes[i] = (blo, bhi)
    assert (seen == 1).all()
    assert max_depth <= 40 and max_depth == depth
    assert len(order) == len(nodes)


def _random_rays(n, seed):
    rng = np.random.default_rng(seed)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform([-3.0, 0.05, -1.2], [3.8, 2.6, 3.6], (n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 3] = 3e38
    return rays, rng


def test_bvh_closest_hit_equals_brute_force(small_scene, oracle):
    rays, _ = _random_rays(6000, 11)
    h, _ = oracle.trace(small_scene, rays)
    b, _ = oracle.trace(small_scene, rays, brute=True)
    assert np.array_equal(h, b)


def test_occlusion_any_hit_equals_brute_force(small_scene, oracle):
    """The occlusion tree answers ray_test exactly as a brute-force closest
    hit does: occluded iff some triangle lies in (0, maxt] (finite and
    unbounded maxt)."""
    rays, rng = _random_rays(6000, 12)
    rays[::2, 3] = rng.uniform(0.05, 2.0, 3000).astype(np.float32)
    a, _ = oracle.trace(small_scene, rays, any_hit=True)
    b, _ = oracle.trace(small_scene, rays, brute=True)
    assert 0 < a.sum() < len(a)
    assert np.array_equal(a.astype(bool), b.reshape(-1, 4)[:, 1] != 0xFFFFFFFF)


def test_scene_save_load_roundtrip(small_scene, tmp_path):
    from mtx import scene

    p = os.path.join(tmp_path, "s.npz")
    small_scene.save(p)
    t = scene.Scene.load(p)
    assert np.array_equal(t.nodes, small_scene.nodes) and bytes(t.materials) == bytes(small_scene.materials)
    assert np.array_equal(t.occ_nodes, small_scene.occ_nodes) and t.occ_depth == small_scene.occ_depth
    assert np.array_equal(t.occ_tri_geom, small_scene.occ_tri_geom)
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


@pytest.mark.parametrize("cnode", ["1", "4"])
@pytest.mark.parametrize("kind", ["one", "two", "nine", "identical", "planar", "random"])
def test_bvh_build_small_and_degenerate_meshes(kind, cnode, monkeypatch):
    """Both collapses (4-wide closest hit, 8-wide occlusion) keep the node
    invariants on tiny, coplanar and coincident-triangle meshes (two collapse
    node costs: other trees)."""
    import ctypes as C

    from mtx import _lib

    monkeypatch.setenv("MTX_BVH_CNODE", cnode)
    v, idx = _tiny_mesh(kind)
    n = len(idx)
    nodes = np.zeros((n + 1) * 16, np.int32)
    geom = np.zeros(12 * n, np.float32)
    perm = np.zeros(n, np.uint32)
    nn, dep = C.c_uint32(), C.c_uint32()
    L = _lib.lib()
    rc = L.mtx_bvh_build(v.ctypes.data, len(v), np.ascontiguousarray(idx).ctypes.data, n, nodes.ctypes.data,
                         C.byref(nn), geom.ctypes.data, perm.ctypes.data, C.byref(dep))
    assert rc == 0, L.mtx_last_error()
    assert sorted(perm.tolist()) == list(range(n))
    _check_bvh4(nodes[: 16 * nn.value], geom, n, dep.value)
    onodes = np.zeros((n + 1) * 20, np.int32)
    ogeom = np.zeros(12 * n, np.float32)
    operm = np.zeros(n, np.uint32)
    rc = L.mtx_bvh_build_occlusion(geom.ctypes.data, n, onodes.ctypes.data, C.byref(nn), ogeom.ctypes.data,
                                   operm.ctypes.data, C.byref(dep))
    assert rc == 0, L.mtx_last_error()
    assert sorted(operm.tolist()) == list(range(n))
    assert np.array_equal(ogeom.reshape(-1, 12), geom.reshape(-1, 12)[operm])
    _check_occ(onodes[: 20 * nn.value], ogeom, n, dep.value)
