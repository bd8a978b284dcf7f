"""Diagnostic (not a product path): how much do the bedroom proxy's few large
triangles (extent > THR; 233 of 1.83 M hold 53 % of the area) cost the
traversal? Midpoint-subdivide them until every edge extent is below THR,
rebuild the BVH and compare trace times and visits per ray against the
original scene (path_test, 1280x720, spp 64). Bounds what spatial splits
(SBVH) could gain."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))
from mtx import load_dict, scene  # noqa: E402

THR = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25


def subdivide(sc, thr):
    P, N, UV = [sc.vpos.copy()], [sc.vnormal.copy()], [sc.vuv.copy()]
    nv = len(sc.vpos)
    F = sc.tri_vidx.reshape(-1, 3).astype(np.int64)
    S = np.asarray(sc.tri_shape).copy()
    vp, vn, vt = sc.vpos, sc.vnormal, sc.vuv
    out_f, out_s = [], []
    keep = np.ones(len(F), bool)
    big = []
    for t in range(len(F)):
        p = vp[F[t]]
        if (p.max(0) - p.min(0)).max() > thr:
            keep[t] = False
            big.append(t)
    verts_p, verts_n, verts_t = list(vp), list(vn), list(vt)

    def mid(a, b):
        verts_p.append((verts_p[a] + verts_p[b]) * 0.5)
        n = verts_n[a] + verts_n[b]
        verts_n.append(n / max(np.linalg.norm(n), 1e-12))
        verts_t.append((verts_t[a] + verts_t[b]) * 0.5)
        return len(verts_p) - 1

    work = [(tuple(F[t]), S[t]) for t in big]
    while work:
        (a, b, c), s_ = work.pop()
        p = np.array([verts_p[a], verts_p[b], verts_p[c]])
        if (p.max(0) - p.min(0)).max() <= thr:
            out_f.append((a, b, c))
            out_s.append(s_)
            continue
        ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
        work += [((a, ab, ca), s_), ((ab, b, bc), s_), ((ca, bc, c), s_), ((ab, bc, ca), s_)]
    sc.vpos = np.ascontiguousarray(np.array(verts_p, np.float32))
    sc.vnormal = np.ascontiguousarray(np.array(verts_n, np.float32))
    sc.vuv = np.ascontiguousarray(np.array(verts_t, np.float32))
    f2 = np.concatenate([F[keep], np.array(out_f, np.int64).reshape(-1, 3)]).astype(np.uint32)
    s2 = np.concatenate([S[keep], np.array(out_s, np.uint32)]).astype(np.uint32)
    sc._build_bvh(f2, s2)
    return len(big), len(out_f)


def run(sc, label):
    integ = load_dict({"type": "path_test"})
    integ.render_film(sc, seed=99, spp=64, stats=True)
    _, st = integ.render_film(sc, seed=1, spp=64, stats=True)
    _, cnt = integ.render_film(sc, seed=1, spp=64, stats=True, counters=True)
    print(label, "n_tris", sc.n_tris, "trace_ms", round(st["trace_ms"], 2), "shadow_ms", round(st["shadow_ms"], 2),
          "shade_ms", round(st["shade_ms"], 2), "nodes/ray", round(cnt["nodes_closest"] / cnt["rays_closest"], 2),
          "tris/ray", round(cnt["tris_closest"] / cnt["rays_closest"], 2), "shadow nodes/ray",
          round(cnt["nodes_shadow"] / max(1, cnt["rays_shadow"]), 2), flush=True)


if __name__ == "__main__":
    import copy
    sc = scene.bedroom(width=1280, height=720)
    run(sc, "original")
    t = copy.copy(sc)  # a new identity: the device upload is keyed by id(scene)
    nb, nn = subdivide(t, THR)
    print("subdivided", nb, "triangles into", nn, "depth", t.bvh_depth, "nodes", t.n_nodes, flush=True)
    run(t, f"tessellated(thr={THR})")
