"""Share of BVH node visits that land in the top levels of the tree (oracle
traversal, CPU): camera rays, diffuse secondary rays from their hits and
shadow rays to the emitters (occlusion tree), as in tools/bvh_experiment.py.
Sizes the LDS-resident tree tops of the traversal kernels."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "oracle"), HERE]


def node_levels(nodes, n_nodes):
    """Tree level of every 4-wide closest-hit node (mtx.h: child refs >= 0
    are inner nodes, breadth-first)."""
    w = nodes.reshape(-1, 16)
    lev = np.full(n_nodes, -1, np.int64)
    lev[0] = 0
    for i in range(n_nodes):  # breadth-first layout: parents precede children
        for k in range(int(w[i, 3].view(np.uint32) >> 24)):
            if w[i, 4 + k] >= 0:
                lev[int(w[i, 4 + k])] = lev[i] + 1
    return lev


def occ_node_levels(nodes, n_nodes):
    """Tree level of every 8-wide occlusion node (mtx.h: inner children are
    child_base + rank among the inner slots, breadth-first)."""
    w = nodes.reshape(-1, 20).view(np.uint32)
    lev = np.full(n_nodes, -1, np.int64)
    lev[0] = 0
    for i in range(n_nodes):
        n_inner = bin(int(w[i, 3] >> 24)).count("1")
        for r in range(n_inner):
            lev[int(w[i, 4]) + r] = lev[i] + 1
    return lev


def main(n=200_000):
    import binding as oracle
    from mtx import scene

    sc = scene.bedroom(cache_dir=os.path.join(ROOT, ".cache"))
    lev = node_levels(np.asarray(sc.nodes), int(sc.n_nodes))
    olev = occ_node_levels(np.asarray(sc.occ_nodes), int(sc.n_occ_nodes))
    H = 4096
    rng = np.random.default_rng(0)
    cam = sc.camera
    pos = rng.random((n, 2)).astype(np.float32)
    tx, ty = np.float32(cam.tan_x), np.float32(cam.tan_y)
    dl = np.stack([(1 - 2 * pos[:, 0]) * tx, (1 - 2 * pos[:, 1]) * ty, np.ones(n, np.float32)], 1)
    dl /= np.linalg.norm(dl, axis=1, keepdims=True)
    M = np.stack([np.array(cam.axis_x), np.array(cam.axis_y), np.array(cam.axis_z)], 1).astype(np.float32)
    d = (dl @ M.T).astype(np.float32)
    o = np.tile(np.array(cam.origin, np.float32), (n, 1))
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7], rays[:, 3] = o, d, 3e38
    h, v = oracle.trace(sc, rays)
    h = h.reshape(-1, 4)
    t = h[:, 0].view(np.float32)
    prim = h[:, 1]
    ok = prim != 0xFFFFFFFF
    g = sc.tri_geom.reshape(-1, 3, 4)[prim[ok]]
    nrm = np.cross(g[:, 1, :3], g[:, 2, :3])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm *= -np.sign(np.sum(nrm * d[ok], 1, keepdims=True))
    p = o[ok] + t[ok, None] * d[ok] + nrm * 1e-3
    u1, u2 = rng.random(len(p)), rng.random(len(p))
    r, phi = np.sqrt(u1), 2 * np.pi * u2
    a = np.where(np.abs(nrm[:, :1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
    tt = np.cross(nrm, a)
    tt /= np.linalg.norm(tt, axis=1, keepdims=True)
    bb = np.cross(nrm, tt)
    dd = (tt * (r * np.cos(phi))[:, None] + bb * (r * np.sin(phi))[:, None] + nrm * np.sqrt(1 - u1)[:, None])
    r2 = np.zeros((len(p), 8), np.float32)
    r2[:, 0:3], r2[:, 4:7], r2[:, 3] = p, dd, 3e38
    e = sc.emitters[0]
    q = (np.array(e.center) + np.outer(rng.random(len(p)) * 2 - 1, e.col0) + np.outer(rng.random(len(p)) * 2 - 1, e.col1))
    sd = q - p
    dist = np.linalg.norm(sd, axis=1)
    r3 = np.zeros((len(p), 8), np.float32)
    r3[:, 0:3], r3[:, 4:7], r3[:, 3] = p, sd / dist[:, None], dist * 0.999
    for nm, lv in (("closest-hit", lev), ("occlusion", olev)):
        print(f"{nm} nodes {len(lv)}, nodes per level (top 6):", [int((lv == k).sum()) for k in range(6)],
              "first index of level:", [int(np.argmax(lv == k)) for k in range(6)])
    for name, rr, anyh in (("primary", rays, False), ("secondary", r2, False), ("shadow", r3, True)):
        lev = olev if anyh else lev
        _, vv = oracle.trace(sc, rr, any_hit=anyh)
        tot = float(vv[:, 0].sum())
        hist = oracle.node_visit_hist(sc, rr, H, any_hit=anyh).astype(np.float64)
        cum = np.cumsum(hist) / tot
        by_lev = [float(hist[: H][lev[:H] == k].sum() / tot) for k in range(5)]
        print(f"{name:9s} visits/ray {tot / len(rr):5.2f}  share in nodes <21 {cum[20]:.3f} <32 {cum[31]:.3f} "
              f"<85 {cum[84]:.3f} <128 {cum[127]:.3f} <341 {cum[340]:.3f} <1024 {cum[1023]:.3f}  "
              f"by level 0-4 {[round(x, 3) for x in by_lev]}", flush=True)


if __name__ == "__main__":
    main()
