"""Visit counts of closest-hit traversal orders on the 8-wide tree against
the 4-wide sorted tree (oracle traversals, CPU): camera
rays and cosine-weighted diffuse secondary rays of the full bedroom proxy.
Modes of oracle trace_cw_closest: 0 octant order, 1 nearest child first then
octant order, 2 entry-distance order, 3 distance order + pop culling."""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "oracle"), HERE]


def camera_and_bounce_rays(sc, oracle, n, seed=0):
    rng = np.random.default_rng(seed)
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
    h, _ = oracle.trace(sc, rays)
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
    return rays, r2


def main(n=100_000):
    import binding as oracle
    from mtx import scene

    oracle.build()
    sc = scene.bedroom(cache_dir=os.path.join(ROOT, ".cache"))
    L = oracle.lib()
    L.orc_trace_cw_closest.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    d = sc.desc()
    for name, rays in zip(("camera", "bounce"), camera_and_bounce_rays(sc, oracle, n)):
        h4, v4 = oracle.trace(sc, rays)
        t4 = h4.reshape(-1, 4)[:, 0].view(np.float32)
        v4 = v4.reshape(-1, 2)
        line = {"rays": name, "n": len(rays), "bvh4_sorted": [float(v4[:, 0].mean()), float(v4[:, 1].mean())]}
        for mode in range(4):
            t = np.zeros(len(rays), np.float32)
            v = np.zeros((len(rays), 2), np.uint32)
            rr = np.ascontiguousarray(rays)
            L.orc_trace_cw_closest(C.byref(d), len(rr), rr.ctypes.data, mode, t.ctypes.data, v.ctypes.data)
            assert np.array_equal(t, t4), (name, mode, int((t != t4).sum()))
            ms = v[:, 0] >> 16
            line[f"cw8_mode{mode}"] = [float((v[:, 0] & 0xffff).mean()), float(v[:, 1].mean()),
                                       int(np.percentile(ms, 50)), int(np.percentile(ms, 99)), int(ms.max())]
        hp, vp = oracle.trace(sc, rays, 2)  # the production 8-wide traversal (trace_closest_cw)
        assert np.array_equal(hp, h4)
        line["cw8_production"] = [float(vp[:, 0].mean()), float(vp[:, 1].mean())]
        t = np.zeros(len(rays), np.float32)
        v = np.zeros((len(rays), 2), np.uint32)
        rr = np.ascontiguousarray(rays)
        L.orc_trace_cw_closest(C.byref(d), len(rr), rr.ctypes.data, 16, t.ctypes.data, v.ctypes.data)
        assert np.array_equal(t, t4), (name, "bvh4 cull")
        msp = v[:, 0] >> 16
        line["bvh4_sorted_popcull"] = [float((v[:, 0] & 0xffff).mean()), float(v[:, 1].mean())]
        line["bvh4_popcull_max_stack_p50_p99_max"] = [int(np.percentile(msp, 50)), int(np.percentile(msp, 99)), int(msp.max())]
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000)
