"""BVH build-parameter experiment on the CPU (oracle traversal counts).

Rebuilds the bedroom BVH under MTX_BVH_* settings and reports the mean node /
triangle visits of the oracle's 4-wide traversal for camera rays, diffuse
secondary rays from their hits and shadow rays to the emitters: the proxy
the GPU traversal time follows. Usage:
    python tools/bvh_experiment.py "MTX_BVH_CT=1" "MTX_BVH_CT=2" ...
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def one(env_str, n=200_000):
    import numpy as np

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "oracle")]
    import binding as oracle
    from mtx import scene

    sc = scene.bedroom(cache_dir=os.path.join(ROOT, ".cache"))
    sc._build_bvh(sc.tri_vidx.reshape(-1, 3), sc.tri_shape)
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
    # cosine-weighted diffuse directions around the normal
    u1, u2 = rng.random(len(p)), rng.random(len(p))
    r, phi = np.sqrt(u1), 2 * np.pi * u2
    a = np.where(np.abs(nrm[:, :1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
    tt = np.cross(nrm, a)
    tt /= np.linalg.norm(tt, axis=1, keepdims=True)
    bb = np.cross(nrm, tt)
    dd = (tt * (r * np.cos(phi))[:, None] + bb * (r * np.sin(phi))[:, None] + nrm * np.sqrt(1 - u1)[:, None])
    r2 = np.zeros((len(p), 8), np.float32)
    r2[:, 0:3], r2[:, 4:7], r2[:, 3] = p, dd, 3e38
    _, v2 = oracle.trace(sc, r2)
    # shadow rays to random emitter points
    em = sc.emitters[rng.integers(0, len(sc.emitters), len(p))] if False else None
    e = sc.emitters[0]
    q = (np.array(e.center) + np.outer(rng.random(len(p)) * 2 - 1, e.col0) + np.outer(rng.random(len(p)) * 2 - 1, e.col1))
    sd = q - p
    dist = np.linalg.norm(sd, axis=1)
    r3 = np.zeros((len(p), 8), np.float32)
    r3[:, 0:3], r3[:, 4:7], r3[:, 3] = p, sd / dist[:, None], dist * 0.999
    _, v3 = oracle.trace(sc, r3, any_hit=True)
    res = {"env": env_str, "nodes": int(sc.n_nodes), "depth": int(sc.bvh_depth)}
    for name, vv in (("primary", v), ("secondary", v2), ("shadow", v3)):
        res[name] = (round(float(vv[:, 0].mean()), 2), round(float(vv[:, 1].mean()), 2))
    print(res, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(sys.argv[2])
    else:
        for e in sys.argv[1:] or [""]:
            env = dict(os.environ)
            for kv in e.split():
                k, v = kv.split("=")
                env[k] = v
            subprocess.run([sys.executable, __file__, "--one", e], env=env, check=True)
