"""Deterministic bedroom-proxy geometry.

The reference benchmark scene (``data/bedroom/scene.xml``) keeps its camera,
film, BSDF table and emitters in the XML, but all 70 OBJ meshes and the 4
textures are Git-LFS pointers. This module replaces each OBJ shape by a
procedurally generated mesh with a fixed, versioned triangle budget

    budget(shape) = ceil(lfs_size(shape.obj) / 96 B)

(≈1.83 M triangles in total; ``Carpet_0002`` alone is ≈1.38 M, the skew that
dominates BVH size and traversal cost). Each mesh is a parametric surface
placed inside the room volume that the camera (scene.xml:13) and the two
window emitters (scene.xml:706-731) imply; shapes keep their XML material,
``face_normals`` flag and ``to_world`` transform. Everything is computed in
float64 with fixed formulas and a seeded generator, then rounded to float32,
so the scene is bit-identical on every machine.
"""
from __future__ import annotations

import math

import numpy as np

PROXY_VERSION = 2
BYTES_PER_TRI = 96


def budget_from_lfs(size: int | None, scale: float = 1.0, minimum: int = 2) -> int:
    """ceil(size / 96 B); scaled-down test scenes keep >= min(full budget, 64)
    triangles per shape so that closed shapes (walls, boxes) stay closed."""
    if not size:
        return minimum
    b = math.ceil(size / BYTES_PER_TRI)
    if scale == 1.0:
        return max(minimum, b)
    return max(minimum, min(b, 64), int(round(b * scale)))


class MeshBuilder:
    """Accumulates parametric patches into one indexed mesh."""

    def __init__(self):
        self.P, self.N, self.UV, self.F = [], [], [], []
        self.nv = 0

    def add(self, P, N, UV, F):
        self.P.append(P)
        self.N.append(N)
        self.UV.append(UV)
        self.F.append(F + self.nv)
        self.nv += len(P)

    def ntris(self) -> int:
        return int(sum(len(f) for f in self.F))

    def build(self):
        P = np.concatenate(self.P) if self.P else np.zeros((0, 3))
        N = np.concatenate(self.N) if self.N else np.zeros((0, 3))
        UV = np.concatenate(self.UV) if self.UV else np.zeros((0, 2))
        F = np.concatenate(self.F) if self.F else np.zeros((0, 3), np.int64)
        return P, N, UV, F


def _grid_dims(ntri: int, aspect: float):
    """Columns C and full rows R with 2*R*C <= ntri, plus the ragged remainder."""
    nq = max(ntri // 2, 1)
    C = max(1, int(round(math.sqrt(nq * aspect))))
    C = min(C, nq)
    R = max(1, nq // C)
    rem = ntri - 2 * R * C
    if rem < 0:
        R -= 1
        rem = ntri - 2 * R * C
    return C, R, rem


def param_patch(mb: MeshBuilder, fn, ntri: int, aspect: float = 1.0, uv_scale=(1.0, 1.0)):
    """Tessellate fn(u, v) -> points [.., 3] over [0,1]^2 into exactly ntri triangles.

    Quads (i, j) -> triangles (a, b, c), (a, c, d) so that the geometric normal
    is dP/du x dP/dv. A ragged extra row takes the remainder.
    """
    if ntri <= 0:
        return
    C, R, rem = _grid_dims(ntri, aspect)
    if R == 0:  # a single triangle
        C, R, rem = 1, 1, ntri - 2
    u = np.linspace(0.0, 1.0, C + 1)
    v = np.linspace(0.0, 1.0, R + 1)
    U, V = np.meshgrid(u, v)  # [R+1, C+1]
    idx = np.arange((R + 1) * (C + 1)).reshape(R + 1, C + 1)
    a = idx[:R, :C].ravel()
    b = idx[:R, 1:].ravel()
    c = idx[1:R + 1, 1:].ravel()
    d = idx[1:R + 1, :C].ravel()
    F = np.concatenate([np.stack([a, b, c], 1).reshape(-1, 1, 3), np.stack([a, c, d], 1).reshape(-1, 1, 3)],
                       1).reshape(-1, 3)
    Uf, Vf = U.ravel(), V.ravel()
    if rem < 0:  # fewer triangles than one quad: keep the first
        F = F[:ntri]
    elif rem > 0:
        # Exact budget without holes: split (rem // 2) triangles at their
        # parametric centroid (1 -> 3) and, for an odd remainder, one
        # triangle at the midpoint of its edge on the v = 0 boundary (1 -> 2).
        extra_u, extra_v, newF, drop = [], [], [], []
        nv = len(Uf)
        bt = 2 * (C - 1)  # first triangle of the last quad of row 0: edge (a, b) lies on v = 0
        if rem % 2:
            ta, tb, tc = F[bt]
            extra_u.append(0.5 * (Uf[ta] + Uf[tb]))
            extra_v.append(0.0)
            newF += [(ta, nv, tc), (nv, tb, tc)]
            drop.append(bt)
            nv += 1
        k = 0
        t = 0
        while k < rem // 2:
            if t != bt or rem % 2 == 0:
                ta, tb, tc = F[t]
                extra_u.append((Uf[ta] + Uf[tb] + Uf[tc]) / 3.0)
                extra_v.append((Vf[ta] + Vf[tb] + Vf[tc]) / 3.0)
                newF += [(ta, tb, nv), (tb, tc, nv), (tc, ta, nv)]
                drop.append(t)
                nv += 1
                k += 1
            t += 1
        keep = np.ones(len(F), bool)
        keep[drop] = False
        F = np.concatenate([F[keep], np.array(newF, np.int64)])
        Uf = np.concatenate([Uf, extra_u])
        Vf = np.concatenate([Vf, extra_v])
    P = fn(Uf, Vf)
    eps = 1e-5
    du = fn(np.clip(Uf + eps, 0, 1), Vf) - fn(np.clip(Uf - eps, 0, 1), Vf)
    dv = fn(Uf, np.clip(Vf + eps, 0, 1)) - fn(Uf, np.clip(Vf - eps, 0, 1))
    N = np.cross(du, dv)
    ln = np.linalg.norm(N, axis=-1, keepdims=True)
    N = np.where(ln > 1e-20, N / np.maximum(ln, 1e-30), np.array([0.0, 1.0, 0.0]))
    UV = np.stack([Uf * uv_scale[0], Vf * uv_scale[1]], -1)
    mb.add(P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), F.astype(np.int64))


# ---------------------------------------------------------------- surfaces --

def quad(o, ex, ey):
    o, ex, ey = map(np.asarray, (o, ex, ey))
    return lambda U, V: o + U[..., None] * ex + V[..., None] * ey


def box_patches(mb, lo, hi, ntri, bump=0.0, seed=0):
    """Axis-aligned box with outward normals; faces share the budget by area."""
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    d = hi - lo
    faces = [  # (origin, e_u, e_v) with e_u x e_v pointing outward
        (lo, [0, 0, d[2]], [0, d[1], 0]),                    # -x
        ([hi[0], lo[1], lo[2]], [0, d[1], 0], [0, 0, d[2]]),  # +x
        (lo, [d[0], 0, 0], [0, 0, d[2]]),                    # -y
        ([lo[0], hi[1], lo[2]], [0, 0, d[2]], [d[0], 0, 0]),  # +y
        (lo, [0, d[1], 0], [d[0], 0, 0]),                    # -z
        ([lo[0], lo[1], hi[2]], [d[0], 0, 0], [0, d[1], 0]),  # +z
    ]
    areas = np.array([np.linalg.norm(np.cross(f[1], f[2])) for f in faces])
    alloc = _split(ntri, areas)
    for (o, eu, ev), n in zip(faces, alloc):
        eu, ev = np.asarray(eu, float), np.asarray(ev, float)
        asp = max(np.linalg.norm(eu), 1e-9) / max(np.linalg.norm(ev), 1e-9)
        base = quad(o, eu, ev)
        if bump > 0.0:
            nrm = np.cross(eu, ev)
            nrm = nrm / np.linalg.norm(nrm)
            ph = 1.7 * seed + 0.3

            def fn(U, V, base=base, nrm=nrm, ph=ph):
                w = np.sin(9.0 * U + ph) * np.sin(7.0 * V + 2 * ph) * 4 * U * (1 - U) * 4 * V * (1 - V)
                return base(U, V) + bump * w[..., None] * nrm
            param_patch(mb, fn, n, asp)
        else:
            param_patch(mb, base, n, asp)


def _split(ntri, weights):
    weights = np.asarray(weights, float)
    weights = weights / weights.sum()
    alloc = np.floor(weights * ntri).astype(int)
    alloc[np.argmax(weights)] += ntri - alloc.sum()
    return alloc


def ellipsoid(c, r):
    c, r = np.asarray(c, float), np.asarray(r, float)

    def fn(U, V):
        th = math.pi * (1.0 - V)  # V=0 south pole -> outward with this winding
        ph = 2 * math.pi * U
        return c + r * np.stack([np.sin(th) * np.cos(ph), np.cos(th), -np.sin(th) * np.sin(ph)], -1)
    return fn


def revolve(c, prof_r, prof_y):
    """Surface of revolution about +y through c; prof_r/prof_y map v in [0,1]."""
    c = np.asarray(c, float)

    def fn(U, V):
        ph = 2 * math.pi * U
        r = prof_r(V)
        y = prof_y(V)
        return c + np.stack([r * np.cos(ph), y, -r * np.sin(ph)], -1)
    return fn


def tube(p0, p1, radius):
    """Open cylinder from p0 to p1."""
    p0, p1 = np.asarray(p0, float), np.asarray(p1, float)
    ax = p1 - p0
    L = np.linalg.norm(ax)
    w = ax / L
    t = np.array([1.0, 0, 0]) if abs(w[0]) < 0.9 else np.array([0, 1.0, 0])
    a = np.cross(w, t)
    a /= np.linalg.norm(a)
    b = np.cross(w, a)

    def fn(U, V):
        ph = 2 * math.pi * U
        return p0 + V[..., None] * ax + radius * (np.cos(ph)[..., None] * a + np.sin(ph)[..., None] * b)
    return fn


def heightfield(x0, x1, z0, z1, hfn):
    def fn(U, V):
        x = x0 + (x1 - x0) * (1.0 - U)
        z = z0 + (z1 - z0) * V
        return np.stack([x, hfn(x, z), z], -1)
    return fn


def noise2(x, z, seed, octaves=4):
    """Deterministic smooth value noise (sum of fixed sinusoids)."""
    rng = np.random.default_rng(seed)
    h = np.zeros_like(x)
    amp = 1.0
    for o in range(octaves):
        f = 3.0 * (2.1 ** o)
        a1, a2, p1, p2 = rng.uniform(0.5, 1.5), rng.uniform(0.5, 1.5), rng.uniform(0, 6.3), rng.uniform(0, 6.3)
        h += amp * np.sin(f * a1 * x + p1) * np.sin(f * a2 * z + p2)
        amp *= 0.55
    return h


# ------------------------------------------------------------- room layout --
# Room volume implied by the sensor (scene.xml:13, at (3.46, 1.21, 3.30)
# looking towards -x/-z) and the window emitters on the z = -1.27 wall.
ROOM = dict(x0=-3.1, x1=3.9, y0=0.0, y1=2.7, z0=-1.32, z1=3.75)


def _walls(mb, n):
    r = ROOM
    faces = [  # inward-facing walls + ceiling
        ((r["x0"], r["y0"], r["z1"]), (0, 0, r["z0"] - r["z1"]), (0, r["y1"], 0)),
        ((r["x1"], r["y0"], r["z0"]), (0, 0, r["z1"] - r["z0"]), (0, r["y1"], 0)),
        ((r["x0"], r["y0"], r["z0"]), (r["x1"] - r["x0"], 0, 0), (0, r["y1"], 0)),
        ((r["x1"], r["y0"], r["z1"]), (r["x0"] - r["x1"], 0, 0), (0, r["y1"], 0)),
        ((r["x0"], r["y1"], r["z0"]), (r["x1"] - r["x0"], 0, 0), (0, 0, r["z1"] - r["z0"])),
    ]
    areas = [np.linalg.norm(np.cross(f[1], f[2])) for f in faces]
    for (o, eu, ev), k in zip(faces, _split(n, areas)):
        param_patch(mb, quad(o, eu, ev), k, np.linalg.norm(eu) / np.linalg.norm(ev))


def _shape_mesh(sid: str, n: int, k: int, mb: MeshBuilder):
    """Geometry for OBJ shape `sid` with exactly n triangles (k = instance index)."""
    r = ROOM
    if sid == "Walls":
        _walls(mb, n)
    elif sid == "Walls2":  # wainscot panels on the bed wall (x = x0)
        param_patch(mb, quad((r["x0"] + 0.02, 0.0, 3.2), (0, 0, -4.3), (0, 1.0, 0)), n, 4.3)
    elif sid == "WoodFloor":
        param_patch(mb, quad((r["x0"], 0.0, r["z0"]), (0, 0, r["z1"] - r["z0"]), (r["x1"] - r["x0"], 0, 0)), n,
                    0.72, uv_scale=(6.0, 8.0))
    elif sid == "Carpet_0002":
        def h(x, z):
            return 0.014 + 0.006 * noise2(x * 8.0, z * 8.0, 11, 5)
        param_patch(mb, heightfield(-1.05, 2.05, -0.55, 2.45, h), n, 1.0)
    elif sid == "Carpet_0001":  # underlay border
        box_patches(mb, (-1.12, 0.0, -0.62), (2.12, 0.008, 2.52), n)
    elif sid == "Matress":
        box_patches(mb, (-3.05, 0.28, 0.25), (-1.05, 0.52, 2.55), n, bump=0.01, seed=1)
    elif sid.startswith("Bedsheets"):
        if k == 0:  # sheet draped over the mattress
            def fn(U, V):
                x = -1.02 - 2.06 * U
                z = 0.22 + 2.36 * V
                y = 0.535 + 0.012 * noise2(x * 3, z * 3, 5, 4)
                edge = np.maximum(np.maximum(0.08 - U * 2.06, U * 2.06 - 1.98), 0.0) / 0.08
                return np.stack([x, y - 0.25 * np.clip(edge, 0, 1), z], -1)
            param_patch(mb, fn, n, 0.9)
        else:  # pillows
            param_patch(mb, ellipsoid((-2.7, 0.62, 0.75 + 0.8 * (k - 1)), (0.22, 0.08, 0.34)), n, 2.0)
    elif sid.startswith("Blankets"):
        def fn(U, V, k=k):
            x = -1.0 - 2.1 * U
            z = 1.45 + 1.15 * V
            y = 0.56 + 0.018 * k + 0.02 * np.sin(14 * z + k) * np.sin(5 * x) + 0.01 * noise2(x * 4, z * 4, 20 + k, 3)
            edge = np.maximum(np.maximum(0.1 - U * 2.1, U * 2.1 - 2.0), 0.0) / 0.1
            return np.stack([x, y - 0.3 * np.clip(edge, 0, 1), z], -1)
        param_patch(mb, fn, n, 1.6)
    elif sid.startswith("WoodFurniture"):
        boxes = [((-3.1, 0.0, 0.15), (-0.95, 0.3, 2.65)),   # bed frame
                 ((-3.05, 0.0, -0.45), (-2.55, 0.55, 0.05)),  # nightstand
                 ((-3.05, 0.0, 2.75), (-2.55, 0.55, 3.25)),  # nightstand
                 ((2.9, 0.0, 1.0), (3.85, 2.1, 2.6)),        # wardrobe
                 ((0.8, 0.0, -1.28), (2.4, 0.75, -0.85)),    # dresser under a window
                 ((-3.08, 0.9, 0.5), (-2.95, 1.7, 2.3)),     # headboard
                 ((2.5, 0.0, -1.25), (3.6, 0.45, -0.7))]     # bench
        lo, hi = boxes[k % len(boxes)]
        box_patches(mb, lo, hi, n)
    elif sid.startswith("Aluminium"):
        x = 2.88 + 0.0 * k
        param_patch(mb, tube((x, 0.7 + 0.14 * k, 1.3 + 0.1 * (k % 3)), (x - 0.05, 0.7 + 0.14 * k, 1.3 + 0.1 * (k % 3)),
                             0.012 + 0.002 * (k % 2)), n, 6.0)
    elif sid.startswith("StainlessSmooth"):
        x0 = 0.9 + 0.3 * k
        param_patch(mb, tube((x0, 0.75, -0.9), (x0, 0.95 + 0.03 * k, -0.9), 0.015 + 0.004 * k), n, 6.0)
    elif sid == "LampMetal_0001":  # floor lamp: stand + base
        n1 = n // 2
        param_patch(mb, tube((3.3, 0.02, -0.75), (3.3, 1.55, -0.75), 0.018), n1, 4.0)
        param_patch(mb, revolve((3.3, 0.0, -0.75), lambda V: 0.2 * np.sin(math.pi * V) + 0.01, lambda V: 0.03 * V), n - n1, 3.0)
    elif sid.startswith("LampMetal"):  # bedside lamp stands
        z = -0.2 if k == 1 else 3.0
        param_patch(mb, revolve((-2.8, 0.55, z), lambda V: 0.05 + 0.03 * np.cos(6 * V), lambda V: 0.35 * V), n, 2.0)
    elif sid.startswith("LampGlass"):
        if k == 0:
            param_patch(mb, ellipsoid((-2.8, 1.05, -0.2), (0.12, 0.14, 0.12)), n, 2.0)
        elif k == 1:
            param_patch(mb, ellipsoid((-2.8, 1.05, 3.0), (0.12, 0.14, 0.12)), n, 2.0)
        elif k == 2:  # floor-lamp shade (roughdielectric, 45 k triangles)
            param_patch(mb, ellipsoid((3.3, 1.7, -0.75), (0.26, 0.2, 0.26)), n, 2.0)
        else:
            param_patch(mb, ellipsoid((-2.8, 0.95, -0.2 if k == 3 else 3.0), (0.05, 0.05, 0.05)), n, 2.0)
    elif sid.startswith("LampEmitter"):
        c = [(3.3, 1.68, -0.75), (-2.8, 1.02, -0.2), (-2.8, 1.02, 3.0)][k % 3]
        param_patch(mb, ellipsoid(c, (0.05, 0.07, 0.05)), n, 2.0)
    elif sid == "DecoPlant":
        rng = np.random.default_rng(7)
        nl = max(1, n // 120)
        per = _split(n, np.ones(nl))
        for i, m in enumerate(per):
            a = rng.uniform(0, 2 * math.pi)
            tilt = rng.uniform(0.3, 1.2)
            base = np.array([3.35, 0.35, 3.3]) + rng.uniform(-0.05, 0.05, 3) * [1, 0, 1]
            L = rng.uniform(0.3, 0.6)

            def fn(U, V, a=a, tilt=tilt, base=base, L=L):
                s = V * L
                wdt = 0.04 * np.sin(math.pi * V) * (U - 0.5) * 2
                dirv = np.array([math.cos(a) * math.sin(tilt), math.cos(tilt), math.sin(a) * math.sin(tilt)])
                side = np.array([-math.sin(a), 0.0, math.cos(a)])
                droop = -0.25 * (s ** 2)
                return base + s[..., None] * dirv + wdt[..., None] * side + droop[..., None] * np.array([0, 1.0, 0])
            param_patch(mb, fn, m, 0.2)
    elif sid.startswith("Rocks"):
        param_patch(mb, ellipsoid((1.1 + 0.09 * k, 0.79, -1.05 + 0.04 * k), (0.05, 0.035, 0.045)), n, 2.0)
    elif sid.startswith("Painting"):  # between the windows; XML to_world shifts the copies along x
        param_patch(mb, quad((0.12, 1.25, r["z0"] + 0.02), (0.3, 0, 0), (0, 0.42, 0)), n, 0.72)
    elif sid == "Picture":
        param_patch(mb, quad((r["x1"] - 0.03, 1.0, -0.3), (0, 0, 0.8), (0, 0.6, 0)), n, 1.33)
    elif sid == "PictureFrame":
        box_patches(mb, (r["x1"] - 0.05, 0.96, -0.34), (r["x1"] - 0.02, 1.64, 0.54), n)
    elif sid == "PictureBacking":
        param_patch(mb, quad((r["x1"] - 0.01, 0.95, -0.35), (0, 0, 0.9), (0, 0.7, 0)), n, 1.3)
    elif sid == "Mirror_0001" or sid == "Mirror_0002":
        z0 = 2.75 if k == 0 else 3.2
        param_patch(mb, quad((r["x1"] - 0.02, 0.7, z0), (0, 0, 0.4), (0, 1.2, 0)), n, 0.33)
    elif sid == "Glass":
        param_patch(mb, revolve((-2.75, 0.55, 2.9), lambda V: 0.035 + 0.005 * V, lambda V: 0.12 * V), n, 3.0)
    elif sid.startswith("Vase"):
        x = 1.6 + 0.35 * k

        def pr(V):
            return 0.05 + 0.06 * np.sin(math.pi * V * 0.9) + 0.01
        param_patch(mb, revolve((x, 0.75, -1.0), pr, lambda V: 0.35 * V), n, 3.0)
    elif sid == "BookCover":
        box_patches(mb, (-3.0, 0.55, -0.35), (-2.75, 0.6, -0.15), n)
    elif sid == "BookPages":
        box_patches(mb, (-2.99, 0.6, -0.34), (-2.76, 0.62, -0.16), n)
    elif sid == "Boxes":
        box_patches(mb, (3.0, 2.1, 1.2), (3.7, 2.4, 2.3), n)
    elif sid.startswith("PlasticCable"):
        z = -0.2 if k == 0 else 3.0

        def fn(U, V, z=z):
            t = V
            p = np.array([-2.8, 0.55, z]) * (1 - t)[..., None] + np.array([-3.05, 0.01, z + 0.6]) * t[..., None]
            ph = 2 * math.pi * U
            return p + 0.006 * np.stack([np.cos(ph), np.sin(ph), np.zeros_like(ph)], -1)
        param_patch(mb, fn, n, 8.0)
    elif sid.startswith("CurtainRod"):
        xc = -1.475 if k == 0 else 1.444
        param_patch(mb, tube((xc - 0.95, 2.32, -1.18), (xc + 0.95, 2.32, -1.18), 0.015), n, 8.0)
    elif sid.startswith("Curtains"):
        xc = -1.475 if k == 0 else 1.444
        n1 = n // 2
        for side, m in ((-1, n1), (1, n - n1)):
            def fn(U, V, side=side, xc=xc):
                x = xc + side * (0.62 + 0.28 * U)
                y = 2.3 * (1.0 - V)
                z = -1.12 + 0.05 * np.sin(2 * math.pi * 5 * U)
                return np.stack([x, y, z], -1)
            param_patch(mb, fn, m, 0.2)
    elif sid.startswith("Window"):
        xc = -1.475 if k == 0 else 1.444
        bars = [((xc - 0.6, 0.22, -1.3), (xc + 0.6, 0.3, -1.2)), ((xc - 0.6, 2.08, -1.3), (xc + 0.6, 2.16, -1.2)),
                ((xc - 0.62, 0.22, -1.3), (xc - 0.54, 2.16, -1.2)), ((xc + 0.54, 0.22, -1.3), (xc + 0.62, 2.16, -1.2)),
                ((xc - 0.012, 0.3, -1.25), (xc + 0.012, 2.08, -1.23))]
        for (lo, hi), m in zip(bars, _split(n, [1, 1, 1, 1, 1])):
            box_patches(mb, lo, hi, m)
    else:  # unknown shape name: small box on the floor
        box_patches(mb, (0.0, 0.0, 0.0), (0.1, 0.1, 0.1), n)


def generate_mesh(sid: str, ntri: int, instance: int):
    mb = MeshBuilder()
    _shape_mesh(sid, ntri, instance, mb)
    P, N, UV, F = mb.build()
    if len(F) != ntri:
        raise AssertionError(f"proxy {sid}: {len(F)} triangles generated for a budget of {ntri}")
    return P, N, UV, F


# ---------------------------------------------------------------- textures --

def procedural_texture(name: str, res: int) -> np.ndarray:
    """Linear-RGB float texture standing in for the LFS bitmap `name`."""
    y, x = np.meshgrid(np.linspace(0, 1, res, endpoint=False), np.linspace(0, 1, res, endpoint=False), indexing="ij")
    if "wood" in name:
        ring = 0.5 + 0.5 * np.sin(40 * (x + 0.15 * np.sin(6 * y)) + 3 * noise2(x * 3, y * 3, 3, 3))
        base = np.array([0.32, 0.17, 0.07]) if "panel" in name else np.array([0.45, 0.26, 0.12])
        img = base * (0.65 + 0.35 * ring)[..., None]
    elif "wallpaper" in name:
        stripe = (np.floor(x * 16) % 2)[..., None]
        img = np.array([0.55, 0.5, 0.42]) * (0.8 + 0.2 * stripe) + 0.05 * np.sin(30 * y)[..., None]
    else:  # Teapot.png: smooth colourful picture
        img = np.stack([0.2 + 0.6 * x, 0.3 + 0.4 * y, 0.5 + 0.3 * np.sin(6 * x * y)], -1)
    return np.clip(img, 0.01, 0.95).astype(np.float32)
