"""Wavefront OBJ and bitmap ingestion (the real bedroom
meshes ``models/*.obj`` and textures ``textures/*.jpg`` referenced at
``scene.xml:221-738``, or any scene of the same XML subset).

Restates upstream Mitsuba 3's ``obj`` shape plugin semantics:
  * ``v``, ``vt``, ``vn``, ``f`` records; negative (relative) indices;
    polygons are triangulated as fans (v0, vi, vi+1);
  * one mesh vertex per distinct (v, vt, vn) index triple, in order of first
    use;
  * ``flip_tex_coords`` (default true): uv.y = 1 - uv.y;
  * ``face_normals`` (default false) drops vertex normals; without ``vn``
    records the vertex normals are recomputed angle-weighted (Thuermer &
    Wuethrich, as Mesh::recompute_vertex_normals).
Bitmaps (``bitmap`` texture): 8-bit images are sRGB-encoded and linearised
(upstream ``raw=false``); float images are taken as linear.
"""
from __future__ import annotations

import numpy as np


def load_obj(path: str, face_normals: bool = False, flip_tex_coords: bool = True):
    """Returns (P [n,3] f64, N [n,3] f64 or None, UV [n,2] f64 or None, F [m,3] int64)."""
    pos, tex, nrm = [], [], []
    key_index: dict = {}
    verts: list = []
    faces: list = []

    def resolve(i: int, n: int) -> int:
        i = int(i)
        return i - 1 if i > 0 else n + i

    with open(path, "r", encoding="utf-8", errors="replace") as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            tag = t[0]
            if tag == "v":
                pos.append([float(x) for x in t[1:4]])
            elif tag == "vt":
                tex.append([float(x) for x in t[1:3]] + [0.0] * max(0, 2 - len(t[1:3])))
            elif tag == "vn":
                nrm.append([float(x) for x in t[1:4]])
            elif tag == "f":
                idx = []
                for c in t[1:]:
                    parts = c.split("/")
                    vi = resolve(parts[0], len(pos))
                    ti = resolve(parts[1], len(tex)) if len(parts) > 1 and parts[1] else -1
                    ni = resolve(parts[2], len(nrm)) if len(parts) > 2 and parts[2] else -1
                    key = (vi, ti, ni)
                    if key not in key_index:
                        key_index[key] = len(verts)
                        verts.append(key)
                    idx.append(key_index[key])
                for k in range(1, len(idx) - 1):
                    faces.append((idx[0], idx[k], idx[k + 1]))
    if not faces:
        raise ValueError(f"{path}: no faces")
    P_src = np.asarray(pos, np.float64)
    keys = np.asarray(verts, np.int64)
    P = P_src[keys[:, 0]]
    F = np.asarray(faces, np.int64)
    UV = None
    if tex and (keys[:, 1] >= 0).all():
        UV = np.asarray(tex, np.float64)[keys[:, 1]]
        if flip_tex_coords:
            UV[:, 1] = 1.0 - UV[:, 1]
    N = None
    if not face_normals:
        if nrm and (keys[:, 2] >= 0).all():
            N = np.asarray(nrm, np.float64)[keys[:, 2]]
        else:
            N = vertex_normals(P, F)
        ln = np.linalg.norm(N, axis=1, keepdims=True)
        N = N / np.where(ln > 0, ln, 1.0)
    return P, N, UV, F


def vertex_normals(P: np.ndarray, F: np.ndarray) -> np.ndarray:
    """Angle-weighted vertex normals (upstream Mesh::recompute_vertex_normals)."""
    N = np.zeros_like(P)
    p = [P[F[:, k]] for k in range(3)]
    n = np.cross(p[1] - p[0], p[2] - p[0])
    ln = np.linalg.norm(n, axis=1, keepdims=True)
    ok = ln[:, 0] > 0
    n = n / np.where(ln > 0, ln, 1.0)
    for k in range(3):
        d0 = p[(k + 1) % 3] - p[k]
        d1 = p[(k + 2) % 3] - p[k]
        d0 = d0 / np.maximum(np.linalg.norm(d0, axis=1, keepdims=True), 1e-300)
        d1 = d1 / np.maximum(np.linalg.norm(d1, axis=1, keepdims=True), 1e-300)
        ang = np.arccos(np.clip(np.sum(d0 * d1, 1), -1.0, 1.0))
        np.add.at(N, F[ok, k], n[ok] * ang[ok, None])
    return N


def srgb_to_linear(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float64)
    return np.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055) ** 2.4)


def load_bitmap(path: str) -> np.ndarray:
    """[H, W, 3] linear float32, rows top to bottom (uv.y = 0 is the first row)."""
    if path.lower().endswith(".exr"):
        from .util import read_exr

        return read_exr(path).astype(np.float32)
    from PIL import Image

    im = Image.open(path)
    a = np.asarray(im.convert("RGB"), np.float64) / 255.0
    return srgb_to_linear(a).astype(np.float32)


def is_real_file(path: str) -> bool:
    """False for a missing file or a Git-LFS pointer stub."""
    import os

    if not os.path.isfile(path):
        return False
    with open(path, "rb") as f:
        head = f.read(64)
    return not head.startswith(b"version https://git-lfs")
