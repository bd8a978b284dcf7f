"""Scene assembly: bedroom description -> SoA arrays -> BVH -> mtx_scene_desc.

Replaces ``mi.load_file('data/bedroom/scene.xml')`` (and the Embree/OptiX
acceleration-structure build behind it) for the integrators. The geometry is
the deterministic bedroom proxy (:mod:`mtx.proxy`); materials, textures,
sensor and emitters follow the XML (committed as ``data/bedroom.json`` by
``tools/extract_bedroom.py``).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os

import numpy as np

from . import _abi, proxy

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def load_bedroom_spec() -> dict:
    with open(os.path.join(DATA, "bedroom.json")) as f:
        return json.load(f)


def _m4(vals):
    return np.asarray(vals, dtype=np.float64).reshape(4, 4)


def _rgb3(v):
    """A radiance given as one float or three."""
    a = np.asarray(v, dtype=np.float64).reshape(-1)
    return np.repeat(a, 3) if a.size == 1 else a[:3]


class Scene:
    """Host-side scene: numpy arrays in the mtx.h layout plus the BVH.

    Attributes mirror mtx_scene_desc. ``desc()`` returns the C struct pointing
    at these arrays (they must stay alive while the struct is used).
    """

    def __init__(self):
        self.meta = {}
        self.env_radiance = None  # constant environment radiance (rgb) or None

    # ------------------------------------------------------------ building --
    @classmethod
    def bedroom(cls, width: int | None = None, height: int | None = None, scale: float = 1.0,
                tex_res: int = 512, spec: dict | None = None, base_dir: str | None = None,
                strict: bool = False) -> "Scene":
        """The bedroom proxy. `scale` multiplies every triangle budget
        (1.0 = the versioned ≈1.83 M-triangle benchmark scene).

        With `base_dir` (the directory of the scene XML), meshes and bitmaps
        whose files exist there (and are not Git-LFS pointers) are loaded
        from disk (:mod:`mtx.obj`); the others fall back to the proxy.
        `strict` (scenes converted from Mitsuba dictionaries): a mesh or
        bitmap without a readable file raises MtxError instead of falling back
        to the proxy -- the scene would otherwise differ from the one the
        dictionary describes."""
        from . import obj as objio
        spec = spec or load_bedroom_spec()
        s = cls()
        film = spec["sensor"]["film"]
        W = int(width or film["width"])
        H = int(height or film["height"])

        # ---------------- materials (scene.xml:26-219 + inline emitter BSDFs)
        tex_names, texels, textures = [], [], []
        tables = []
        mats, mat_index = [], {}
        loaded = []  # files read from base_dir

        def texture_id(t):
            fn = t.get("filename", "tex")
            if fn in tex_names:
                return tex_names.index(fn)
            full = os.path.join(base_dir, fn) if base_dir else None
            if full and objio.is_real_file(full):
                img = objio.load_bitmap(full)
                loaded.append(fn)
            elif strict:
                from ._lib import MtxError
                raise MtxError(f"bitmap {fn!r}: no readable file under {base_dir!r}")
            else:
                img = proxy.procedural_texture(fn, tex_res)
            off = sum(x.size for x in texels)
            texels.append(np.ascontiguousarray(img, np.float32).reshape(-1))
            textures.append((img.shape[1], img.shape[0], off))
            tex_names.append(fn)
            return len(tex_names) - 1

        def convert(b) -> _abi.Material:
            m = _abi.Material()
            m.tex = -1
            m.opacity = 1.0
            m.table = -1
            flags = 0
            while b["type"] in ("twosided", "mask"):
                if b["type"] == "twosided":
                    flags |= _abi.MTX_MF_TWOSIDED
                else:
                    flags |= _abi.MTX_MF_MASK
                    m.opacity = float(b.get("opacity", 0.5))
                b = b["nested"]
            t = b["type"]
            if b.get("distribution", "beckmann") == "beckmann":
                flags |= _abi.MTX_MF_BECKMANN
            m.alpha = float(b.get("alpha", 0.1))
            eta = float(b.get("int_ior", 1.5046)) / float(b.get("ext_ior", 1.000277))
            if t == "diffuse":
                m.type = _abi.MTX_MAT_DIFFUSE
                refl = b.get("reflectance", [0.5, 0.5, 0.5])
                if isinstance(refl, dict):
                    m.tex = texture_id(refl)
                else:
                    m.rgb[:] = refl
            elif t == "roughplastic":
                m.type = _abi.MTX_MAT_ROUGHPLASTIC
                m.eta = eta
                if b.get("nonlinear", False):
                    flags |= _abi.MTX_MF_NONLINEAR
                d = b.get("diffuse_reflectance", [0.5, 0.5, 0.5])
                if isinstance(d, dict):
                    m.tex = texture_id(d)
                    d_mean = float(texels[m.tex].mean())
                else:
                    m.rgb[:] = d
                    d_mean = float(np.mean(d))
                m.spec_weight = 1.0 / (d_mean + 1.0)  # s_mean / (d_mean + s_mean), s_mean = 1
                tab = np.zeros(_abi.MTX_ROUGH_TRANSMITTANCE_RES, np.float32)
                internal = C.c_float()
                from ._lib import check, lib
                check(lib().mtx_roughplastic_tables(1 if flags & _abi.MTX_MF_BECKMANN else 0, m.alpha, m.eta,
                                                    tab.ctypes.data, C.byref(internal)), "mtx_roughplastic_tables")
                m.internal_refl = internal.value
                m.table = sum(x.size for x in tables)
                tables.append(tab)
            elif t == "conductor":
                m.type = _abi.MTX_MAT_CONDUCTOR
                m.rgb[:] = b.get("specular_reflectance", [1.0, 1.0, 1.0])
                m.eta_rgb[:] = b.get("eta", [0.0, 0.0, 0.0])  # material "none": eta = 0, k = 1
                m.k_rgb[:] = b.get("k", [1.0, 1.0, 1.0])
            elif t == "roughconductor":
                m.type = _abi.MTX_MAT_ROUGHCONDUCTOR
                m.rgb[:] = b.get("specular_reflectance", [1.0, 1.0, 1.0])
                m.eta_rgb[:] = b.get("eta", [0.0, 0.0, 0.0])
                m.k_rgb[:] = b.get("k", [1.0, 1.0, 1.0])
            elif t == "dielectric":
                m.type = _abi.MTX_MAT_DIELECTRIC
                m.eta = eta
            elif t == "roughdielectric":
                m.type = _abi.MTX_MAT_ROUGHDIELECTRIC
                m.eta = eta
            else:
                raise ValueError(f"unsupported bsdf type {t}")
            m.flags = flags
            return m

        for bid, b in spec["bsdfs"].items():
            mat_index[bid] = len(mats)
            mats.append(convert(b))

        # ---------------- shapes
        P_all, N_all, UV_all, F_all, shape_of_tri = [], [], [], [], []
        shapes, emitters = [], []
        nv = 0
        family_count = {}
        budgets = {}
        for sd in spec["shapes"]:
            M = _m4(sd["to_world"]) if sd.get("to_world") else np.eye(4)
            if sd["type"] == "rectangle":
                loc = np.array([[-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0]], np.float64)
                P = loc @ M[:3, :3].T + M[:3, 3]
                F = np.array([[0, 1, 2], [0, 2, 3]], np.int64)
                N = np.zeros_like(P)
                UV = (loc[:, :2] + 1) * 0.5
                flags = 1  # face normals
            elif sd["type"] == "cube":
                # Mitsuba's cube: [-1, 1]^3, two outward-wound triangles per face
                P, F = _cube_mesh()
                P = P @ M[:3, :3].T + M[:3, 3]
                N = np.zeros_like(P)
                UV = np.zeros((len(P), 2))
                flags = 1  # face normals
            elif base_dir and sd.get("filename") and objio.is_real_file(os.path.join(base_dir, sd["filename"])):
                if sd["type"] != "obj":
                    raise ValueError(f"shape type {sd['type']!r} is not supported (obj, rectangle)")
                face_n = bool(sd.get("face_normals", False))
                P, N, UV, F = objio.load_obj(os.path.join(base_dir, sd["filename"]), face_normals=face_n,
                                             flip_tex_coords=bool(sd.get("flip_tex_coords", True)))
                loaded.append(sd["filename"])
                P = P @ M[:3, :3].T + M[:3, 3]
                flags = 0
                if N is None:
                    N = np.zeros_like(P)
                    flags |= 1
                else:
                    N = N @ np.linalg.inv(M[:3, :3])  # normals transform with the inverse transpose
                    N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-30)
                if UV is None:
                    UV = np.zeros((len(P), 2))
                else:
                    flags |= 2
                budgets[sd["id"]] = len(F)
            elif strict:
                from ._lib import MtxError
                raise MtxError(f"shape {sd['id']!r} ({sd['type']}): "
                               + (f"no readable file {sd['filename']!r} under {base_dir!r}" if sd.get("filename")
                                  else "no filename"))
            else:
                fam = sd["id"].split("_")[0]
                k = family_count.get(fam, 0)
                family_count[fam] = k + 1
                n = proxy.budget_from_lfs(sd.get("lfs_size"), scale)
                budgets[sd["id"]] = n
                P, N, UV, F = proxy.generate_mesh(sd["id"], n, k)
                P = P @ M[:3, :3].T + M[:3, 3]
                Ninv = np.linalg.inv(M[:3, :3]).T
                N = N @ Ninv.T
                N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-30)
                flags = (1 if sd.get("face_normals", False) else 0) | 2
            if "bsdf" in sd:
                mid = mat_index[sd["bsdf"]]
            else:
                mid = len(mats)
                mats.append(convert(sd["bsdf_inline"]))
            em = -1
            if "emitter" in sd:
                em = len(emitters)
                e = _abi.Emitter()
                e.center[:] = M[:3, 3]
                e.col0[:] = M[:3, 0]
                e.col1[:] = M[:3, 1]
                nrm = np.linalg.inv(M[:3, :3]).T @ np.array([0.0, 0.0, 1.0])
                e.normal[:] = nrm / np.linalg.norm(nrm)
                e.inv_area = 1.0 / np.linalg.norm(np.cross(2 * M[:3, 0], 2 * M[:3, 1]))
                e.radiance[:] = sd["emitter"]["radiance"]
                emitters.append(e)
            sh = _abi.Shape()
            sh.material, sh.emitter, sh.flags = mid, em, flags
            shapes.append(sh)
            P_all.append(P)
            N_all.append(N)
            UV_all.append(UV)
            F_all.append(F + nv)
            shape_of_tri.append(np.full(len(F), len(shapes) - 1, np.uint32))
            nv += len(P)

        s.vpos = np.ascontiguousarray(np.concatenate(P_all).astype(np.float32))
        s.vnormal = np.ascontiguousarray(np.concatenate(N_all).astype(np.float32))
        s.vuv = np.ascontiguousarray(np.concatenate(UV_all).astype(np.float32))
        tri_vidx = np.concatenate(F_all).astype(np.uint32)
        tri_shape = np.concatenate(shape_of_tri)
        s.shapes = (_abi.Shape * len(shapes))(*shapes)
        s.materials = (_abi.Material * len(mats))(*mats)
        s.emitters = (_abi.Emitter * len(emitters))(*emitters)
        s.textures = (_abi.Texture * max(1, len(textures)))(*[_abi.Texture(w, h, o) for (w, h, o) in textures])
        s.n_textures = len(textures)
        s.texels = np.ascontiguousarray(np.concatenate(texels) if texels else np.zeros(3, np.float32))
        s.tables = np.ascontiguousarray(np.concatenate(tables) if tables else np.zeros(1, np.float32))
        s.n_tables = int(sum(x.size for x in tables))
        s.camera = _camera(spec["sensor"], W, H)
        env = spec.get("environment")
        s.env_radiance = None if env is None else tuple(float(x) for x in _rgb3(env["radiance"]))
        s._build_bvh(tri_vidx, tri_shape)
        s.meta = {"scene": "bedroom-proxy" if not loaded else "xml", "proxy_version": proxy.PROXY_VERSION,
                  "fov_axis": spec["sensor"].get("fov_axis", "x"),
                  "scale": scale, "width": W, "height": H, "n_tris": int(s.n_tris), "budgets": budgets,
                  "bvh_depth": s.bvh_depth, "n_nodes": int(s.n_nodes), "occ_depth": s.occ_depth,
                  "n_occ_nodes": int(s.n_occ_nodes), "loaded_files": loaded}
        return s

    @classmethod
    def from_xml(cls, path: str, width: int | None = None, height: int | None = None, tex_res: int = 512,
                 scale: float = 1.0) -> "Scene":
        """mi.load_file(path) for the supported XML subset (mtx/xmlscene.py):
        OBJ meshes and bitmaps are read from disk where present; meshes that
        are Git-LFS pointers get the deterministic proxy of their budget."""
        from .xmlscene import parse_scene_xml
        spec = parse_scene_xml(path)
        return cls.bedroom(width, height, scale=scale, tex_res=tex_res, spec=spec,
                           base_dir=os.path.dirname(os.path.abspath(path)))

    def _build_bvh(self, tri_vidx, tri_shape):
        from ._lib import check, lib
        n = len(tri_shape)
        nodes = np.zeros((n + 1) * _abi.MTX_BVH_NODE_WORDS, np.int32)
        geom = np.zeros(12 * n, np.float32)
        perm = np.zeros(n, np.uint32)
        nn = C.c_uint32()
        depth = C.c_uint32()
        tri_vidx = np.ascontiguousarray(tri_vidx.reshape(-1))
        check(lib().mtx_bvh_build(self.vpos.ctypes.data, len(self.vpos), tri_vidx.ctypes.data, n, nodes.ctypes.data,
                                  C.byref(nn), geom.ctypes.data, perm.ctypes.data, C.byref(depth)), "mtx_bvh_build")
        self.n_nodes = nn.value
        self.nodes = np.ascontiguousarray(nodes[: _abi.MTX_BVH_NODE_WORDS * nn.value])
        self.tri_geom = geom
        self.tri_vidx = np.ascontiguousarray(tri_vidx.reshape(-1, 3)[perm].reshape(-1))
        self.tri_shape = np.ascontiguousarray(tri_shape[perm])
        self.tri_perm = perm  # input triangle of each leaf-order triangle
        self.n_tris = n
        self.bvh_depth = depth.value
        self._build_occlusion()

    def _build_occlusion(self):
        """The any-hit BVH (mtx.h occlusion node) over the closest-hit tree's
        triangle records; occ_perm maps its leaf order to the scene's."""
        from ._lib import check, lib
        n = self.n_tris
        nodes = np.zeros((n + 1) * _abi.MTX_OCC_NODE_WORDS, np.int32)
        geom = np.zeros(12 * n, np.float32)
        perm = np.zeros(n, np.uint32)
        nn = C.c_uint32()
        depth = C.c_uint32()
        check(lib().mtx_bvh_build_occlusion(self.tri_geom.ctypes.data, n, nodes.ctypes.data, C.byref(nn),
                                            geom.ctypes.data, perm.ctypes.data, C.byref(depth)),
              "mtx_bvh_build_occlusion")
        self.n_occ_nodes = nn.value
        self.occ_nodes = np.ascontiguousarray(nodes[: _abi.MTX_OCC_NODE_WORDS * nn.value])
        self.occ_tri_geom = geom
        self.occ_perm = perm
        self.occ_depth = depth.value

    # ------------------------------------------------------------- export --
    @property
    def width(self) -> int:
        return int(self.camera.width)

    @property
    def height(self) -> int:
        return int(self.camera.height)

    def with_film(self, width: int, height: int) -> "Scene":
        """Same scene, different film resolution: the fov along the sensor's
        fov_axis is kept (Mitsuba's perspective sensor: x, y, or the smaller /
        larger side of the new film), the other axis follows the aspect."""
        cam = _abi.Camera()
        C.pointer(cam)[0] = self.camera
        W0, H0 = int(cam.width), int(cam.height)
        t = cam.tan_x if _fov_axis(self.meta.get("fov_axis", "x"), W0, H0) == "x" else cam.tan_y
        if _fov_axis(self.meta.get("fov_axis", "x"), width, height) == "x":
            cam.tan_x = t
            cam.tan_y = cam.tan_x * height / width
        else:
            cam.tan_y = t
            cam.tan_x = cam.tan_y * width / height
        cam.width, cam.height = width, height
        return self.with_camera(cam)

    def with_camera(self, cam) -> "Scene":
        """Same geometry and materials seen through another sensor (an
        ``mtx_camera``; the film size may differ). Shares the arrays."""
        import copy
        s = copy.copy(self)
        c2 = _abi.Camera()
        C.pointer(c2)[0] = cam
        s.camera = c2
        s.meta = dict(self.meta, width=int(c2.width), height=int(c2.height))
        return s

    def sensors(self) -> list:
        """scene.sensors() (testpssmlt.py:45): the scene's one sensor."""
        return [Sensor(self.camera)]

    def desc(self) -> _abi.SceneDesc:
        d = _abi.SceneDesc()
        d.n_tris = self.n_tris
        d.n_nodes = self.n_nodes
        d.n_verts = len(self.vpos)
        d.n_shapes = len(self.shapes)
        d.n_materials = len(self.materials)
        d.n_emitters = len(self.emitters)
        d.n_textures = self.n_textures
        d.nodes = self.nodes.ctypes.data
        d.tri_geom = self.tri_geom.ctypes.data
        d.tri_vidx = self.tri_vidx.ctypes.data
        d.tri_shape = self.tri_shape.ctypes.data
        d.vpos = self.vpos.ctypes.data
        d.vnormal = self.vnormal.ctypes.data
        d.vuv = self.vuv.ctypes.data
        d.shapes = C.addressof(self.shapes)
        d.materials = C.addressof(self.materials)
        d.emitters = C.addressof(self.emitters)
        d.textures = C.addressof(self.textures)
        d.texels = self.texels.ctypes.data
        d.n_texels = self.texels.size
        d.tables = self.tables.ctypes.data
        d.n_tables = self.n_tables
        d.camera = self.camera
        d.occ_nodes = self.occ_nodes.ctypes.data
        d.occ_tri_geom = self.occ_tri_geom.ctypes.data
        d.n_occ_nodes = self.n_occ_nodes
        self.occ_perm = np.ascontiguousarray(self.occ_perm, np.uint32)
        d.occ_perm = self.occ_perm.ctypes.data
        env = getattr(self, "env_radiance", None)
        d.has_env = 0 if env is None else 1
        d.env_radiance[:] = (0.0, 0.0, 0.0) if env is None else env
        return d

    def save(self, path: str):
        np.savez(path, vpos=self.vpos, vnormal=self.vnormal, vuv=self.vuv, nodes=self.nodes, tri_geom=self.tri_geom,
                 occ_nodes=self.occ_nodes, occ_tri_geom=self.occ_tri_geom, occ_perm=self.occ_perm,
                 tri_vidx=self.tri_vidx, tri_shape=self.tri_shape, texels=self.texels, tables=self.tables,
                 shapes=np.frombuffer(bytes(self.shapes), np.uint8),
                 materials=np.frombuffer(bytes(self.materials), np.uint8),
                 emitters=np.frombuffer(bytes(self.emitters), np.uint8),
                 textures=np.frombuffer(bytes(self.textures), np.uint8),
                 camera=np.frombuffer(bytes(self.camera), np.uint8),
                 meta=np.frombuffer(json.dumps(self.meta).encode(), np.uint8),
                 counts=np.array([self.n_tris, self.n_nodes, self.n_textures, self.n_tables, self.bvh_depth,
                                  self.n_occ_nodes, self.occ_depth], np.int64),
                 env=np.array([0.0, 0.0, 0.0, 0.0] if getattr(self, "env_radiance", None) is None
                              else [1.0, *self.env_radiance], np.float32))

    @classmethod
    def load(cls, path: str) -> "Scene":
        z = np.load(path, allow_pickle=False)
        s = cls()
        for k in ("vpos", "vnormal", "vuv", "nodes", "tri_geom", "tri_vidx", "tri_shape", "texels", "tables",
                  "occ_nodes", "occ_tri_geom", "occ_perm"):
            setattr(s, k, np.ascontiguousarray(z[k]))

        def arr(T, raw):
            n = len(raw) // C.sizeof(T)
            a = (T * n)()
            C.memmove(a, raw.tobytes(), len(raw))
            return a
        s.shapes = arr(_abi.Shape, z["shapes"])
        s.materials = arr(_abi.Material, z["materials"])
        s.emitters = arr(_abi.Emitter, z["emitters"])
        s.textures = arr(_abi.Texture, z["textures"])
        s.camera = _abi.Camera.from_buffer_copy(z["camera"].tobytes())
        s.meta = json.loads(z["meta"].tobytes().decode())
        (s.n_tris, s.n_nodes, s.n_textures, s.n_tables, s.bvh_depth, s.n_occ_nodes,
         s.occ_depth) = (int(x) for x in z["counts"])
        env = z["env"] if "env" in z.files else np.zeros(4, np.float32)
        s.env_radiance = tuple(float(x) for x in env[1:]) if env[0] else None
        return s


class Sensor:
    """A perspective sensor: the ``mtx_camera`` it renders through (what
    ``scene.sensors()[i]`` hands to ``render(scene, sensor, ...)``)."""

    def __init__(self, camera):
        cam = _abi.Camera()
        C.pointer(cam)[0] = camera
        self.camera = cam

    def film_size(self) -> tuple:
        return int(self.camera.width), int(self.camera.height)


def _cube_mesh():
    """The 12 triangles of [-1, 1]^3, counter-clockwise seen from outside."""
    P, F = [], []
    for axis in range(3):
        for sign in (-1.0, 1.0):
            u, v = (axis + 1) % 3, (axis + 2) % 3
            quad = []
            for a, b in ((-1, -1), (1, -1), (1, 1), (-1, 1)):
                p = np.zeros(3)
                p[axis], p[u], p[v] = sign, a, b
                quad.append(p)
            if sign < 0:
                quad = quad[::-1]
            base = len(P)
            P.extend(quad)
            F.extend([[base, base + 1, base + 2], [base, base + 2, base + 3]])
    return np.array(P, np.float64), np.array(F, np.int64)


def _fov_axis(axis: str, W: int, H: int) -> str:
    """Mitsuba's perspective-sensor fov_axis x (default), y, smaller, larger
    -> the film axis the fov is measured along."""
    if axis == "smaller":
        return "x" if W <= H else "y"
    if axis == "larger":
        return "x" if W >= H else "y"
    if axis not in ("x", "y"):
        raise ValueError(f"fov_axis {axis!r} is not supported (x, y, smaller, larger)")
    return axis


def camera_from_sensor(sensor: dict, W: int | None = None, H: int | None = None) -> _abi.Camera:
    """A perspective sensor description (the spec form of mtx.xmlscene /
    mtx.mitsuba_dict: fov, fov_axis, near / far clip, to_world, film) -> an
    ``mtx_camera``; the film size from the sensor's film unless given."""
    film = sensor.get("film", {}) or {}
    return _camera(sensor, int(W or film.get("width", 768)), int(H or film.get("height", 576)))


def _camera(sensor: dict, W: int, H: int) -> _abi.Camera:
    M = _m4(sensor["to_world"])
    cam = _abi.Camera()
    cam.origin[:] = M[:3, 3]
    cam.axis_x[:] = M[:3, 0]
    cam.axis_y[:] = M[:3, 1]
    cam.axis_z[:] = M[:3, 2]
    fov = float(sensor.get("fov", 45.0))
    axis = _fov_axis(sensor.get("fov_axis", "x"), W, H)
    t = math.tan(math.radians(fov) * 0.5)
    if axis == "x":  # the other axis from the fp32-rounded one (as the fixtures were made)
        cam.tan_x = t
        cam.tan_y = cam.tan_x * H / W
    else:
        cam.tan_y = t
        cam.tan_x = cam.tan_y * W / H
    cam.near_clip = float(sensor.get("near_clip", 1e-2))
    cam.far_clip = float(sensor.get("far_clip", 1e4))
    cam.width, cam.height = W, H
    cam.inv_rows[:] = np.linalg.inv(M[:3, :3]).reshape(-1)
    return cam


_cache: dict = {}


def bedroom(width=None, height=None, scale: float = 1.0, tex_res: int = 512, cache_dir: str | None = None) -> Scene:
    """Cached bedroom proxy (in-process, and on disk when `cache_dir` is set)."""
    key = (scale, tex_res)
    if key not in _cache:
        path = None
        if cache_dir:
            path = os.path.join(cache_dir, f"bedroom_v{proxy.PROXY_VERSION}a{_abi.MTX_ABI_VERSION}_s{scale:g}_t{tex_res}.npz")
        if path and os.path.exists(path):
            _cache[key] = Scene.load(path)
        else:
            sc = Scene.bedroom(scale=scale, tex_res=tex_res)
            if path:
                os.makedirs(cache_dir, exist_ok=True)
                sc.save(path)
            _cache[key] = sc
    s = _cache[key]
    W = int(width or s.width)
    H = int(height or s.height)
    return s if (W, H) == (s.width, s.height) else s.with_film(W, H)
