"""ctypes binding of oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
to check (or time beside) the HIP product path. Never imported by the product
package `mtx`.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
sys.path.insert(0, os.path.join(HERE, "..", "mitsuba3-experiments_amd"))

from mtx import _abi  # noqa: E402  (struct layouts of include/mtx.h)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        SD, RA = C.POINTER(_abi.SceneDesc), C.POINTER(_abi.RenderArgs)
        sig = {
            "orc_trace": [SD, u64, vp, C.c_int, C.c_int, vp, vp],
            "orc_node_visit_hist": [SD, u64, vp, C.c_int, vp, C.c_uint32],
            "orc_sample_rays": [SD, RA, u64, vp, vp, u32, vp, vp],
            "orc_render_samples": [SD, RA, vp, vp],
            "orc_render_samples_q": [SD, RA, vp, vp, vp],
            "orc_film": [u32, u32, u32, u32, vp, vp, vp],
            "orc_render": [SD, RA, vp],
            "orc_rng_stream": [u32, u32, u32, u32, vp],
            "orc_prefix_sum_f32_hs": [vp, vp, u64],
            "orc_prefix_sum_u32": [vp, vp, u64, C.c_int],
            "orc_hashgrid": [vp, u64, u32, u32, vp, vp, vp, vp],
            "orc_scatter_reduce_f32": [C.c_int, vp, u64, vp, vp, u64],
            "orc_dmath": [C.c_int, vp, vp, u64],
            "orc_pssmlt_render": [SD, RA, u32, vp, vp],
            "orc_restir_frame": [SD, RA, C.POINTER(_abi.Camera), vp, vp, vp, vp, vp, vp],
            "orc_field_features": [C.POINTER(_abi.FieldDesc), u64, vp, vp, vp],
            "orc_nerad_lhs": [SD, C.POINTER(_abi.NeradTables), u32, u32, vp],
            "orc_nerad_rhs": [SD, C.POINTER(_abi.NeradTables), u32, u32, u32, u32, vp],
            "orc_nerad_render_samples": [SD, RA, vp, vp],
        }
        for k, a in sig.items():
            getattr(L, k).argtypes = a
            getattr(L, k).restype = C.c_int
        _lib = L
    return _lib


def render_args(integrator, max_depth, rr_depth, seed, spp, y0, y1, spp_total=None, sample_offset=0, nrc_c=0.01):
    a = _abi.RenderArgs()
    a.integrator, a.max_depth, a.rr_depth, a.seed = integrator, max_depth, rr_depth, seed
    a.spp, a.spp_total, a.sample_offset = spp, spp_total or spp, sample_offset
    a.y0, a.y1, a.nrc_c = y0, y1, nrc_c
    return a


def render_samples(scene, args):
    """Per-sample (L [n,3], pos [n,2]) in (pixel, sample) order for rows [y0,y1)."""
    n = (args.y1 - args.y0) * scene.width * args.spp
    L = np.zeros((n, 3), np.float32)
    pos = np.zeros((n, 2), np.float32)
    d = scene.desc()
    lib().orc_render_samples(C.byref(d), C.byref(args), L.ctypes.data, pos.ctypes.data)
    return L, pos


def render_samples_nrc_cache(scene, args):
    """NRC with the radiance-cache option (args.flags bit 2): per-sample
    (L [n,3], pos [n,2], query [n,10]); query rows are {valid, p.xyz, wi.xyz,
    T.xyz} of the cache lookup the stopped segment makes (zeros: none)."""
    n = (args.y1 - args.y0) * scene.width * args.spp
    L = np.zeros((n, 3), np.float32)
    pos = np.zeros((n, 2), np.float32)
    q = np.zeros((n, 10), np.float32)
    d = scene.desc()
    lib().orc_render_samples_q(C.byref(d), C.byref(args), L.ctypes.data, pos.ctypes.data, q.ctypes.data)
    return L, pos, q


def film(width, y0, y1, spp, L, pos, spp_total=None, sample_offset=0, nslots=8):
    """The film of per-sample radiance in (pixel, sample) order: 8 partial
    slots combined by a fixed tree (the mtx_render film, orc_film_slots), or
    one slot (nslots=1: the PSSMLT / ReSTIR film order)."""
    f = np.zeros((y1 - y0 + 2, width + 2, 4), np.float32)
    L_ = lib()
    L_.orc_film_slots.argtypes = [C.c_uint32] * 7 + [C.c_void_p] * 3
    L_.orc_film_slots(width, y0, y1, spp, spp if spp_total is None else spp_total, sample_offset, nslots,
                      np.ascontiguousarray(L, np.float32).ctypes.data, np.ascontiguousarray(pos, np.float32).ctypes.data,
                      f.ctypes.data)
    return f


def render(scene, args):
    f = np.zeros((args.y1 - args.y0 + 2, scene.width + 2, 4), np.float32)
    d = scene.desc()
    lib().orc_render(C.byref(d), C.byref(args), f.ctypes.data)
    return f


def sample_rays(scene, args, rays, lanes, rng_skip=2):
    n = len(lanes)
    L = np.zeros((n, 3), np.float32)
    valid = np.zeros(n, np.uint8)
    d = scene.desc()
    lib().orc_sample_rays(C.byref(d), C.byref(args), n, np.ascontiguousarray(rays, np.float32).ctypes.data,
                          np.ascontiguousarray(lanes, np.uint32).ctypes.data, rng_skip, L.ctypes.data,
                          valid.ctypes.data)
    return L, valid


def trace(scene, rays, any_hit=False, brute=False):
    n = len(rays)
    hits = np.zeros(n if int(any_hit) == 1 else 4 * n, np.uint32)
    visits = np.zeros(2 * n, np.uint32)
    d = scene.desc()
    lib().orc_trace(C.byref(d), n, np.ascontiguousarray(rays, np.float32).ctypes.data, int(any_hit), int(brute),
                    hits.ctypes.data, visits.ctypes.data)
    return hits, visits.reshape(n, 2)


def node_visit_hist(scene, rays, hist_len, any_hit=False):
    """Visits per node index < hist_len over `rays` (diagnostic for tools/)."""
    hist = np.zeros(hist_len, np.uint64)
    d = scene.desc()
    lib().orc_node_visit_hist(C.byref(d), len(rays), np.ascontiguousarray(rays, np.float32).ctypes.data,
                              int(any_hit), hist.ctypes.data, int(hist_len))
    return hist


def rng_stream(seed, lane0, n_lanes, n_draws):
    out = np.zeros((n_lanes, n_draws), np.float32)
    lib().orc_rng_stream(seed, lane0, n_lanes, n_draws, out.ctypes.data)
    return out


def prefix_sum_f32_hs(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    lib().orc_prefix_sum_f32_hs(x.ctypes.data, out.ctypes.data, len(x))
    return out


def prefix_sum_u32(x, inclusive=True):
    x = np.ascontiguousarray(x, np.uint32)
    out = np.zeros_like(x)
    lib().orc_prefix_sum_u32(x.ctypes.data, out.ctypes.data, len(x), int(inclusive))
    return out


def hashgrid(p, resolution, n_cells):
    p = np.ascontiguousarray(p, np.float32).reshape(3, -1)
    n = p.shape[1]
    cell = np.zeros(n, np.uint32)
    size = np.zeros(n_cells, np.uint32)
    off = np.zeros(n_cells, np.uint32)
    idx = np.zeros(n, np.uint32)
    lib().orc_hashgrid(p.ctypes.data, n, resolution, n_cells, cell.ctypes.data, size.ctypes.data, off.ctypes.data,
                       idx.ctypes.data)
    return cell, size, off, idx


def scatter_reduce(op, target, value, index):
    t = np.array(target, np.float32)
    lib().orc_scatter_reduce_f32(op, t.ctypes.data, len(t), np.ascontiguousarray(value, np.float32).ctypes.data,
                                 np.ascontiguousarray(index, np.uint32).ctypes.data, len(value))
    return t


def dmath(op, x):
    """op in sin, cos, log, exp, erf, erfinv (mtx_core/dmath.h)."""
    ops = {"sin": 0, "cos": 1, "log": 2, "exp": 3, "erf": 4, "erfinv": 5}
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    lib().orc_dmath(ops[op], x.ctypes.data, out.ctypes.data, len(x))
    return out


def bsdf_probe(scene, mat, wi, wo, uv, u):
    n = len(wi)
    out = np.zeros((n, 16), np.float32)
    out2 = np.zeros(n, np.float32)
    d = scene.desc()
    L = lib()
    L.orc_bsdf_probe.argtypes = [C.POINTER(_abi.SceneDesc), C.c_uint32, C.c_uint64] + [C.c_void_p] * 6
    c = [np.ascontiguousarray(a, np.float32) for a in (wi, wo, uv, u)]
    L.orc_bsdf_probe(C.byref(d), mat, n, *[a.ctypes.data for a in c], out.ctypes.data, out2.ctypes.data)
    return out, out2


def warp(op, u):
    ops = {"cosine_hemisphere": 0, "disk_concentric": 1, "disk": 2, "std_normal": 3, "uniform_hemisphere": 4}
    u = np.ascontiguousarray(u, np.float32)
    out = np.zeros((len(u), 3), np.float32)
    L = lib()
    L.orc_warp.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64]
    L.orc_warp(ops[op], u.ctypes.data, out.ctypes.data, len(u))
    return out


def pssmlt_render(scene, args, iterations=200, chains=False):
    """Pssmlt.render (pssmlt.py:167-228) for rows [y0, y1): film (+ chain state)."""
    f = np.zeros((args.y1 - args.y0 + 2, scene.width + 2, 4), np.float32)
    n = (args.y1 - args.y0) * scene.width * args.spp
    ch = np.zeros((n, 6), np.float32) if chains else None
    d = scene.desc()
    lib().orc_pssmlt_render(C.byref(d), C.byref(args), iterations, f.ctypes.data, ch.ctypes.data if chains else None)
    return (f, ch) if chains else f


class RestirOracle:
    """RestirIntegrator (restirgi.py:151-588) frame by frame on the CPU; the
    state arrays use the device layout (mtx_core/restir.h)."""

    def __init__(self, scene, spp=1):
        n = scene.width * scene.height * spp
        self.n = n
        self.cur = np.zeros((5, n, 4), np.float32)
        self.prev = np.zeros((5, n, 4), np.float32)
        self.tres = np.zeros((6, n, 4), np.float32)
        self.sres = np.zeros((6, n, 4), np.float32)
        self.radius = np.zeros(n, np.float32)
        self.prev_cam = None

    def frame(self, scene, args):
        """One render() call; `args` carries frame, seed and the properties."""
        if args.frame == 0:
            self.prev_cam = scene.camera
        f = np.zeros((scene.height + 2, scene.width + 2, 4), np.float32)
        d = scene.desc()
        cam = _abi.Camera.from_buffer_copy(bytes(self.prev_cam))
        lib().orc_restir_frame(C.byref(d), C.byref(args), C.byref(cam), self.cur.ctypes.data,
                               self.prev.ctypes.data, self.tres.ctypes.data, self.sres.ctypes.data,
                               self.radius.ctypes.data, f.ctypes.data)
        self.prev[...] = self.cur  # restirgi.py:247
        self.prev_cam = _abi.Camera.from_buffer_copy(bytes(scene.camera))
        return f


def field_features(field, p, wi):
    """mtx_core/field.h features of (p, wi) for a mtx.field.Field (fp16 rows of 64)."""
    p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
    wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
    out = np.zeros((len(p), 64), np.uint16)
    d = field.desc()
    lib().orc_field_features(C.byref(d), len(p), p.ctypes.data, wi.ctypes.data, out.ctypes.data)
    return out.view(np.float16)


def nerad_lhs(scene, tables, seed, n):
    """IntersectionSampler.sample restated (nerad.py:291-310): (n, 9) rows as mtx_nerad_lhs."""
    from mtx.nerad import tables_struct

    out = np.zeros((n, 9), np.float32)
    d = scene.desc()
    t = tables_struct(tables)
    lib().orc_nerad_lhs(C.byref(d), C.byref(t), seed, n, out.ctypes.data)
    return out


def nerad_rhs(scene, tables, lhs_seed, rhs_seed, batch, M):
    """sample_rhs lanes without the field term (nerad.py:174-233): (batch*M, 16) rows =
    L_nee(3), f(3), Le(3), stop-vertex valid, query p(3), query wi(3)."""
    from mtx.nerad import tables_struct

    out = np.zeros((batch * M, 16), np.float32)
    d = scene.desc()
    t = tables_struct(tables)
    lib().orc_nerad_rhs(C.byref(d), C.byref(t), lhs_seed, rhs_seed, batch, M, out.ctypes.data)
    return out


def nerad_compose(lanes, field_out, M):
    """L = L_nee + f * (Le + Field) per lane (field 0 at invalid stop vertices),
    then dr.block_sum(L, M) / M with the samples added in order (float32)."""
    f32 = np.float32
    L = lanes[:, 0:3] + lanes[:, 3:6] * (lanes[:, 6:9] + field_out.astype(f32))
    n = len(lanes) // M
    acc = np.zeros((n, 3), f32)
    Lm = L.reshape(n, M, 3)
    for j in range(M):
        acc = acc + Lm[:, j]
    return L, acc / f32(M)


def nerad_render_samples(scene, args):
    """Integrator.sample lanes of a render (nerad.py:235-254): (n, 16) rows as
    nerad_rhs (L_nee = 0) and the film positions (n, 2), (pixel, sample) order."""
    n = (args.y1 - args.y0) * scene.width * args.spp
    lanes = np.zeros((n, 16), np.float32)
    pos = np.zeros((n, 2), np.float32)
    d = scene.desc()
    lib().orc_nerad_render_samples(C.byref(d), C.byref(args), lanes.ctypes.data, pos.ctypes.data)
    return lanes, pos


def probe(scene, op, inputs):
    """orc_probe: the shared sensor / spawn / emitter primitives item by item
    (op 0 camera_ray, 1 spawn_ray, 2 spawn_ray_to, 3 sample_emitter_direction,
    4 pdf_emitter_direction + emitter_eval); 16 floats in and out per item."""
    ops = {"camera_ray": 0, "spawn_ray": 1, "spawn_ray_to": 2, "sample_emitter": 3, "pdf_emitter": 4}
    x = np.zeros((len(inputs), 16), np.float32)
    a = np.asarray(inputs, np.float32)
    x[:, : a.shape[1]] = a
    out = np.zeros_like(x)
    d = scene.desc()
    L = lib()
    L.orc_probe.argtypes = [C.POINTER(_abi.SceneDesc), C.c_int, C.c_uint64, C.c_void_p, C.c_void_p]
    rc = L.orc_probe(C.byref(d), ops[op], len(x), x.ctypes.data, out.ctypes.data)
    assert rc == 0
    return out


def restir_probe(op, inputs):
    """orc_restir_probe: the ReSTIR GI reservoir primitives of
    mtx_core/restir.h item by item (op p_hat, similar, update, merge, J,
    to_idx); 16 floats in and out per item."""
    ops = {"p_hat": 0, "similar": 1, "update": 2, "merge": 3, "J": 4, "to_idx": 5}
    a = np.asarray(inputs, np.float32)
    x = np.zeros((len(a), 16), np.float32)
    x[:, : a.shape[1]] = a
    out = np.zeros_like(x)
    L = lib()
    L.orc_restir_probe.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_void_p]
    assert L.orc_restir_probe(ops[op], len(x), x.ctypes.data, out.ctypes.data) == 0
    return out


def si_probe(items):
    """orc_si_probe: si_from_vertices item by item; items is (n, 40) float32
    (layout in oracle.cpp), returns (n, 24): p, n, s, t, ns, uv(+0), wi."""
    x = np.ascontiguousarray(items, np.float32)
    assert x.ndim == 2 and x.shape[1] == 40
    out = np.zeros((len(x), 24), np.float32)
    L = lib()
    L.orc_si_probe.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p]
    assert L.orc_si_probe(len(x), x.ctypes.data, out.ctypes.data) == 0
    return out


def tex_probe(scene, tex, uv):
    """orc_tex_probe: bilinear repeat-wrapped lookups of one scene texture."""
    uv = np.ascontiguousarray(uv, np.float32)
    out = np.zeros((len(uv), 3), np.float32)
    d = scene.desc()
    L = lib()
    L.orc_tex_probe.argtypes = [C.POINTER(_abi.SceneDesc), C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p]
    assert L.orc_tex_probe(C.byref(d), tex, len(uv), uv.ctypes.data, out.ctypes.data) == 0
    return out


# ---- multi-core CPU baselines (bench.py cpu_baseline legs; equal results) --
def prefix_sum_u32_mt(x, inclusive=True):
    x = np.ascontiguousarray(x, np.uint32)
    out = np.zeros_like(x)
    L = lib()
    L.orc_prefix_sum_u32_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
    L.orc_prefix_sum_u32_mt(x.ctypes.data, out.ctypes.data, len(x), int(inclusive))
    return out


def prefix_sum_f32_hs_mt(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    L = lib()
    L.orc_prefix_sum_f32_hs_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    L.orc_prefix_sum_f32_hs_mt(x.ctypes.data, out.ctypes.data, len(x))
    return out


def hashgrid_mt(p, resolution, n_cells):
    p = np.ascontiguousarray(p, np.float32).reshape(3, -1)
    n = p.shape[1]
    out = [np.zeros(n, np.uint32), np.zeros(n_cells, np.uint32), np.zeros(n_cells, np.uint32), np.zeros(n, np.uint32)]
    L = lib()
    L.orc_hashgrid_mt.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32] + [C.c_void_p] * 4
    L.orc_hashgrid_mt(p.ctypes.data, n, resolution, n_cells, *[a.ctypes.data for a in out])
    return tuple(out)


def scatter_reduce_mt(op, target, value, index):
    t = np.array(target, np.float32)
    v = np.ascontiguousarray(value, np.float32)
    i = np.ascontiguousarray(index, np.uint32)
    L = lib()
    L.orc_scatter_reduce_f32_mt.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64]
    L.orc_scatter_reduce_f32_mt(op, t.ctypes.data, len(t), v.ctypes.data, i.ctypes.data, len(v))
    return t
