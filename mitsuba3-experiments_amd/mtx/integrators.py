"""Integrator façade with the reference's plugin names, properties and entry
points, backed by libmtx (HIP, gfx950). No CPU fallback.

Reference surface:
  * ``mi.register_integrator(name, lambda props: Cls(props))`` —
    path.py:305 ("mypath"), path-mis.py:158 ("path_test")
  * ``mi.load_dict({"type": name, **props})`` — path.py:316-322
  * ``render(scene, sensor, seed, spp, develop, evaluate)`` (SamplingIntegrator
    render, transcribed path.py:103-192)
  * ``sample(scene, sampler, ray, medium, active) -> (L, valid, aovs)``
    (path.py:195-202, path-mis.py:24-31)

When ``mitsuba`` is importable the classes can additionally be registered as
``mi.SamplingIntegrator`` plugins (:func:`register_with_mitsuba`); without it
(this container, the GPU box) they operate on :class:`mtx.scene.Scene`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._lib import MtxError, check, context, lib

_REGISTRY: dict = {}


def register_integrator(name: str, ctor) -> None:
    """Mirror of mi.register_integrator (path.py:305)."""
    _REGISTRY[name] = ctor


def load_dict(d: dict):
    """Mirror of mi.load_dict({"type": name, **props}) for integrators."""
    d = dict(d)
    name = d.pop("type")
    if name not in _REGISTRY:
        raise ValueError(f"unknown integrator type {name!r}; registered: {sorted(_REGISTRY)}")
    return _REGISTRY[name](d)


class Properties(dict):
    """Minimal mi.Properties: props.get(name, def_value)."""

    def get(self, name, def_value=None):  # noqa: D401 - mitsuba signature
        return super().get(name, def_value)


class IndependentSampler:
    """Sampler state handed to sample(): PCG32 lanes seeded with
    sample_tea_32(seed, lane) and advanced by `skip` draws."""

    def __init__(self, seed: int, lanes, skip: int = 0):
        self.seed = int(seed)
        self.lanes = np.ascontiguousarray(lanes, np.uint32)
        self.skip = int(skip)


def develop(film: np.ndarray) -> np.ndarray:
    """hdrfilm develop: inner W x H pixels, RGB / weight (0 where weight is 0)."""
    inner = film[1:-1, 1:-1]
    w = inner[..., 3:4]
    return np.where(w != 0, inner[..., :3] / np.where(w != 0, w, 1), 0).astype(np.float32)


def _rows3(v, drjit_layout: bool = False) -> np.ndarray:
    """A wavefront of 3-vectors as (N, 3) float32.

    `drjit_layout`: the field comes from a ray object, whose Array3f is (3, N)
    in Dr.Jit's layout at every N. A bare array is (N, 3) or (3, N); a 3x3
    array is ambiguous (3 rays either way) and is refused."""
    a = np.asarray(v, np.float32)
    if a.ndim == 2 and a.shape[0] == 3:
        if drjit_layout:
            a = a.T
        elif a.shape[1] == 3:
            raise MtxError("ambiguous 3x3 ray array: pass a ray object (Dr.Jit (3, N) fields) "
                           "or (N, 3) arrays with N != 3")
        else:
            a = a.T
    elif drjit_layout and a.ndim == 1 and a.size == 3:
        a = a.reshape(3, 1).T
    return a.reshape(-1, 3)


class SamplingIntegrator:
    integrator_id = 0
    name = ""

    def __init__(self, props=None):
        self.props = Properties(props or {})

    # ------------------------------------------------------------ arguments --
    def render_args(self, scene, seed: int, spp: int, y0: int = 0, y1: int | None = None, spp_total: int | None = None,
                    sample_offset: int = 0, chunk_paths: int = 0, flags: int = 0) -> _abi.RenderArgs:
        a = _abi.RenderArgs()
        a.integrator = self.integrator_id
        a.max_depth = int(self.max_depth)
        a.rr_depth = int(getattr(self, "rr_depth", 0))
        a.seed = int(seed)
        a.spp = int(spp)
        a.spp_total = int(spp_total or spp)
        a.sample_offset = int(sample_offset)
        a.y0 = int(y0)
        a.y1 = int(scene.height if y1 is None else y1)
        a.chunk_paths = int(chunk_paths)
        a.nrc_c = float(getattr(self, "c", 0.01))
        a.flags = int(flags)
        a.iterations = int(getattr(self, "iterations", 0))
        return a

    # --------------------------------------------------------------- render --
    def render_film(self, scene, seed: int = 0, spp: int = 1, y0: int = 0, y1: int | None = None,
                    spp_total: int | None = None, sample_offset: int = 0, device: int | None = None,
                    out=None, stats: bool = False, chunk_paths: int = 0, counters: bool = False, ctx=None,
                    extra_flags: int = 0, sensor=None):
        """Raw film (rows y0-1..y1, cols -1..W) x RGBW. `out` may be a
        device tensor (torch, on the context's device) to keep the film in HBM.
        stats=True returns (film, stats) with per-kernel-class HIP-event
        times; counters=True also collects the traversal visit counters
        (slower kernels: use it outside timed regions). `sensor`: the camera
        to render through (:func:`scene_with_sensor`; None = the scene's)."""
        ctx = ctx or context(device)
        scene = scene_with_sensor(scene, sensor)
        _bind_scene(ctx, scene)
        a = self.render_args(scene, seed, spp, y0, y1, spp_total, sample_offset, chunk_paths,
                             flags=(2 if stats else 0) | (1 if stats and counters else 0))
        a.restir_flags |= int(extra_flags)
        shape = (a.y1 - a.y0 + 2, scene.width + 2, 4)
        st = _abi.Stats()
        if out is None:
            film = np.zeros(shape, np.float32)
            check(lib().mtx_render(ctx.handle, C.byref(a), film.ctypes.data, 0, C.byref(st)), "mtx_render")
        else:
            if tuple(out.shape) != shape or not out.is_contiguous():
                raise MtxError(f"film tensor must be contiguous with shape {shape}")
            film = out
            check(lib().mtx_render(ctx.handle, C.byref(a), C.c_void_p(out.data_ptr()), 1, C.byref(st)), "mtx_render")
        return (film, st.as_dict()) if stats else film

    def render(self, scene, sensor=None, seed: int = 0, spp: int = 1, develop: bool = True, evaluate: bool = True):
        """SamplingIntegrator.render (path.py:103-192) through `sensor` (the
        scene's own when None / 0, as mi.render does; testpssmlt.py:45 passes
        scene.sensors()[0]): TensorXf[H, W, 3] of the sensor's film."""
        film = self.render_film(scene, seed=seed, spp=spp, sensor=sensor)
        return globals()["develop"](film) if develop else film

    # --------------------------------------------------------------- sample --
    def sample(self, scene, sampler: IndependentSampler, ray, medium=None, active=True):
        """sample(scene, sampler, ray) over a wavefront of rays -> (L, valid, []).

        `ray` is an (o, d) pair or a ray object with `.o` / `.d` fields (the
        RayDifferential3f of path.py:195-202); each field is (N, 3) or (3, N)
        (Dr.Jit's Array3f layout)."""
        obj = hasattr(ray, "o") and hasattr(ray, "d")
        o, d = (ray.o, ray.d) if obj else ray
        if _is_cuda(o) or _is_cuda(d):
            return self._sample_device(scene, sampler, o, d, obj)
        rays = np.ascontiguousarray(np.concatenate([_rows3(o, obj), _rows3(d, obj)], 1))
        n = len(rays)
        if len(sampler.lanes) != n:
            raise MtxError("sampler lanes and rays differ in length")
        ctx = context()
        _bind_scene(ctx, scene)
        a = self.render_args(scene, sampler.seed, 1)
        L = np.zeros((n, 3), np.float32)
        valid = np.zeros(n, np.uint8)
        check(lib().mtx_sample_rays(ctx.handle, C.byref(a), n, rays.ctypes.data, sampler.lanes.ctypes.data,
                                    sampler.skip, L.ctypes.data, valid.ctypes.data), "mtx_sample_rays")
        return L, valid.astype(bool), []

    def _sample_device(self, scene, sampler, o, d, obj):
        """sample() on a wavefront already in HBM (torch CUDA tensors, as the
        reference's Dr.Jit arrays are, path.py:194-202): rays, lanes, L and
        valid stay on the device (mtx_sample_rays_dev); returns tensors."""
        import torch

        def rows(v):
            t = torch.as_tensor(v, dtype=torch.float32, device=dev)
            if t.dim() == 2 and t.shape[0] == 3 and (obj or t.shape[1] != 3):
                t = t.T
            elif t.dim() == 2 and t.shape == (3, 3):
                raise MtxError("ambiguous 3x3 ray array: pass a ray object (Dr.Jit (3, N) fields) "
                               "or (N, 3) tensors with N != 3")
            return t.reshape(-1, 3)

        dev = next(x.device for x in (o, d) if _is_cuda(x))
        rays = torch.cat([rows(o), rows(d)], 1).contiguous()
        n = rays.shape[0]
        lanes = torch.as_tensor(np.asarray(sampler.lanes, np.uint32).view(np.int32), device=dev) \
            if not _is_cuda(sampler.lanes) else sampler.lanes.to(torch.int32)
        lanes = lanes.contiguous()
        if len(lanes) != n:
            raise MtxError("sampler lanes and rays differ in length")
        L = torch.empty((n, 3), dtype=torch.float32, device=dev)
        valid = torch.empty(n, dtype=torch.uint8, device=dev)
        ctx = context(dev.index if dev.index is not None else torch.cuda.current_device())
        _bind_scene(ctx, scene)
        a = self.render_args(scene, sampler.seed, 1)
        torch.cuda.current_stream(dev).synchronize()  # libmtx runs on its own stream
        check(lib().mtx_sample_rays_dev(ctx.handle, C.byref(a), n, rays.data_ptr(), lanes.data_ptr(), sampler.skip,
                                        L.data_ptr(), valid.data_ptr()), "mtx_sample_rays_dev")
        return L, valid.bool(), []


def _is_cuda(x) -> bool:
    import sys

    torch = sys.modules.get("torch")
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def trace_rays(scene, rays, any_hit: bool = False, visits: bool = False, device: int | None = None):
    """Scene.ray_intersect / Scene.ray_test (path-mis.py:69-71, restirgi.py:320)
    over a wavefront of rays: (N, 8) float32 rows (o.xyz, tmax, d.xyz, 0).
    Closest hit: (N, 4) words (t, prim bits, u, v bits; t = inf on a miss);
    any hit: (N,) 1 = occluded. A torch CUDA tensor is traced where it lies
    (mtx_trace_dev) and the results are int32 tensors there; numpy goes
    through mtx_trace. visits=True also returns (N, 2) node / triangle visits."""
    if _is_cuda(rays):
        import torch

        r = rays.to(torch.float32).reshape(-1, 8).contiguous()
        n = r.shape[0]
        hits = torch.empty((n,) if any_hit else (n, 4), dtype=torch.int32, device=r.device)
        vis = torch.empty((n, 2), dtype=torch.int32, device=r.device) if visits else None
        ctx = context(r.device.index if r.device.index is not None else torch.cuda.current_device())
        _bind_scene(ctx, scene)
        torch.cuda.current_stream(r.device).synchronize()
        if n:
            check(lib().mtx_trace_dev(ctx.handle, n, r.data_ptr(), int(any_hit), hits.data_ptr(),
                                      vis.data_ptr() if visits else None), "mtx_trace_dev")
        return (hits, vis) if visits else hits
    r = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    n = len(r)
    hits = np.zeros((n,) if any_hit else (n, 4), np.uint32)
    vis = np.zeros((n, 2), np.uint32) if visits else None
    ctx = context(device)
    _bind_scene(ctx, scene)
    if n:
        check(lib().mtx_trace(ctx.handle, n, r.ctypes.data, int(any_hit), hits.ctypes.data,
                              vis.ctypes.data if visits else None), "mtx_trace")
    return (hits, vis) if visits else hits


class Path(SamplingIntegrator):
    """path.py:21-302 ("mypath"): starts from the first surface interaction;
    NEE + BSDF sampling with power-heuristic MIS (variant A, path.py:10-18),
    Russian roulette. Uses self.max_depth where path.py:235 reads a global."""

    integrator_id = _abi.MTX_INT_PATH
    name = "mypath"

    def __init__(self, props=None):
        super().__init__(props)
        self.max_depth = self.props.get("max_depth", 16)  # path.py:23
        self.rr_depth = self.props.get("rr_depth", 4)  # path.py:24


class PathIntegrator(SamplingIntegrator):
    """path-mis.py:18-155 ("path_test"): upstream-style NEE + MIS loop."""

    integrator_id = _abi.MTX_INT_PATH_MIS
    name = "path_test"

    def __init__(self, props=None):
        super().__init__(props)
        self.max_depth = self.props.get("max_depth", 8)  # path-mis.py:21
        self.rr_depth = self.props.get("rr_depth", 2)  # path-mis.py:22


class Simple(SamplingIntegrator):
    """simple.py:8-116 ("integrator"): BSDF sampling only (no emitter
    sampling, no MIS), Russian roulette. The estimator without NEE that the
    NEE + MIS integrators must agree with in expectation (the reference's
    parity-vs-other-integrator pattern, path.py:332-359, testpssmlt.py)."""

    integrator_id = _abi.MTX_INT_SIMPLE
    name = "integrator"

    def __init__(self, props=None):
        super().__init__(props)
        self.max_depth = self.props.get("max_depth", 8)  # simple.py:11
        self.rr_depth = self.props.get("rr_depth", 2)  # simple.py:12


class NRCIntegrator(SamplingIntegrator):
    """nrc.py:17-125: NEE + MIS path segments truncated by the NRC spread
    heuristic (a < c * a0, c = 0.01); no primary emission (nrc.py:118)."""

    integrator_id = _abi.MTX_INT_NRC
    name = "nrc"

    def __init__(self, props=None):
        super().__init__(props)
        self.max_depth = self.props.get("max_depth", 10)  # nrc.py:23
        self.c = self.props.get("c", 0.01)  # nrc.py:123
        self.rr_depth = 0
        # Radiance cache (nerad.py Field): a segment stopped
        # by the spread criterion adds T * field(x, -d) at its next hit.
        self.field = self.props.get("field", None)

    def render_args(self, *args, **kwargs) -> _abi.RenderArgs:
        a = super().render_args(*args, **kwargs)
        if self.field is not None:
            a.flags |= _abi.MTX_RENDER_NRC_CACHE
        return a

    def render_film(self, scene, *args, ctx=None, device: int | None = None, **kwargs):
        ctx = ctx or context(device)
        if self.field is not None:
            self.field._ensure(ctx)
        return super().render_film(scene, *args, ctx=ctx, **kwargs)

    def sample(self, scene, sampler: IndependentSampler, ray, medium=None, active=True):
        if self.field is not None:
            self.field._ensure(context())
        return super().sample(scene, sampler, ray, medium, active)


class NeradIntegrator(SamplingIntegrator):
    """nerad.py:118-254 Integrator used as a renderer (sample(), :235-254):
    a camera ray's first hit is followed through delta / null vertices
    (next_smooth_si, :124-164, at most 10 more traces) and L = Field(si) * f
    + Le(si). Needs the trained (or any) radiance field: props["field"]."""

    integrator_id = _abi.MTX_INT_NERAD
    name = "nerad"

    def __init__(self, props=None):
        super().__init__(props)
        self.field = self.props.get("field", None)
        if self.field is None:
            raise MtxError('"nerad" needs a radiance field: load_dict({"type": "nerad", "field": Field(scene)})')
        self.max_depth = 11  # the first hit + next_smooth_si's max_depth = 10 (:146)
        self.rr_depth = 0

    def render_film(self, scene, *args, ctx=None, device: int | None = None, **kwargs):
        ctx = ctx or context(device)
        self.field._ensure(ctx)
        return super().render_film(scene, *args, ctx=ctx, **kwargs)

    def sample(self, scene, sampler: IndependentSampler, ray, medium=None, active=True):
        self.field._ensure(context())
        return super().sample(scene, sampler, ray, medium, active)


class PssmltSimple(SamplingIntegrator):
    """pssmlt.py:96-255 + pssmltsimple.py:11-145 ("pssmlt_simple"): per-pixel
    primary-sample-space MLT over W*H*spp chains; 200 Metropolis iterations
    (large step every 50, aggregation when i % 50 > 40, pssmlt.py:206-210),
    BSDF-only proposals whose local directions are mutated as
    normalize(0.9 old + 0.1 new) (pssmltsimple.py:135-142). Chains are
    independent and never leave their pixel, so a multi-GPU render shards
    the chains of every pixel by range (``spp_total`` / ``sample_offset``,
    :func:`mtx.distributed.render_sharded` mode "samples"), or by row bands."""

    integrator_id = _abi.MTX_INT_PSSMLT_SIMPLE
    name = "pssmlt_simple"

    def __init__(self, props=None):
        super().__init__(props)
        self.max_depth = self.props.get("max_depth", 16)  # pssmlt.py:105
        self.rr_depth = self.props.get("rr_depth", 4)  # pssmlt.py:106
        self.iterations = self.props.get("iterations", 200)  # pssmlt.py:208

    def sample(self, *args, **kwargs):
        raise MtxError("PssmltSimple.sample() needs the Metropolis chain state; use render()")


class PssmltPath(PssmltSimple):
    """pssmlt.py:96-255 + pssmltpath.py:12-193 ("pssmlt"): the same chains
    and Metropolis schedule as PssmltSimple, with an NEE + MIS proposal
    tracer; each path vertex holds the local direction and the emitter
    sample, mutated as normalize(0.99 old + 0.01 new) and
    clamp(old + 0.1 N(0,1)) (pssmltpath.py:170-190)."""

    integrator_id = _abi.MTX_INT_PSSMLT_PATH
    name = "pssmlt"


class RestirIntegrator(SamplingIntegrator):
    """restirgi.py:151-588 ("restirgi"): ReSTIR GI. Each render() call is one
    frame: an initial sample per lane (camera hit x_v + a path-mis secondary
    path giving L_o at x_s), temporal resampling against the previous frame's
    sample reprojected through the previous camera, spatial resampling of up
    to 9 neighbours' temporal reservoirs (visibility-tested, optional jacobian
    and bias correction), then bsdf.eval * L_o * W + emittance splatted at the
    integer pixel. Reservoirs, the previous samples and the search radii stay
    in HBM inside the device context between frames.

    Properties and defaults follow restirgi.py:157-166. ``max_M_spatial=None``
    (the reference default, which raises a TypeError at :297) is treated as
    "no clamp, always 9 neighbours"."""

    integrator_id = _abi.MTX_INT_RESTIR_GI
    name = "restirgi"

    def __init__(self, props=None):
        super().__init__(props)
        g = self.props.get
        self.max_depth = g("max_depth", 8)
        self.rr_depth = g("rr_depth", 2)
        self.bias_correction = bool(g("bias_correction", True))
        self.jacobian = bool(g("jacobian", True))
        self.bsdf_sampling = bool(g("bsdf_sampling", True))
        self.max_M_temporal = g("max_M_temporal", None)
        self.max_M_spatial = g("max_M_spatial", None)
        self.initial_search_radius = float(g("initial_search_radius", 10.0))
        self.minimal_search_radius = float(g("minimal_search_radius", 3.0))
        self.spatial_spatial_reuse = bool(g("spatial_spatial_reuse", False))
        self.n = 0
        self.film_size = None

    def render_args(self, scene, seed: int, spp: int, *args, **kwargs) -> _abi.RenderArgs:
        a = super().render_args(scene, seed, spp, *args, **kwargs)
        a.frame = int(self.n)
        a.restir_flags = ((_abi.MTX_RESTIR_BIAS_CORRECTION if self.bias_correction else 0)
                          | (_abi.MTX_RESTIR_JACOBIAN if self.jacobian else 0)
                          | (_abi.MTX_RESTIR_BSDF_SAMPLING if self.bsdf_sampling else 0)
                          | (_abi.MTX_RESTIR_SPATIAL_SPATIAL if self.spatial_spatial_reuse else 0))
        a.max_M_temporal = int(self.max_M_temporal or 0)
        a.max_M_spatial = int(self.max_M_spatial or 0)
        a.initial_search_radius = self.initial_search_radius
        a.minimal_search_radius = self.minimal_search_radius
        return a

    def render_film(self, scene, seed: int = 0, spp: int = 1, device: int | None = None, out=None,
                    stats: bool = False, counters: bool = False, y0: int = 0, y1: int | None = None,
                    stage: str | None = None, ctx=None, sensor=None, **kwargs):
        """One frame (restirgi.py:182-258) through `sensor` (None: the
        scene's camera); advances the frame counter. The previous frame's
        camera is the context's prev_sensor (restirgi.py:226-227, :247).

        Row bands (multi-GPU): render rows [y0, y1) in two calls,
        stage="A" (initial sample + temporal) and stage="B" (spatial + final +
        film), importing the neighbours' halo rows in between
        (:func:`mtx.distributed.restir_band_frame`)."""
        if kwargs.get("sample_offset", 0) or kwargs.get("spp_total") not in (None, spp):
            raise MtxError("ReSTIR GI renders all samples of its pixels")
        scene = scene_with_sensor(scene, sensor)
        y1 = scene.height if y1 is None else int(y1)
        if stage not in (None, "A", "B"):
            raise MtxError(f"stage must be None, 'A' or 'B', not {stage!r}")
        ctx = ctx or context(device)
        _bind_scene(ctx, scene)
        size = (scene.width, scene.height, int(spp))
        if self.film_size is None:
            self.film_size = size
        if size != self.film_size:
            raise MtxError(f"film size / spp changed between frames: {self.film_size} -> {size}")
        owner = getattr(ctx, "_restir_owner", None)
        if self.n > 0 and owner is not self:
            raise MtxError("another ReSTIR integrator rendered on this device context since the last frame")
        ctx._restir_owner = self
        self._ctx = ctx  # _bind_scene pointed the device camera at this frame's sensor
        flags = {None: 0, "A": _abi.MTX_RESTIR_STAGE_A, "B": _abi.MTX_RESTIR_STAGE_B}[stage]
        result = super().render_film(scene, seed=seed, spp=spp, device=device, out=out, stats=stats,
                                     counters=counters, y0=y0, y1=y1, ctx=ctx, extra_flags=flags)
        if stage != "A":
            self.n += 1  # restirgi.py:245
        return result

    def rows(self, which: str, row0: int, nrows: int, buf, to_state: bool, ctx=None) -> None:
        """Copy state rows to / from a device tensor (halo exchange):
        which = 'sample' (5 planes), 'temporal' (6 planes) or 'prev_sample'
        (5 planes: the previous frame's samples, between frames; a moving
        camera's reprojection reads them anywhere in the film); buf is a
        contiguous [planes, nrows, W*spp, 4] float32 tensor on the device."""
        ctx = ctx or getattr(self, "_ctx", None) or context()
        idx = {"sample": 0, "temporal": 1, "prev_sample": 2}[which]
        check(lib().mtx_restir_rows(ctx.handle, idx, int(row0), int(nrows), C.c_void_p(buf.data_ptr()),
                                    int(bool(to_state))), "mtx_restir_rows")

    def state(self, which: str, device: int | None = None, ctx=None) -> np.ndarray:
        """Device state of the last frame: 'sample' (5 planes x lanes x 4),
        'temporal' / 'spatial' (6 planes), 'radius' (lanes)."""
        idx, planes = {"sample": (0, 5), "temporal": (1, 6), "spatial": (2, 6), "radius": (3, 0)}[which]
        W, H, spp = self.film_size
        n = W * H * spp
        shape = (planes, n, 4) if planes else (n,)
        out = np.zeros(shape, np.float32)
        ctx = ctx or getattr(self, "_ctx", None) or context(device)
        check(lib().mtx_restir_state(ctx.handle, idx, out.ctypes.data, out.size), "mtx_restir_state")
        return out

    def sample(self, *args, **kwargs):
        raise MtxError("RestirIntegrator.sample() needs the frame's reservoirs; use render()")


register_integrator("restirgi", lambda props: RestirIntegrator(props))
register_integrator("mypath", lambda props: Path(props))
register_integrator("pssmlt_simple", lambda props: PssmltSimple(props))
register_integrator("pssmlt", lambda props: PssmltPath(props))  # pssmltpath.py:193
register_integrator("path_test", lambda props: PathIntegrator(props))
register_integrator("nrc", lambda props: NRCIntegrator(props))
register_integrator("integrator", lambda props: Simple(props))  # simple.py:119
register_integrator("nerad", lambda props: NeradIntegrator(props))


def scene_with_sensor(scene, sensor):
    """The scene seen through `sensor` -- the ``sensor`` argument of
    SamplingIntegrator.render / mi.render (testpssmlt.py:45, pssmlt.py:167-175,
    restirgi.py:182-190): None or 0 (the scene's own sensor), an
    ``mtx_camera``, an object with a ``camera`` (``Scene.sensors()[i]``), a
    ``perspective`` sensor dictionary, or an ``mi.Sensor`` loaded with the
    wrapped ``mi.load_dict``. Shares the scene's arrays (same geometry: the
    device scene is re-pointed at the camera, not re-uploaded, unless the film
    size differs)."""
    if sensor is None or (isinstance(sensor, int) and not isinstance(sensor, bool) and sensor == 0):
        return scene
    if isinstance(sensor, int):
        raise MtxError(f"sensor index {sensor}: the scene has one sensor")
    from .scene import camera_from_sensor
    if isinstance(sensor, _abi.Camera):
        cam = sensor
    elif isinstance(getattr(sensor, "camera", None), _abi.Camera):
        cam = sensor.camera
    elif isinstance(sensor, dict):
        from .mitsuba_dict import sensor_from_dict
        cam = camera_from_sensor(sensor_from_dict(sensor))
    else:
        entry = _MI_OBJECTS.get(id(sensor))
        if entry is None or entry[0]() is not sensor or entry[1][0] != "sensor":
            raise MtxError(f"unsupported sensor {type(sensor).__name__}: pass None, an mtx_camera, "
                           "Scene.sensors()[i], a perspective sensor dictionary or an mi.Sensor loaded by the "
                           "wrapped mi.load_dict")
        cam = camera_from_sensor(entry[1][1])
    if bytes(cam) == bytes(scene.camera):
        return scene
    return scene.with_camera(cam)


def _bind_scene(ctx, scene) -> None:
    """Upload `scene` to the context's device once (keyed by its geometry and
    film size); a scene sharing the bound geometry and film size with another
    camera (Scene.with_camera, scene_with_sensor) only re-points the device
    camera (mtx_set_camera)."""
    key = (id(scene.nodes), scene.width, scene.height)
    if getattr(ctx, "_scene_key", None) == key:
        if getattr(ctx, "_camera", None) != bytes(scene.camera):
            check(lib().mtx_set_camera(ctx.handle, C.byref(scene.camera)), "mtx_set_camera")
            ctx._camera = bytes(scene.camera)
        ctx.scene = scene
        return
    d = scene.desc()
    check(lib().mtx_scene_upload(ctx.handle, C.byref(d)), "mtx_scene_upload")
    ctx._scene_key = key
    ctx._camera = bytes(scene.camera)
    ctx._nerad_key = None  # surface tables (mtx_nerad_upload) belong to the previous scene
    ctx.scene = scene  # keep the host arrays alive while bound


# mi.Scene / mi.Sensor objects loaded through the wrapped mi.load_dict /
# mi.load_file: id -> [weak reference to the object, (kind, converted spec or
# XML path, base dir) taken at load time, the mtx scene built on first
# render]. An entry goes when its object is collected (objects that take no
# weak reference are kept, at most _MI_STRONG_MAX of them).
_MI_OBJECTS: dict = {}
_MI_STRONG: list = []
_MI_STRONG_MAX = 64


def _record(obj, source) -> None:
    import weakref

    key = id(obj)
    try:
        ref = weakref.ref(obj)
        weakref.finalize(obj, _MI_OBJECTS.pop, key, None)
    except TypeError:
        _MI_STRONG.append(obj)
        if len(_MI_STRONG) > _MI_STRONG_MAX:
            old = _MI_STRONG.pop(0)
            _MI_OBJECTS.pop(id(old), None)
        ref = (lambda o: (lambda: o))(obj)
    _MI_OBJECTS[key] = [ref, source, None]


def mtx_scene_of(scene):
    """The :class:`mtx.scene.Scene` a registered plugin renders for `scene`:
    itself, or the scene built from the dictionary / XML file an ``mi.Scene``
    was loaded from (mi.load_dict / mi.load_file wrapped by
    :func:`register_with_mitsuba`). Raises MtxError for an ``mi.Scene`` of
    unknown origin."""
    from .scene import Scene

    if isinstance(scene, Scene):
        return scene
    entry = _MI_OBJECTS.get(id(scene))
    if entry is None or entry[0]() is not scene or entry[1][0] == "sensor":
        raise MtxError("mtx renders mtx.scene.Scene objects, or an mi.Scene loaded by mi.load_dict / mi.load_file "
                       "after mtx.register_with_mitsuba() (its source dictionary / XML is converted); this mi.Scene "
                       "has no recorded source")
    if entry[2] is None:
        kind, src, base = entry[1]
        if kind == "error":
            raise MtxError(src)
        if kind == "dict":
            from .mitsuba_dict import scene_from_spec
            entry[2] = scene_from_spec(src, base_dir=base)
        else:
            from .scene import Scene as _S
            entry[2] = _S.from_xml(src)
    return entry[2]


def _wrap_loaders(mi) -> None:
    """mi.load_dict / mi.load_file record each loaded scene's (and
    perspective sensor's) source, converted at load time (so later edits of
    the dictionary do not change the recorded scene; an unsupported scene
    loads in Mitsuba and raises when an mtx integrator renders it)."""
    import os

    from .mitsuba_dict import SENSOR_TYPES, sensor_from_dict, spec_from_dict

    if getattr(mi, "_mtx_wrapped", False):
        return
    load_dict, load_file = getattr(mi, "load_dict", None), getattr(mi, "load_file", None)
    if load_dict is not None:
        def _load_dict(d, *args, **kwargs):
            obj = load_dict(d, *args, **kwargs)
            if isinstance(d, dict) and d.get("type") == "scene":
                try:
                    _record(obj, ("dict", spec_from_dict(d), os.getcwd()))
                except MtxError as e:
                    _record(obj, ("error", str(e), None))  # the message only: no traceback frames kept
            elif isinstance(d, dict) and d.get("type") in SENSOR_TYPES:
                _record(obj, ("sensor", sensor_from_dict(d), None))
            return obj

        mi.load_dict = _load_dict
    if load_file is not None:
        def _load_file(path, *args, **kwargs):
            obj = load_file(path, *args, **kwargs)
            _record(obj, ("xml", os.path.abspath(str(path)), None))
            return obj

        mi.load_file = _load_file
    mi._mtx_wrapped = True


def register_with_mitsuba(mi=None) -> bool:
    """With Mitsuba importable (it is not in this image: returns False), register
    every façade name (path.py:305, path-mis.py:158, pssmltsimple.py:145,
    restirgi.py:591, ...) as an ``mi.SamplingIntegrator`` subclass.

    The registered plugin reads its properties through ``props.get``
    (path.py:22-25) and forwards ``render`` / ``sample`` to the mtx
    integrator. It renders an :class:`mtx.scene.Scene`, or an ``mi.Scene``
    that the script loaded with ``mi.load_dict`` / ``mi.load_file`` after this
    call: those loaders are wrapped to record the scene's source, and the
    plugin converts it (:mod:`mtx.mitsuba_dict` for dictionaries such as
    ``mi.cornell_box()``, path.py:308-309 / path-mis.py:162 /
    restirgi.py:595-599 / nrc.py:130-136; :meth:`mtx.scene.Scene.from_xml` for
    files), so the reference scripts run unchanged. An ``mi.Scene`` of unknown
    origin (or one using plugins outside the supported subset) raises
    MtxError instead of rendering something else. `mi` may be passed
    explicitly (tests use a stand-in module)."""
    if mi is None:
        try:
            import mitsuba as mi  # noqa: F401
        except Exception:
            return False
    _wrap_loaders(mi)
    for name, ctor in list(_REGISTRY.items()):
        mi.register_integrator(name, _mitsuba_plugin(mi, name, ctor))
    return True


def _mitsuba_plugin(mi, name: str, ctor):
    """Constructor of the mi.SamplingIntegrator subclass wrapping `ctor`."""

    def _scene(scene):
        return mtx_scene_of(scene)

    class Plugin(mi.SamplingIntegrator):
        def __init__(self, props):
            super().__init__(props)
            keys = props.keys() if hasattr(props, "keys") else []
            self.mtx = ctor({k: props[k] for k in keys})

        def render(self, scene, sensor=None, seed=0, spp=1, develop=True, evaluate=True):
            return self.mtx.render(_scene(scene), sensor, seed, spp, develop, evaluate)

        def sample(self, scene, sampler, ray, medium=None, active=True):
            return self.mtx.sample(_scene(scene), sampler, ray, medium, active)

    Plugin.__name__ = Plugin.__qualname__ = f"Mtx_{name}"
    return lambda props: Plugin(props)
