"""Neural radiosity training of the radiance field (nerad.py; SURVEY §8f
item 3: "training (Adam, GradScaler, nerad.py:336-400) after" inference).

The reference trains ``Field`` (hash grid + fp16 MLP, nerad.py:54-106) by
minimising the radiosity residual ``mean((L_lhs - detach(L_rhs))^2)``
(``training_step``, :336-348): left-hand side points from
``IntersectionSampler`` (:254-285), ``L_lhs = Field(si)``, the right-hand side
one bounce of the rendering equation with ``M = 32`` samples per point whose
continuation is the field itself (``Integrator.sample_rhs``, :175-238), then
``dr.backward(scaler.scale(loss))`` and ``scaler.step(opt)`` with Adam on
fp32 copies of the parameters (:351-366).

Here one ``mtx_nerad_step`` call runs that whole step on the GPU: the LHS
sampler kernel, the RHS lanes on the wavefront path tracer (persistent trace
kernels + ``k_shade<NERAD_RHS>``, their stop vertices querying the MFMA field
through the NRC cache queue), the fused forward/backward of the network, the
hash-grid scatter of the gradients, GradScaler's finite check and Adam. The
names below follow the reference script.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._lib import MtxError, check, context, lib
from .field import Field
from .integrators import _bind_scene


class SeedGenerator:
    """The reference's global ``seed()`` counter (nerad.py:33-40)."""

    def __init__(self, start: int = 0):
        self.next = int(start)

    def __call__(self) -> int:
        s = self.next
        self.next += 1
        return s


# ---------------------------------------------------------------- tables --
def surface_tables(scene) -> dict:
    """Surface-area distributions of IntersectionSampler (nerad.py:281-289):
    the shapes weighted by area, and per shape its triangles by area (upstream
    Mesh::m_area_pmf; triangles in BVH leaf order). cdf = float(double
    prefix sum), normalization = float(1 / double(sum))."""
    v = np.asarray(scene.vpos, np.float32).reshape(-1, 3)
    idx = np.asarray(scene.tri_vidx, np.int64).reshape(-1, 3)
    p0, p1, p2 = v[idx[:, 0]], v[idx[:, 1]], v[idx[:, 2]]
    cr = np.cross(p1 - p0, p2 - p0).astype(np.float32)
    area = (np.float32(0.5) * np.sqrt((cr.astype(np.float64) ** 2).sum(1))).astype(np.float32)
    tri_shape = np.asarray(scene.tri_shape, np.int64)
    n_shapes = len(scene.shapes)
    order = np.argsort(tri_shape, kind="stable")  # per shape, ascending leaf index
    counts = np.bincount(tri_shape, minlength=n_shapes)
    if (counts == 0).any():
        raise MtxError("every shape needs at least one triangle")
    tri_off = np.zeros(n_shapes + 1, np.uint32)
    tri_off[1:] = np.cumsum(counts)
    tri_prim = order.astype(np.uint32)
    tri_pmf = area[order]
    tri_cdf = np.zeros_like(tri_pmf)
    tri_sum = np.zeros(n_shapes, np.float32)
    tri_norm = np.zeros(n_shapes, np.float32)
    tri_valid = np.zeros(2 * n_shapes, np.uint32)
    shape_area = np.zeros(n_shapes, np.float64)
    for s in range(n_shapes):
        a, b = tri_off[s], tri_off[s + 1]
        pm = tri_pmf[a:b]
        cd = np.cumsum(pm.astype(np.float64))
        tri_cdf[a:b] = cd.astype(np.float32)
        tri_sum[s] = np.float32(cd[-1])
        nz = np.nonzero(pm > 0)[0]
        if len(nz) == 0:
            raise MtxError(f"shape {s} has zero surface area")
        tri_norm[s] = np.float32(1.0 / np.float64(tri_sum[s]))
        tri_valid[2 * s], tri_valid[2 * s + 1] = nz[0], nz[-1]
        shape_area[s] = float(tri_sum[s])  # shape.surface_area() (:285)
    w = (shape_area / shape_area.sum()).astype(np.float32)  # weights /= dr.sum(weights) (:287)
    shape_cdf = np.cumsum(w.astype(np.float64))
    nz = np.nonzero(w > 0)[0]
    return {
        "shape_pmf": w, "shape_cdf": shape_cdf.astype(np.float32), "shape_sum": np.float32(shape_cdf[-1]),
        "shape_norm": np.float32(1.0 / np.float64(np.float32(shape_cdf[-1]))),
        "shape_valid": (int(nz[0]), int(nz[-1])), "tri_off": tri_off, "tri_pmf": tri_pmf, "tri_cdf": tri_cdf,
        "tri_prim": tri_prim, "tri_sum": tri_sum, "tri_norm": tri_norm, "tri_valid": tri_valid,
    }


def tables_struct(t: dict) -> _abi.NeradTables:
    """ctypes view of surface_tables() (the dict keeps the arrays alive)."""
    d = _abi.NeradTables()
    d.n_shapes = len(t["shape_pmf"])
    d.n_entries = len(t["tri_pmf"])
    for k in ("shape_pmf", "shape_cdf", "tri_off", "tri_pmf", "tri_cdf", "tri_prim", "tri_sum", "tri_norm",
              "tri_valid"):
        t[k] = np.ascontiguousarray(t[k])
        setattr(d, k, t[k].ctypes.data)
    d.shape_sum = float(t["shape_sum"])
    d.shape_norm = float(t["shape_norm"])
    d.shape_valid[0], d.shape_valid[1] = t["shape_valid"]
    return d


# ------------------------------------------------------- reference names --
class IntersectionSampler:
    """nerad.py:275-310: surface points by area and incident directions
    (uniform sphere for two-sided BSDFs, hemisphere otherwise)."""

    def __init__(self, scene):
        self.scene = scene
        self.tables = surface_tables(scene)

    def bind(self, ctx):
        _bind_scene(ctx, self.scene)
        if getattr(ctx, "_nerad_key", None) is not self:
            d = tables_struct(self.tables)
            check(lib().mtx_nerad_upload(ctx.handle, C.byref(d)), "mtx_nerad_upload")
            ctx._nerad_key = self
        return ctx

    def sample(self, seed: int, n: int, ctx=None) -> np.ndarray:
        """n points: (n, 9) float32 = prim (uint32 bits), b1, b2, p.xyz, wi_world.xyz."""
        ctx = self.bind(ctx or context())
        out = np.zeros((n, 9), np.float32)
        a = _abi.NeradArgs(lhs_seed=seed, rhs_seed=0, batch=n, M=1)
        check(lib().mtx_nerad_lhs(ctx.handle, C.byref(a), out.ctypes.data), "mtx_nerad_lhs")
        return out


class Adam:
    """drjit.opt.Adam settings (nerad.py:336-342; upstream defaults)."""

    def __init__(self, lr: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999, epsilon: float = 1e-8):
        self.lr, self.beta_1, self.beta_2, self.epsilon = lr, beta_1, beta_2, epsilon


class GradScaler:
    """drjit.opt.GradScaler settings (nerad.py:347): dynamic loss scaling
    (upstream defaults unverifiable offline: torch.amp's are used)."""

    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000):
        self.init_scale, self.growth_factor = init_scale, growth_factor
        self.backoff_factor, self.growth_interval = backoff_factor, growth_interval


class Integrator:
    """nerad.py:118-255: sample_lhs = Field(si); sample_rhs = one bounce of
    the rendering equation with M samples per point, continued by the field."""

    def __init__(self, field: Field, batch_size: int = 2 ** 14, M: int = 32):
        self.field, self.batch_size, self.M = field, int(batch_size), int(M)

    def render(self, scene, sensor=None, seed: int = 0, spp: int = 1, develop: bool = True, evaluate: bool = True):
        """integrator.render(scene, sensor, seed, spp) (nerad.py:399): sample()
        (:235-254) for every camera lane, on the wavefront (MTX_INT_NERAD)."""
        from .integrators import NeradIntegrator

        return NeradIntegrator({"field": self.field}).render(scene, seed=seed, spp=spp, develop=develop)

    def sample_lhs(self, scene, si: np.ndarray, ctx=None) -> np.ndarray:
        """Field(si) at IntersectionSampler points ((n, 9) rows)."""
        return self.field(si[:, 3:6], si[:, 6:9], ctx=ctx)

    def sample_rhs(self, scene, isampler: IntersectionSampler, lhs_seed: int, rhs_seed: int, ctx=None,
                   lanes: bool = False):
        """L_rhs (batch, 3) at the points isampler.sample(lhs_seed, batch);
        with lanes=True also every sample's L (batch * M, 3) before the mean."""
        ctx = isampler.bind(self.field._ensure(ctx))
        a = _abi.NeradArgs(lhs_seed=lhs_seed, rhs_seed=rhs_seed, batch=self.batch_size, M=self.M)
        out = np.zeros((self.batch_size, 3), np.float32)
        ln = np.zeros((self.batch_size * self.M, 3), np.float32) if lanes else None
        check(lib().mtx_nerad_rhs(ctx.handle, C.byref(a), out.ctypes.data, ln.ctypes.data if lanes else None),
              "mtx_nerad_rhs")
        return (out, ln) if lanes else out


class FieldTrainer:
    """The training loop of nerad.py:383-400 on one device context: each
    step seeds the LHS sampler and the RHS sampler from the reference's
    seed() counter and runs training_step (:363-375) on the GPU."""

    def __init__(self, scene, field: Field, batch_size: int = 2 ** 14, M: int = 32, opt: Adam | None = None,
                 scaler: GradScaler | None = None, seed_start: int = 1, ctx=None):
        self.scene, self.field = scene, field
        self.isampler = IntersectionSampler(scene)
        self.integrator = Integrator(field, batch_size, M)
        self.opt, self.scaler = opt or Adam(), scaler or GradScaler()
        self.seed = SeedGenerator(seed_start)  # seed 0 renders img_ref in the script (:329)
        self.ctx = self.isampler.bind(field._ensure(ctx or context()))
        o = _abi.FieldOpt(lr=self.opt.lr, beta_1=self.opt.beta_1, beta_2=self.opt.beta_2,
                          epsilon=self.opt.epsilon, init_scale=self.scaler.init_scale,
                          growth_factor=self.scaler.growth_factor, backoff_factor=self.scaler.backoff_factor,
                          growth_interval=self.scaler.growth_interval)
        check(lib().mtx_field_train_init(self.ctx.handle, C.byref(o)), "mtx_field_train_init")

    def step(self, counters: bool = False) -> dict:
        """One training_step; returns its loss, scale and phase times (ms);
        counters=True also counts the RHS traversal visits (slower)."""
        a = _abi.NeradArgs(lhs_seed=self.seed(), rhs_seed=self.seed(), batch=self.integrator.batch_size,
                           M=self.integrator.M, flags=1 if counters else 0)
        st = _abi.TrainStats()
        check(lib().mtx_nerad_step(self.ctx.handle, C.byref(a), C.byref(st)), "mtx_nerad_step")
        return st.as_dict()

    def params(self):
        """fp32 master copies: (table (n_levels, T, n_features), [weights])."""
        T = 1 << self.field.log2_table
        tab = np.zeros((self.field.n_levels, T, self.field.n_features), np.float32)
        nw = sum(w.size for w in self.field.weights)
        w = np.zeros(nw, np.float32)
        check(lib().mtx_field_params(self.ctx.handle, tab.ctypes.data, w.ctypes.data, None, None),
              "mtx_field_params")
        out, o = [], 0
        for x in self.field.weights:
            out.append(w[o:o + x.size].reshape(x.shape))
            o += x.size
        return tab, out

    def download(self) -> None:
        """field.table / field.weights <- fp16 casts of the trained parameters
        (the device field already is; this refreshes the host copy)."""
        tab, ws = self.params()
        self.field.table = tab.astype(np.float16)
        self.field.weights = [w.astype(np.float16) for w in ws]


def field_grad(field: Field, p, wi, target, scale: float = 1.0, ctx=None):
    """Loss, output and gradients of scale * mean((Field(p, wi) - target)^2)
    w.r.t. the table and the weights (mtx_field_grad; test entry)."""
    ctx = field._ensure(ctx)
    p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
    wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
    target = np.ascontiguousarray(target, np.float32).reshape(-1, 3)
    n = len(p)
    out = np.zeros((n, 3), np.float32)
    gt = np.zeros(field.table.shape, np.float32)
    gw = np.zeros(sum(w.size for w in field.weights), np.float32)
    loss = C.c_double()
    check(lib().mtx_field_grad(ctx.handle, n, p.ctypes.data, wi.ctypes.data, target.ctypes.data, float(scale),
                               out.ctypes.data, C.byref(loss), gt.ctypes.data, gw.ctypes.data), "mtx_field_grad")
    ws, o = [], 0
    for x in field.weights:
        ws.append(gw[o:o + x.size].reshape(x.shape))
        o += x.size
    return loss.value, out, gt, ws


def field_train_step(field: Field, p, wi, target, ctx=None) -> dict:
    """One optimiser step on given points / targets (mtx_field_train_step)."""
    ctx = field._ensure(ctx)
    p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
    wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
    target = np.ascontiguousarray(target, np.float32).reshape(-1, 3)
    st = _abi.TrainStats()
    check(lib().mtx_field_train_step(ctx.handle, len(p), p.ctypes.data, wi.ctypes.data, target.ctypes.data,
                                     C.byref(st)), "mtx_field_train_step")
    return st.as_dict()


def field_train_init(field: Field, opt: Adam | None = None, scaler: GradScaler | None = None, ctx=None):
    ctx = field._ensure(ctx)
    opt, scaler = opt or Adam(), scaler or GradScaler()
    o = _abi.FieldOpt(lr=opt.lr, beta_1=opt.beta_1, beta_2=opt.beta_2, epsilon=opt.epsilon,
                      init_scale=scaler.init_scale, growth_factor=scaler.growth_factor,
                      backoff_factor=scaler.backoff_factor, growth_interval=scaler.growth_interval)
    check(lib().mtx_field_train_init(ctx.handle, C.byref(o)), "mtx_field_train_init")
    return ctx


def field_params(field: Field, ctx=None):
    """fp32 master table, weights and Adam moments (m, v) of a training field."""
    ctx = field._ensure(ctx)
    n_tab = field.table.size
    nw = sum(w.size for w in field.weights)
    tab = np.zeros(n_tab, np.float32)
    w = np.zeros(nw, np.float32)
    m = np.zeros(n_tab + nw, np.float32)
    v = np.zeros(n_tab + nw, np.float32)
    check(lib().mtx_field_params(ctx.handle, tab.ctypes.data, w.ctypes.data, m.ctypes.data, v.ctypes.data),
          "mtx_field_params")
    return tab, w, m, v
