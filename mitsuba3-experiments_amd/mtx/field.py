"""Radiance field for NRC (nerad.py:54-106 ``Field``).

``Field(scene)`` holds the hash-grid table and the MLP weights (fp16,
``nn.pack(..., "training")`` layout restated as plain row-major matrices) and
evaluates ``Field(si)`` = MLP(p_norm, hashgrid(p_norm), wi, SH3(wi)) on the
GPU: the encoder is ``mtx_core/field.h``, the fused MLP runs on the gfx950
matrix cores (``csrc/field.hip``). Parameters are seeded-random (inference
only; the reference trains them with Adam, ``nerad.py:336-375``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._lib import MtxError, check, context, lib


class Field:
    def __init__(self, scene=None, width: int = 64, n_hidden: int = 4, sh_order: int = 3, bias: bool = False,
                 n_levels: int = 16, n_features: int = 2, log2_table: int = 19, base_res: int = 16,
                 per_level_scale: float = 2.0, seed: int = 0, table_scale: float = 1e-1, bbox=None):
        if width != 64 or sh_order != 3 or bias:
            raise MtxError("Field supports width 64, sh_order 3, no bias (nerad.py:57-61 defaults)")
        self.n_levels, self.n_features, self.log2_table = n_levels, n_features, log2_table
        self.base_res, self.per_level_scale, self.n_hidden = base_res, per_level_scale, n_hidden
        self.n_in = 3 + n_levels * n_features + 3 + 16
        if self.n_in > 64:
            raise MtxError("too many encoding features for one 64-wide input layer")
        if bbox is None:
            v = np.asarray(scene.vpos, np.float32).reshape(-1, 3)
            bbox = (v.min(0), v.max(0))  # scene.bbox() (nerad.py:93)
        self.bbox_min = np.asarray(bbox[0], np.float32)
        self.bbox_max = np.asarray(bbox[1], np.float32)
        rng = np.random.default_rng(seed)
        T = 1 << log2_table
        self.table = (rng.uniform(-1, 1, (n_levels, T, n_features)) * table_scale).astype(np.float16)
        dims = [(64, self.n_in)] + [(64, 64)] * n_hidden + [(3, 64)]
        self.weights = [(rng.uniform(-1, 1, d) * np.sqrt(6.0 / d[1])).astype(np.float16) for d in dims]
        self._ctx_uploaded = set()

    # ---------------------------------------------------------------- device --
    def desc(self) -> _abi.FieldDesc:
        d = _abi.FieldDesc()
        d.n_levels, d.n_features, d.log2_table, d.base_res = self.n_levels, self.n_features, self.log2_table, \
            self.base_res
        d.per_level_scale = self.per_level_scale
        d.bbox_min[:] = self.bbox_min.tolist()
        d.bbox_max[:] = self.bbox_max.tolist()
        d.n_in, d.n_hidden = self.n_in, self.n_hidden
        self._t = np.ascontiguousarray(self.table).view(np.uint16)
        self._w = np.ascontiguousarray(np.concatenate([w.reshape(-1) for w in self.weights])).view(np.uint16)
        d.table = self._t.ctypes.data
        d.weights = self._w.ctypes.data
        return d

    def upload(self, ctx=None):
        ctx = ctx or context()
        d = self.desc()
        check(lib().mtx_field_upload(ctx.handle, C.byref(d)), "mtx_field_upload")
        self._ctx_uploaded.add(id(ctx))
        return ctx

    def _ensure(self, ctx):
        ctx = ctx or context()
        if id(ctx) not in self._ctx_uploaded:
            self.upload(ctx)
        return ctx

    def __call__(self, p, wi, ctx=None) -> np.ndarray:
        """Field(si): radiance (n, 3) for positions p and world directions wi."""
        ctx = self._ensure(ctx)
        p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
        wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
        out = np.zeros((len(p), 3), np.float32)
        check(lib().mtx_field_eval(ctx.handle, len(p), p.ctypes.data, wi.ctypes.data, out.ctypes.data),
              "mtx_field_eval")
        return out

    def features(self, p, wi, ctx=None) -> np.ndarray:
        """fp16 feature rows (n, 64) (zero-padded beyond n_in)."""
        ctx = self._ensure(ctx)
        p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
        wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
        out = np.zeros((len(p), 64), np.uint16)
        check(lib().mtx_field_features(ctx.handle, len(p), p.ctypes.data, wi.ctypes.data, out.ctypes.data),
              "mtx_field_features")
        return out.view(np.float16)

    def mlp(self, feat, ctx=None) -> np.ndarray:
        ctx = self._ensure(ctx)
        f = np.ascontiguousarray(np.asarray(feat, np.float16).reshape(-1, 64)).view(np.uint16)
        out = np.zeros((len(f), 3), np.float32)
        check(lib().mtx_field_mlp(ctx.handle, len(f), f.ctypes.data, out.ctypes.data), "mtx_field_mlp")
        return out

    # ------------------------------------------------------ CPU reference --
    def mlp_reference(self, feat) -> np.ndarray:
        """Plain fp32 reference of the network (fp16 weights, f32 layer
        products, activations rounded to fp16 and LeakyReLU(0.01) evaluated
        in fp16 as the device does); test use only."""
        x = np.asarray(feat, np.float16).astype(np.float32)[:, : self.n_in]
        for i, w in enumerate(self.weights):
            x = x @ w.astype(np.float32).T
            if i < len(self.weights) - 1:
                h = x.astype(np.float16)
                x = np.maximum(h, h * np.float16(0.01)).astype(np.float32)
        return x.astype(np.float16).astype(np.float32)

    def flops_per_query(self) -> int:
        return 2 * sum(w.shape[0] * w.shape[1] for w in self.weights)
