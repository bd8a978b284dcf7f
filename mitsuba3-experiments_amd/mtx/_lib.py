"""Loader for the in-tree libmtx.so (the HIP product library).

The library is loaded from this package directory only; there is no CPU or
Python fallback for the hot path: if the library is missing or no gfx950
device is visible, the calls that need it raise :class:`MtxError`.

torch, when importable, is imported first so that torch and libmtx share one
HIP runtime (torch bundles its own libamdhip64.so.7; loading the system copy
first would put two runtimes in one process).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

from . import _abi

try:  # one HIP runtime per process: torch's, if torch is present
    import torch as _torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for host-only use
    _torch = None

# MTX_LIB_VARIANT selects an in-tree tuning build (e.g. "shade4" ->
# libmtx_shade4.so, see csrc/Makefile `variants`); default libmtx.so.
_VARIANT = os.environ.get("MTX_LIB_VARIANT", "")
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        f"libmtx_{_VARIANT}.so" if _VARIANT else "libmtx.so")


class MtxError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libmtx.so (raises MtxError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MtxError(
            f"libmtx.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback for the hot path."
        )
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "mtx_abi_version": ([], C.c_int),
        "mtx_last_error": ([], C.c_char_p),
        "mtx_ctx_create": ([C.c_int, C.POINTER(vp)], C.c_int),
        "mtx_ctx_destroy": ([vp], None),
        "mtx_bvh_build": ([vp, u32, vp, u32, vp, C.POINTER(u32), vp, vp, C.POINTER(u32)], C.c_int),
        "mtx_bvh_build_occlusion": ([vp, u32, vp, C.POINTER(u32), vp, vp, C.POINTER(u32)], C.c_int),
        "mtx_roughplastic_tables": ([u32, C.c_float, C.c_float, vp, C.POINTER(C.c_float)], C.c_int),
        "mtx_scene_upload": ([vp, C.POINTER(_abi.SceneDesc)], C.c_int),
        "mtx_render": ([vp, C.POINTER(_abi.RenderArgs), vp, C.c_int, C.POINTER(_abi.Stats)], C.c_int),
        "mtx_last_device_ms": ([vp], C.c_double),
        "mtx_field_upload": ([vp, C.POINTER(_abi.FieldDesc)], C.c_int),
        "mtx_field_features": ([vp, u64, vp, vp, vp], C.c_int),
        "mtx_field_mlp": ([vp, u64, vp, vp], C.c_int),
        "mtx_field_eval": ([vp, u64, vp, vp, vp], C.c_int),
        "mtx_set_camera": ([vp, C.POINTER(_abi.Camera)], C.c_int),
        "mtx_restir_rows": ([vp, C.c_int, u32, u32, vp, C.c_int], C.c_int),
        "mtx_restir_state": ([vp, C.c_int, vp, u64], C.c_int),
        "mtx_sample_rays": ([vp, C.POINTER(_abi.RenderArgs), u64, vp, vp, u32, vp, vp], C.c_int),
        "mtx_sample_rays_dev": ([vp, C.POINTER(_abi.RenderArgs), u64, vp, vp, u32, vp, vp], C.c_int),
        "mtx_trace": ([vp, u64, vp, C.c_int, vp, vp], C.c_int),
        "mtx_trace_dev": ([vp, u64, vp, C.c_int, vp, vp], C.c_int),
        "mtx_prefix_sum_u32": ([vp, vp, vp, u64, C.c_int], C.c_int),
        "mtx_prefix_sum_f32_hs": ([vp, vp, vp, u64], C.c_int),
        "mtx_prefix_sum_u32_dev": ([vp, vp, vp, u64, C.c_int], C.c_int),
        "mtx_prefix_sum_f32_hs_dev": ([vp, vp, vp, u64], C.c_int),
        "mtx_hashgrid_build": ([vp, vp, u64, u32, u32, vp, vp, vp, vp], C.c_int),
        "mtx_hashgrid_build_dev": ([vp, vp, u64, u32, u32, vp, vp, vp, vp], C.c_int),
        "mtx_scatter_reduce_f32": ([vp, C.c_int, vp, u64, vp, vp, u64], C.c_int),
        "mtx_scatter_reduce_f32_dev": ([vp, C.c_int, vp, u64, vp, vp, u64], C.c_int),
        "mtx_group_by_u32": ([vp, vp, u64, u32, vp, vp, vp], C.c_int),
        "mtx_group_by_u32_dev": ([vp, vp, u64, u32, vp, vp, vp], C.c_int),
        "mtx_field_train_init": ([vp, C.POINTER(_abi.FieldOpt)], C.c_int),
        "mtx_field_grad": ([vp, u64, vp, vp, vp, C.c_float, vp, C.POINTER(C.c_double), vp, vp], C.c_int),
        "mtx_field_train_step": ([vp, u64, vp, vp, vp, C.POINTER(_abi.TrainStats)], C.c_int),
        "mtx_field_params": ([vp, vp, vp, vp, vp], C.c_int),
        "mtx_nerad_upload": ([vp, C.POINTER(_abi.NeradTables)], C.c_int),
        "mtx_nerad_lhs": ([vp, C.POINTER(_abi.NeradArgs), vp], C.c_int),
        "mtx_nerad_rhs": ([vp, C.POINTER(_abi.NeradArgs), vp, vp], C.c_int),
        "mtx_nerad_step": ([vp, C.POINTER(_abi.NeradArgs), C.POINTER(_abi.TrainStats)], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.mtx_abi_version() != _abi.MTX_ABI_VERSION:
        raise MtxError("libmtx ABI version mismatch; rebuild the library")
    _lib = L
    return L


def check(rc: int, what: str = "libmtx call") -> None:
    if rc != 0:
        msg = lib().mtx_last_error().decode("utf-8", "replace")
        raise MtxError(f"{what} failed with {_abi.ERRORS.get(rc, rc)}: {msg}")


def ptr(a) -> int | None:
    """Address of a contiguous numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data


class Context:
    """One libmtx context bound to one HIP device (mirrors mtx_ctx)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        check(L.mtx_ctx_create(int(device), C.byref(h)), f"mtx_ctx_create(device={device})")
        self._h = h
        self.device = device
        self.scene = None

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().mtx_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def context(device: int | None = None) -> Context:
    """Process-wide context per device (default: torch's current device once
    torch has initialised HIP, else LOCAL_RANK or 0)."""
    if device is None:
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            device = torch.cuda.current_device()
        else:
            device = int(os.environ.get("LOCAL_RANK", "0"))
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]
