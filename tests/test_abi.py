"""The C ABI library loads, exports exactly what include/mtx.h declares, and
its host-only entry points behave (no GPU needed)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "mtx.h")).read()
    return sorted(set(re.findall(r"\b(mtx_[a-z0-9_]+)\s*\(", src)))


def test_header_and_exports_agree():
    from mtx import _abi

    assert _declared() == sorted(_abi.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    from mtx import _lib

    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.mtx_abi_version() == _lib._abi.MTX_ABI_VERSION == 8


def test_struct_sizes_match_header():
    from mtx import _abi

    assert C.sizeof(_abi.Material) == 72
    assert C.sizeof(_abi.Emitter) == 64
    assert C.sizeof(_abi.Shape) == 16
    assert C.sizeof(_abi.Camera) == 112
    assert C.sizeof(_abi.RenderArgs) == 80
    assert C.sizeof(_abi.FieldOpt) == 32
    assert C.sizeof(_abi.TrainStats) == 88
    assert C.sizeof(_abi.NeradTables) == 96
    assert C.sizeof(_abi.NeradArgs) == 20


def test_struct_layouts_match_the_c_compiler(tmp_path):
    """Every ctypes mirror of an include/mtx.h struct has the C compiler's
    size and field offsets (gcc on the header itself)."""
    import shutil
    import subprocess

    from mtx import _abi

    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    structs = {"SceneDesc": "mtx_scene_desc", "RenderArgs": "mtx_render_args", "Camera": "mtx_camera",
               "Material": "mtx_material", "Emitter": "mtx_emitter"}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mtx.h"', "int main(void) {"]
    for py, c in structs.items():
        lines.append(f'  printf("{py} size %zu\\n", sizeof({c}));')
        for f, _ in getattr(_abi, py)._fields_:
            lines.append(f'  printf("{py} {f} %zu\\n", offsetof({c}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        py, field, val = line.split()
        T = getattr(_abi, py)
        got = C.sizeof(T) if field == "size" else getattr(T, field).offset
        assert got == int(val), (py, field, got, int(val))


def test_ctx_create_without_gpu_fails_cleanly():
    import torch

    from mtx import _lib

    if torch.cuda.is_available():
        return
    h = C.c_void_p()
    rc = _lib.lib().mtx_ctx_create(0, C.byref(h))
    assert rc < 0
    assert _lib.lib().mtx_last_error()


def test_bvh_build_rejects_bad_input():
    from mtx import _lib

    L = _lib.lib()
    v = np.zeros(9, np.float32)
    idx = np.array([0, 1, 7], np.uint32)  # vertex 7 does not exist
    nodes = np.zeros(64, np.int32)
    geom = np.zeros(12, np.float32)
    perm = np.zeros(1, np.uint32)
    nn, dep = C.c_uint32(), C.c_uint32()
    rc = L.mtx_bvh_build(v.ctypes.data, 3, idx.ctypes.data, 1, nodes.ctypes.data, C.byref(nn), geom.ctypes.data,
                         perm.ctypes.data, C.byref(dep))
    assert rc == -1 and b"out of range" in L.mtx_last_error()
    rc = L.mtx_bvh_build_occlusion(geom.ctypes.data, 0, nodes.ctypes.data, C.byref(nn), geom.ctypes.data, None,
                                   C.byref(dep))
    assert rc == -1 and b"empty" in L.mtx_last_error()


def test_roughplastic_tables():
    from mtx import _lib

    tab = np.zeros(64, np.float32)
    internal = C.c_float()
    assert _lib.lib().mtx_roughplastic_tables(0, 0.15, 1.5, tab.ctypes.data, C.byref(internal)) == 0
    assert ((tab > 0) & (tab <= 1)).all()
    assert tab[-1] > 0.9  # normal incidence: ~4 % Fresnel reflectance
    assert 0.3 < internal.value < 0.8


def test_shadow_record_form_is_checked():
    """make_shadow<INT, FINAL> (kernels.hip) static_asserts that an
    integrator's shadow-record form matches where its L is stored
    (shadow_final_form): the round-5 nerad regression made at compile time.
    A final-value record for the nerad RHS (L by path, read-modify-write
    form) must not compile; the library's own instantiations do."""
    import os
    import shutil
    import subprocess

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "mitsuba3-experiments_amd", "csrc", "kernels.hip")
    cmd = [hipcc, "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(root, "include"), "-fsyntax-only", src]
    ok = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stderr[-2000:]
    bad = subprocess.run(cmd + ["-DMTX_TEST_BAD_SHADOW_FORM"], capture_output=True, text=True, timeout=300)
    assert bad.returncode != 0 and "shadow record form does not match" in bad.stderr
