"""Where a shade step's cycles go (diagnostic): runs one headline render
(path-mis, bedroom 1280x720, spp 256) with the MTX_DIAG_STAMPS library
variant (`make -C mitsuba3-experiments_amd/csrc variant NAME=stamps
DEFS=-DMTX_DIAG_STAMPS=1`) and prints each phase's share of the shade
kernel's wave-cycles (s_memtime stamps summed per wave, kernels.hip).
The stamp build's own run time is not quoted: read the shares."""
import ctypes as C
import json
import os
import sys

os.environ["MTX_LIB_VARIANT"] = "stamps"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))

SEGS = ["loop top -> shade start (queue entry, prefetched hit)",
        "-> surface interaction (ray_d, thr, L, misc, shading record)",
        "-> material + texture colour (bsdf_at)",
        "-> emitter sample (NEE)",
        "-> BSDF eval + sample",
        "-> RR, spawn, path-state stores",
        "-> block append (2 barriers + 1 atomic) + queue / shadow stores",
        "-> next step's queue entry and hit"]


def main():
    import torch

    from mtx import PathIntegrator, _lib, scene

    lib = _lib.lib()
    lib.mtx_diag_shade_stamps.argtypes = [C.c_void_p]
    lib.mtx_diag_shade_stamps.restype = C.c_int
    sc = scene.bedroom()
    integ = PathIntegrator({"max_depth": 8, "rr_depth": 2})
    out = torch.empty((sc.height + 2, sc.width + 2, 4), dtype=torch.float32, device="cuda:0")
    buf = (C.c_ulonglong * 10)()
    integ.render_film(sc, seed=1, spp=256, out=out)  # warm-up
    assert lib.mtx_diag_shade_stamps(buf) == 8, "not an MTX_DIAG_STAMPS build"
    integ.render_film(sc, seed=0, spp=256, out=out)
    torch.cuda.synchronize()
    assert lib.mtx_diag_shade_stamps(buf) == 8
    acc = [int(buf[k]) for k in range(8)]
    steps, waves = int(buf[8]), int(buf[9])
    tot = sum(acc)
    res = {"steps_per_wave": steps / max(1, waves), "cycles_per_step": tot / max(1, steps),
           "shares": {SEGS[k]: round(acc[k] / tot, 4) for k in range(8)}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
