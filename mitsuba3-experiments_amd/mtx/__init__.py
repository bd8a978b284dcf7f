"""mtx — MI355X-native wavefront path-tracing integrator.

Drop-in for the per-bounce sample() loop of DoeringChristian/
mitsuba3-experiments (path.py, path-mis.py, nrc.py, ...) and its GPU
primitives (prefix_sum.py, hashgrid.py, reductions.py). Host code is Python;
every hot-path operation runs in libmtx.so (hand-written HIP for gfx950)
through the C ABI declared in include/mtx.h.
"""
from ._lib import MtxError, context, lib  # noqa: F401
from .integrators import (  # noqa: F401
    IndependentSampler,
    NeradIntegrator,
    NRCIntegrator,
    Path,
    PathIntegrator,
    PssmltPath,
    PssmltSimple,
    RestirIntegrator,
    Simple,
    develop,
    load_dict,
    mtx_scene_of,
    register_integrator,
    register_with_mitsuba,
    scene_with_sensor,
    trace_rays,
)

__version__ = "0.1.0"
