"""Python façade (SURVEY §8b layer 2) without a GPU: the Mitsuba plugin
registration against a stand-in `mitsuba` module (Mitsuba is not importable
here), property defaults of the reference scripts, ray-layout handling."""
import types

import numpy as np
import pytest


def _fake_mitsuba():
    mi = types.SimpleNamespace()
    mi.registered = {}

    class SamplingIntegrator:  # the base class path.py:21 subclasses
        def __init__(self, props):
            self.base_props = props

    class Props(dict):  # mi.Properties: keys() / [] / get()
        def get(self, k, d=None):
            return super().get(k, d)

    mi.SamplingIntegrator = SamplingIntegrator
    mi.Properties = Props
    mi.register_integrator = lambda name, ctor: mi.registered.__setitem__(name, ctor)
    return mi


def test_register_with_mitsuba_subclasses():
    from mtx import integrators
    from mtx._lib import MtxError

    mi = _fake_mitsuba()
    assert integrators.register_with_mitsuba(mi) is True
    for name in ("mypath", "path_test", "pssmlt_simple", "pssmlt", "restirgi", "nrc"):
        assert name in mi.registered  # path.py:305, path-mis.py:158, pssmltsimple.py:145, restirgi.py:591
    plug = mi.registered["mypath"](mi.Properties(max_depth=3, rr_depth=1))  # path.py:313-314
    assert isinstance(plug, mi.SamplingIntegrator)
    assert (plug.mtx.max_depth, plug.mtx.rr_depth) == (3, 1)
    assert mi.registered["path_test"](mi.Properties()).mtx.max_depth == 8  # path-mis.py:21
    with pytest.raises(MtxError, match="mi.Scene"):
        plug.render(object(), None, 0, 4)
    with pytest.raises(MtxError, match="mi.Scene"):
        plug.sample(object(), None, None)


def test_register_without_mitsuba():
    from mtx import integrators

    try:
        import mitsuba  # noqa: F401
        pytest.skip("mitsuba importable")
    except ImportError:
        pass
    assert integrators.register_with_mitsuba() is False


def test_ray_layouts():
    from mtx.integrators import _rows3

    a = np.arange(30, dtype=np.float32).reshape(10, 3)
    assert np.array_equal(_rows3(a), a)
    assert np.array_equal(_rows3(a.T), a)  # Dr.Jit Array3f layout (3, N)
    assert _rows3(np.zeros(3, np.float32)).shape == (1, 3)
    # a 3x3 bare array is ambiguous and refused; from a ray object it is (3, N)
    from mtx import MtxError

    sq = np.arange(9, dtype=np.float32).reshape(3, 3)
    with pytest.raises(MtxError):
        _rows3(sq)
    assert np.array_equal(_rows3(sq, drjit_layout=True), sq.T)
    assert np.array_equal(_rows3(a.T, drjit_layout=True), a)
