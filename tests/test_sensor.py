"""The ``sensor`` argument of SamplingIntegrator.render / mi.render
(testpssmlt.py:45 ``integrator.render(scene, scene.sensors()[0], ...)``,
pssmlt.py:167-175, restirgi.py:182-190 ``film = sensor.film()``): the film is
rendered through the given sensor, not the scene's own camera."""
import numpy as np
import pytest

from test_mitsuba_dict import T, _fake_mi, cornell_box


def _moved_sensor(width=48, height=48):
    return {"type": "perspective", "fov": 30.0, "fov_axis": "smaller",
            "to_world": T.look_at(origin=[0.3, 0.2, 3.5], target=[0, 0, 0], up=[0, 1, 0]),
            "film": {"type": "hdrfilm", "width": width, "height": height}}


def test_sensor_forms_resolve():
    from mtx import MtxError, integrators
    from mtx.mitsuba_dict import scene_from_dict, sensor_from_dict
    from mtx.scene import camera_from_sensor

    sc = scene_from_dict(cornell_box(48, 48))
    assert integrators.scene_with_sensor(sc, None) is sc
    assert integrators.scene_with_sensor(sc, 0) is sc
    assert integrators.scene_with_sensor(sc, sc.sensors()[0]) is sc  # the scene's own sensor
    with pytest.raises(MtxError, match="one sensor"):
        integrators.scene_with_sensor(sc, 1)
    with pytest.raises(MtxError, match="unsupported sensor"):
        integrators.scene_with_sensor(sc, object())
    with pytest.raises(MtxError, match="perspective only"):
        integrators.scene_with_sensor(sc, {"type": "orthographic"})
    v = integrators.scene_with_sensor(sc, _moved_sensor())
    ref = camera_from_sensor(sensor_from_dict(_moved_sensor()))
    assert bytes(v.camera) == bytes(ref) and bytes(v.camera) != bytes(sc.camera)
    assert v.nodes is sc.nodes and v.tri_geom is sc.tri_geom  # same geometry, no copy
    assert integrators.scene_with_sensor(sc, ref).camera.origin[0] == ref.origin[0]
    w = integrators.scene_with_sensor(sc, _moved_sensor(32, 20))
    assert (w.width, w.height) == (32, 20)
    # an mi.Sensor loaded by the wrapped mi.load_dict
    mi = _fake_mi()
    mi.load_dict = lambda d: object.__new__(type("MiObj", (), {}))
    integrators._wrap_loaders.__globals__  # noqa: B018 (module loaded)
    mi._mtx_wrapped = False
    integrators._wrap_loaders(mi)
    s_obj = mi.load_dict(_moved_sensor())
    assert bytes(integrators.scene_with_sensor(sc, s_obj).camera) == bytes(ref)


def test_oracle_film_follows_the_sensor(oracle):
    """Rendering through a moved sensor changes the image; the scene view the
    sensor yields is what the oracle renders (CPU)."""
    from mtx import integrators, load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(cornell_box(32, 32))
    integ = load_dict({"type": "path_test"})
    v = integrators.scene_with_sensor(sc, _moved_sensor(32, 32))
    a = oracle.render(sc, integ.render_args(sc, 1, 4))
    b = oracle.render(v, integ.render_args(v, 1, 4))
    assert not np.array_equal(a, b) and np.isfinite(b).all()


@pytest.mark.gpu
def test_render_through_sensor_bit_exact(oracle):
    """render(scene, sensor) on the GPU equals the oracle's render of the scene
    seen through that sensor; a later render without a sensor is the scene's
    own camera again (the device camera is re-pointed, not left behind), and
    a sensor with another film size renders that film size."""
    from mtx import integrators, load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(cornell_box(48, 48))
    integ = load_dict({"type": "path_test"})
    own = integ.render_film(sc, seed=2, spp=8)
    moved = integ.render_film(sc, seed=2, spp=8, sensor=_moved_sensor())
    v = integrators.scene_with_sensor(sc, _moved_sensor())
    np.testing.assert_array_equal(moved, oracle.render(v, integ.render_args(v, 2, 8)))
    np.testing.assert_array_equal(own, oracle.render(sc, integ.render_args(sc, 2, 8)))
    np.testing.assert_array_equal(integ.render_film(sc, seed=2, spp=8), own)
    img = integ.render(sc, _moved_sensor(40, 24), seed=2, spp=4)
    assert img.shape == (24, 40, 3) and np.isfinite(img).all()
