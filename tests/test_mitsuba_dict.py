"""The reference scripts' scenes: mi.load_dict(mi.cornell_box()) (path.py:308-309,
path-mis.py:162, restirgi.py:595-599, nrc.py:130-136) through the mtx
plugin. Mitsuba is not importable here, so a stand-in module plays
mi.load_dict / mi.ScalarTransform4f (a 4x4 ``.matrix``), and the Cornell box
dictionary is restated from Mitsuba 3's ``cornell_box()``: five rectangles, two
cubes, three diffuse BSDFs, one area light, a perspective sensor with
fov_axis "smaller". The converted scene's geometry, light and camera are
checked against numpy, its oracle image against the box's layout (red wall
left, green wall right, light on top); on the GPU the plugin renders the
loaded mi.Scene bit-exactly like the oracle."""
import types

import numpy as np
import pytest


class T:
    """Stand-in for mi.ScalarTransform4f: composable 4x4 matrices."""

    def __init__(self, m=None):
        self.matrix = np.eye(4) if m is None else np.asarray(m, np.float64)

    def _then(self, m):
        return T(self.matrix @ m)

    def translate(self, v):
        m = np.eye(4)
        m[:3, 3] = v
        return self._then(m)

    def scale(self, v):
        m = np.diag(list(np.broadcast_to(np.asarray(v, np.float64), 3)) + [1.0])
        return self._then(m)

    def rotate(self, axis, angle):
        a = np.asarray(axis, np.float64) / np.linalg.norm(axis)
        c, s = np.cos(np.radians(angle)), np.sin(np.radians(angle))
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        m = np.eye(4)
        m[:3, :3] = np.eye(3) + s * K + (1 - c) * K @ K
        return self._then(m)

    @staticmethod
    def look_at(origin, target, up):
        o, t, u = (np.asarray(x, np.float64) for x in (origin, target, up))
        d = (t - o) / np.linalg.norm(t - o)
        left = np.cross(u, d)
        left /= np.linalg.norm(left)
        nu = np.cross(d, left)
        m = np.eye(4)
        m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, nu, d, o
        return T(m)


def cornell_box(width=64, height=64):
    """Mitsuba 3's cornell_box() dictionary (film reduced for the tests)."""
    return {
        "type": "scene",
        "integrator": {"type": "path", "max_depth": 8},
        "sensor": {"type": "perspective", "fov_axis": "smaller", "near_clip": 0.001, "far_clip": 100.0,
                   "focus_distance": 1000, "fov": 39.3077,
                   "to_world": T.look_at(origin=[0, 0, 3.9], target=[0, 0, 0], up=[0, 1, 0]),
                   "sampler": {"type": "independent", "sample_count": 64},
                   "film": {"type": "hdrfilm", "width": width, "height": height, "rfilter": {"type": "gaussian"},
                            "pixel_format": "rgb", "component_format": "float32"}},
        "white": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.885809, 0.698859, 0.666422]}},
        "green": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.105421, 0.37798, 0.076425]}},
        "red": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.570068, 0.0430135, 0.0443706]}},
        "light": {"type": "rectangle", "to_world": T().translate([0.0, 0.99, 0.01]).rotate([1, 0, 0], 90).scale(
            [0.23, 0.19, 0.19]), "bsdf": {"type": "ref", "id": "white"},
                  "emitter": {"type": "area", "radiance": {"type": "rgb", "value": [18.387, 13.9873, 6.75357]}}},
        "floor": {"type": "rectangle", "to_world": T().translate([0.0, -1.0, 0.0]).rotate([1, 0, 0], -90),
                  "bsdf": {"type": "ref", "id": "white"}},
        "ceiling": {"type": "rectangle", "to_world": T().translate([0.0, 1.0, 0.0]).rotate([1, 0, 0], 90),
                    "bsdf": {"type": "ref", "id": "white"}},
        "back": {"type": "rectangle", "to_world": T().translate([0.0, 0.0, -1.0]), "bsdf": {"type": "ref", "id": "white"}},
        "green-wall": {"type": "rectangle", "to_world": T().translate([1.0, 0.0, 0.0]).rotate([0, 1, 0], -90),
                       "bsdf": {"type": "ref", "id": "green"}},
        "red-wall": {"type": "rectangle", "to_world": T().translate([-1.0, 0.0, 0.0]).rotate([0, 1, 0], 90),
                     "bsdf": {"type": "ref", "id": "red"}},
        "small-box": {"type": "cube", "to_world": T().translate([0.335, -0.7, 0.38]).rotate([0, 1, 0], -17).scale(0.3),
                      "bsdf": {"type": "ref", "id": "white"}},
        "large-box": {"type": "cube", "to_world": T().translate([-0.33, -0.4, -0.28]).rotate([0, 1, 0], 18.25).scale(
            [0.3, 0.61, 0.3]), "bsdf": {"type": "ref", "id": "white"}},
    }


def _fake_mi():
    mi = types.SimpleNamespace()
    mi.registered = {}

    class SamplingIntegrator:
        def __init__(self, props):
            self.base_props = props

    class Props(dict):
        def get(self, k, d=None):
            return super().get(k, d)

    class MiScene:  # what mi.load_dict returns for a scene dictionary
        pass

    mi.SamplingIntegrator = SamplingIntegrator
    mi.Properties = Props
    mi.register_integrator = lambda name, ctor: mi.registered.__setitem__(name, ctor)
    mi.load_dict = lambda d: MiScene() if d.get("type") == "scene" else d
    mi.load_file = lambda path: MiScene()
    return mi


def test_cornell_box_converts():
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(cornell_box())
    assert sc.n_tris == 6 * 2 + 2 * 12  # five walls + the light, two cubes
    assert len(sc.emitters) == 1
    e = sc.emitters[0]
    np.testing.assert_allclose(list(e.radiance), [18.387, 13.9873, 6.75357], rtol=1e-6)
    np.testing.assert_allclose(list(e.center), [0.0, 0.99, 0.01], atol=1e-7)
    np.testing.assert_allclose(list(e.normal), [0.0, -1.0, 0.0], atol=1e-6)  # faces down into the box
    assert abs(1.0 / e.inv_area - 4 * 0.23 * 0.19) < 1e-6
    # fov 39.3077 along the smaller (here: equal) axis
    assert abs(sc.camera.tan_x - np.tan(np.radians(39.3077) / 2)) < 1e-6 and abs(sc.camera.tan_y - sc.camera.tan_x) < 1e-7
    np.testing.assert_allclose(list(sc.camera.origin), [0, 0, 3.9], atol=1e-6)
    # every vertex inside the box [-1, 1]^3 (the large box sinks 0.01 into the floor)
    v = np.asarray(sc.vpos).reshape(-1, 3)
    assert np.all(np.abs(v) <= 1.01 + 1e-5)
    # three materials, the walls' colours
    cols = sorted(tuple(round(x, 4) for x in m.rgb) for m in sc.materials)
    assert (0.5701, 0.043, 0.0444) in cols and (0.1054, 0.378, 0.0764) in cols


def test_cornell_box_oracle_image_layout(oracle):
    from mtx import load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(cornell_box(48, 48))
    integ = load_dict({"type": "path_test"})
    film = oracle.render(sc, integ.render_args(sc, 3, 16))
    inner = film[1:-1, 1:-1]
    img = inner[..., :3] / np.maximum(inner[..., 3:4], 1e-12)
    assert np.all(np.isfinite(img)) and img.mean() > 0.05
    left, right = img[:, : 48 // 5].mean((0, 1)), img[:, -48 // 5:].mean((0, 1))
    assert left[0] > 2 * left[1]  # the red wall on the left (camera +x maps to the image left)
    assert right[1] > 1.3 * right[0]  # the green wall on the right (white boxes in view too)
    assert left[0] > 2 * right[0] and right[1] > left[1]
    top = img[: 48 // 6, 48 // 3: 2 * 48 // 3].mean()
    assert top > img.mean()  # the light in the ceiling


def test_plugin_resolves_loaded_scenes():
    from mtx import MtxError, integrators
    from mtx.scene import Scene

    mi = _fake_mi()
    assert integrators.register_with_mitsuba(mi)
    mi_scene = mi.load_dict(cornell_box(16, 16))
    sc = integrators.mtx_scene_of(mi_scene)
    assert isinstance(sc, Scene) and sc.n_tris == 36
    assert integrators.mtx_scene_of(mi_scene) is sc  # converted once
    with pytest.raises(MtxError, match="no recorded source"):
        integrators.mtx_scene_of(object())
    from mtx.mitsuba_dict import spec_from_dict

    bad = cornell_box()
    bad["env"] = {"type": "envmap", "filename": "sky.exr"}
    with pytest.raises(MtxError, match="environment emitter"):
        spec_from_dict(bad)
    gold = cornell_box()
    gold["white"] = {"type": "conductor", "material": "Au"}
    with pytest.raises(MtxError, match="named conductor"):
        spec_from_dict(gold)
    nolight = {k: v for k, v in cornell_box().items() if k != "light"}
    with pytest.raises(MtxError, match="no emitter"):
        spec_from_dict(nolight)


@pytest.mark.gpu
def test_plugin_renders_the_loaded_cornell_box(oracle):
    """mi.render(mi.load_dict(mi.cornell_box()), integrator=path_test) through
    the registered plugin (path-mis.py:162-170): bit-exact against the oracle."""
    from mtx import integrators

    mi = _fake_mi()
    integrators.register_with_mitsuba(mi)
    mi_scene = mi.load_dict(cornell_box(64, 64))
    plug = mi.registered["path_test"](mi.Properties())
    film = plug.mtx.render_film(integrators.mtx_scene_of(mi_scene), seed=5, spp=16)
    sc = integrators.mtx_scene_of(mi_scene)
    ref = oracle.render(sc, plug.mtx.render_args(sc, 5, 16))
    np.testing.assert_array_equal(film, ref)
    img = plug.render(mi_scene, None, 5, 16)
    assert img.shape == (64, 64, 3) and np.all(np.isfinite(img))


def test_obj_shape_and_fov_axes(tmp_path):
    """An `obj` shape with a `filename` (the scenes' meshes, scene.xml:221-738)
    loads through the dictionary path; fov_axis x / y / smaller / larger follow
    Mitsuba's perspective sensor on a non-square film."""
    from mtx import MtxError
    from mtx.mitsuba_dict import scene_from_dict

    (tmp_path / "quad.obj").write_text("v -1 -1 0\nv 1 -1 0\nv 1 1 0\nv -1 1 0\nf 1 2 3 4\n")
    d = cornell_box(64, 32)
    d["mesh"] = {"type": "obj", "filename": "quad.obj", "to_world": T().translate([0.0, 0.0, -0.5]).scale(0.2),
                 "bsdf": {"type": "ref", "id": "red"}}
    sc = scene_from_dict(d, base_dir=str(tmp_path))
    assert sc.n_tris == 36 + 2  # the quad, fan-triangulated
    t = np.tan(np.radians(39.3077) / 2)
    for axis, (tx, ty) in {"x": (t, t * 32 / 64), "y": (t * 64 / 32, t), "smaller": (t * 64 / 32, t),
                           "larger": (t, t * 32 / 64)}.items():
        d2 = cornell_box(64, 32)
        d2["sensor"]["fov_axis"] = axis
        cam = scene_from_dict(d2).camera
        assert abs(cam.tan_x - tx) < 1e-5 and abs(cam.tan_y - ty) < 1e-5, axis
    d3 = cornell_box()
    d3["sensor"]["fov_axis"] = "diagonal"
    with pytest.raises((MtxError, ValueError)):
        scene_from_dict(d3)


@pytest.mark.parametrize("entry,match", [({"type": "envmap", "filename": "sky.exr"}, "environment emitter 'envmap'"),
                                         ({"type": "point", "position": [0, 0.5, 0]}, "'point' emitters"),
                                         ({"type": "directional", "direction": [0, -1, 0]}, "'directional' emitters")])
def test_environment_and_delta_emitters_rejected(entry, match):
    """An environment emitter is what a reference integrator reads where a
    ray escapes (path-mis.py:41 valid_ray, :84 / path.py:239 si.emitter on a
    miss); mtx evaluates a constant one (tests/test_environment.py), an envmap
    is refused with that reason instead of rendering it black, and so are
    delta lights."""
    from mtx import MtxError
    from mtx.mitsuba_dict import spec_from_dict

    d = cornell_box()
    d["sky"] = entry
    with pytest.raises(MtxError, match=match):
        spec_from_dict(d)


def test_obj_shape_needs_its_file(tmp_path):
    """An obj shape whose file is missing (or that names none) raises instead
    of falling back to the procedural proxy mesh (which would render another
    scene)."""
    from mtx import MtxError
    from mtx.mitsuba_dict import scene_from_dict

    d = cornell_box(16, 16)
    d["mesh"] = {"type": "obj", "filename": "missing.obj", "bsdf": {"type": "ref", "id": "red"}}
    with pytest.raises(MtxError, match="missing.obj"):
        scene_from_dict(d, base_dir=str(tmp_path))
    d["mesh"] = {"type": "obj", "bsdf": {"type": "ref", "id": "red"}}
    with pytest.raises(MtxError, match="needs a filename"):
        scene_from_dict(d, base_dir=str(tmp_path))
    d["mesh"] = {"type": "diffuse"}
    d["white"] = {"type": "diffuse", "reflectance": {"type": "bitmap", "filename": "nope.png"}}
    del d["mesh"]
    with pytest.raises(MtxError, match="nope.png"):
        scene_from_dict(d, base_dir=str(tmp_path))


def test_loaded_scene_is_recorded_at_load_time():
    """The wrapped mi.load_dict converts the dictionary when it is loaded:
    later edits of the dictionary do not change the rendered scene; a scene
    outside the subset still loads (in Mitsuba) and raises when an mtx
    integrator is asked to render it; entries go with their mi.Scene."""
    import gc

    from mtx import MtxError, integrators

    mi = _fake_mi()
    integrators.register_with_mitsuba(mi)
    d = cornell_box(16, 16)
    obj = mi.load_dict(d)
    d["red"]["reflectance"]["value"] = [0.0, 0.0, 1.0]
    d["small-box"]["type"] = "sphere"
    sc = integrators.mtx_scene_of(obj)
    cols = sorted(tuple(round(x, 4) for x in m.rgb) for m in sc.materials)
    assert (0.5701, 0.043, 0.0444) in cols and sc.n_tris == 36
    bad = cornell_box(16, 16)
    bad["sky"] = {"type": "envmap", "filename": "sky.exr"}
    bad_obj = mi.load_dict(bad)
    try:
        integrators.mtx_scene_of(bad_obj)
        raise AssertionError("expected MtxError")
    except MtxError as e:
        assert "environment emitter" in str(e)
    n = len(integrators._MI_OBJECTS)
    del obj, bad_obj
    gc.collect()
    assert len(integrators._MI_OBJECTS) == n - 2


def test_with_film_keeps_the_fov_axis():
    """Scene.with_film keeps the fov along the sensor's fov_axis (Mitsuba's
    perspective sensor), as a scene loaded at the new film size has it."""
    from mtx.mitsuba_dict import scene_from_dict

    for axis in ("x", "y", "smaller", "larger"):
        d = cornell_box(64, 32)
        d["sensor"]["fov_axis"] = axis
        a = scene_from_dict(d).with_film(24, 40)
        d2 = cornell_box(24, 40)
        d2["sensor"]["fov_axis"] = axis
        b = scene_from_dict(d2).camera
        assert (a.camera.width, a.camera.height) == (24, 40)
        assert abs(a.camera.tan_x - b.tan_x) < 1e-6 and abs(a.camera.tan_y - b.tan_y) < 1e-6, axis
