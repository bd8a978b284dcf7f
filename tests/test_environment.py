"""A constant environment emitter: Mitsuba's ``constant`` plugin, the
``scene.environment()`` the reference integrators read where a ray escapes
(path-mis.py:41 valid_ray, path-mis.py:84 / path.py:239 ``si.emitter(scene)``
on a miss) and that NEE picks uniformly among the scene's emitters.

Mitsuba is not importable here, so the emitter is pinned three ways: against
a float64 transcription of ConstantBackgroundEmitter (sample_direction /
pdf_direction / eval, and Scene's uniform emitter pick) through the oracle
probe; by a white furnace (a white diffuse cube under a unit sky renders 1 in
expectation; a pixel that sees only sky is exactly 1); and, on the GPU, the
kernels bit-exactly against the oracle (parity unpinned against Mitsuba)."""
import numpy as np
import pytest
from test_mitsuba_dict import T, cornell_box

RAY_EPS = 1500.0 * 2.0**-24  # math::RayEpsilon<float>


def furnace(width=24, height=24, albedo=1.0, sky=1.0):
    return {
        "type": "scene",
        "sensor": {"type": "perspective", "fov": 40.0, "to_world": T.look_at([0, 0, 4], [0, 0, 0], [0, 1, 0]),
                   "film": {"type": "hdrfilm", "width": width, "height": height}},
        "cube": {"type": "cube", "to_world": T().rotate([0, 1, 0], 30).rotate([1, 0, 0], 20).scale(0.6),
                 "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": albedo}}},
        "sky": {"type": "constant", "radiance": {"type": "rgb", "value": sky}},
    }


def with_sky(d, radiance):
    d = dict(d)
    d["sky"] = {"type": "constant", "radiance": {"type": "rgb", "value": radiance}}
    return d


def test_constant_environment_converts(tmp_path):
    from mtx import MtxError
    from mtx.mitsuba_dict import scene_from_dict, spec_from_dict
    from mtx.scene import Scene
    from mtx.xmlscene import parse_scene_xml

    sc = scene_from_dict(with_sky(cornell_box(16, 16), [0.2, 0.3, 0.4]))
    assert sc.env_radiance == pytest.approx((0.2, 0.3, 0.4))
    d = sc.desc()
    assert d.has_env == 1 and list(d.env_radiance) == pytest.approx([0.2, 0.3, 0.4])
    assert scene_from_dict(furnace(sky=0.7)).env_radiance == pytest.approx((0.7, 0.7, 0.7))  # a float radiance
    assert scene_from_dict(cornell_box(16, 16)).desc().has_env == 0
    sc.save(str(tmp_path / "s.npz"))
    assert Scene.load(str(tmp_path / "s.npz")).env_radiance == pytest.approx((0.2, 0.3, 0.4))
    two = with_sky(cornell_box(), 1.0)
    two["sky2"] = {"type": "constant"}
    with pytest.raises(MtxError, match="more than one environment"):
        spec_from_dict(two)
    # an environment alone lights the scene
    assert "environment" in spec_from_dict(furnace())
    # XML: a top-level constant emitter; anything else at the top level raises
    xml = """<scene version="3.0.0">
  <sensor type="perspective"><float name="fov" value="40"/>
    <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
  <emitter type="constant"><rgb name="radiance" value="0.25, 0.5, 1"/></emitter>
</scene>"""
    (tmp_path / "a.xml").write_text(xml)
    assert parse_scene_xml(str(tmp_path / "a.xml"))["environment"]["radiance"] == pytest.approx([0.25, 0.5, 1.0])
    (tmp_path / "b.xml").write_text(xml.replace('"constant"', '"envmap"'))
    with pytest.raises(MtxError, match="constant environment"):
        parse_scene_xml(str(tmp_path / "b.xml"))


def _bsphere(sc):
    v = np.asarray(sc.vpos, np.float64).reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    c = (lo + hi) * 0.5
    return c, max(RAY_EPS, np.linalg.norm(c - lo) * (1 + RAY_EPS))


def _sphere(u):  # warp::square_to_uniform_sphere
    z = 1.0 - 2.0 * u[1]
    r = np.sqrt(max(0.0, 1.0 - z * z))
    return np.array([r * np.cos(2 * np.pi * u[0]), r * np.sin(2 * np.pi * u[0]), z])


@pytest.mark.parametrize("with_area", [False, True])
def test_environment_sampling_pins(oracle, with_area):
    """ConstantBackgroundEmitter::sample_direction (uniform sphere direction,
    target point 2 max(r, |ref - c|) away, weight radiance / pdf), its
    pdf_direction (1 / 4 pi) and eval, behind Scene::sample_emitter_direction's
    uniform pick (index floor(u.x N), u.x rescaled, pdf / N, weight x N) --
    float64 transcription against the oracle's float32 (tolerances below)."""
    from mtx.mitsuba_dict import scene_from_dict

    rad = np.array([0.3, 0.6, 0.9])
    sc = scene_from_dict(with_sky(cornell_box(8, 8), list(rad)) if with_area else furnace(sky=list(rad)))
    N = len(sc.emitters) + 1
    env = N - 1
    c, R = _bsphere(sc)
    refs = [[0.1, 0.2, 0.3], [0.0, -0.9, 0.5], [3.0, 2.0, -5.0]]  # the last outside the sphere
    us = [[0.999, 0.25], [0.75, 0.9], [0.52, 0.013], [0.9, 0.5]]
    items = [ref + u for ref in refs for u in us]
    out = oracle.probe(sc, "sample_emitter", items)
    n_env = 0
    for it, o in zip(items, out):
        ref, u = np.array(it[:3]), np.array(it[3:5])
        idx = min(int(np.float32(u[0]) * np.float32(N)), N - 1)
        if idx != env:
            continue
        n_env += 1
        u0 = float(np.float32(np.float32(u[0]) * np.float32(N)) - np.float32(idx))
        d = _sphere([u0, u[1]])
        dist = 2.0 * max(R, np.linalg.norm(ref - c))
        assert int(o[14]) == env
        np.testing.assert_allclose(o[9:12], d, atol=2e-6)  # direction
        np.testing.assert_allclose(o[6:9], -d, atol=2e-6)  # normal
        assert o[12] == pytest.approx(dist, rel=1e-6)  # distance
        np.testing.assert_allclose(o[3:6], ref + d * dist, rtol=1e-5, atol=2e-5)  # target point
        assert o[13] == pytest.approx(1.0 / (4.0 * np.pi) / N, rel=1e-6)  # pdf incl. the pick
        np.testing.assert_allclose(o[0:3], rad * 4.0 * np.pi * N, rtol=1e-6)  # radiance / pdf
    assert n_env >= 3
    pe = oracle.probe(sc, "pdf_emitter", [[env, 0.0, 0.0, 1.0, 5.0, 0.0, 0.0, -1.0, 0.3, -0.2, -0.9],
                                           [env, 0.6, 0.8, 0.0, 1e30, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0]])
    for o in pe:
        assert o[0] == pytest.approx(1.0 / (4.0 * np.pi) / N, rel=1e-6)  # any direction, any distance
        np.testing.assert_array_equal(o[1:4], rad.astype(np.float32))  # eval: the radiance, any side


def test_white_furnace_oracle(oracle):
    """A white (albedo 1) diffuse convex cube under a unit sky: every pixel is
    1 in expectation (path-mis NEE + MIS, and mypath); a pixel whose samples
    all miss the cube is exactly 1 (valid_ray is set by the environment)."""
    from mtx import load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(furnace(24, 24))
    for name in ("path_test", "mypath"):
        integ = load_dict({"type": name, "max_depth": 64, "rr_depth": 5})
        film = oracle.render(sc, integ.render_args(sc, 3, 32))
        inner = film[1:-1, 1:-1]
        img = inner[..., :3] / inner[..., 3:4]
        assert np.all(np.isfinite(img))
        np.testing.assert_array_equal(img[0, 0], np.ones(3, np.float32))  # a corner sees only sky
        assert abs(img.mean() - 1.0) < 0.02, (name, img.mean())
        assert np.abs(img - 1.0).max() < 0.35, (name, np.abs(img - 1.0).max())
    # half-albedo cube: darker than the sky, brighter than black
    sc2 = scene_from_dict(furnace(24, 24, albedo=0.5))
    integ = load_dict({"type": "path_test", "max_depth": 64, "rr_depth": 5})
    img2 = oracle.render(sc2, integ.render_args(sc2, 3, 32))[1:-1, 1:-1]
    img2 = img2[..., :3] / img2[..., 3:4]
    assert img2[12, 12].mean() < 0.75 and img2[0, 0].mean() == 1.0


@pytest.mark.gpu
def test_restir_with_environment_is_refused():
    """restirgi.py's reservoirs hold the secondary path's first hit; an escape
    to the environment has none, and is not restated: refused with the reason."""
    from mtx import MtxError, load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(furnace(8, 8))
    integ = load_dict({"type": "restirgi"})
    with pytest.raises(MtxError, match="environment"):
        integ.render_film(sc, seed=0, spp=1)


@pytest.mark.gpu
@pytest.mark.parametrize("scene_kind", ["furnace", "cornell_sky"])
@pytest.mark.parametrize("name", ["path_test", "mypath", "integrator", "nrc"])
def test_environment_gpu_bit_exact(oracle, scene_kind, name):
    """The kernels' environment (miss emission with MIS, NEE pick, far-point
    shadow rays, valid_ray) against the oracle, bit for bit."""
    from mtx import load_dict
    from mtx.mitsuba_dict import scene_from_dict

    d = furnace(32, 32, albedo=0.8) if scene_kind == "furnace" else with_sky(cornell_box(32, 32), [0.4, 0.5, 0.6])
    sc = scene_from_dict(d)
    integ = load_dict({"type": name, "max_depth": 8} if name != "nrc" else {"type": name})
    film = integ.render_film(sc, seed=11, spp=8)
    ref = oracle.render(sc, integ.render_args(sc, 11, 8))
    np.testing.assert_array_equal(film, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pssmlt_simple", "pssmlt"])
def test_environment_pssmlt_gpu_bit_exact(oracle, name):
    """PSSMLT chains under a sky (pssmltpath.py:39 valid_ray from the
    environment; escaped proposals see its radiance): 60 Metropolis
    iterations, film bit-identical to the oracle."""
    from mtx import load_dict
    from mtx.mitsuba_dict import scene_from_dict

    sc = scene_from_dict(with_sky(cornell_box(24, 24), [0.4, 0.5, 0.6]))
    integ = load_dict({"type": name, "iterations": 60})
    film = integ.render_film(sc, seed=4, spp=2)
    ref = oracle.pssmlt_render(sc, integ.render_args(sc, 4, 2), 60)
    np.testing.assert_array_equal(film, ref)
    assert film[..., 3].sum() > 0
