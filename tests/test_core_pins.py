"""Independent numpy pins of the shared per-lane primitives (include/mtx_core)
that the HIP kernels and the oracle both compile.

Bit-exact HIP-vs-oracle parity pins traversal, queueing, RNG consumption and
film order, but compares these formulas with themselves. Here each one is
restated from its upstream definition (Mitsuba 3
semantics) in float64 numpy and checked against the shared implementation,
with the tolerance written in each test:

* PerspectiveCamera::sample_ray from the XML's to_world matrix and fov
  (scene.xml:10-14), through Mitsuba's camera_to_sample projective matrix;
* the hdrfilm + tent(radius 1) splat and develop (scene.xml:18-24);
* Interaction::spawn_ray / spawn_ray_to offsets (RayEpsilon, ShadowEpsilon);
* the rectangle area emitter: solid-angle pdf integrated over the sphere
  of directions (ray/rectangle intersection in numpy), one-sidedness, and
  E[sample_emitter_direction weight] against the closed-form solid angle of
  the rectangle (Van Oosterom-Strackee), emitter geometry from the XML;
* conductor and dielectric (delta lobes) against the complex / real Fresnel
  equations and Snell's law; roughdielectric sample-vs-eval.
"""
import math

import numpy as np
import pytest

from conftest import ROOT  # noqa: F401


@pytest.fixture(scope="module")
def spec():
    from mtx import scene

    return scene.load_bedroom_spec()


def _m4(v):
    return np.asarray(v, np.float64).reshape(4, 4)


# ------------------------------------------------------------------ camera --
def _perspective(fov_x, near, far):
    recip = 1.0 / (far - near)
    cot = 1.0 / math.tan(math.radians(fov_x) * 0.5)
    return np.array([[cot, 0, 0, 0], [0, cot, 0, 0], [0, 0, far * recip, -near * far * recip], [0, 0, 1, 0]])


def _scale(x, y, z):
    return np.diag([x, y, z, 1.0])


def _translate(x, y, z):
    m = np.eye(4)
    m[:3, 3] = (x, y, z)
    return m


def test_camera_ray_matches_mitsuba_projection(oracle, small_scene, spec):
    """Upstream perspective.cpp: camera_to_sample = S(-0.5, -0.5 aspect, 1)
    T(-1, -1/aspect, 0) perspective(fov_x, near, far); sample_ray un-projects
    (x, y, 0), normalises, moves the origin to the near plane and sets
    maxt = (far - near) / d.z. float64 numpy vs the fp32 shared code: 2e-6."""
    sen = spec["sensor"]
    W, H = small_scene.width, small_scene.height
    aspect = W / H
    near, far = 1e-2, 1e4
    c2s = _scale(-0.5, -0.5 * aspect, 1.0) @ _translate(-1.0, -1.0 / aspect, 0.0) @ _perspective(sen["fov"], near, far)
    s2c = np.linalg.inv(c2s)
    M = _m4(sen["to_world"])
    rng = np.random.default_rng(0)
    pos = np.concatenate([rng.random((2000, 2)), [[0, 0], [1, 1], [0.5, 0.5], [1, 0]]]).astype(np.float32)
    out = oracle.probe(small_scene, "camera_ray", pos)
    hp = np.concatenate([pos.astype(np.float64), np.zeros((len(pos), 1)), np.ones((len(pos), 1))], 1) @ s2c.T
    near_p = hp[:, :3] / hp[:, 3:4]
    dl = near_p / np.linalg.norm(near_p, axis=1, keepdims=True)
    d = dl @ M[:3, :3].T
    inv_z = 1.0 / dl[:, 2]
    o = M[:3, 3] + d * (near * inv_z)[:, None]
    maxt = (far - near) * inv_z
    np.testing.assert_allclose(out[:, 3:6], d, rtol=0, atol=2e-6)
    np.testing.assert_allclose(out[:, 0:3], o, rtol=0, atol=2e-6 * np.abs(o).max())
    np.testing.assert_allclose(out[:, 6], maxt, rtol=2e-6)
    # the image centre looks along the camera's +z axis (scene.xml:13)
    c = out[-2, 3:6]
    np.testing.assert_allclose(c, M[:3, 2] / np.linalg.norm(M[:3, 2]), atol=1e-6)


# -------------------------------------------------------------------- film --
def test_tent_film_matches_numpy_splat(oracle):
    """hdrfilm with a radius-1 tent (scene.xml:23): each sample at continuous
    position (sx, sy) adds w = tent(sx - (x + 0.5)) tent(sy - (y + 0.5)) times
    (rgb, 1) to every pixel of the (W+2) x (rows+2) block with a 1-pixel
    border; develop divides by the weight. float64 numpy: rtol 1e-5."""
    W, y0, y1, spp = 9, 2, 7, 5
    rng = np.random.default_rng(1)
    rows = y1 - y0
    n = rows * W * spp
    px = np.repeat(np.arange(rows * W), spp)
    x = px % W
    y = y0 + px // W
    pos = np.stack([x + rng.random(n), y + rng.random(n)], 1).astype(np.float32)
    L = rng.random((n, 3)).astype(np.float32) * 4
    film = oracle.film(W, y0, y1, spp, L, pos)
    ref = np.zeros((rows + 2, W + 2, 4))
    for k in range(n):
        sx, sy = float(pos[k, 0]), float(pos[k, 1])
        for fy in range(rows + 2):
            wy = max(0.0, 1 - abs(sy - (y0 - 1 + fy + 0.5)))
            for fx in range(W + 2):
                wx = max(0.0, 1 - abs(sx - (fx - 1 + 0.5)))
                w = wx * wy
                if w:
                    ref[fy, fx, :3] += w * L[k]
                    ref[fy, fx, 3] += w
    np.testing.assert_allclose(film, ref, rtol=1e-5, atol=1e-6)
    from mtx import develop

    img = develop(film)
    np.testing.assert_allclose(img, ref[1:-1, 1:-1, :3] / ref[1:-1, 1:-1, 3:], rtol=1e-5)


# ------------------------------------------------------------------- spawn --
RAY_EPS = 1500.0 * 2.0 ** -24  # Appendix A: RayEpsilon = 2^-24 * 1500
SHADOW_EPS = 10.0 * RAY_EPS


def test_spawn_offsets(oracle, small_scene):
    """Interaction::spawn_ray: o = p + n sign(n.d) (1 + max|p|) RayEpsilon,
    maxt = largest float; spawn_ray_to(t): the same offset towards t,
    d = (t - o)/|t - o|, maxt = |t - o| (1 - ShadowEpsilon). Tolerances: fp32
    rounding of the float64 formulas."""
    rng = np.random.default_rng(2)
    n = 3000
    p = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    nn = rng.normal(size=(n, 3))
    nn = (nn / np.linalg.norm(nn, axis=1, keepdims=True)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    out = oracle.probe(small_scene, "spawn_ray", np.concatenate([p, nn, d], 1))
    P, N, D = (a.astype(np.float64) for a in (p, nn, d))
    mag = (1 + np.abs(P).max(1)) * RAY_EPS * np.sign((N * D).sum(1))
    o = P + N * mag[:, None]
    np.testing.assert_allclose(out[:, 0:3], o, rtol=0, atol=4e-7 * (1 + np.abs(P).max()))
    assert np.all(np.linalg.norm((out[:, 0:3] - p).astype(np.float64), axis=1) > 0)  # the offset is applied
    np.testing.assert_array_equal(out[:, 3:6], d)
    assert np.all(out[:, 6] == np.finfo(np.float32).max)
    t = (p + d * rng.uniform(0.01, 5, (n, 1))).astype(np.float32)
    out = oracle.probe(small_scene, "spawn_ray_to", np.concatenate([p, nn, t], 1))
    T = t.astype(np.float64)
    mag = (1 + np.abs(P).max(1)) * RAY_EPS * np.sign((N * (T - P)).sum(1))
    o = P + N * mag[:, None]
    dd = T - o
    dist = np.linalg.norm(dd, axis=1)
    np.testing.assert_allclose(out[:, 0:3], o, rtol=0, atol=4e-7 * (1 + np.abs(P).max()))
    np.testing.assert_allclose(out[:, 3:6], dd / dist[:, None], rtol=0, atol=3e-6 / dist.min())
    # fp32 rounding of o (|o| <= 4) bounds the distance error: 1.5e-6 absolute
    np.testing.assert_allclose(out[:, 6], dist * (1 - SHADOW_EPS), rtol=2e-6, atol=1.5e-6)
    assert np.all(out[:, 6] < dist)  # stops short of the target


# ----------------------------------------------------------------- emitter --
def _rects(spec):
    """(corners[4,3], normal, radiance) of each area-light rectangle straight
    from the XML's to_world (Rectangle: [-1,1]^2 at z=0, normal +z)."""
    out = []
    for s in spec["shapes"]:
        if "emitter" not in s:
            continue
        M = _m4(s["to_world"])
        loc = np.array([[-1, -1, 0, 1], [1, -1, 0, 1], [1, 1, 0, 1], [-1, 1, 0, 1]], np.float64)
        P = (loc @ M.T)[:, :3]
        n = np.linalg.inv(M[:3, :3]).T @ np.array([0, 0, 1.0])
        out.append((P, n / np.linalg.norm(n), np.asarray(s["emitter"]["radiance"], np.float64)))
    return out


def _solid_angle_tri(a, b, c):
    """Van Oosterom-Strackee: solid angle of triangle (a, b, c) seen from 0."""
    la, lb, lc = np.linalg.norm(a), np.linalg.norm(b), np.linalg.norm(c)
    num = abs(np.dot(a, np.cross(b, c)))
    den = la * lb * lc + np.dot(a, b) * lc + np.dot(a, c) * lb + np.dot(b, c) * la
    return 2 * math.atan2(num, den)


def _solid_angle_rect(P, ref):
    q = P - ref
    return _solid_angle_tri(q[0], q[1], q[2]) + _solid_angle_tri(q[0], q[2], q[3])


def _ref_points(rects, n, rng):
    """Points in the room that see the front (emitting) side of every light."""
    pts = []
    while len(pts) < n:
        p = rng.uniform([-2.5, 0.1, -1.0], [2.5, 2.4, 3.0])
        if all(np.dot(p - P.mean(0), nrm) > 0.05 for P, nrm, _ in rects):
            pts.append(p)
    return np.array(pts)


def test_emitter_pdf_integrates_to_pick_probability(oracle, small_scene, spec):
    """∫ pdf_emitter_direction dω over the sphere = 1 (1/2 per light) for a
    point in front of both lights, 0 behind one: directions uniform on the
    sphere, hits and (dist, normal) from a numpy ray/rectangle test. MC with
    4 M directions: tolerance 4 %."""
    rects = _rects(spec)
    rng = np.random.default_rng(4)
    ref = _ref_points(rects, 1, rng)[0]
    n = 1 << 22
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    total = 0.0
    for e, (P, nrm, _) in enumerate(rects):
        c = P.mean(0)
        e1, e2 = (P[1] - P[0]) / 2, (P[3] - P[0]) / 2
        denom = v @ nrm
        t = ((c - ref) @ nrm) / np.where(denom != 0, denom, np.nan)
        hitp = ref + v * t[:, None]
        lx = ((hitp - c) @ e1) / (e1 @ e1)
        ly = ((hitp - c) @ e2) / (e2 @ e2)
        hit = (t > 0) & (np.abs(lx) <= 1) & (np.abs(ly) <= 1)
        k = np.flatnonzero(hit)
        inp = np.zeros((len(k), 8), np.float32)
        inp[:, 0] = e
        inp[:, 1:4] = v[k]
        inp[:, 4] = t[k]
        inp[:, 5:8] = nrm
        pdf = oracle.probe(small_scene, "pdf_emitter", inp)[:, 0].astype(np.float64)
        est = pdf.sum() / n * 4 * math.pi
        assert abs(est - 0.5) < 0.02, (e, est)
        total += est
        # one-sided: the same direction from behind the light has pdf 0
        inp[:, 5:8] = -nrm
        assert not oracle.probe(small_scene, "pdf_emitter", inp)[:, 0].any()
    assert abs(total - 1.0) < 0.04


def test_emitter_sampling_against_closed_form_solid_angle(oracle, small_scene, spec):
    """E_u[sample_emitter_direction weight] = sum_e Le_e Omega_e(ref) (no
    occlusion test): area sampling turned into solid angle must integrate the
    radiance over each light's closed-form solid angle. The sample lies on
    the rectangle, d = (p - ref)/|p - ref|, and the returned pdf equals
    pdf_emitter_direction at that direction. MC 2^18 samples: 1.5 %."""
    rects = _rects(spec)
    rng = np.random.default_rng(5)
    for ref in _ref_points(rects, 3, rng):
        n = 1 << 18
        u = rng.random((n, 2)).astype(np.float32)
        inp = np.concatenate([np.tile(ref.astype(np.float32), (n, 1)), u], 1)
        out = oracle.probe(small_scene, "sample_emitter", inp).astype(np.float64)
        w, p, nn, d, dist, pdf, em = out[:, 0:3], out[:, 3:6], out[:, 6:9], out[:, 9:12], out[:, 12], out[:, 13], out[:, 14]
        expect = sum(Le * _solid_angle_rect(P, ref) for P, _, Le in rects)
        np.testing.assert_allclose(w.mean(0), expect, rtol=0.015)
        for e, (P, nrm, Le) in enumerate(rects):
            m = em == e
            assert 0.45 < m.mean() < 0.55
            c = P.mean(0)
            e1, e2 = (P[1] - P[0]) / 2, (P[3] - P[0]) / 2
            q = p[m] - c
            assert np.all(np.abs(q @ nrm) < 1e-5)
            assert np.all(np.abs(q @ e1 / (e1 @ e1)) <= 1 + 1e-5) and np.all(np.abs(q @ e2 / (e2 @ e2)) <= 1 + 1e-5)
            np.testing.assert_allclose(nn[m], np.tile(nrm, (m.sum(), 1)), atol=1e-6)
        rel = p - ref
        np.testing.assert_allclose(dist, np.linalg.norm(rel, axis=1), rtol=2e-6)
        np.testing.assert_allclose(d, rel / dist[:, None], atol=2e-6)
        inp2 = np.zeros((n, 8), np.float32)
        inp2[:, 0], inp2[:, 1:4], inp2[:, 4], inp2[:, 5:8] = em, d, dist, nn
        pdf2 = oracle.probe(small_scene, "pdf_emitter", inp2)[:, 0]
        np.testing.assert_allclose(pdf2, pdf, rtol=1e-6)
        # weight = Le / pdf for a front-facing sample
        np.testing.assert_allclose(w[:, 0], 16.4648 / pdf, rtol=2e-6)


def test_emitter_eval_one_sided(oracle, small_scene):
    inp = np.zeros((4, 11), np.float32)
    inp[:, 0] = [0, 1, 0, -1]
    inp[:, 8:11] = [[0.3, 0.1, 0.9], [0, 0, 1], [0.2, 0.2, -0.9], [0, 0, 1]]
    out = oracle.probe(small_scene, "pdf_emitter", inp)
    assert np.all(out[:2, 1:4] == np.float32(16.4648))
    assert not out[2:, 1:4].any()  # back side / no emitter


# ------------------------------------------------------------------- BSDFs --
def _fresnel_dielectric(cos_i, eta):
    """Exact unpolarised Fresnel reflectance (real IOR), float64."""
    cos_i = np.asarray(cos_i, np.float64)
    e = np.where(cos_i >= 0, eta, 1 / eta)
    ci = np.abs(cos_i)
    sin2_t = (1 - ci ** 2) / e ** 2
    tir = sin2_t >= 1
    ct = np.sqrt(np.maximum(0, 1 - sin2_t))
    rs = (ci - e * ct) / (ci + e * ct)
    rp = (e * ci - ct) / (e * ci + ct)
    return np.where(tir, 1.0, 0.5 * (rs ** 2 + rp ** 2)), ct, e


def _fresnel_conductor(cos_i, eta, k):
    """Unpolarised conductor Fresnel from the complex IOR n = eta + i k."""
    n = complex(eta, k)
    c = np.asarray(cos_i, np.complex128)
    s2 = 1 - c ** 2
    root = np.sqrt(n ** 2 - s2)
    rs = (c - root) / (c + root)
    rp = (n ** 2 * c - root) / (n ** 2 * c + root)
    return (0.5 * (np.abs(rs) ** 2 + np.abs(rp) ** 2)).real


def _mats(scene, mtype):
    return [i for i, m in enumerate(scene.materials) if m.type == mtype]


def _wi(rng, n, side=1.0):
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v[:, 2] = side * (np.abs(v[:, 2]) + 0.02)
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def test_conductor_delta_against_complex_fresnel(oracle, small_scene):
    """conductor (scene.xml: material=none, i.e. a perfect mirror, and any
    other eta/k): wo = mirror(wi), pdf 1, weight = specular_reflectance x
    F_conductor(cos_i; eta + i k) (numpy complex arithmetic): rtol 1e-5;
    eval and pdf of a delta lobe are 0. Twosided: the back side mirrors too."""
    from mtx import _abi

    rng = np.random.default_rng(6)
    ids = _mats(small_scene, _abi.MTX_MAT_CONDUCTOR)
    assert ids
    for mid in ids:
        m = small_scene.materials[mid]
        for side in (1.0, -1.0):
            wi = _wi(rng, 2000, side)
            u = rng.random((2000, 3), dtype=np.float32)
            out, _ = oracle.bsdf_probe(small_scene, mid, wi, wi, np.full((2000, 2), 0.3, np.float32), u)
            if side < 0 and not (m.flags & _abi.MTX_MF_TWOSIDED):
                assert not out[:, 10:13].any()
                continue
            np.testing.assert_allclose(out[:, 4:7], wi * np.array([-1, -1, 1], np.float32), atol=1e-7)
            assert np.all(out[:, 7] == 1) and np.all(out[:, 0:4] == 0)
            ci = np.abs(wi[:, 2])
            for c in range(3):
                F = _fresnel_conductor(ci, m.eta_rgb[c], m.k_rgb[c]) * m.rgb[c]
                np.testing.assert_allclose(out[:, 10 + c], F, rtol=1e-5, atol=1e-7)


def test_dielectric_delta_against_fresnel_and_snell(oracle, small_scene):
    """dielectric (scene.xml, int_ior/ext_ior): reflection chosen with
    probability F(cos_i) (the sample1 threshold), wo = mirror(wi) or Snell's
    refraction, pdf = F or 1 - F, weight 1 for reflection and 1/eta_rel^2
    (radiance transport) for refraction, bs.eta = eta_rel. Exact Fresnel in
    float64 numpy: rtol 2e-5. Both sides (entering / leaving, incl. TIR)."""
    from mtx import _abi

    rng = np.random.default_rng(7)
    ids = _mats(small_scene, _abi.MTX_MAT_DIELECTRIC)
    assert ids
    n = 4000
    for mid in ids:
        eta = small_scene.materials[mid].eta
        for side in (1.0, -1.0):
            wi = _wi(rng, n, side)
            u = rng.random((n, 3), dtype=np.float32)
            out, _ = oracle.bsdf_probe(small_scene, mid, wi, wi, np.full((n, 2), 0.3, np.float32), u)
            F, ct, e = _fresnel_dielectric(wi[:, 2], eta)
            refl = u[:, 0] <= F
            # skip samples within rounding of the threshold, and the last
            # 1e-3 of sin^2 before total internal reflection (fp32 cos_t
            # there is ill-conditioned)
            sin2_t = (1 - wi[:, 2].astype(np.float64) ** 2) / e ** 2
            ok = (np.abs(u[:, 0] - F) > 1e-5) & (np.abs(sin2_t - 1) > 1e-3)
            typ = out[:, 9].view(np.uint32)
            assert np.all((typ[ok] == 0x20) == refl[ok])
            np.testing.assert_allclose(out[ok, 7], np.where(refl, F, 1 - F)[ok], rtol=2e-5, atol=1e-7)
            r = refl & ok
            np.testing.assert_allclose(out[r, 4:7], wi[r] * np.array([-1, -1, 1]), atol=1e-6)
            assert np.all(out[r, 10:13] == 1) and np.all(out[r, 8] == 1)
            t = ~refl & ok
            # Snell: wo = -wi_t / e + (0,0,-sign(cos_i) cos_t)
            wo = np.stack([-wi[t, 0] / e[t], -wi[t, 1] / e[t], -np.sign(wi[t, 2]) * ct[t]], 1)
            np.testing.assert_allclose(out[t, 4:7], wo, atol=2e-6)
            np.testing.assert_allclose(out[t, 10], 1 / e[t] ** 2, rtol=2e-5)
            np.testing.assert_allclose(out[t, 8], e[t], rtol=1e-6)
            assert np.all(out[:, 0:4] == 0)  # delta lobes: eval = pdf = 0


def test_roughdielectric_sample_matches_eval(oracle, small_scene):
    """roughdielectric (visible-normal sampling): the sample weight equals
    eval(wo)/pdf(wo) at the sampled wo and the sample pdf equals the
    evaluated pdf, for reflection and refraction, from both sides: rtol 1e-4."""
    from mtx import _abi

    rng = np.random.default_rng(8)
    for mid in _mats(small_scene, _abi.MTX_MAT_ROUGHDIELECTRIC):
        for side in (1.0, -1.0):
            wi = _wi(rng, 4000, side)
            u = rng.random((4000, 3), dtype=np.float32)
            out, pdf2 = oracle.bsdf_probe(small_scene, mid, wi, wi, np.full((4000, 2), 0.3, np.float32), u)
            w, val2, spdf = out[:, 10:13], out[:, 13:16], out[:, 7]
            ok = (spdf > 1e-3) & (w.max(1) > 0)
            typ = out[ok, 9].view(np.uint32)
            assert set(np.unique(typ)) <= {0x08, 0x10} and len(np.unique(typ)) == 2
            np.testing.assert_allclose(w[ok], val2[ok] / pdf2[ok, None], rtol=1e-4)
            np.testing.assert_allclose(spdf[ok], pdf2[ok], rtol=1e-4)


# ----------------------------------------------------------- white furnace --
@pytest.mark.parametrize("name", ["path_test", "mypath", "integrator"])
def test_white_furnace_oracle(oracle, name):
    """The CPU restatement in a closed box of emitting diffuse walls
    (tests/test_gpu_convergence.py furnace_spec): pixel value
    Le (1 - rho^M) / (1 - rho); image mean at spp 256 within 0.4 %, 2x2 of
    the 32x32 image's 16x16 blocks within 5 standard errors of the pixel
    spread."""
    from mtx import develop, load_dict
    from mtx.scene import Scene
    from test_gpu_convergence import furnace_spec

    rho, Le, M = 0.5, 1.5, 6
    sc = Scene.bedroom(spec=furnace_spec(rho, Le))
    integ = load_dict({"type": name, "max_depth": M, "rr_depth": 2})
    img = develop(oracle.render(sc, integ.render_args(sc, 3, 256))).astype(np.float64)
    expect = Le * (1 - rho ** M) / (1 - rho)
    assert abs(img.mean() / expect - 1) < 4e-3, (name, img.mean(), expect)
    blocks = img.reshape(2, 16, 2, 16, 3)
    se = img.std() / 16
    assert np.abs(blocks.mean(axis=(1, 3)) - expect).max() < 5 * se
