"""Independent pins of roughconductor and roughdielectric (include/mtx_core/
bsdf.h base_eval_pdf / base_sample, microfacet.h): float64 numpy restatements
of the microfacet models (Walter et al. 2007, "Microfacet Models for
Refraction through Rough Surfaces"; Heitz 2018 visible-normal pdf) that share
no code with the C++ ones, evaluated at random (wi, wo) pairs through the
oracle's bsdf_probe. Reference call sites: bsdf.eval_pdf_sample at
path-mis.py:107-109, bsdf.sample at pssmltsimple.py:84.

Bit-exact HIP-vs-oracle parity cannot see a formula error in the shared
headers; these tests can:
* roughconductor: D (GGX / Beckmann), Smith G1 per direction, the complex-IOR
  conductor Fresnel (numpy complex arithmetic) times specular_reflectance, and
  the visible-normal pdf D G1(wi) / (4 cos_i);
* roughdielectric: the reflection lobe F D G / (4 |cos_i|) and the
  transmission lobe |wi.h| |wo.h| (1 - F) D G / (|cos_i| (wi.h + eta wo.h)^2)
  with the radiance scale 1/eta^2 (eta^2 of the Jacobian cancelled), the
  half-vector Jacobians of both lobes, from both sides;
* the alpha -> 0 limits: the sampled lobes become the smooth conductor and
  dielectric (already pinned in tests/test_core_pins.py): mirror / Snell
  directions, weights F_conductor x R and 1 / eta^2, reflection chosen with
  probability F.
Tolerances are stated in each assert.
"""
import copy

import numpy as np
import pytest

from test_core_pins import _fresnel_conductor, _fresnel_dielectric
from test_roughplastic_pin import D as D_np
from test_roughplastic_pin import G1 as G1_np


def _materials(scene, mtype):
    return [i for i, m in enumerate(scene.materials) if m.type == mtype]


def _with_alpha(scene, mid, alpha):
    from mtx import _abi

    s = copy.copy(scene)
    mats = [_abi.Material.from_buffer_copy(bytes(m)) for m in scene.materials]
    mats[mid].alpha = alpha
    s.materials = (_abi.Material * len(mats))(*mats)
    return s


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _hemi(rng, n, side=1.0, zmin=0.05):
    v = rng.normal(size=(n, 3))
    v[:, 2] = side * (np.abs(v[:, 2]) + zmin)
    return _unit(v)


def _near(rng, base, n, spread, side):
    v = base + spread * rng.normal(size=(n, 3))
    v[:, 2] = side * (np.abs(v[:, 2]) + 0.05)
    return _unit(v)


def _probe(oracle, sc, mid, wi, wo, u=None):
    n = len(wi)
    if u is None:
        u = np.full((n, 3), 0.5, np.float32)
    out, pdf2 = oracle.bsdf_probe(sc, mid, wi.astype(np.float32), wo.astype(np.float32),
                                  np.full((n, 2), 0.3, np.float32), u.astype(np.float32))
    return out, pdf2


def _refract_dir(wi, eta):
    """Snell refraction of wi about +z (relative eta = eta_t / eta_i on wi's side)."""
    ci = wi[:, 2]
    e = np.where(ci >= 0, eta, 1.0 / eta)
    s2 = (1.0 - ci * ci) / e ** 2
    ct = np.sqrt(np.maximum(0.0, 1.0 - s2))
    return np.stack([-wi[:, 0] / e, -wi[:, 1] / e, -np.sign(ci) * ct], 1)


# ------------------------------------------------------------ roughconductor --
def test_roughconductor_eval_pdf_against_numpy(oracle, small_scene):
    """eval = R F(wi.h; eta + i k) D(h) G1(wi) G1(wo) / (4 cos_i) and
    pdf = D(h) G1(wi) / (4 cos_i) (visible normals: D G1 |wi.h| / cos_i times
    the reflection Jacobian 1 / (4 |wo.h|), wi.h = wo.h), every roughconductor
    of the bedroom (GGX alpha 0.2 / 0.1, Beckmann 0.1): rtol 1e-4 (float32 vs
    float64), atol 1e-6 of the lobe's peak."""
    from mtx import _abi

    rng = np.random.default_rng(21)
    ids = _materials(small_scene, _abi.MTX_MAT_ROUGHCONDUCTOR)
    assert len(ids) >= 3
    kinds = set()
    n = 12000
    for mid in ids:
        m = small_scene.materials[mid]
        beck = bool(m.flags & _abi.MTX_MF_BECKMANN)
        kinds.add(beck)
        alpha = float(m.alpha)
        wi = _hemi(rng, n)
        wo = np.concatenate([_near(rng, wi[: n // 2] * [-1, -1, 1], n // 2, 2.5 * alpha, 1.0), _hemi(rng, n - n // 2)])
        wi = wi.astype(np.float32).astype(np.float64)
        wo = wo.astype(np.float32).astype(np.float64)
        out, _ = _probe(oracle, small_scene, mid, wi, wo)
        h = _unit(wi + wo)
        ci = wi[:, 2]
        dh = np.sum(wi * h, 1)
        Dh = D_np(h[:, 2], alpha, beck)
        G = G1_np(wi, h, alpha, beck) * G1_np(wo, h, alpha, beck)
        for c in range(3):
            F = _fresnel_conductor(dh, m.eta_rgb[c], m.k_rgb[c]) * m.rgb[c]
            ref = F * Dh * G / (4 * ci)
            np.testing.assert_allclose(out[:, c], ref, rtol=1e-4, atol=1e-6 * ref.max())
        ref_pdf = Dh * G1_np(wi, h, alpha, beck) / (4 * ci)
        np.testing.assert_allclose(out[:, 3], ref_pdf, rtol=1e-4, atol=1e-6 * ref_pdf.max())
        assert (ref_pdf > 1.0).mean() > 0.1  # the lobe's peak region was exercised
        # below the surface: no reflection (twosided materials mirror the side)
        if not (m.flags & _abi.MTX_MF_TWOSIDED):
            out_b, _ = _probe(oracle, small_scene, mid, wi, wo * [1, 1, -1])
            assert not out_b[:, 0:4].any()
    assert kinds == {False, True}, "the bedroom has GGX and Beckmann roughconductors"


def test_roughconductor_alpha_to_zero_is_the_smooth_conductor(oracle, small_scene):
    """alpha = 1e-4: the sampled direction is the mirror direction (atol 2e-3
    for >= 99 % of the samples: GGX's slope distribution has Cauchy-like tails,
    P(|slope| > s) ~ alpha / s), the weight F_conductor(cos_i) x R (rtol 1e-3)
    for those, as the delta conductor pinned in test_core_pins."""
    from mtx import _abi

    rng = np.random.default_rng(22)
    mid = _materials(small_scene, _abi.MTX_MAT_ROUGHCONDUCTOR)[0]
    sc = _with_alpha(small_scene, mid, 1e-4)
    m = sc.materials[mid]
    n = 4000
    wi = _hemi(rng, n, zmin=0.1)
    out, _ = _probe(oracle, sc, mid, wi, wi, rng.random((n, 3)))
    close = np.abs(out[:, 4:7] - wi * [-1, -1, 1]).max(1) < 2e-3
    assert close.mean() > 0.99, close.mean()
    assert np.all(out[:, 9].view(np.uint32) == 0x08)  # glossy reflection
    for c in range(3):
        F = _fresnel_conductor(wi[:, 2], m.eta_rgb[c], m.k_rgb[c]) * m.rgb[c]
        np.testing.assert_allclose(out[close, 10 + c], F[close], rtol=1e-3)


# ----------------------------------------------------------- roughdielectric --
def _dielectric_ref(wi, wo, eta_ext, alpha, beck):
    """Walter et al. 2007 eval / pdf (value includes cos_o, radiance scale)."""
    ci, co = wi[:, 2], wo[:, 2]
    refl = ci * co > 0
    eta = np.where(ci > 0, eta_ext, 1.0 / eta_ext)  # eta_t / eta_i for wi's side
    h = np.where(refl[:, None], wi + wo, wi + eta[:, None] * wo)
    h = _unit(h)
    h = h * np.sign(h[:, 2:3])
    dih, doh = np.sum(wi * h, 1), np.sum(wo * h, 1)
    F, _, _ = _fresnel_dielectric(dih, eta_ext)
    Dh = D_np(h[:, 2], alpha, beck)
    G = G1_np(wi, h, alpha, beck) * G1_np(wo, h, alpha, beck)
    f_r = F * Dh * G / (4 * np.abs(ci))
    den = (dih + eta * doh) ** 2
    f_t = np.abs(dih * doh) * (1 - F) * Dh * G / (np.abs(ci) * den)  # eta^2 (Jacobian) x 1/eta^2 (radiance)
    val = np.where(refl, f_r, f_t)
    ok_side = (dih * ci > 0) & (doh * co > 0)
    wi_up = wi * np.sign(ci)[:, None]
    vis = Dh * G1_np(wi_up, h, alpha, beck) * np.abs(dih) / np.abs(ci)
    jac = np.where(refl, 1 / (4 * np.abs(doh)), eta ** 2 * np.abs(doh) / den)
    pdf = np.where(ok_side, vis * np.where(refl, F, 1 - F) * jac, 0.0)
    return val, pdf, refl, den


@pytest.mark.parametrize("side", [1.0, -1.0])
def test_roughdielectric_eval_pdf_against_numpy(oracle, small_scene, side):
    """Both lobes from both sides of the bedroom's roughdielectric (Beckmann,
    alpha 0.1, eta 1.5): rtol 2e-4 (float32 vs float64; the transmission
    lobe's denominator (wi.h + eta wo.h)^2 loses a few more bits), atol 1e-6 of
    the peak. Pairs with a near-singular refraction denominator are skipped."""
    from mtx import _abi

    rng = np.random.default_rng(23 if side > 0 else 24)
    ids = _materials(small_scene, _abi.MTX_MAT_ROUGHDIELECTRIC)
    assert ids
    n = 16000
    for mid in ids:
        m = small_scene.materials[mid]
        beck = bool(m.flags & _abi.MTX_MF_BECKMANN)
        alpha, eta = float(m.alpha), float(m.eta)
        wi = _hemi(rng, n, side, zmin=0.08)
        q = n // 3
        wo = np.concatenate([
            _near(rng, wi[:q] * [-1, -1, 1], q, 2.5 * alpha, side),        # reflection lobe
            _near(rng, _refract_dir(wi[q:2 * q], eta), q, 2.5 * alpha, -side),  # transmission lobe
            _hemi(rng, n - 2 * q, -side)])                                  # anywhere below
        wi = wi.astype(np.float32).astype(np.float64)
        wo = wo.astype(np.float32).astype(np.float64)
        out, _ = _probe(oracle, small_scene, mid, wi, wo)
        val, pdf, refl, den = _dielectric_ref(wi, wo, eta, alpha, beck)
        ok = den > 1e-2
        assert ok.mean() > 0.9
        for c in range(3):
            np.testing.assert_allclose(out[ok, c], val[ok], rtol=2e-4, atol=1e-6 * val.max())
        np.testing.assert_allclose(out[ok, 3], pdf[ok], rtol=2e-4, atol=1e-6 * pdf.max())
        # both lobes carry real values in the sample
        assert (val[refl] > 0.5).any() and (val[~refl] > 0.5).any()


def test_roughdielectric_alpha_to_zero_is_the_smooth_dielectric(oracle, small_scene):
    """alpha = 1e-4: reflection is chosen with probability F(cos_i) (sample1
    threshold; samples within 2e-3 of it skipped), reflected directions are the
    mirror, refracted ones Snell's (atol 2e-3 for >= 99 % of the samples: the
    sampled normal's tails), weights 1 and 1/eta^2 (rtol 1e-3) for those,
    bs.eta = the relative IOR, as the delta dielectric pinned in test_core_pins.
    Both sides."""
    from mtx import _abi

    rng = np.random.default_rng(25)
    mid = _materials(small_scene, _abi.MTX_MAT_ROUGHDIELECTRIC)[0]
    sc = _with_alpha(small_scene, mid, 1e-4)
    eta = float(sc.materials[mid].eta)
    n = 6000
    for side in (1.0, -1.0):
        wi = _hemi(rng, n, side, zmin=0.1)
        u = rng.random((n, 3))
        out, _ = _probe(oracle, sc, mid, wi, wi, u)
        F, ct, e = _fresnel_dielectric(wi[:, 2], eta)
        sin2_t = (1 - wi[:, 2] ** 2) / e ** 2
        ok = (np.abs(u[:, 0] - F) > 2e-3) & (np.abs(sin2_t - 1) > 2e-2) & (out[:, 10] > 0)
        assert ok.mean() > 0.8
        typ = out[:, 9].view(np.uint32)
        refl = u[:, 0] <= F
        assert np.all((typ[ok] == 0x08) == refl[ok])
        expect = np.where(refl[:, None], wi * [-1, -1, 1], _refract_dir(wi, eta))
        close = np.abs(out[:, 4:7] - expect).max(1) < 2e-3
        assert close[ok].mean() > 0.99, close[ok].mean()
        r, t = refl & ok & close, ~refl & ok & close
        np.testing.assert_allclose(out[r, 10:13], 1.0, rtol=1e-3)
        np.testing.assert_allclose(out[t, 10], 1.0 / e[t] ** 2, rtol=1e-3)
        np.testing.assert_allclose(out[t, 8], e[t], rtol=1e-6)
        assert r.sum() > 50 and t.sum() > 50
