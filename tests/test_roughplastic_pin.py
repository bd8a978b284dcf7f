"""Independent pin of the roughplastic BSDF (include/mtx_core/bsdf.h
roughplastic_eval_pdf, csrc/bvh_build.cpp mtx_roughplastic_tables): a float64
numpy restatement of upstream Mitsuba's roughplastic (SURVEY.md Appendix A,
"roughplastic nonlinear": bsdf.eval_pdf_sample at path-mis.py:107-109,
bsdf.sample at pssmltsimple.py:84) that shares no code with the C++ one.

* The 64-entry external transmittance table and the internal reflectance are
  integrated over the microfacet normal m (Gauss-Legendre in tan(theta_m) /
  alpha and in phi, float64), not over the visible-normal sample space in
  float32 as the C++ precompute does.
* Closed-form limits: as alpha -> 0 the table tends to 1 - F(cos theta, eta)
  and the internal reflectance to the hemispherical average of F(mu, 1/eta)
  (which equals 1 - (1 - r_external) / eta^2).
* eval and pdf at random (wi, wo) against the numpy formula (GGX / Beckmann D,
  Smith G, exact dielectric Fresnel, the `nonlinear` denominator
  1 - R * internal, the diffuse term R / (1 - .) * cos_o / pi / eta^2 * t_i t_o).
Tolerances are stated in each assert.
"""
import copy
import functools
import ctypes as C
import math

import numpy as np
import pytest

RES = 64  # MTX_ROUGH_TRANSMITTANCE_RES


# ----------------------------------------------------------- numpy formulas --
def fresnel(ci, eta):
    """Exact unpolarised dielectric Fresnel reflectance (upstream fresnel_dielectric)."""
    ci = np.asarray(ci, np.float64)
    eta_it = np.where(ci >= 0, eta, 1.0 / eta)
    a = np.abs(ci)
    ct2 = 1.0 - (1.0 - a * a) / (eta_it * eta_it)
    ct = np.sqrt(np.maximum(ct2, 0.0))
    rs = (a - eta_it * ct) / (a + eta_it * ct)
    rp = (eta_it * a - ct) / (eta_it * a + ct)
    return np.where(ct2 <= 0, 1.0, 0.5 * (rs * rs + rp * rp))


def D(mz, alpha, beckmann):
    mz = np.asarray(mz, np.float64)
    c2 = mz * mz
    t2 = (1.0 - c2) / np.maximum(c2, 1e-300)
    if beckmann:
        v = np.exp(-t2 / alpha**2) / (math.pi * alpha**2 * c2 * c2)
    else:
        v = 1.0 / (math.pi * alpha**2 * c2 * c2 * (1.0 + t2 / alpha**2) ** 2)
    return np.where(mz > 0, v, 0.0)


def G1(v, m, alpha, beckmann):
    vz = v[..., 2]
    t2 = (1.0 - vz * vz) / np.maximum(vz * vz, 1e-300)
    if beckmann:
        a = 1.0 / np.sqrt(np.maximum(alpha**2 * t2, 1e-300))
        g = np.where(a >= 1.6, 1.0, (3.535 * a + 2.181 * a * a) / (1.0 + 2.276 * a + 2.577 * a * a))
    else:
        g = 2.0 / (1.0 + np.sqrt(1.0 + alpha**2 * t2))
    return np.where(np.sum(v * m, -1) * vz > 0, g, 0.0)


def _gl(n, a, b):
    x, w = np.polynomial.legendre.leggauss(n)
    return 0.5 * (b - a) * x + 0.5 * (b + a), 0.5 * (b - a) * w


def spec_albedo(mu, alpha, eta, beckmann, n_s=256, n_phi=128):
    """Directional albedo of the specular microfacet lobe at cos(theta_i) = mu:
    integral over m of F(wi.m) G1(wi, m) G1(wo, m) D(m) (wi.m) / mu, wo = reflect(wi, m)."""
    mu = float(mu)
    wi = np.array([math.sqrt(max(0.0, 1 - mu * mu)), 0.0, mu])
    t, wt = _gl(n_s, 0.0, 1.0)  # s = tan(theta_m) / alpha = t / (1 - t)
    s = t / (1.0 - t)
    ds = wt / (1.0 - t) ** 2
    th = np.arctan(alpha * s)
    dth = ds * alpha / (1.0 + (alpha * s) ** 2)
    ph, wp = _gl(n_phi, 0.0, math.pi)  # symmetric in +-phi: [0, pi] twice
    TH, PH = np.meshgrid(th, ph, indexing="ij")
    W = np.outer(dth * np.sin(th), wp) * 2.0
    m = np.stack([np.sin(TH) * np.cos(PH), np.sin(TH) * np.sin(PH), np.cos(TH)], -1)
    dm = m @ wi
    wo = 2.0 * dm[..., None] * m - wi
    f = fresnel(dm, eta) * G1(np.broadcast_to(wi, m.shape), m, alpha, beckmann) * G1(wo, m, alpha, beckmann)
    f = f * D(m[..., 2], alpha, beckmann) * np.maximum(dm, 0.0) / mu
    return float(np.sum(f * W))


@functools.lru_cache(maxsize=None)
def np_tables(alpha, eta, beckmann):
    """Upstream roughplastic precompute semantics: mu = max(1e-6, linspace(0, 1, 64));
    table = 1 - albedo(mu, eta); internal = mean(albedo(mu, 1/eta) * mu) * 2."""
    mus = np.maximum(1e-6, np.linspace(0.0, 1.0, RES))
    tab = np.array([1.0 - spec_albedo(m, alpha, eta, beckmann) for m in mus])
    internal = np.mean([spec_albedo(m, alpha, 1.0 / eta, beckmann) * m for m in mus]) * 2.0
    return tab, internal


def c_tables(alpha, eta, beckmann):
    from mtx import _lib

    tab = np.zeros(RES, np.float32)
    internal = C.c_float()
    assert _lib.lib().mtx_roughplastic_tables(1 if beckmann else 0, alpha, eta, tab.ctypes.data, C.byref(internal)) == 0
    return tab.astype(np.float64), float(internal.value)


def lerp_table(tab, x):
    x = x * (RES - 1)
    i = np.minimum(x.astype(np.int64), RES - 2)
    return tab[i] + (tab[i + 1] - tab[i]) * (x - i)


# ------------------------------------------------------------------- tests --
@pytest.mark.parametrize("beckmann", [False, True])
@pytest.mark.parametrize("alpha", [0.15, 0.4])
def test_transmittance_table_and_internal_reflectance(alpha, beckmann):
    """The C++ precompute (float32 Gauss-Legendre over the visible-normal sample
    space) against the float64 integral over microfacet normals."""
    ref_tab, ref_int = np_tables(alpha, 1.5, beckmann)
    tab, internal = c_tables(alpha, 1.5, beckmann)
    # entry 0 is mu = 1e-6 (grazing): both ~0; everything within 2e-3 absolute
    np.testing.assert_allclose(tab, ref_tab, atol=2e-3)
    assert abs(internal - ref_int) < 2e-3, (internal, ref_int)


@pytest.mark.parametrize("beckmann", [False, True])
def test_smooth_limit_closed_forms(beckmann):
    """alpha -> 0: t(mu) -> 1 - F(mu, eta); internal -> 2 mean(F(mu, 1/eta) mu)
    over the same 64 nodes, which approximates the hemispherical average
    2 int_0^1 F(mu, 1/eta) mu dmu = 1 - (1 - r_e) / eta^2."""
    eta = 1.5
    tab, internal = c_tables(1e-3, eta, beckmann)
    mus = np.maximum(1e-6, np.linspace(0.0, 1.0, RES))
    smooth = 1.0 - fresnel(mus, eta)
    sel = mus >= 0.15  # near grazing the G1 shadowing of a finite alpha still matters
    np.testing.assert_allclose(tab[sel], smooth[sel], atol=2e-3)
    discrete = 2.0 * np.mean(fresnel(mus, 1.0 / eta) * mus)
    assert abs(internal - discrete) < 3e-3, (internal, discrete)
    x, w = _gl(4000, 0.0, 1.0)
    r_i = 2.0 * np.sum(w * fresnel(x, 1.0 / eta) * x)
    r_e = 2.0 * np.sum(w * fresnel(x, eta) * x)
    assert abs(r_i - (1.0 - (1.0 - r_e) / eta**2)) < 1e-4  # reciprocity identity
    assert abs(discrete - r_i) < 1.5e-2  # 64-node mean vs integral (the upstream discretisation)
    assert abs(r_i - 0.5963) < 2e-3  # eta = 1.5: the classic internal diffuse reflectance


def _flat_roughplastic(scene, mid, rgb):
    """The scene with material `mid` given a constant diffuse colour (no texture)."""
    from mtx import _abi

    s = copy.copy(scene)
    mats = [_abi.Material.from_buffer_copy(bytes(m)) for m in scene.materials]
    mats[mid].tex = -1
    mats[mid].rgb[:] = rgb
    mats[mid].spec_weight = 1.0 / (float(np.mean(rgb)) + 1.0)  # s_mean / (d_mean + s_mean), upstream ctor
    s.materials = (_abi.Material * len(mats))(*mats)
    return s, mats[mid]


@pytest.fixture(scope="module")
def plastic_ids(small_scene):
    from mtx import _abi

    ids = {}
    for i, m in enumerate(small_scene.materials):
        if m.type == _abi.MTX_MAT_ROUGHPLASTIC:
            ids.setdefault(bool(m.flags & _abi.MTX_MF_BECKMANN), i)
    assert set(ids) == {False, True}, "the bedroom has GGX and Beckmann roughplastic"
    return ids


@pytest.mark.parametrize("beckmann", [False, True])
def test_eval_pdf_against_numpy(oracle, small_scene, plastic_ids, beckmann):
    """bsdf.eval_pdf of roughplastic (bsdf.h:128-157, through the twosided
    wrapper on the front side) vs the numpy restatement of the formula. The
    table and internal reflectance are the precomputed ones (pinned against the
    float64 integral above), so this isolates the eval / pdf arithmetic:
    rtol 1e-4 (float32 vs float64)."""
    from mtx import _abi

    mid = plastic_ids[beckmann]
    rgb = [0.6, 0.25, 0.05]
    sc, m = _flat_roughplastic(small_scene, mid, rgb)
    assert m.flags & _abi.MTX_MF_NONLINEAR
    alpha, eta = float(m.alpha), float(m.eta)
    tab, internal = c_tables(alpha, eta, beckmann)
    np.testing.assert_array_equal(tab.astype(np.float32), sc.tables[m.table: m.table + RES])
    rng = np.random.default_rng(11)
    n = 20000

    def hemi(k):
        v = rng.normal(size=(k, 3))
        v[:, 2] = np.abs(v[:, 2]) + 0.02
        return v / np.linalg.norm(v, axis=1, keepdims=True)

    wi, wo = hemi(n), hemi(n)
    # half of the pairs near the mirror direction, where the specular lobe lives
    k = n // 2
    refl = wi[:k] * np.array([-1.0, -1.0, 1.0])
    wo[:k] = refl + 0.15 * rng.normal(size=(k, 3))
    wo[:k, 2] = np.abs(wo[:k, 2]) + 0.02
    wo[:k] /= np.linalg.norm(wo[:k], axis=1, keepdims=True)
    wi32, wo32 = wi.astype(np.float32), wo.astype(np.float32)
    wi, wo = wi32.astype(np.float64), wo32.astype(np.float64)
    out, _ = oracle.bsdf_probe(sc, mid, wi32, wo32, np.full((n, 2), 0.3, np.float32), rng.random((n, 3), dtype=np.float32))
    val, pdf = out[:, 0:3].astype(np.float64), out[:, 3].astype(np.float64)

    ci, co = wi[:, 2], wo[:, 2]
    H = wi + wo
    H /= np.linalg.norm(H, axis=1, keepdims=True)
    Dh = D(H[:, 2], alpha, beckmann)
    spec = fresnel(np.sum(wi * H, 1), eta) * Dh * G1(wi, H, alpha, beckmann) * G1(wo, H, alpha, beckmann) / (4 * ci)
    t_i, t_o = lerp_table(tab, ci), lerp_table(tab, co)
    R = np.array(rgb)
    diff = R / (1.0 - R * internal)  # nonlinear=true
    ref_val = spec[:, None] + diff[None, :] * (co * t_i * t_o / (math.pi * eta**2))[:, None]
    sw = float(m.spec_weight)
    assert abs(sw - 1.0 / (np.mean(rgb) + 1.0)) < 1e-6  # s_mean / (d_mean + s_mean)
    ps, pd = (1 - t_i) * sw, t_i * (1 - sw)
    ps, pd = ps / (ps + pd), 1 - ps / (ps + pd)
    ref_pdf = ps * Dh * G1(wi, H, alpha, beckmann) / (4 * ci) + pd * co / math.pi

    np.testing.assert_allclose(val, ref_val, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(pdf, ref_pdf, rtol=1e-4, atol=1e-7)
    # the specular lobe was exercised: a good share of pairs where it dominates
    assert (spec > 0.5 * ref_val.max(1)).mean() > 0.05


def test_roughplastic_sample_is_eval_over_pdf(oracle, small_scene, plastic_ids):
    """bsdf.sample: the returned pdf is eval_pdf's pdf at the sampled wo and the
    weight is eval / pdf (upstream roughplastic sample), both lobes selected."""
    rng = np.random.default_rng(13)
    n = 20000
    for mid in plastic_ids.values():
        sc, _ = _flat_roughplastic(small_scene, mid, [0.4, 0.4, 0.4])
        wi = rng.normal(size=(n, 3))
        wi[:, 2] = np.abs(wi[:, 2]) + 0.05
        wi = (wi / np.linalg.norm(wi, axis=1, keepdims=True)).astype(np.float32)
        out, pdf2 = oracle.bsdf_probe(sc, mid, wi, wi, np.full((n, 2), 0.3, np.float32), rng.random((n, 3), dtype=np.float32))
        w, val2, spdf = out[:, 10:13], out[:, 13:16], out[:, 7]
        typ = out[:, 9].view(np.uint32)
        ok = spdf > 1e-4
        assert len(set(typ[ok].tolist())) == 2  # glossy and diffuse lobes both drawn
        np.testing.assert_allclose(spdf[ok], pdf2[ok], rtol=1e-6)
        np.testing.assert_allclose(w[ok], val2[ok] / pdf2[ok, None], rtol=1e-5, atol=1e-7)
