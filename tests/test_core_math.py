"""The shared per-lane primitive layer (include/mtx_core) against independent
numpy formulas: deterministic transcendentals, warps, and BSDF invariants
(sample/eval consistency, energy conservation, pdf normalisation)."""
import math

import numpy as np
import pytest
from scipy import special


def test_transcendentals_accuracy(oracle):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-7, 7, 20000), np.linspace(-1.6, 1.6, 1001)]).astype(np.float32)
    xd = x.astype(np.float64)
    assert np.max(np.abs(oracle.dmath("sin", x) - np.sin(xd))) < 3e-7
    assert np.max(np.abs(oracle.dmath("cos", x) - np.cos(xd))) < 3e-7
    p = np.exp(rng.uniform(-30, 30, 20000)).astype(np.float32)
    rel = np.abs(oracle.dmath("log", p) - np.log(p.astype(np.float64))) / np.maximum(1, np.abs(np.log(p.astype(np.float64))))
    assert rel.max() < 3e-7
    e = rng.uniform(-80, 80, 20000).astype(np.float32)
    assert np.max(np.abs(oracle.dmath("exp", e) / np.exp(e.astype(np.float64)) - 1)) < 5e-7
    z = rng.uniform(-4, 4, 20000).astype(np.float32)
    assert np.max(np.abs(oracle.dmath("erf", z) - special.erf(z.astype(np.float64)))) < 2e-6
    y = rng.uniform(-0.999, 0.999, 20000).astype(np.float32)
    ref = special.erfinv(y.astype(np.float64))
    assert np.max(np.abs(oracle.dmath("erfinv", y) - ref) / np.maximum(1, np.abs(ref))) < 2e-6
    assert oracle.dmath("log", np.array([0.0], np.float32))[0] == -np.inf


def test_warps(oracle):
    rng = np.random.default_rng(1)
    u = rng.random((50000, 2), dtype=np.float32)
    v = oracle.warp("cosine_hemisphere", u)
    assert np.allclose(np.linalg.norm(v, axis=1), 1, atol=1e-5) and (v[:, 2] >= 0).all()
    # E[cos theta] under the cosine density = 2/3
    assert abs(v[:, 2].mean() - 2 / 3) < 5e-3
    d = oracle.warp("disk_concentric", u)
    assert (np.hypot(d[:, 0], d[:, 1]) <= 1 + 1e-6).all() and abs(np.hypot(d[:, 0], d[:, 1]).mean() - 2 / 3) < 5e-3
    g = oracle.warp("std_normal", u)[:, :2]
    assert abs(g.mean()) < 0.02 and abs(g.std() - 1) < 0.02
    h = oracle.warp("uniform_hemisphere", u)
    assert np.allclose(np.linalg.norm(h, axis=1), 1, atol=1e-5) and abs(h[:, 2].mean() - 0.5) < 5e-3


def _sphere(n, rng):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


@pytest.fixture(scope="module")
def materials(small_scene):
    out = {}
    from mtx import _abi

    for i, m in enumerate(small_scene.materials):
        out.setdefault((m.type, m.flags & (_abi.MTX_MF_BECKMANN | _abi.MTX_MF_MASK)), i)
    return out


def test_bsdf_sample_matches_eval(oracle, small_scene, materials):
    """For non-delta lobes: weight == eval(wo)/pdf(wo) at the sampled wo, and
    the sample pdf equals the evaluated pdf (mask: nested lobe only)."""
    from mtx import _abi

    rng = np.random.default_rng(3)
    n = 4000
    for (mtype, fl), mid in materials.items():
        if mtype in (_abi.MTX_MAT_CONDUCTOR, _abi.MTX_MAT_DIELECTRIC):
            continue  # delta lobes: tests/test_core_pins.py (Fresnel / Snell)
        wi = _sphere(n, rng)
        wi[:, 2] = np.abs(wi[:, 2]) + 0.05
        wi /= np.linalg.norm(wi, axis=1, keepdims=True)
        u = rng.random((n, 3), dtype=np.float32)
        out, pdf2 = oracle.bsdf_probe(small_scene, mid, wi, wi, np.full((n, 2), 0.3, np.float32), u)
        typ = out[:, 9].view(np.uint32)
        w, val2, spdf = out[:, 10:13], out[:, 13:16], out[:, 7]
        ok = (spdf > 1e-3) & (w.max(1) > 0) & (typ != 1)
        if fl & _abi.MTX_MF_MASK:
            opacity = small_scene.materials[mid].opacity
            val2 = val2 / opacity
            pdf2 = pdf2 / opacity
        np.testing.assert_allclose(w[ok], val2[ok] / pdf2[ok, None], rtol=2e-3, atol=1e-5)
        np.testing.assert_allclose(spdf[ok], pdf2[ok], rtol=2e-3)


def test_bsdf_energy_and_pdf_normalisation(oracle, small_scene, materials):
    """Furnace-style checks: E[weight] <= 1 (albedo <= 1) and the evaluated
    pdf integrates to <= 1 over the sphere (uniform-direction MC)."""
    from mtx import _abi

    rng = np.random.default_rng(5)
    n = 60000
    for (mtype, fl), mid in materials.items():
        wi = np.tile(np.array([[0.3, 0.1, 0.9]], np.float32), (n, 1))
        wi /= np.linalg.norm(wi, axis=1, keepdims=True)
        u = rng.random((n, 3), dtype=np.float32)
        wo = _sphere(n, rng)
        out, _ = oracle.bsdf_probe(small_scene, mid, wi, wo, np.full((n, 2), 0.3, np.float32), u)
        albedo = out[:, 10:13].mean(0)
        assert (albedo <= 1.0 + 0.02).all(), (mtype, albedo)
        if mtype not in (_abi.MTX_MAT_CONDUCTOR, _abi.MTX_MAT_DIELECTRIC):
            integral = out[:, 3].mean() * 4 * math.pi
            assert integral <= 1.05, (mtype, integral)
            if mtype == _abi.MTX_MAT_DIFFUSE and not fl & _abi.MTX_MF_MASK:
                assert abs(integral - 1) < 0.03
