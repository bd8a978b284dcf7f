"""Radiance field (nerad.py:54-106) for NRC: shared encoder (oracle vs HIP,
bit-exact) and the fused fp16 MFMA MLP (vs a plain fp32 reference with fp16
activation rounding; tolerance stated below)."""
import numpy as np
import pytest


def _field(**kw):
    from mtx.field import Field

    return Field(bbox=([-3.0, 0.0, -2.0], [4.0, 3.0, 4.0]), **kw)


def _queries(n, seed=1):
    rng = np.random.default_rng(seed)
    p = rng.uniform([-3, 0, -2], [4, 3, 4], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    return p, d


def test_sh_basis_orthonormal(oracle):
    """The 16 SH features (dr.sh_eval order 3) are orthonormal on the sphere."""
    f = _field()
    p, d = _queries(200_000, seed=3)
    feat = oracle.field_features(f, p, d).astype(np.float64)
    Y = feat[:, 38:54]
    G = 4 * np.pi * (Y.T @ Y) / len(Y)
    np.testing.assert_allclose(G, np.eye(16), atol=0.03)
    assert np.array_equal(feat[:, 35:38], d.astype(np.float16).astype(np.float64))  # wi
    assert (feat[:, 54:] == 0).all()


def test_hashgrid_partition_of_unity_and_vertices(oracle):
    f = _field()
    f.table[:] = np.float16(1.0)
    p, d = _queries(5000)
    feat = oracle.field_features(f, p, d)
    assert (feat[:, 3:35] == np.float16(1.0)).all()  # trilinear weights sum to one
    # a point on a level-0 grid vertex returns that vertex's entry (dense level:
    # scale 15, resolution 16, index x + 16 y + 256 z)
    f2 = _field()
    rng = np.random.default_rng(0)
    f2.table[0] = rng.uniform(-1, 1, f2.table[0].shape).astype(np.float16)
    gx, gy, gz = 3, 7, 11
    pn = (np.array([gx, gy, gz], np.float64) - 0.5) / 15.0
    pw = (f2.bbox_min + pn * (f2.bbox_max - f2.bbox_min)).astype(np.float32)[None]
    feat = oracle.field_features(f2, pw, d[:1])
    idx = gx + 16 * gy + 256 * gz
    np.testing.assert_allclose(feat[0, 3:5].astype(np.float32), f2.table[0, idx].astype(np.float32), atol=2e-3)


@pytest.mark.gpu
def test_field_features_bit_exact(oracle):
    f = _field()
    p, d = _queries(20_000)
    assert np.array_equal(f.features(p, d).view(np.uint16), oracle.field_features(f, p, d).view(np.uint16))


@pytest.mark.gpu
def test_field_mlp_exact_on_integer_selection_network():
    """Weights that select one input per output (asymmetric permutations) and
    small non-negative integer features: every value is exact in fp16 and f32,
    so any fragment-layout error shows as a wrong integer."""
    f = _field()
    n_in = f.n_in
    for li, w in enumerate(f.weights):
        w[:] = 0
        rows, cols = w.shape
        for o in range(rows):
            k = (o * 7 + 3) % cols if li == 0 else ((o * 5 + 1) % cols if li < len(f.weights) - 1 else o * 11 + 2)
            w[o, k] = 1
    rng = np.random.default_rng(5)
    n = 1000
    feat = np.zeros((n, 64), np.float16)
    feat[:, :n_in] = rng.integers(0, 8, (n, n_in)).astype(np.float16)
    got = f.mlp(feat)
    ref = f.mlp_reference(feat)
    assert np.array_equal(got, ref)
    assert len(np.unique(got)) > 4


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 1000, 65_537])
def test_field_eval_vs_reference(oracle, n):
    """Field(si) on the GPU vs encoder (oracle) + fp32 reference MLP.
    Tolerance: fp16 activations and f32 MFMA accumulation in a different
    order than numpy -> |err| <= 2e-3 + 2e-2 |ref|."""
    f = _field()
    p, d = _queries(n, seed=n)
    got = f(p, d)
    ref = f.mlp_reference(oracle.field_features(f, p, d))
    np.testing.assert_allclose(got, ref, rtol=2e-2, atol=2e-3)
    assert np.isfinite(got).all() and np.abs(got).max() > 0


def test_nrc_cache_queries_leave_L_unchanged(small_scene, oracle):
    """The cache option only adds queries: the oracle's per-sample L and film
    positions are identical with and without it, and stopped segments that
    hit a surface produce queries with unit-length wi (CPU)."""
    from mtx import load_dict

    integ = load_dict({"type": "nrc"})
    a = integ.render_args(small_scene, 3, 2)
    L0, pos0 = oracle.render_samples(small_scene, a)
    a.flags |= 4
    L1, pos1, q = oracle.render_samples_nrc_cache(small_scene, a)
    assert np.array_equal(L0, L1) and np.array_equal(pos0, pos1)
    m = q[:, 0] == 1
    assert 0.05 < m.mean() < 1.0
    assert (q[~m] == 0).all()
    np.testing.assert_allclose(np.linalg.norm(q[m, 4:7], axis=1), 1.0, atol=1e-5)
    assert (q[m, 7:10] >= 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [0, 1000])
def test_nrc_cache_film_bit_exact(small_scene, oracle, chunk):
    """NRC with the radiance cache: the GPU film equals the
    oracle's per-sample L + T * Field(query) composed on the host (field
    evaluated by the same fused MFMA kernel through mtx_field_eval), splatted
    by the oracle film. Bit-exact: every step is the same IEEE sequence."""
    from mtx import load_dict
    from mtx.field import Field

    field = Field(small_scene, seed=5, table_scale=1.0)
    integ = load_dict({"type": "nrc", "field": field})
    spp = 4
    film = integ.render_film(small_scene, seed=3, spp=spp, chunk_paths=chunk)
    a = integ.render_args(small_scene, 3, spp)
    assert a.flags & 4
    L, pos, q = oracle.render_samples_nrc_cache(small_scene, a)
    m = q[:, 0] == 1
    assert m.any()
    out = field(q[m, 1:4], q[m, 4:7])
    L[m] = L[m] + q[m, 7:10] * out
    ref = oracle.film(small_scene.width, 0, small_scene.height, spp, L, pos)
    np.testing.assert_array_equal(film, ref)
    plain = load_dict({"type": "nrc"}).render_film(small_scene, seed=3, spp=spp)
    assert not np.array_equal(plain, film)


@pytest.mark.gpu
@pytest.mark.parametrize("n_hidden", [14, 16])
def test_nrc_cache_deep_field_bit_exact(small_scene, oracle, n_hidden):
    """Fields deeper than the fused cache kernel's LDS allows (n_hidden 15 /
    16 need more than the 160 KiB of a workgroup) take the three-kernel path
    (encode, MLP, apply; api.cpp run_cache) instead of a failed launch: the
    film still equals the oracle's composition bit for bit; n_hidden 14 is
    the deepest fused case."""
    from mtx import load_dict
    from mtx.field import Field

    field = Field(small_scene, seed=9, table_scale=1.0, n_hidden=n_hidden)
    integ = load_dict({"type": "nrc", "field": field})
    film = integ.render_film(small_scene, seed=4, spp=2)
    a = integ.render_args(small_scene, 4, 2)
    L, pos, q = oracle.render_samples_nrc_cache(small_scene, a)
    m = q[:, 0] == 1
    assert m.any()
    L[m] = L[m] + q[m, 7:10] * field(q[m, 1:4], q[m, 4:7])
    np.testing.assert_array_equal(film, oracle.film(small_scene.width, 0, small_scene.height, 2, L, pos))


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [0, 40000])
def test_nrc_cache_two_streams_bit_exact(small_scene, oracle, chunk):
    """A render of >= 2^16 paths runs on two wavefronts / streams, each chunk's
    cache pass (encode, MLP, apply) on its wavefront's own query buffers
    while the other chunk traces: the film still equals the oracle's
    composition bit for bit (256x144, spp 4: 147 K paths; two chunks, or four
    alternating over the two wavefronts with chunk_paths 40000)."""
    from mtx import load_dict
    from mtx.field import Field

    sc = small_scene.with_film(256, 144)
    field = Field(sc, seed=5, table_scale=1.0)
    integ = load_dict({"type": "nrc", "field": field})
    spp = 4
    film = integ.render_film(sc, seed=3, spp=spp, chunk_paths=chunk)
    a = integ.render_args(sc, 3, spp)
    L, pos, q = oracle.render_samples_nrc_cache(sc, a)
    m = q[:, 0] == 1
    out = field(q[m, 1:4], q[m, 4:7])
    L[m] = L[m] + q[m, 7:10] * out
    np.testing.assert_array_equal(film, oracle.film(sc.width, 0, sc.height, spp, L, pos))


@pytest.mark.gpu
def test_nrc_cache_morton_order_unchanged(tmp_path):
    """MTX_CACHE_SORT=1 encodes the cache queries in Morton order (sorted with
    the hash-grid group-by; measured slower); 2 groups them by region on the
    device, one eighth of the rows per XCD (also on the second wavefront of a
    two-stream render: chunk_paths); queue order otherwise; the encode, MLP
    and apply fused into one launch (MTX_CACHE_FUSED) or not, the level-major
    or the query-major encoder (MTX_ENCODE_LM). All films are identical (each
    query's features and MLP column are its own)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from mtx import load_dict, scene
from mtx.field import Field
sc = scene.bedroom(width=64, height=36, scale=0.02, tex_res=64)
integ = load_dict({"type": "nrc", "field": Field(sc, seed=5, table_scale=1.0)})
kw = {"chunk_paths": int(sys.argv[3])} if int(sys.argv[3]) else {}
np.save(sys.argv[2], integ.render_film(sc, seed=7, spp=4, **kw))
'''
    films = []
    # (order, chunk paths, fused encode+MLP+apply, level-major encoder)
    for flag, chunk, fused, lm in (("1", 0, "0", "0"), ("0", 0, "0", "0"), ("2", 0, "1", "1"), ("2", 5000, "1", "1"),
                                   ("0", 5000, "1", "1"), ("2", 0, "0", "1"), ("0", 0, "1", "0")):
        f = tmp_path / f"f{flag}_{chunk}_{fused}_{lm}.npy"
        subprocess.run([sys.executable, "-c", code, os.path.join(root, "mitsuba3-experiments_amd"), str(f), str(chunk)],
                       check=True, env=dict(os.environ, MTX_CACHE_SORT=flag, MTX_CACHE_FUSED=fused, MTX_ENCODE_LM=lm),
                       timeout=300)
        films.append(np.load(f))
    for f in films[1:]:
        np.testing.assert_array_equal(films[0], f)
