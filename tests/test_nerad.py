"""Neural radiosity training (nerad.py).

CPU: the surface-area tables and the CPU restatement of IntersectionSampler /
sample_rhs (oracle/) against the properties the reference's algorithm
implies. GPU: the HIP LHS points and RHS lanes bit for bit against that
restatement (the field term composed from the same field evaluation), the
fused forward/backward of the network against a float64 numpy reference of
the same fp16 network (tolerances below), the Adam / GradScaler step against
numpy, and a short training run whose loss falls. Parity with Dr.Jit's
autodiff / optimisers themselves is unpinned (upstream, not in the tree)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def nscene():
    from mtx import scene

    return scene.bedroom(width=32, height=18, scale=0.02, tex_res=32)


@pytest.fixture(scope="module")
def tables(nscene):
    from mtx.nerad import surface_tables

    return surface_tables(nscene)


# ----------------------------------------------------------------- CPU ----
def test_surface_tables(nscene, tables):
    t = tables
    S = len(nscene.shapes)
    assert len(t["shape_pmf"]) == S and abs(float(t["shape_pmf"].astype(np.float64).sum()) - 1.0) < 1e-5
    assert np.all(np.diff(t["shape_cdf"]) >= 0)
    # every leaf-order triangle appears once, grouped by shape
    assert np.array_equal(np.sort(t["tri_prim"]), np.arange(nscene.n_tris, dtype=np.uint32))
    shp = np.asarray(nscene.tri_shape)
    for s in range(S):
        a, b = t["tri_off"][s], t["tri_off"][s + 1]
        assert np.all(shp[t["tri_prim"][a:b]] == s)
        assert np.all(np.diff(t["tri_cdf"][a:b]) >= 0) and t["tri_sum"][s] == t["tri_cdf"][b - 1]
        lo, hi = t["tri_valid"][2 * s], t["tri_valid"][2 * s + 1]
        assert t["tri_pmf"][a + lo] > 0 and t["tri_pmf"][a + hi] > 0


def test_oracle_lhs_points(nscene, tables, oracle):
    """Points lie on their triangle (barycentrics in the simplex), directions
    are unit length, one-sided materials get hemisphere directions, and the
    shapes are chosen in proportion to their area."""
    n = 20000
    lhs = oracle.nerad_lhs(nscene, tables, 7, n)
    prim = lhs[:, 0].view(np.uint32)
    b1, b2 = lhs[:, 1], lhs[:, 2]
    assert prim.max() < nscene.n_tris
    assert np.all(b1 >= 0) and np.all(b2 >= 0) and np.all(b1 + b2 <= 1.0 + 1e-6)
    v = np.asarray(nscene.vpos, np.float32).reshape(-1, 3)
    idx = np.asarray(nscene.tri_vidx).reshape(-1, 3)[prim]
    p = (1 - b1 - b2)[:, None] * v[idx[:, 0]] + b1[:, None] * v[idx[:, 1]] + b2[:, None] * v[idx[:, 2]]
    np.testing.assert_allclose(lhs[:, 3:6], p, atol=1e-4)
    assert np.abs(np.linalg.norm(lhs[:, 6:9], axis=1) - 1).max() < 1e-5
    shp = np.asarray(nscene.tri_shape)[prim]
    freq = np.bincount(shp, minlength=len(nscene.shapes)) / n
    big = tables["shape_pmf"] > 0.02
    np.testing.assert_allclose(freq[big], tables["shape_pmf"][big], rtol=0.15)


def test_oracle_rhs_lanes(nscene, tables, oracle):
    lanes = oracle.nerad_rhs(nscene, tables, 3, 4, 128, 8)
    assert np.isfinite(lanes).all()
    assert np.all(lanes[:, 0:3] >= 0) and np.all(lanes[:, 3:6] >= 0)
    valid = lanes[:, 9] > 0
    assert 0.2 < valid.mean() <= 1.0
    assert np.all(lanes[~valid, 3:6] == 0)  # f *= select(active, 1, 0) (nerad.py:222)
    # a different RHS seed gives different samples, the same seed the same ones
    assert np.array_equal(lanes, oracle.nerad_rhs(nscene, tables, 3, 4, 128, 8))
    assert not np.array_equal(lanes, oracle.nerad_rhs(nscene, tables, 3, 5, 128, 8))


# ------------------------------------------------------------------ GPU ----
def _field(sc, seed=1, **kw):
    from mtx.field import Field

    return Field(sc, seed=seed, **kw)


@pytest.mark.gpu
def test_nerad_lhs_bit_exact(nscene, oracle):
    from mtx.nerad import IntersectionSampler

    isamp = IntersectionSampler(nscene)
    for seed, n in ((0, 1), (3, 1000), (11, 4097)):
        got = isamp.sample(seed, n)
        ref = oracle.nerad_lhs(nscene, isamp.tables, seed, n)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), seed


@pytest.mark.gpu
@pytest.mark.parametrize("zero_field", [True, False])
def test_nerad_rhs_bit_exact(nscene, oracle, zero_field):
    """Every RHS lane and the per-point mean bit-exact: the oracle's lanes
    composed with the field evaluated (by the same HIP encoder + MLP) at the
    oracle's stop vertices."""
    from mtx.nerad import IntersectionSampler, Integrator

    field = _field(nscene)
    if zero_field:
        field.weights = [np.zeros_like(w) for w in field.weights]
    isamp = IntersectionSampler(nscene)
    batch, M = 700, 4
    integ = Integrator(field, batch_size=batch, M=M)
    L_rhs, lanes = integ.sample_rhs(nscene, isamp, 5, 6, lanes=True)
    ref = oracle.nerad_rhs(nscene, isamp.tables, 5, 6, batch, M)
    valid = ref[:, 9] > 0
    fv = np.zeros((len(ref), 3), np.float32)
    if valid.any():
        fv[valid] = field(ref[valid, 10:13], ref[valid, 13:16])
    if zero_field:
        assert np.all(fv == 0)
    L_ref, mean_ref = oracle.nerad_compose(ref, fv, M)
    assert np.array_equal(lanes, L_ref), np.argwhere(lanes != L_ref)[:5]
    assert np.array_equal(L_rhs, mean_ref)


def _ref_forward_backward(field, feat, target, scale):
    """float64 reference of the fp16 network (fp16-rounded pre-activations,
    LeakyReLU(0.01) in fp16, fp16 output) and its gradients."""
    n_in = field.n_in
    x = feat.astype(np.float64)[:, :n_in]
    Ws = [w.astype(np.float64) for w in field.weights]
    acts = [x]
    for W in Ws[:-1]:
        h = (x @ W.T).astype(np.float16)
        a = np.maximum(h, h * np.float16(0.01))
        x = a.astype(np.float64)
        acts.append(x)
    out = (x @ Ws[-1].T).astype(np.float16).astype(np.float64)
    d = out - target.astype(np.float64)
    n = len(feat)
    loss = float((d * d).mean())
    dY = scale * 2.0 * d / (3.0 * n)
    gW = [None] * len(Ws)
    for l in range(len(Ws) - 1, -1, -1):
        if l < len(Ws) - 1:
            dY = dY * np.where(acts[l + 1] > 0, 1.0, 0.01)
        gW[l] = dY.T @ acts[l]
        dY = dY @ Ws[l]
    return loss, out, gW, dY  # dY: d/d(features[:, :n_in])


def _corners(field, p):
    """Per level: the 8 table indices and trilinear weights of point p
    (mtx_core/field.h field_level_corners, float32)."""
    f32 = np.float32
    pn = ((p.astype(f32) - field.bbox_min) / (field.bbox_max - field.bbox_min)).astype(f32)
    T = 1 << field.log2_table
    res_out = []
    for l in range(field.n_levels):
        scale = f32(np.exp2(l * np.log2(field.per_level_scale)) * field.base_res - 1.0)
        res = int(np.ceil(float(scale))) + 1
        dense = res ** 3 <= T
        pos = pn * scale + f32(0.5)
        g = np.floor(pos)
        t = pos - g
        g = g.astype(np.int64)
        idx, w = [], []
        for c in range(8):
            b = np.array([c & 1, (c >> 1) & 1, (c >> 2) & 1])
            x, y, z = (g + b).astype(np.uint64)
            if dense:
                i = int(x + y * res + z * res * res)
            else:
                i = int((x * 1) ^ ((y * 2654435761) & 0xFFFFFFFF) ^ ((z * 805459861) & 0xFFFFFFFF))
            idx.append(i & (T - 1))
            ww = f32(1)
            for k in range(3):
                ww = ww * (t[k] if b[k] else f32(1) - t[k])
            w.append(ww)
        res_out.append((idx, w))
    return res_out


@pytest.mark.gpu
def test_field_gradients(nscene):
    """Output, loss and weight gradients against the float64 reference
    (tolerance: relative Frobenius error 2e-3 per layer -- fp32 sums and the
    rare fp16 activation that rounds the other way); table gradients: their
    per-level sums equal the grid-feature gradients (trilinear weights sum to
    one) and, for a single point, sit at its 8 corners with weight * dF."""
    from mtx.nerad import field_grad

    field = _field(nscene, seed=3, log2_table=14)
    rng = np.random.default_rng(0)
    n = 777
    v = np.asarray(nscene.vpos, np.float32).reshape(-1, 3)
    p = rng.uniform(v.min(0), v.max(0), (n, 3)).astype(np.float32)
    wi = rng.normal(size=(n, 3)).astype(np.float32)
    wi /= np.linalg.norm(wi, axis=1, keepdims=True)
    target = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    scale = 1024.0
    loss, out, gt, gw = field_grad(field, p, wi, target, scale)
    feat = field.features(p, wi)
    rl, rout, rgw, rdx = _ref_forward_backward(field, feat, target, scale)
    assert np.abs(out - rout).max() <= 2e-3 * max(1.0, np.abs(rout).max())
    assert abs(loss - rl) <= 1e-3 * rl
    for l, (a, b) in enumerate(zip(gw, rgw)):
        err = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        assert err < 2e-3, (l, err)
    LF = field.n_levels * field.n_features
    dgrid = rdx[:, 3:3 + LF].reshape(n, field.n_levels, field.n_features)
    np.testing.assert_allclose(gt.sum(axis=1), dgrid.sum(axis=0), rtol=2e-3, atol=1e-3 * np.abs(dgrid).max())
    # one point: gradients at its corners only
    loss1, out1, gt1, gw1 = field_grad(field, p[:1], wi[:1], target[:1], scale)
    _, _, _, rdx1 = _ref_forward_backward(field, field.features(p[:1], wi[:1]), target[:1], scale)
    ref_t = np.zeros_like(gt1, dtype=np.float64)
    for l, (idx, w) in enumerate(_corners(field, p[0])):
        for f in range(field.n_features):
            dF = rdx1[0, 3 + l * field.n_features + f]
            for i, ww in zip(idx, w):
                ref_t[l, i, f] += float(ww) * dF
    assert np.count_nonzero(gt1) <= np.count_nonzero(ref_t) + 0
    np.testing.assert_allclose(gt1, ref_t, rtol=2e-3, atol=2e-3 * np.abs(ref_t).max())


@pytest.mark.gpu
def test_adam_and_grad_scaler(nscene):
    """One GradScaler + Adam step on fp32 master copies (drjit.opt.Adam form)
    against numpy; a non-finite gradient skips the step and halves the scale."""
    from mtx.nerad import Adam, GradScaler, field_grad, field_params, field_train_init, field_train_step

    field = _field(nscene, seed=5, log2_table=12)
    rng = np.random.default_rng(1)
    n = 300
    v = np.asarray(nscene.vpos, np.float32).reshape(-1, 3)
    p = rng.uniform(v.min(0), v.max(0), (n, 3)).astype(np.float32)
    wi = np.tile(np.array([[0, 0, 1]], np.float32), (n, 1))
    target = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    opt, sc = Adam(lr=1e-3), GradScaler(init_scale=256.0)
    field_train_init(field, opt, sc)
    t0, w0, _, _ = field_params(field)
    assert np.array_equal(t0, field.table.reshape(-1).astype(np.float32))
    _, _, gt, gw = field_grad(field, p, wi, target, 256.0)
    g = np.concatenate([gt.reshape(-1), np.concatenate([x.reshape(-1) for x in gw])]).astype(np.float64) / 256.0
    st = field_train_step(field, p, wi, target)
    assert st["found_inf"] == 0 and st["step"] == 1 and st["scale"] == 256.0
    t1, w1, m1, v1 = field_params(field)
    p0 = np.concatenate([t0, w0]).astype(np.float64)
    m = 0.1 * g
    vv = 0.001 * g * g
    lr_t = 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9)
    ref = p0 - lr_t * m / (np.sqrt(vv) + 1e-8)
    np.testing.assert_allclose(np.concatenate([t1, w1]), ref, rtol=1e-5, atol=2e-7)
    np.testing.assert_allclose(m1, m, rtol=1e-3, atol=1e-12)
    # a NaN target -> non-finite gradients: no update, scale backs off
    bad = target.copy()
    bad[0, 0] = np.nan
    st = field_train_step(field, p, wi, bad)
    assert st["found_inf"] == 1 and st["step"] == 1 and st["scale"] == 128.0
    t2, w2, _, _ = field_params(field)
    assert np.array_equal(t2, t1) and np.array_equal(w2, w1)


@pytest.mark.gpu
def test_training_reduces_loss(nscene):
    """training_step (nerad.py:363-375) on the device lowers the radiosity
    residual of a fixed validation batch (same LHS / RHS seeds, M = 64, so
    the residual is deterministic given the field), and the fp16 field the
    renderer sees is the cast of the fp32 master weights."""
    from mtx.nerad import FieldTrainer, Integrator

    field = _field(nscene, seed=2, log2_table=14)
    tr = FieldTrainer(nscene, field, batch_size=2048, M=8)
    val = Integrator(field, batch_size=4096, M=64)

    # The residual is (LHS - RHS)^2 with a Monte-Carlo RHS: its floor is the
    # M = 64 RHS variance of the batch's points, which depends on where the
    # seeds land (the IntersectionSampler draws triangles in BVH leaf order,
    # so every new tree moves them). With the 4-wide BVH this batch started at
    # 0.09-0.23 and fell 2-5x in 60 steps; with the 8-wide one it starts at
    # 0.42 and falls to 0.28 (0.66x): asserted below 0.8x.
    def residual():
        lhs = tr.isampler.sample(123457, 4096, ctx=tr.ctx)
        rhs = val.sample_rhs(nscene, tr.isampler, 123457, 123458, ctx=tr.ctx)
        return float(np.mean((val.sample_lhs(nscene, lhs, ctx=tr.ctx) - rhs) ** 2))

    before = residual()
    losses = [tr.step()["loss"] for _ in range(60)]
    after = residual()
    assert np.isfinite(losses).all()
    assert after < 0.8 * before, (before, after, losses)
    tab, ws = tr.params()
    rng = np.random.default_rng(3)
    v = np.asarray(nscene.vpos, np.float32).reshape(-1, 3)
    p = rng.uniform(v.min(0), v.max(0), (64, 3)).astype(np.float32)
    wi = np.tile(np.array([[0, 1, 0]], np.float32), (64, 1))
    live = field(p, wi, ctx=tr.ctx)
    tr.download()
    assert np.array_equal(field.weights[0], ws[0].astype(np.float16))
    feat = field.features(p, wi, ctx=tr.ctx)
    np.testing.assert_allclose(live, field.mlp_reference(feat), atol=2e-2 * max(1.0, np.abs(live).max()))


@pytest.mark.gpu
def test_nerad_render_bit_exact(nscene, oracle):
    """Integrator.sample as a renderer (nerad.py:235-254): every sample's
    L = Field(si) * f + Le and the film bit-exact against the oracle's lanes
    composed with the same field evaluation."""
    from mtx import load_dict

    field = _field(nscene, seed=4)
    integ = load_dict({"type": "nerad", "field": field})
    spp = 3
    film = integ.render_film(nscene, seed=2, spp=spp)
    a = integ.render_args(nscene, 2, spp)
    lanes, pos = oracle.nerad_render_samples(nscene, a)
    valid = lanes[:, 9] > 0
    fv = np.zeros((len(lanes), 3), np.float32)
    fv[valid] = field(lanes[valid, 10:13], lanes[valid, 13:16])
    L = fv * lanes[:, 3:6] + lanes[:, 6:9]
    ref = oracle.film(nscene.width, 0, nscene.height, spp, np.ascontiguousarray(L, np.float32), pos)
    assert np.array_equal(film, ref), int((film != ref).sum())
    assert valid.mean() > 0.5 and film[..., 3].sum() > 0
