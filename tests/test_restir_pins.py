"""Independent pins of mtx_core/restir.h (the ReSTIR GI reservoir arithmetic
the device kernels and the oracle both compile, so bit-exact HIP-vs-oracle
parity cannot see an error in it).

Each function below is a float64 numpy transcription of the reference's own
Python text, written from restirgi.py and not from the header:

  J                restirgi.py:42-53
  p_hat            restirgi.py:84-85
  RestirReservoir  restirgi.py:118-148 (update :120-134, merge :136-141)
  similar          restirgi.py:175-180 (dist_threshold 0.1, angle 25 deg, :152-153)
  to_idx           restirgi.py:170-173

Dr.Jit semantics restated: ``dr.clamp(x, lo, hi) = maximum(minimum(x, hi), lo)``
with NaN-ignoring min / max (LLVM minnum / maxnum, CUDA min.f32: the non-NaN
operand wins) -> ``np.fmax(np.fmin(x, hi), lo)``; ``dr.select(c, a, b)``;
a UInt count enters ``p * r.W * r.M`` as a float, left to right. The header
computes in float32, the transcription in float64, so values are compared
with the relative tolerance written in each assert, and decisions (taken /
similar) exactly wherever the float64 quantity is not within 1e-5 of the
threshold. Edge cases from the verdict: d = 0, div = 0, NaN inputs, and the
``u < wnew / w`` draw with w = 0 (0 / 0: never taken).
"""
import numpy as np

COS25 = np.cos(25 * np.pi / 180)


def _clamp(x, lo, hi):
    return np.fmax(np.fmin(x, hi), lo)


def _norm(v):
    return np.sqrt(np.sum(v * v, axis=-1))


def J_ref(receiver, x_s, n_s, x_v):
    """restirgi.py:42-53."""
    with np.errstate(all="ignore"):
        v_new = receiver - x_s
        d_new = _norm(v_new)
        cos_new = _clamp(np.sum(v_new * n_s, -1) / d_new, 0.0, 1.0)
        v_old = x_v - x_s
        d_old = _norm(v_old)
        cos_old = _clamp(np.sum(v_old * n_s, -1) / d_old, 0.0, 1.0)
        div = cos_old * d_new ** 2
        return np.where(div > 0, cos_new * d_old ** 2 / div, 0.0)


def update_ref(w, M, wnew, active, u):
    """RestirReservoir.update, restirgi.py:120-134 -> (w, M, taken, wnew / w)."""
    with np.errstate(all="ignore"):
        w = w + np.where(active, wnew, 0.0)
        M = M + np.where(active, 1, 0)
        ratio = wnew / w
        return w, M, active & (u < ratio), ratio


def merge_ref(w, M, oW, oM, p, active, u):
    """RestirReservoir.merge, restirgi.py:136-141."""
    M0 = M
    w, _, taken, ratio = update_ref(w, M, p * oW * oM.astype(np.float64), active, u)
    return w, np.where(active, M0 + oM, M0), taken, ratio


def similar_ref(xa, na, xb, nb):
    """RestirIntegrator.similar, restirgi.py:175-180 -> (similar, dist, cos)."""
    dist = _norm(xa - xb)
    c = np.sum(na * nb, -1)
    return (dist < 0.1) & (c > COS25), dist, c


def to_idx_ref(x, y, W, H, spp, smp):
    """restirgi.py:170-173 literally: Point2u(pos) (negative -> wraps as u32),
    clamp to [0, film_size] (one past the last pixel)."""
    xu, yu = np.asarray(x, np.int64) % (1 << 32), np.asarray(y, np.int64) % (1 << 32)
    xu, yu = np.clip(xu, 0, W), np.clip(yu, 0, H)
    return ((yu * W + xu) * spp + smp) % (1 << 32)


def _unit(rng, n):
    v = rng.normal(size=(n, 3))
    return v / _norm(v)[:, None]


def test_p_hat(oracle):
    rng = np.random.default_rng(1)
    f = (rng.uniform(0, 4, (4000, 3)) * rng.choice([1e-3, 1.0, 1e3], (4000, 1))).astype(np.float32)
    got = oracle.restir_probe("p_hat", f)[:, 0]
    np.testing.assert_allclose(got, _norm(f.astype(np.float64)), rtol=2e-6)


def test_similar(oracle):
    rng = np.random.default_rng(2)
    n = 20000
    xa = rng.uniform(-2, 2, (n, 3))
    xb = xa + _unit(rng, n) * rng.uniform(0.0, 0.2, (n, 1))
    na = _unit(rng, n)
    ang = np.radians(rng.uniform(0, 50, n))
    perp = _unit(rng, n)
    perp -= np.sum(perp * na, -1)[:, None] * na
    perp /= _norm(perp)[:, None]
    nb = na * np.cos(ang)[:, None] + perp * np.sin(ang)[:, None]
    xa, xb, na, nb = (v.astype(np.float32) for v in (xa, xb, na, nb))
    got = oracle.restir_probe("similar", np.concatenate([xa, na, xb, nb], 1))[:, 0] == 1
    ref, dist, c = similar_ref(*(v.astype(np.float64) for v in (xa, na, xb, nb)))
    clear = (np.abs(dist - 0.1) > 1e-5) & (np.abs(c - COS25) > 1e-5)
    assert clear.mean() > 0.99 and ref[clear].mean() > 0.1
    np.testing.assert_array_equal(got[clear], ref[clear])


def test_update_and_merge(oracle):
    rng = np.random.default_rng(3)
    n = 20000
    w = np.where(rng.random(n) < 0.1, 0.0, rng.exponential(2.0, n)).astype(np.float32)
    M = rng.integers(0, 40, n).astype(np.float32)
    wnew = np.where(rng.random(n) < 0.1, 0.0, rng.exponential(1.0, n)).astype(np.float32)
    active = rng.random(n) < 0.8
    u = rng.random(n).astype(np.float32)
    got = oracle.restir_probe("update", np.stack([w, M, wnew, active, u], 1).astype(np.float32))
    rw, rM, rt, ratio = update_ref(w.astype(np.float64), M.astype(np.int64), wnew.astype(np.float64), active,
                                   u.astype(np.float64))
    np.testing.assert_allclose(got[:, 0], rw, rtol=1e-6)
    np.testing.assert_array_equal(got[:, 1], rM)
    with np.errstate(invalid="ignore"):
        clear = ~(np.abs(u - ratio) <= 1e-5 * np.fmax(1.0, np.abs(ratio)))
    np.testing.assert_array_equal(got[clear, 2] == 1, rt[clear])
    # w = 0 after the update (inactive with w = 0, or wnew = 0 into w = 0): 0 / 0, never taken
    zero = np.array([[0, 5, 0, 1, 0.0], [0, 5, 0, 1, 0.5], [0, 5, 3, 0, 0.0]], np.float32)
    z = oracle.restir_probe("update", zero)
    np.testing.assert_array_equal(z[:, :3], [[0, 6, 0], [0, 6, 0], [0, 5, 0]])
    # merge: the neighbour's weight p * W * M, its M added when active
    oW = rng.exponential(1.0, n).astype(np.float32)
    oM = rng.integers(0, 30, n).astype(np.float32)
    p = rng.exponential(1.0, n).astype(np.float32)
    got = oracle.restir_probe("merge", np.stack([w, M, oW, oM, p, active, u], 1).astype(np.float32))
    rw, rM, rt, ratio = merge_ref(w.astype(np.float64), M.astype(np.int64), oW.astype(np.float64),
                                  oM.astype(np.int64), p.astype(np.float64), active, u.astype(np.float64))
    np.testing.assert_allclose(got[:, 0], rw, rtol=2e-6)
    np.testing.assert_array_equal(got[:, 1], rM)
    with np.errstate(invalid="ignore"):
        clear = ~(np.abs(u - ratio) <= 1e-5 * np.fmax(1.0, np.abs(ratio)))
    np.testing.assert_array_equal(got[clear, 2] == 1, rt[clear])
    # a neighbour with M = 0 adds no weight: 0 / w (w > 0) is never above u >= 0
    m0 = oracle.restir_probe("merge", np.array([[2.0, 3, 1.5, 0, 1.0, 1, 0.0]], np.float32))
    np.testing.assert_array_equal(m0[0, :3], [2.0, 3, 0])


def test_jacobian(oracle):
    rng = np.random.default_rng(4)
    n = 20000
    x_s = rng.uniform(-1, 1, (n, 3))
    n_s = _unit(rng, n)
    receiver = x_s + _unit(rng, n) * rng.uniform(0.05, 3.0, (n, 1))
    x_v = x_s + _unit(rng, n) * rng.uniform(0.05, 3.0, (n, 1))
    inp = np.concatenate([receiver, x_s, n_s, x_v], 1).astype(np.float32)
    got = oracle.restir_probe("J", inp)[:, 0]
    r64 = inp.astype(np.float64)
    ref = J_ref(r64[:, 0:3], r64[:, 3:6], r64[:, 6:9], r64[:, 9:12])
    # cosines well inside (0, 1): the float32 chain's relative error is small
    with np.errstate(all="ignore"):
        c_new = np.sum((r64[:, 0:3] - r64[:, 3:6]) * r64[:, 6:9], -1) / _norm(r64[:, 0:3] - r64[:, 3:6])
        c_old = np.sum((r64[:, 9:12] - r64[:, 3:6]) * r64[:, 6:9], -1) / _norm(r64[:, 9:12] - r64[:, 3:6])
    inner = (c_new > 1e-3) & (c_old > 1e-3)
    assert inner.mean() > 0.2
    np.testing.assert_allclose(got[inner], ref[inner], rtol=2e-4)
    # a neighbour seen from behind (cos_old clamped to 0: div = 0) or the
    # receiver behind the sample (cos_new = 0): J = 0 exactly
    edge = ((c_old < -1e-3) | (c_new < -1e-3))
    assert edge.any()
    np.testing.assert_array_equal(got[edge], ref[edge])
    np.testing.assert_array_equal(ref[edge], 0.0)
    # d_new = 0 (receiver at x_s), d_old = 0 (x_v at x_s): 0; NaN inputs as
    # the reference text has them (clamp ignores a NaN cosine: a NaN receiver
    # or x_s gives div = NaN -> 0, a NaN normal gives cosines 1 and a finite
    # J, a NaN x_v gives NaN)
    s = np.array([0.2, 0.1, -0.3], np.float32)
    nn = np.array([0.0, 0.0, 1.0], np.float32)
    up = s + np.array([0.1, 0.2, 0.9], np.float32)
    nan3 = np.full(3, np.nan, np.float32)
    cases = np.array([np.concatenate(c) for c in ([s, s, nn, up], [up, s, nn, s], [nan3, s, nn, up],
                                                  [up, nan3, nn, up], [up, s, nan3, up], [up, s, nn, nan3])],
                     np.float32)
    g = oracle.restir_probe("J", cases)[:, 0]
    c64 = cases.astype(np.float64)
    ref = J_ref(c64[:, 0:3], c64[:, 3:6], c64[:, 6:9], c64[:, 9:12])
    np.testing.assert_array_equal(ref[:4], 0.0)
    assert np.isfinite(ref[4]) and ref[4] > 0 and np.isnan(ref[5])
    np.testing.assert_array_equal(g, ref)  # NaN where the reference gives NaN


def test_to_idx(oracle):
    """In-film positions: the reference's index exactly. Outside the film the
    reference clamps to [0, film_size] -- one past the last pixel -- after
    wrapping negative offsets through u32 (restirgi.py:170-173); mtx clamps
    to [0, size - 1] in signed arithmetic (reference bugs
    decided explicitly). Both choices are asserted here."""
    W, H, spp = 37, 23, 3
    xs, ys = np.meshgrid(np.arange(-3, W + 3), np.arange(-3, H + 3))
    xs, ys = xs.reshape(-1), ys.reshape(-1)
    smp = (xs * 7 + ys) % spp
    inp = np.stack([xs, ys, np.full_like(xs, W), np.full_like(xs, H), np.full_like(xs, spp), smp], 1)
    got = oracle.restir_probe("to_idx", inp.astype(np.float32))[:, 0].astype(np.int64)
    ref = to_idx_ref(xs, ys, W, H, spp, smp)
    inside = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
    np.testing.assert_array_equal(got[inside], ref[inside])
    mine = ((np.clip(ys, 0, H - 1) * W + np.clip(xs, 0, W - 1)) * spp + smp)
    np.testing.assert_array_equal(got, mine)
    assert (got < W * H * spp).all() and (ref[~inside] >= W * H * spp).any()
