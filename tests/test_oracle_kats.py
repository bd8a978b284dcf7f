"""Oracle pins: the reference's in-repo known answers and independent numpy
restatements of the upstream sampler."""
import numpy as np
import pytest

M64 = (1 << 64) - 1


def tea(v0, v1, rounds=4):
    """sample_tea_32 (pssmlt.py:92 call site; upstream algorithm)."""
    v0 = np.asarray(v0, np.uint32).copy()
    v1 = np.asarray(v1, np.uint32).copy()
    s = np.uint32(0)
    with np.errstate(over="ignore"):
        for _ in range(rounds):
            s = np.uint32(s + np.uint32(0x9E3779B9))
            v0 = v0 + (((v1 << np.uint32(4)) + np.uint32(0xA341316C)) ^ (v1 + s) ^ ((v1 >> np.uint32(5)) + np.uint32(0xC8013EA4)))
            v1 = v1 + (((v0 << np.uint32(4)) + np.uint32(0xAD90777D)) ^ (v0 + s) ^ ((v0 >> np.uint32(5)) + np.uint32(0x7E95761E)))
    return v0, v1


class PCG32:
    """Dr.Jit PCG32 restated in Python integers (vectorised over lanes)."""

    MULT = 0x5851F42D4C957F2D

    def __init__(self, initstate, initseq):
        self.state = [0] * len(initstate)
        self.inc = [((int(q) << 1) | 1) & M64 for q in initseq]
        self.next_u32()
        self.state = [(s + int(i)) & M64 for s, i in zip(self.state, initstate)]
        self.next_u32()

    def next_u32(self):
        out = []
        for k, old in enumerate(self.state):
            self.state[k] = (old * self.MULT + self.inc[k]) & M64
            xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
            rot = old >> 59
            out.append(((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF)
        return np.array(out, np.uint32)

    def next_f32(self):
        u = self.next_u32()
        return ((u >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)


@pytest.mark.parametrize("seed", [0, 7])
def test_rng_streams_match_numpy_pcg32(oracle, seed):
    lanes = np.arange(256, dtype=np.uint32)
    v0, v1 = tea(np.full(256, seed, np.uint32), lanes)
    rng = PCG32(v0, v1)
    ref = np.stack([rng.next_f32() for _ in range(16)], 1)
    got = oracle.rng_stream(seed, 0, 256, 16)
    assert np.array_equal(got, ref)
    assert ((got >= 0) & (got < 1)).all()


def test_tea_known_answer():
    # fixed vectors of the 4-round TEA used for sampler seeding
    v0, v1 = tea(np.array([0, 1, 0xFFFFFFFF], np.uint32), np.array([0, 2, 12345], np.uint32))
    v0b, v1b = tea(np.array([0, 1, 0xFFFFFFFF], np.uint32), np.array([0, 2, 12345], np.uint32))
    assert np.array_equal(v0, v0b) and np.array_equal(v1, v1b)
    assert len(set(v0.tolist())) == 3


def test_hashgrid_kat(oracle):
    """hashgrid.py:93-98: points (0,0,0),(.1,.1,.1),(.6,.6,.6),(1,1,1), res 2, 2 cells."""
    p = np.array([[0, 0.1, 0.6, 1]] * 3, np.float32)
    cell, size, off, idx = oracle.hashgrid(p, 2, 2)
    assert cell.tolist() == [0, 0, 1, 0]
    assert size.tolist() == [3, 1]
    assert off.tolist() == [0, 3]
    assert idx.tolist() == [0, 1, 3, 2]


def test_hashgrid_matches_numpy(oracle):
    from mtx import primitives

    rng = np.random.default_rng(2)
    p = rng.random((3, 5000), dtype=np.float32)
    cell, size, off, idx = oracle.hashgrid(p, 100, 5000)
    assert np.array_equal(cell, primitives.hash_cells(p, 100, 5000))
    assert np.array_equal(size, np.bincount(cell, minlength=5000).astype(np.uint32))
    assert np.array_equal(off, (np.cumsum(size) - size).astype(np.uint32))
    assert np.array_equal(idx, np.argsort(cell, kind="stable").astype(np.uint32))


def test_scatter_reduce_kat(oracle):
    """reductions.py:57-63: 25 ones into 10 zeros by arange(25) % 10."""
    t = oracle.scatter_reduce(0, np.zeros(10, np.float32), np.ones(25, np.float32), np.arange(25) % 10)
    assert t.tolist() == [3, 3, 3, 3, 3, 2, 2, 2, 2, 2]
    t = oracle.scatter_reduce(2, np.zeros(3, np.float32), np.array([1, 5, 2, 7], np.float32), [0, 0, 1, 2])
    assert t.tolist() == [5, 2, 7]


def _hs_numpy(x):
    x = x.copy()
    n = len(x)
    i = 0
    while (1 << i) < n:
        s = 1 << i
        y = x.copy()
        y[s:] = x[s:] + x[:-s]
        x = y
        i += 1
    return x


def test_prefix_sum_kat(oracle):
    """prefix_sum.py:39-54: 10^6 PCG32 floats (seed 0) — Hillis-Steele order."""
    x = oracle.rng_stream(0, 0, 1_000_000, 1)[:, 0].copy()
    got = oracle.prefix_sum_f32_hs(x)
    assert np.array_equal(got, _hs_numpy(x))
    np.testing.assert_allclose(got, np.cumsum(x.astype(np.float64)), rtol=1e-4)
    u = np.arange(1, 100, dtype=np.uint32)
    assert np.array_equal(oracle.prefix_sum_u32(u), np.cumsum(u).astype(np.uint32))
    assert np.array_equal(oracle.prefix_sum_u32(u, False), (np.cumsum(u) - u).astype(np.uint32))


def test_multicore_primitive_baselines_equal_sequential(oracle):
    """The OpenMP CPU baselines bench.py times (all host cores) compute the
    same arrays as the sequential restatements, bit for bit."""
    rng = np.random.default_rng(9)
    x = rng.integers(0, 1 << 16, 100003, dtype=np.uint32)
    for inc in (True, False):
        assert np.array_equal(oracle.prefix_sum_u32_mt(x, inc), oracle.prefix_sum_u32(x, inc))
    f = rng.random(70001, dtype=np.float32)
    assert np.array_equal(oracle.prefix_sum_f32_hs_mt(f), oracle.prefix_sum_f32_hs(f))
    p = rng.random((3, 50000), dtype=np.float32)
    for nc in (50000, 97, 1, 1 << 20):
        for a, b in zip(oracle.hashgrid_mt(p, 100, nc), oracle.hashgrid(p, 100, nc)):
            assert np.array_equal(a, b), nc
    idx = rng.integers(0, 1000, 60000, dtype=np.uint32)
    val = rng.random(60000, dtype=np.float32) - 0.5
    for op in (0, 1, 2):
        tgt = rng.random(1000, dtype=np.float32)
        assert np.array_equal(oracle.scatter_reduce_mt(op, tgt, val, idx), oracle.scatter_reduce(op, tgt, val, idx))


def _np_group_by(idx, n_keys):
    """numpy restatement of the device group-by (stable: ascending index)."""
    order = np.argsort(idx, kind="stable").astype(np.uint32)
    size = np.bincount(idx, minlength=n_keys).astype(np.uint32)
    offset = (np.cumsum(size) - size).astype(np.uint32)
    return size, offset, order


def test_scatter_reduce_mul_and_unknown_op(oracle):
    """reductions.py:12 takes any func; the device op table adds mul
    (sequential product per target); an unknown op name raises."""
    from mtx import primitives

    rng = np.random.default_rng(3)
    idx = rng.integers(0, 7, 200).astype(np.uint32)
    val = (0.9 + 0.2 * rng.random(200)).astype(np.float32)
    tgt = np.ones(7, np.float32)
    ref = tgt.copy()
    for i, v in zip(idx, val):
        ref[i] = np.float32(ref[i] * v)
    assert np.array_equal(oracle.scatter_reduce(3, tgt, val, idx), ref)
    assert np.array_equal(oracle.scatter_reduce_mt(3, tgt, val, idx), ref)
    with pytest.raises(TypeError):
        primitives.scatter_reduce_with("xor", tgt, val, idx)


def test_scatter_reduce_callable_fold_rounds():
    """A Python func (reductions.py:12, :53) is folded round by round over the
    group-by (mtx.primitives.fold_rounds; the device provides the grouping,
    here its numpy restatement): the KAT of reductions.py:57-63 (ten targets,
    25 ones, index i % 10 -> 3 3 3 3 3 2 2 2 2 2) and, for a non-commutative
    func and an integer dtype, the sequential loop in ascending index."""
    from mtx import primitives

    idx = (np.arange(25) % 10).astype(np.uint32)
    t = primitives.fold_rounds(lambda a, b: a + b, np.zeros(10, np.float32), np.ones(25, np.float32),
                               *_np_group_by(idx, 10))
    assert np.array_equal(t, np.array([3] * 5 + [2] * 5, np.float32))
    rng = np.random.default_rng(5)
    idx = rng.integers(0, 33, 500).astype(np.uint32)
    val = rng.integers(-9, 9, 500).astype(np.int64)
    func = lambda a, b: 3 * a - b  # noqa: E731  (order-dependent)
    tgt = rng.integers(-5, 5, 40).astype(np.int64)  # targets 33..39 receive nothing
    ref = tgt.copy()
    for i, v in zip(idx, val):
        ref[i] = func(ref[i], v)
    got = primitives.fold_rounds(func, tgt, val, *_np_group_by(idx, 40))
    assert np.array_equal(got, ref) and got.dtype == np.int64
