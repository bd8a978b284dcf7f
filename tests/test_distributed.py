"""N>1 path on CPU: world_size 2 over gloo. Each rank renders its shard with
the CPU restatement (the HIP renderer needs a GPU; the combine logic is the
same code bench.py uses), rank 0 checks the combined film."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_path):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import binding as oracle
    from mtx import distributed, load_dict, scene

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scene.bedroom(width=48, height=27, scale=0.02, tex_res=32)
    if mode == "chains":  # PSSMLT: chain range of every pixel per rank
        sc = sc.with_film(24, 12)
        integ = load_dict({"type": "pssmlt_simple", "iterations": 45})

        def render(spp, spp_total, off, y0, y1):
            return oracle.pssmlt_render(sc, integ.render_args(sc, 4, spp, y0, y1, spp_total, off), 45)

        full = distributed.render_sharded(render, sc.height, 4, "samples")
    else:
        integ = load_dict({"type": "path_test"})

        def render(spp, spp_total, off, y0, y1):
            a = integ.render_args(sc, 4, spp, y0, y1, spp_total, off)
            return oracle.render(sc, a)

        full = distributed.render_sharded(render, sc.height, 8 if mode == "samples" else 4, mode)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [8, 4, 3])
def test_sample_shards_combine_to_the_one_rank_film(tmp_path, oracle, world):
    """GPU-count invariance: 8 ranks of 1 sample (one film
    slot per rank, the 8-GPU node) and 4 ranks of 2 samples (2 whole slots
    each) combine to the one-rank spp-8 film bit for bit (lane seeding
    path.py:156-161: a sample's lane is the same at every N); 3 ranks (the
    shards split slots) equal it up to summation order (rtol 2e-6)."""
    from mtx import load_dict, scene

    out = os.path.join(tmp_path, "full.npy")
    mp.start_processes(_worker, args=(world, _free_port(), "samples", out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    sc = scene.bedroom(width=48, height=27, scale=0.02, tex_res=32)
    integ = load_dict({"type": "path_test"})
    ref = oracle.render(sc, integ.render_args(sc, 4, 8, 0, sc.height, 8, 0))
    if world in (4, 8):
        assert np.array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-6)
    assert ref[..., 3].sum() > 0


@pytest.mark.parametrize("mode", ["samples", "rows", "chains"])
def test_two_rank_combine(tmp_path, oracle, mode):
    from mtx import load_dict, scene

    out = os.path.join(tmp_path, "full.npy")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    sc = scene.bedroom(width=48, height=27, scale=0.02, tex_res=32)
    integ = load_dict({"type": "path_test"})
    if mode == "chains":
        # pssmlt.py chains [2r, 2r+2) of every pixel on rank r (4 chains), 45
        # iterations (aggregation window 41-44 included): the sum of the shards
        # equals the one-rank film up to the summation order (rtol 2e-6)
        sc = sc.with_film(24, 12)
        integ = load_dict({"type": "pssmlt_simple", "iterations": 45})
        parts = [oracle.pssmlt_render(sc, integ.render_args(sc, 4, 2, 0, sc.height, 4, 2 * r), 45) for r in range(2)]
        assert np.array_equal(got, parts[0] + parts[1])  # rank-order sum, bit-exact
        ref = oracle.pssmlt_render(sc, integ.render_args(sc, 4, 4, 0, sc.height), 45)
        assert ref[..., 3].sum() > 0
        np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-6)
        return
    if mode == "samples":
        # the film's 8 partial slots (one sample each at spp 8): each rank
        # renders 4 whole slots and the rank sum is the top of the slot tree,
        # so the combined film IS the one-rank film, bit for bit
        ref = oracle.render(sc, integ.render_args(sc, 4, 8, 0, sc.height, 8, 0))
        assert np.array_equal(got, ref)
        return
    else:
        ref = oracle.render(sc, integ.render_args(sc, 4, 4, 0, sc.height))
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-6)


def _halo_worker(rank, world, port, height, halo, out_dir):
    """ReSTIR row-band halo exchange (mtx.distributed.exchange_halos) with a
    fake state: each rank owns rows of two plane stacks filled with a value
    that encodes (which, plane, row, lane); after the exchange every rank must
    hold its neighbours' halo rows exactly."""
    import sys

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd")]
    import torch
    import torch.distributed as dist

    from mtx import distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y0, y1 = distributed.row_bands(height, world)[rank]
    lanes = 5

    def truth(which, planes):
        w = 0 if which == "sample" else 1
        p = torch.arange(planes).view(planes, 1, 1, 1)
        r = torch.arange(height).view(1, height, 1, 1)
        l = torch.arange(lanes).view(1, 1, lanes, 1)
        c = torch.arange(4).view(1, 1, 1, 4)
        return (((w * 10 + p) * 1000 + r) * 100 + l) * 10 + c + 0.0

    state = {}
    for which, planes in (("sample", 5), ("temporal", 6)):
        s = torch.full((planes, height, lanes, 4), -1.0)
        s[:, y0:y1] = truth(which, planes)[:, y0:y1]
        state[which] = s

    def export_rows(which, row0, nrows):
        return state[which][:, row0:row0 + nrows].contiguous()

    def import_rows(which, row0, t):
        state[which][:, row0:row0 + t.shape[1]] = t

    distributed.exchange_halos(export_rows, import_rows, y0, y1, height, halo)
    ok = True
    lo, hi = max(0, y0 - halo), min(height, y1 + halo)
    for which, planes in (("sample", 5), ("temporal", 6)):
        t = truth(which, planes)
        ok &= bool(torch.equal(state[which][:, lo:hi], t[:, lo:hi]))
        ok &= bool((state[which][:, :lo] == -1).all()) and bool((state[which][:, hi:] == -1).all())
    np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.array([ok]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height,halo", [(2, 27, 10), (3, 40, 10), (4, 16, 3)])
def test_restir_halo_exchange(tmp_path, world, height, halo):
    mp.start_processes(_halo_worker, args=(world, _free_port(), height, halo, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert bool(np.load(os.path.join(tmp_path, f"ok{r}.npy"))[0]), f"rank {r}"


def _prev_worker(rank, world, port, height, out_dir):
    """gather_prev_samples with a fake state: each rank holds only its band of
    the previous frame's samples; afterwards every rank holds the whole film's."""
    import sys

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd")]
    import torch
    import torch.distributed as dist

    from mtx import distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y0, y1 = distributed.row_bands(height, world)[rank]
    lanes = 3
    truth = torch.arange(5 * height * lanes * 4, dtype=torch.float32).view(5, height, lanes, 4)
    state = torch.full_like(truth, -1.0)
    state[:, y0:y1] = truth[:, y0:y1]

    def export_rows(which, row0, nrows):
        assert which == "prev_sample"
        return state[:, row0:row0 + nrows].contiguous()

    def import_rows(which, row0, t):
        assert which == "prev_sample" and not (y0 <= row0 < y1)
        state[:, row0:row0 + t.shape[1]] = t

    distributed.gather_prev_samples(export_rows, import_rows, y0, y1, height)
    np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.array([bool(torch.equal(state, truth))]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height", [(2, 27), (3, 10)])
def test_restir_moving_camera_gathers_prev_samples(tmp_path, world, height):
    """A moving camera reprojects into any band (restirgi.py:374-383): the
    previous frame's samples of the whole film reach every rank (ragged bands)."""
    mp.start_processes(_prev_worker, args=(world, _free_port(), height, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert bool(np.load(os.path.join(tmp_path, f"ok{r}.npy"))[0]), f"rank {r}"


def test_sample_range_needs_a_sample_per_rank():
    """spp < world would leave a rank with an empty range (mtx_render
    rejects spp 0) while the others wait in the gather: every rank raises alike."""
    from mtx import distributed

    assert [distributed.sample_range(256, 8, r) for r in (0, 7)] == [(0, 32), (224, 256)]
    assert [distributed.sample_range(3, 2, r) for r in range(2)] == [(0, 1), (1, 3)]
    for r in range(4):
        with pytest.raises(ValueError):
            distributed.sample_range(3, 4, r)


def test_halo_plan_edges():
    from mtx import distributed

    # first band: nothing above; last band: nothing below
    su, sd, ru, rd = distributed.halo_plan(0, 10, 30, 4)
    assert ru == (0, 0) and sd == (6, 4) and rd == (10, 4)
    su, sd, ru, rd = distributed.halo_plan(20, 30, 30, 4)
    assert rd == (30, 0) and su == (20, 4) and ru == (16, 4)


def _scan_worker(rank, world, port, sizes, out_path):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import binding as oracle
    from mtx import distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = _scan_input(sum(sizes))
    lo = sum(sizes[:rank])
    part = x[lo: lo + sizes[rank]]
    res = [distributed.prefix_sum_sharded(part, inclusive=inc, scan=oracle.prefix_sum_u32) for inc in (True, False)]
    np.savez(out_path + f".{rank}.npz", inc=res[0], exc=res[1])
    dist.barrier()
    dist.destroy_process_group()


def _scan_input(n):
    # values near 2^32 so the running sum wraps several times
    rng = np.random.default_rng(11)
    return (rng.integers(0, 1 << 32, n, dtype=np.uint64)).astype(np.uint32)


@pytest.mark.parametrize("sizes", [(5000, 3001), (0, 777), (4096, 0, 123)])
def test_prefix_sum_sharded(tmp_path, oracle, sizes):
    """u32 scan sharded as local scan + all_gather of totals +
    offset equals the single-array scan bit for bit (ragged and empty slices)."""
    world = len(sizes)
    out = os.path.join(tmp_path, "scan")
    mp.start_processes(_scan_worker, args=(world, _free_port(), sizes, out), nprocs=world, join=True,
                       start_method="spawn")
    x = _scan_input(sum(sizes))
    for inc in (True, False):
        got = np.concatenate([np.load(out + f".{r}.npz")["inc" if inc else "exc"] for r in range(world)])
        assert got.dtype == np.uint32
        assert np.array_equal(got, oracle.prefix_sum_u32(x, inclusive=inc))


def _reduce_worker(rank, world, port, out_path):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd")]
    import torch
    import torch.distributed as dist

    from mtx import distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for shape in [(7, 9, 4), (5, 7, 4), (1, 1, 1)]:
        g = torch.Generator().manual_seed(1000 * rank + shape[0])
        film = torch.randn(shape, generator=g, dtype=torch.float32) * 1e3
        a = distributed.gather_sum(film)
        b = distributed.reduce_sum(film)
        if rank == 0:
            res.append(bool(torch.equal(a, b)) and a.shape == film.shape)
    if rank == 0:
        np.save(out_path, np.array(res))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_reduce_sum_matches_gather_sum(tmp_path, world):
    """The sliced reduction (all_to_all + per-slice rank-tree sum + gather)
    is bit-identical to the gather-then-tree-sum on rank 0, incl. films whose
    size is not a multiple of the world size."""
    out = os.path.join(tmp_path, "ok.npy")
    mp.start_processes(_reduce_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    assert np.load(out).all()
