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
    integ = load_dict({"type": "path_test"})

    def render(spp, spp_total, off, y0, y1):
        a = integ.render_args(sc, 4, spp, y0, y1, spp_total, off)
        return oracle.render(sc, a)

    full = distributed.render_sharded(render, sc.height, 4, mode)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["samples", "rows"])
def test_two_rank_combine(tmp_path, oracle, mode):
    from mtx import load_dict, scene

    out = os.path.join(tmp_path, "full.npy")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    sc = scene.bedroom(width=48, height=27, scale=0.02, tex_res=32)
    integ = load_dict({"type": "path_test"})
    if mode == "samples":
        parts = [oracle.render(sc, integ.render_args(sc, 4, 4, 0, sc.height, 8, 4 * r)) for r in range(2)]
        assert np.array_equal(got, parts[0] + parts[1])  # rank-order sum, bit-exact
        ref = oracle.render(sc, integ.render_args(sc, 4, 8, 0, sc.height, 8, 0))
    else:
        ref = oracle.render(sc, integ.render_args(sc, 4, 4, 0, sc.height))
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-6)
