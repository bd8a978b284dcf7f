"""One rank's share of the N-GPU headline render on one GPU (tuning probe):
the bench's path-mis frame at global spp 256, samples [s0, s1) of rank
`--rank` of `--world` (bench.py's distributed.sample_range), timed like
bench.py's steps but without the cross-rank film combine. Prints one JSON
line per world size.

    python tools/rank_shard_probe.py --worlds 1 2 4 8 --steps 5
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mitsuba3-experiments_amd"))
import torch  # noqa: E402

from mtx import PathIntegrator, distributed  # noqa: E402
from mtx import scene as mscene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--rank", type=int, default=-1, help="rank of the shard (default: the last)")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    sc = mscene.bedroom()
    integ = PathIntegrator({"max_depth": 8, "rr_depth": 2})  # bench.py's integrator
    film = torch.empty((sc.height + 2, sc.width + 2, 4), dtype=torch.float32, device="cuda:0")
    for world in a.worlds:
        rank = a.rank if a.rank >= 0 else world - 1
        s0, s1 = distributed.sample_range(a.spp, world, rank)
        for i in range(a.warmup):
            integ.render_film(sc, seed=i, spp=s1 - s0, spp_total=a.spp, sample_offset=s0, out=film)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            integ.render_film(sc, seed=i, spp=s1 - s0, spp_total=a.spp, sample_offset=s0, out=film)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        print(json.dumps({"world": world, "rank": rank, "samples": [s0, s1], "ms_per_step": round(ms, 3)}), flush=True)


if __name__ == "__main__":
    main()
