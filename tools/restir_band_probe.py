"""Per-rank probe of C4 (restirgi.py ReSTIR GI, 1920x1080, props of
restirgi.py:610-620) at N = 8 on ONE GPU: the work one rank of an 8-GPU
row-band render does per frame -- stage A (initial sample + temporal reuse)
and stage B (spatial reuse + final shading + film) over its band of 135 rows
(mtx.distributed.row_bands) -- timed alone, beside the whole frame, with the
per-kernel-class split of both (HIP events). The halo rows a rank would
import from its neighbours between the stages are not exchanged here (no
peers): the timing is the compute a rank does, the P2P halo transfer comes on
top. North-star target: 8 GPUs >= 6x one GPU, i.e. the band frame <= 1/6 of
the whole frame.

    python tools/restir_band_probe.py [--frames 10] [--rank 3] [--world 8]
prints one JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd"), os.path.join(ROOT, "tools"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    import torch

    from bench_workloads import RESTIR_C4
    from mtx import RestirIntegrator, distributed, scene
    from mtx._lib import context

    torch.cuda.set_device(0)
    sc = scene.bedroom(1920, 1080)
    ctx = context(0)
    y0, y1 = distributed.row_bands(sc.height, args.world)[args.rank]

    def run(band):
        integ = RestirIntegrator(RESTIR_C4)
        rows = (y1 - y0) if band else sc.height
        film = torch.empty((rows + 2, sc.width + 2, 4), dtype=torch.float32, device="cuda:0")

        def frame(seed):
            if not band:
                return integ.render_film(sc, seed=seed, spp=1, out=film, stats=True, ctx=ctx)[1]
            a = integ.render_film(sc, seed=seed, spp=1, y0=y0, y1=y1, stage="A", stats=True, ctx=ctx)[1]
            b = integ.render_film(sc, seed=seed, spp=1, y0=y0, y1=y1, stage="B", out=film, stats=True, ctx=ctx)[1]
            return {k: a[k] + b[k] for k in b}

        for k in range(args.warmup):
            frame(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        agg = None
        for k in range(args.frames):
            st = frame(args.warmup + k)
            agg = st if agg is None else {x: agg[x] + st[x] for x in st}
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.frames * 1e3
        f = args.frames
        return ms, {"trace_closest": round(agg["trace_ms"] / f, 3), "trace_shadow_and_visibility": round(agg["shadow_ms"] / f, 3),
                    "shade": round(agg["shade_ms"] / f, 3), "other": round(agg["other_ms"] / f, 3),
                    "trace_launches": int(agg["trace_launches"] / f), "visibility_launches": int(agg["shadow_launches"] / f)}

    full_ms, full_k = run(False)
    band_ms, band_k = run(True)
    out = {"probe": "C4 per-rank band", "film": [sc.width, sc.height], "world": args.world, "rank": args.rank,
           "band_rows": [y0, y1], "frames": args.frames, "full_frame_ms": round(full_ms, 3),
           "band_frame_ms": round(band_ms, 3), "full_over_band": round(full_ms / band_ms, 3),
           "target_full_over_band": 6.0, "full_kernels_ms": full_k, "band_kernels_ms": band_k,
           "note": "band = stage A + stage B of one rank's rows without the halo P2P transfer"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
