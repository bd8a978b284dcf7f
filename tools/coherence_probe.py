"""Ray-order probe (tuning experiment, GPU): how much does the order of a
wavefront of secondary rays matter to the traversal kernels?

Builds bounce-1-like rays on the bedroom proxy -- camera rays in the bench's
pixel-major order (spp samples of a pixel contiguous), their primary hits,
then one random hemisphere direction per hit (facing back toward the camera)
-- and traces the same rays (mtx_trace_dev, closest and any hit) in four
orders: as generated, stably grouped by direction octant, sorted by
(octant, Morton code of the origin), and shuffled. Hits are order-free, so
every order must return the same hits per ray (checked). Prints one JSON line
per (mode, order) with the best of --reps timings.

    python tools/coherence_probe.py --spp 16
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mitsuba3-experiments_amd"))
from mtx import scene as mscene  # noqa: E402
from mtx.integrators import trace_rays  # noqa: E402


def camera_rays(cam, W, H, spp, gen, dev):
    n = W * H * spp
    i = torch.arange(n, device=dev)
    pix = i // spp
    x = (pix % W).float()
    y = (pix // W).float()
    u = torch.rand((n, 2), generator=gen, device=dev)
    px = (x + u[:, 0]) / W
    py = (y + u[:, 1]) / H
    dl = torch.stack([(1 - 2 * px) * cam.tan_x, (1 - 2 * py) * cam.tan_y, torch.ones_like(px)], 1)
    dl = dl / dl.norm(dim=1, keepdim=True)
    ax, ay, az = (torch.tensor(list(a), device=dev) for a in (cam.axis_x, cam.axis_y, cam.axis_z))
    d = dl[:, :1] * ax + dl[:, 1:2] * ay + dl[:, 2:] * az
    o = torch.tensor(list(cam.origin), device=dev) + d * (cam.near_clip / dl[:, 2:])
    return o, d


def pack(o, d, tmax):
    r = torch.zeros((o.shape[0], 8), dtype=torch.float32, device=o.device)
    r[:, :3] = o
    r[:, 3] = tmax
    r[:, 4:7] = d
    return r.contiguous()


def morton30(p, lo, hi):
    q = ((p - lo) / (hi - lo).clamp_min(1e-12) * 1023).clamp(0, 1023).to(torch.int64)
    code = torch.zeros(p.shape[0], dtype=torch.int64, device=p.device)
    for b in range(10):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return code


def timed(fn, reps):
    best = None
    out = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        best = dt if best is None else min(best, dt)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    sc = mscene.bedroom(width=a.width, height=a.height)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    o, d = camera_rays(sc.camera, a.width, a.height, a.spp, gen, dev)
    big = 3.0e38
    h = trace_rays(sc, pack(o, d, big))
    t = h[:, 0].view(torch.float32)
    ok = torch.isfinite(t)
    p = o[ok] + d[ok] * t[ok, None]
    dc = d[ok]
    w = torch.randn((p.shape[0], 3), generator=gen, device=dev)
    w = w / w.norm(dim=1, keepdim=True)
    w = torch.where(((w * dc).sum(1, keepdim=True) > 0), -w, w)  # back toward the camera side
    org = p - dc * (1e-4 * (1 + p.abs().amax(1, keepdim=True)))
    rays = pack(org, w, big)
    n = rays.shape[0]
    octant = ((w[:, 0] < 0).long() | ((w[:, 1] < 0).long() << 1) | ((w[:, 2] < 0).long() << 2))
    lo, hi = org.amin(0), org.amax(0)
    orders = {
        "generated": torch.arange(n, device=dev),
        "octant": torch.sort(octant, stable=True).indices,
        "octant_morton": torch.sort((octant << 30) | morton30(org, lo, hi), stable=True).indices,
        "shuffled": torch.randperm(n, generator=gen, device=dev),
    }
    ref = {}
    for any_hit in (False, True):
        for name, perm in orders.items():
            rp = rays[perm].contiguous()
            ms, (hits, vis) = timed(lambda: trace_rays(sc, rp, any_hit=any_hit, visits=True), a.reps)
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(n, device=dev)
            hits_o = hits[inv]
            key = "any" if any_hit else "closest"
            if key not in ref:
                ref[key] = hits_o
            same = bool(torch.equal(ref[key], hits_o))
            nv = vis[:, 0].double().mean().item()
            print(json.dumps({"mode": key, "order": name, "rays": n, "ms": round(ms, 3),
                              "mrays_per_s": round(n / ms / 1e3, 1), "node_visits": round(nv, 3),
                              "hits_equal": same}), flush=True)


if __name__ == "__main__":
    main()
