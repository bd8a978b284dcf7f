"""How much does the order of a bounce's rays change closest-hit traversal
time? (ray-order experiment.) The wavefront keeps the
raygen order: pixel-major, a pixel's samples contiguous (kernels.hip
k_raygen_camera), so a wave's secondary rays start at one pixel's hit points
and point in random cosine-weighted directions. This script traces the same
rays in several orders through mtx_trace (k_trace_raw, closest hit) and prints
the launch order; the durations come from the rocprofv3 kernel trace
(tools/ray_order_summary.py pairs them up).

Orders: natural; sorted by direction octant within blocks of 256 / 1024 rays
(what an octant-binned append in k_shade would produce); sorted by a finer
direction bin (octahedral 4x4 per hemisphere) within 256; globally shuffled.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-experiments_amd")]


def camera_rays(sc, pixels, spp, seed=0):
    rng = np.random.default_rng(seed)
    cam = sc.camera
    W, H = cam.width, cam.height
    px = np.repeat(pixels, spp)
    x = (px % W).astype(np.float32) + rng.random(len(px), dtype=np.float32)
    y = (px // W).astype(np.float32) + rng.random(len(px), dtype=np.float32)
    tx, ty = np.float32(cam.tan_x), np.float32(cam.tan_y)
    dl = np.stack([(1 - 2 * x / W) * tx, (1 - 2 * y / H) * ty, np.ones(len(px), np.float32)], 1)
    dl /= np.linalg.norm(dl, axis=1, keepdims=True)
    M = np.stack([np.array(cam.axis_x), np.array(cam.axis_y), np.array(cam.axis_z)], 1).astype(np.float32)
    rays = np.zeros((len(px), 8), np.float32)
    rays[:, 0:3] = np.array(cam.origin, np.float32)
    rays[:, 4:7] = dl @ M.T
    rays[:, 3] = 3e38
    return rays


def bounce_rays(sc, rays, hits, seed=1):
    rng = np.random.default_rng(seed)
    h = hits.reshape(-1, 4)
    t = h[:, 0].view(np.float32)
    prim = h[:, 1]
    ok = prim != 0xFFFFFFFF
    g = sc.tri_geom.reshape(-1, 3, 4)[prim[ok]]
    d = rays[ok, 4:7]
    nrm = np.cross(g[:, 1, :3], g[:, 2, :3])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm *= -np.sign(np.sum(nrm * d, 1, keepdims=True))
    p = rays[ok, 0:3] + t[ok, None] * d + nrm * 1e-3
    u1, u2 = rng.random(len(p)), rng.random(len(p))
    r, phi = np.sqrt(u1), 2 * np.pi * u2
    a = np.where(np.abs(nrm[:, :1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
    tt = np.cross(nrm, a)
    tt /= np.linalg.norm(tt, axis=1, keepdims=True)
    bb = np.cross(nrm, tt)
    dd = tt * (r * np.cos(phi))[:, None] + bb * (r * np.sin(phi))[:, None] + nrm * np.sqrt(1 - u1)[:, None]
    out = np.zeros((len(p), 8), np.float32)
    out[:, 0:3], out[:, 4:7], out[:, 3] = p, dd, 3e38
    return out


def octant(r):
    d = r[:, 4:7]
    return ((d[:, 0] < 0).astype(np.int64) | ((d[:, 1] < 0).astype(np.int64) << 1) |
            ((d[:, 2] < 0).astype(np.int64) << 2))


def fine_bin(r):
    d = r[:, 4:7] / np.abs(r[:, 4:7]).sum(1, keepdims=True)  # octahedral map
    u = np.clip(((d[:, 0] + 1) * 2).astype(np.int64), 0, 3)
    v = np.clip(((d[:, 1] + 1) * 2).astype(np.int64), 0, 3)
    return ((d[:, 2] < 0).astype(np.int64) << 4) | (u << 2) | v


def block_sort(r, key, block):
    n = len(r)
    blk = np.arange(n) // block
    return r[np.lexsort((np.arange(n), key, blk))]


def pixel_orders(W, H, y0, rows):
    """The same band of pixels in scanline order and in tile orders."""
    ys, xs = np.meshgrid(np.arange(y0, y0 + rows), np.arange(W), indexing="ij")
    ys, xs = ys.reshape(-1), xs.reshape(-1)
    out = {"scanline": ys * W + xs}
    for tw, th in ((8, 8), (16, 16), (32, 8)):
        key = np.lexsort((xs % tw, (ys - y0) % th, xs // tw, (ys - y0) // th))
        out[f"tile{tw}x{th}"] = (ys * W + xs)[key]
    return out


def main_pixels(spp=256, rows=64, reps=3):
    """Raygen pixel order: scanline (k_raygen_camera) vs tiles, camera and
    bounce rays of a 1280 x `rows` band."""
    from mtx import context, integrators, scene
    from mtx._lib import check, lib

    sc = scene.bedroom()
    ctx = context(0)
    integrators._bind_scene(ctx, sc)

    def trace(r, tag):
        r = np.ascontiguousarray(r, np.float32)
        hits = np.zeros(4 * len(r), np.uint32)
        check(lib().mtx_trace(ctx.handle, len(r), r.ctypes.data, 0, hits.ctypes.data, None), "mtx_trace")
        print(json.dumps({"launch": tag, "rays": len(r)}), flush=True)
        return hits

    sets = {}
    for name, pix in pixel_orders(sc.camera.width, sc.camera.height, 300, rows).items():
        cam = camera_rays(sc, pix, spp)
        sets["camera_" + name] = cam
        sets["bounce_" + name] = bounce_rays(sc, cam, trace(cam, "warmup"))
    for k in range(reps):
        for name, r in sets.items():
            trace(r, name)


def main(spp=256, reps=3):
    from mtx import context, integrators, scene
    from mtx._lib import check, lib

    sc = scene.bedroom()
    W, H = sc.camera.width, sc.camera.height
    # 64 K pixels spread over the frame (every 2nd column, every 7th row)
    pix = (np.arange(0, H, 7)[:, None] * W + np.arange(0, W, 2)[None, :]).reshape(-1)[: 65536 * 256 // spp]
    ctx = context(0)
    integrators._bind_scene(ctx, sc)

    def trace(r, tag):
        r = np.ascontiguousarray(r, np.float32)
        hits = np.zeros(4 * len(r), np.uint32)
        check(lib().mtx_trace(ctx.handle, len(r), r.ctypes.data, 0, hits.ctypes.data, None), "mtx_trace")
        print(json.dumps({"launch": tag, "rays": len(r)}), flush=True)
        return hits

    cam = camera_rays(sc, pix, spp)
    h0 = trace(cam, "warmup")
    b1 = bounce_rays(sc, cam, h0)
    rng = np.random.default_rng(7)
    orders = {
        "camera_natural": cam,
        "camera_shuffled": cam[rng.permutation(len(cam))],
        "bounce_natural": b1,
        "bounce_octant_256": block_sort(b1, octant(b1), 256),
        "bounce_octant_1024": block_sort(b1, octant(b1), 1024),
        "bounce_fine_256": block_sort(b1, fine_bin(b1), 256),
        "bounce_fine_1024": block_sort(b1, fine_bin(b1), 1024),
        "bounce_shuffled": b1[rng.permutation(len(b1))],
    }
    ref = None
    for k in range(reps):
        for name, r in orders.items():
            h = trace(r, name)
            if name == "bounce_natural" and k == 0:
                ref = h
    # the bounce hits are the same rays' hits whatever the order
    assert ref is not None


if __name__ == "__main__":
    main_pixels() if len(sys.argv) > 1 and sys.argv[1] == "pixels" else main()
