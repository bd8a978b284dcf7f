"""Benchmark: Mpaths/s of the path-mis.py NEE+MIS integrator (BASELINE.json
configs[1]) on the bedroom proxy at 1280x720 spp=256 (the metric's
resolution and spp), one process per GPU.

A step renders the full 1280x720 film at `--spp` samples per pixel on every
rank; rank r traces the global sample range [r*spp, (r+1)*spp) of every pixel
(weak scaling: per-GPU work is fixed, the job's spp grows with N), and the
per-rank films are gathered to rank 0 over RCCL and summed in rank order.
Inputs (scene, BVH) are resident in HBM before the timed region; the film
stays in HBM and only the gather crosses GPUs.

Prints ONE JSON line on rank 0 (contract in the task statement) with
`roofline` for the closest-hit traversal kernel (HIP-event time per launch
over the timed region; algorithmic bytes from the in-kernel visit counters of
one extra, untimed step with the same seed as the first timed step) and
`cpu_baseline` (the oracle/ CPU restatement on a bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
NODE_BYTES, TRI_BYTES, RAY_BYTES, HIT_BYTES = 64, 48, 32, 16


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--width", type=int, default=1280)
    p.add_argument("--height", type=int, default=720)
    p.add_argument("--max-depth", type=int, default=8)
    p.add_argument("--rr-depth", type=int, default=2)
    p.add_argument("--chunk", type=int, default=0, help="wavefront paths per chunk (0 = library default)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU time of the baseline sample")
    p.add_argument("--workload", default="path_mis", choices=["path_mis", "pssmlt", "pssmltpath", "restir", "nrc", "prims", "field", "nerad"],
                   help="path_mis = the driver's headline line (default); the others measure the remaining "
                        "SURVEY §8 configurations on one GPU (C3 PSSMLT, C4 ReSTIR GI, C5 NRC, primitives)")
    p.add_argument("--iterations", type=int, default=20, help="PSSMLT Metropolis iterations (C3 short variant)")
    p.add_argument("--frames", type=int, default=10, help="ReSTIR GI timed frames")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="N>1 ranks: nccl (RCCL, the measurement) or gloo (host-staged device tensors; lets "
                        "several ranks share one GPU in a rehearsal of the N>1 code path)")
    return p.parse_args()


def main():
    args = parse()
    if args.workload != "path_mis":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_workloads

        return bench_workloads.run(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks may share a GPU (--backend gloo)
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from mtx import PathIntegrator, scene

    sc = scene.bedroom(width=args.width, height=args.height)
    integ = PathIntegrator({"max_depth": args.max_depth, "rr_depth": args.rr_depth})
    W, H, spp = sc.width, sc.height, args.spp
    film = torch.empty((H + 2, W + 2, 4), dtype=torch.float32, device=f"cuda:{local}")
    from mtx import distributed

    def step(i, stats=False, counters=False):
        r = integ.render_film(sc, seed=i, spp=spp, spp_total=spp * world, sample_offset=spp * rank, out=film,
                              stats=stats, chunk_paths=args.chunk, counters=counters)
        if world > 1:
            distributed.gather_sum(film)  # RCCL all_gather, rank-order sum on rank 0
        return r[1] if stats else None

    for i in range(args.warmup):
        step(1000 + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agg = None
    for i in range(args.steps):
        st = step(i, stats=True)
        if agg is None:
            agg = dict(st)
        else:
            for k, v in st.items():
                agg[k] += v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}" if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # visit counters (deterministic): one untimed step, same seed as step 0
    cnt = step(0, stats=True, counters=True)

    paths_per_rank = W * H * spp
    value = world * paths_per_rank * args.steps / elapsed / 1e6
    # roofline of the dominant kernel: closest-hit traversal
    alg_bytes = (cnt["rays_closest"] * (RAY_BYTES + HIT_BYTES) + cnt["nodes_closest"] * NODE_BYTES
                 + cnt["tris_closest"] * TRI_BYTES)  # per step
    launches = max(1, cnt["trace_launches"])  # per step
    trace_s = agg["trace_ms"] / 1e3 / args.steps  # per step, counters off
    achieved = alg_bytes / trace_s / 1e9 if trace_s > 0 else 0.0

    traffic, traffic_src = measured_traffic("mtxd::k_trace_closest<false>")
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(sc, integ, args)
        out = {
            "metric": "Mpaths/sec on bedroom@1280×720 spp=256, 1/2/4/8 GPUs; HBM GB/s vs peak",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: deterministic bedroom proxy (scene.xml camera/BSDFs/emitters, "
                    f"{sc.n_tris} procedural triangles)",
            "config": {
                "workload": f"path-mis.py NEE+MIS (BASELINE configs[1]) on bedroom-proxy {W}x{H}, spp={spp} per GPU "
                            f"(global sample range per rank), max_depth={args.max_depth}, rr_depth={args.rr_depth}",
                "global_spp": spp * world,
                "paths_per_step": paths_per_rank * world,
                "parallelism": f"sample-range shards x{world}, RCCL all_gather of films",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_trace_closest (4-wide quantised BVH, closest hit)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_ms": round(trace_s * 1e3 / launches, 4),
                "launches_per_step": int(launches),
                "alg_bytes_per_launch": int(alg_bytes / launches),
                "rays_per_step": int(cnt["rays_closest"]),
                "node_visits_per_ray": round(cnt["nodes_closest"] / max(1, cnt["rays_closest"]), 2),
                "tri_visits_per_ray": round(cnt["tris_closest"] / max(1, cnt["rays_closest"]), 2),
                "simd_util_node_phase": round(cnt["nodes_closest"] / max(1, 64 * cnt["wave_node_iters"]), 3),
                "simd_util_leaf_phase": round(cnt["tris_closest"] / max(1, 64 * cnt["wave_leaf_iters"]), 3),
            },
            "kernels_ms_per_step": {
                "trace_closest": round(agg["trace_ms"] / args.steps, 3),
                "trace_shadow": round(agg["shadow_ms"] / args.steps, 3),
                "shade": round(agg["shade_ms"] / args.steps, 3),
                "other": round(agg["other_ms"] / args.steps, 3),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measured_traffic(kernel):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (profiles/*_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE, made by
    tools/profile_session.sh + tools/pmc_summary.py on this bench command)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return int(k["hbm_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def cpu_baseline(sc, integ, args):
    """oracle/ (the CPU restatement, OpenMP over the host cores) on a bounded
    sample of the same workload: the full 1280x720 frame at a reduced spp,
    sized to about `cpu_seconds` of CPU time after a 1-spp calibration run."""
    import binding as oracle

    oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    a1 = integ.render_args(sc, 0, 1)
    t0 = time.perf_counter()
    oracle.render(sc, a1)
    t1 = time.perf_counter() - t0
    spp = max(1, min(64, int(round(args.cpu_seconds / max(t1, 1e-3)))))
    a = integ.render_args(sc, 0, spp)
    t0 = time.perf_counter()
    oracle.render(sc, a)
    dt = time.perf_counter() - t0
    n = sc.width * sc.height * spp
    return {"value": round(n / dt / 1e6, 4), "unit": "Mpaths/s", "cores": threads, "kind": "port",
            "sample": f"full {sc.width}x{sc.height} frame at spp={spp} ({n} paths, {dt:.1f} s), same integrator, "
                      "scene and seed scheme; oracle/oracle.cpp (OpenMP)"}


if __name__ == "__main__":
    main()
