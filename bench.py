"""Benchmark: Mpaths/s of the path-mis.py NEE+MIS integrator (BASELINE.json
configs[1]) on the bedroom proxy at 1280x720 spp=256 (the metric's
resolution and spp), one process per GPU.

A step renders ONE 1280x720 film at a fixed global spp=256 (strong scaling:
the job's work is the same at every N). Rank r of N traces the global sample
range [r*256/N, (r+1)*256/N) of every pixel with global-lane seeding
(path.py:156-161: lane = pixel*spp + sample), so the N=1 and N>1 films hold
the same paths; the per-rank films are combined on rank 0 over RCCL by an
all_to_all of film slices, a pairwise rank-tree sum of each slice on its rank
and a gather of the summed slices. A film is the fixed binary tree of 8
partial-slot films (32 samples each at spp 256), a rank at N = 2 / 4 / 8
renders whole slots and the rank tree is the top of the same tree, so the
combined film equals the N=1 film bit for bit. Inputs (scene, BVH) are resident in
HBM before the timed region; the film stays in HBM and only the combine
crosses GPUs. The timed region includes it.

`python bench.py --gpus N` without a torchrun environment starts the N rank
processes itself (torch.distributed.run, before this process touches the
GPU) and exits with their status; under torchrun WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0 (contract in the task statement) with
`roofline` for the closest-hit traversal kernel and `cpu_baseline` (the
oracle/ CPU restatement on a bounded sample, N=1 only).

The roofline names the unit that bounds the traversal: its vector-memory
address path (TA/TCP, "vmem"). The achieved rate is the algorithmic bytes
(32 + 16 + 64 N_node + 36 N_tri per ray, exact visit counts from
the in-kernel counters of one extra, untimed step) over the HIP-event time of
the launches; the peak is that path's byte rate (64 B per CU-cycle, measured
by tools/probes/ta_rate.hip: 1 KiB wave-loads in <= 16 lines at 17 cycles). The
committed rocprofv3 unit counters of the same build (profiles/*_pmc_units.json,
tools/pmc_units.py) give the occupancy beside it: TA busy ~0.8 of the
kernel's cycles at ~0.3 of the byte peak, because a divergent gather costs
the TA one cycle per distinct 128-B line per instruction (the probe: 64
lanes on 64 L1 lines 65 cycles, on L2 lines 142), so the bound is the line
rate of gathers, not bytes. The `hbm` sub-object is the DRAM/fabric side
(FETCH_SIZE x2 + WRITE_SIZE per launch, profiles/*_pmc_traffic.json) against
the 8 TB/s HBM peak. PMC files are used only when their recorded source hash
and bench arguments match this build and this run (otherwise null).
"""
import argparse
import hashlib
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-experiments_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
# MI355X_MICROARCH.md "Indexed rows: gather into LDS": rows shared by every
# workgroup, served from the XCD's L2: 16.8-18.8 TB/s chip-wide (upper end).
L2_GATHER_PEAK_GBS = 18800.0
# vector-memory (TA/TCP) byte path: 1 KiB per 16.9 CU-cycles for a wave64
# dwordx4 load touching <= 16 lines (tools/probes/ta_rate.hip, profiles/r3_ta_rate.txt),
# x 256 CUs x 2.4 GHz
VMEM_PEAK_GBS = round(1024 / 16.9 * 256 * 2.4, 0)
# node and triangle records as the device reads them (triangles packed to 36 B, mtx_scene_upload)
NODE_BYTES, TRI_BYTES, RAY_BYTES, HIT_BYTES, OCC_BYTES = 64, 36, 32, 16, 4
OCC_NODE_BYTES = 80  # the any-hit tree's 8-wide compressed node (mtx.h MTX_OCC_NODE_WORDS)
# SURVEY §8d wavefront path state per lane per bounce, read + written
SHADE_BYTES_PER_PATH_BOUNCE = 2 * 108 + 32


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--spp", type=int, default=256, help="global samples per pixel (split over the ranks)")
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
    p.add_argument("--iterations", type=int, default=200,
                   help="PSSMLT Metropolis iterations (pssmlt.py:208: 200, aggregation when i %% 50 > 40)")
    p.add_argument("--frames", type=int, default=10, help="ReSTIR GI timed frames")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="N>1 ranks: nccl (RCCL, the measurement) or gloo (host-staged device tensors; lets "
                        "several ranks share one GPU in a rehearsal of the N>1 code path)")
    p.add_argument("--master-port", type=int, default=29517, help="rendezvous port when bench.py starts the ranks")
    p.add_argument("--dump-film", default="", help="save rank 0's combined film of the seed-0 step (.npy; tests)")
    return p.parse_args()


def spawn_ranks(args) -> int:
    """Start the N rank processes (one per GPU) under torch.distributed.run.
    Runs before this process makes any GPU call; the ranks are children, not
    an exec of this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={args.master_port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


# Kernel names (rocprofv3's short form) whose PMC traffic / units bench.py
# attaches: the closest-hit and any-hit traversals and path-mis shade.
PMC_KERNELS = {"closest": "mtxd::k_trace_closest<false>", "shadow": "mtxd::k_trace_shadow<false>",
               "shade": "mtxd::k_shade<2>"}


def src_sha() -> str:
    """Hash of the sources that make libmtx.so (kernels, host runtime, shared
    headers, build flags): a PMC profile is valid for the build it measured."""
    h = hashlib.sha256()
    pats = ["mitsuba3-experiments_amd/csrc/*.hip", "mitsuba3-experiments_amd/csrc/*.h",
            "mitsuba3-experiments_amd/csrc/*.cpp", "mitsuba3-experiments_amd/csrc/Makefile",
            "include/*.h", "include/mtx_core/*.h"]
    for f in sorted(x for p in pats for x in glob.glob(os.path.join(ROOT, p))):
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def traffic_key(args) -> str:
    """The bench arguments a PMC profile depends on (per-launch traffic)."""
    if getattr(args, "workload", "path_mis") != "path_mis":
        return f"{args.workload} spp={args.spp} iterations={args.iterations}"
    return f"path_mis {args.width}x{args.height} spp={args.spp} md={args.max_depth} rr={args.rr_depth} chunk={args.chunk}"


def measured_traffic(kernels, key):
    """HBM-side bytes per launch of each kernel in `kernels` from the newest
    committed rocprofv3 PMC summary (profiles/*_pmc_traffic.json, FETCH_SIZE x2
    + WRITE_SIZE, tools/pmc_summary.py) whose src_sha and bench key match this
    build and run. Returns ({kernel: bytes}, source or reason)."""
    sha = src_sha()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=os.path.getmtime)
    reason = "no profiles/*_pmc_traffic.json"
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("src_sha") != sha:
            reason = f"stale: {os.path.basename(f)} src_sha {d.get('src_sha')} != {sha}"
            continue
        if d.get("bench_key") != key:
            reason = f"{os.path.basename(f)}: bench args differ"
            continue
        ks = d.get("kernels", {})
        return {k: (int(ks[k]["hbm_bytes_per_launch"]) if k in ks else None) for k in kernels}, \
            os.path.relpath(f, ROOT)
    return {k: None for k in kernels}, reason


def measured_units(kernels, key):
    """Unit occupancy per launch of each kernel in `kernels` (TA busy, VALU
    busy, ...) from the newest committed profiles/*_pmc_units.json
    (tools/pmc_units.py) whose src_sha and bench key match. Returns
    ({kernel: dict or None}, source or reason)."""
    sha = src_sha()
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_units.json")), key=os.path.getmtime)
    reason = "no profiles/*_pmc_units.json"
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("src_sha") != sha:
            reason = f"stale: {os.path.basename(f)} src_sha {d.get('src_sha')} != {sha}"
            continue
        if d.get("bench_key") != key:
            reason = f"{os.path.basename(f)}: bench args differ"
            continue
        ks = d.get("kernels", {})
        keep = ("ta_busy", "valu_busy", "salu_busy", "l1_l2_read_bytes_per_launch", "ta_cycles_per_vmem",
                "vmem_insts_per_launch")
        return {k: ({x: ks[k][x] for x in keep if x in ks[k]} if k in ks else None) for k in kernels}, \
            os.path.relpath(f, ROOT)
    return {k: None for k in kernels}, reason


def _kernel_entry(ms_per_step, launches, traffic, alg_bytes_per_step=None, alg_peak=None, alg_bound=None):
    e = {"ms_per_step": round(ms_per_step, 3), "launches_per_step": int(launches)}
    launch_s = ms_per_step / 1e3 / max(1, launches)
    if alg_bytes_per_step is not None and ms_per_step > 0:
        ach = alg_bytes_per_step / (ms_per_step / 1e3) / 1e9
        e.update({"alg_bytes_per_launch": int(alg_bytes_per_step / max(1, launches)),
                  "alg_GBps": round(ach, 1), "alg_bound": alg_bound, "alg_peak_GBps": alg_peak,
                  "alg_frac": round(ach / alg_peak, 4)})
    if traffic is not None and launch_s > 0:
        hb = traffic / launch_s / 1e9
        e.update({"hbm_bytes_per_launch": int(traffic), "hbm_GBps": round(hb, 1),
                  "hbm_frac": round(hb / HBM_PEAK_GBS, 4)})
    return e


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.workload == "path_mis" and args.spp < world:
        # checked on every rank before any collective (no rank waits in a gather)
        print(f"bench.py: --spp {args.spp} < {world} ranks: every rank needs >= 1 sample per pixel", file=sys.stderr)
        sys.exit(2)
    if args.workload != "path_mis":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_workloads

        return bench_workloads.run(args)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks may share a GPU (--backend gloo)
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from mtx import PathIntegrator, distributed, scene

    sc = scene.bedroom(width=args.width, height=args.height)
    integ = PathIntegrator({"max_depth": args.max_depth, "rr_depth": args.rr_depth})
    W, H, spp = sc.width, sc.height, args.spp
    s0, s1 = distributed.sample_range(spp, world, rank)
    film = torch.empty((H + 2, W + 2, 4), dtype=torch.float32, device=f"cuda:{local}")

    combined = [film]

    def step(i, stats=False, counters=False):
        r = integ.render_film(sc, seed=i, spp=s1 - s0, spp_total=spp, sample_offset=s0, out=film,
                              stats=stats, chunk_paths=args.chunk, counters=counters)
        if world > 1:
            combined[0] = distributed.reduce_sum(film)  # RCCL all_to_all of slices, slice sums, gather to rank 0
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
        agg = dict(st) if agg is None else {k: agg[k] + v for k, v in st.items()}
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
    if args.dump_film and rank == 0:
        import numpy as np

        np.save(args.dump_film, combined[0].cpu().numpy())

    value = W * H * spp * args.steps / elapsed / 1e6
    K = args.steps
    # rank-local per-step figures (this rank's launches)
    alg_closest = (cnt["rays_closest"] * (RAY_BYTES + HIT_BYTES) + cnt["nodes_closest"] * NODE_BYTES
                   + cnt["tris_closest"] * TRI_BYTES)
    alg_shadow = (cnt["rays_shadow"] * (RAY_BYTES + OCC_BYTES) + cnt["nodes_shadow"] * OCC_NODE_BYTES
                  + cnt["tris_shadow"] * TRI_BYTES)
    launches = max(1, cnt["trace_launches"])
    trace_ms = agg["trace_ms"] / K  # counters off
    trace_s = trace_ms / 1e3
    achieved = alg_closest / trace_s / 1e9 if trace_s > 0 else 0.0
    names = PMC_KERNELS
    traffic, traffic_src = (measured_traffic(list(names.values()), traffic_key(args)) if world == 1
                            else ({k: None for k in names.values()}, "N>1: PMC profiles are N=1"))
    units, units_src = (measured_units(list(names.values()), traffic_key(args)) if world == 1
                        else ({k: None for k in names.values()}, "N>1: PMC profiles are N=1"))
    tc = traffic[names["closest"]]
    uc = units[names["closest"]]
    launch_s = trace_s / launches
    hbm_ach = tc / launch_s / 1e9 if (tc is not None and launch_s > 0) else None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(sc, integ, args)
        kernels = {
            "trace_closest": _kernel_entry(trace_ms, launches, tc, alg_closest, VMEM_PEAK_GBS, "vmem"),
            "trace_shadow": dict(_kernel_entry(agg["shadow_ms"] / K, cnt["shadow_launches"], traffic[names["shadow"]],
                                               alg_shadow, VMEM_PEAK_GBS, "vmem"),
                                 rays_per_step=int(cnt["rays_shadow"]),
                                 node_visits_per_ray=round(cnt["nodes_shadow"] / max(1, cnt["rays_shadow"]), 2),
                                 tri_visits_per_ray=round(cnt["tris_shadow"] / max(1, cnt["rays_shadow"]), 2)),
            "shade": _kernel_entry(agg["shade_ms"] / K, cnt["trace_launches"], traffic[names["shade"]],
                                   cnt["rays_closest"] * SHADE_BYTES_PER_PATH_BOUNCE, HBM_PEAK_GBS, "hbm"),
        }
        for kk, nn in (("trace_closest", names["closest"]), ("trace_shadow", names["shadow"]),
                       ("shade", names["shade"])):
            kernels[kk]["units"] = units[nn]
        # vector-memory wave instructions per ray (PMC SQ_INSTS_VMEM_RD + _WR per launch)
        for kk, rays, nl in (("trace_closest", cnt["rays_closest"], launches),
                             ("trace_shadow", cnt["rays_shadow"], cnt["shadow_launches"])):
            u = kernels[kk]["units"]
            if u and u.get("vmem_insts_per_launch") and rays:
                u["vmem_wave_insts_per_ray"] = round(u["vmem_insts_per_launch"] / (rays / max(1, nl)), 3)
        # the roofline object follows north_star's traversal kernel; the
        # kernel with the most time per step is named beside it
        big = max(kernels, key=lambda k: kernels[k]["ms_per_step"])
        largest = {"kernel": big, "ms_per_step": kernels[big]["ms_per_step"], "bound": kernels[big].get("alg_bound"),
                   "alg_frac": kernels[big].get("alg_frac"), "hbm_frac": kernels[big].get("hbm_frac")}
        out = {
            "metric": "Mpaths/sec on bedroom@1280×720 spp=256, 1/2/4/8 GPUs; HBM GB/s vs peak",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: deterministic bedroom proxy (scene.xml camera/BSDFs/emitters, "
                    f"{sc.n_tris} procedural triangles)",
            "config": {
                "workload": f"path-mis.py NEE+MIS (BASELINE configs[1]) on bedroom-proxy {W}x{H}, global spp={spp} "
                            f"split over {world} rank(s) by sample range, max_depth={args.max_depth}, "
                            f"rr_depth={args.rr_depth}",
                "global_spp": spp,
                "spp_per_rank": s1 - s0,
                "paths_per_step": W * H * spp,
                "parallelism": f"sample-range shards x{world}" + (", RCCL slice-reduce of films to rank 0" if world > 1 else ""),
            },
            "roofline": {
                # the busier of the two units the traversal can saturate, from the
                # build's unit counters (TA 0.75 vs VALU 0.54 in profiles/r3d_pmc_units.json)
                "bound": "vmem" if (uc is None or uc["ta_busy"] >= uc["valu_busy"]) else "valu",
                "kernel": "k_trace_closest (4-wide quantised BVH, closest hit)",
                "achieved": round(achieved, 1),
                "peak": VMEM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / VMEM_PEAK_GBS, 4),
                "traffic": tc,
                "traffic_source": traffic_src,
                "peak_source": "vector-memory (TA/TCP) byte path, 64 B/CU-cycle: tools/probes/ta_rate.hip "
                               "(profiles/r3_ta_rate.txt) x 256 CUs x 2.4 GHz",
                "units": uc,
                "units_source": units_src,
                "bound_reason": "TA (vector-memory address path) is the busiest unit of the kernel (units.ta_busy "
                                "vs units.valu_busy); gathers cost the TA one cycle per distinct 128-B line per "
                                "instruction, so it saturates at a fraction of its byte peak",
                "frac_vs_l2_gather_peak": round(achieved / L2_GATHER_PEAK_GBS, 4),
                "hbm": None if hbm_ach is None else {
                    "achieved": round(hbm_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(hbm_ach / HBM_PEAK_GBS, 4),
                    "bytes_per_launch": tc, "definition": "PMC FETCH_SIZE x2 + WRITE_SIZE per launch / avg launch time"},
                "avg_launch_ms": round(trace_ms / launches, 4),
                "launches_per_step": int(launches),
                "alg_bytes_per_launch": int(alg_closest / launches),
                "rays_per_step": int(cnt["rays_closest"]),
                "node_visits_per_ray": round(cnt["nodes_closest"] / max(1, cnt["rays_closest"]), 2),
                "tri_visits_per_ray": round(cnt["tris_closest"] / max(1, cnt["rays_closest"]), 2),
                "active_lane_frac_node_phase": round(cnt["nodes_closest"] / max(1, 64 * cnt["wave_node_iters"]), 3),
                "tris_per_lane_leaf_step": round(cnt["tris_closest"] / max(1, 64 * cnt["wave_leaf_iters"]), 3),
                "kernel_choice": "north_star's traversal kernel (closest hit); the kernel with the most time "
                                 "per step is `largest_kernel`",
                "largest_kernel": largest,
            },
            "kernels": dict(kernels, other_ms_per_step=round(agg["other_ms"] / K, 3),
                            streams=int(cnt.get("streams", 1)),
                            overlapped=bool(cnt.get("streams", 1) > 1),
                            note=("per-kernel times are summed HIP-event intervals of launches that overlap on "
                                  "two streams (this rank's render ran on two wavefronts): they do not add up "
                                  "to ms_per_step" if cnt.get("streams", 1) > 1 else
                                  "one stream: per-kernel times add up to the step with other_ms")),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_model() -> str:
    """The host CPU's model name as lscpu prints it."""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            if line.strip().startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
            "cpu_model": cpu_model(), "sample": f"full {sc.width}x{sc.height} frame at spp={spp} ({n} paths, {dt:.1f} s), same integrator, "
                      "scene and seed scheme; oracle/oracle.cpp (OpenMP)"}


if __name__ == "__main__":
    main()
