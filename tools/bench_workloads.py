"""Single-GPU measurements of the SURVEY §8 configurations other than the
headline path-mis line (run through `python bench.py --workload X`; this
module is imported by bench.py, which sets up sys.path):

  pssmlt  C3  pssmltsimple.py PSSMLT, bedroom 1280x720, 256 chains/pixel,
              --iterations Metropolis iterations (200 = pssmlt.py:208, default)
  pssmltpath  the same chains with pssmltpath.py's NEE + MIS proposals
  restir  C4  restirgi.py ReSTIR GI, bedroom 1920x1080, props of
              restirgi.py:610-620, --frames timed frames
  nrc     C5  nrc.py NRC path segments, bedroom 1280x720 spp 4
  prims       prefix_sum.py / hashgrid.py / reductions.py at the §8d sizes

Each prints one JSON line per measurement with the same fields as bench.py:
`roofline` for the dominant kernel and `cpu_baseline` from oracle/ on a
bounded sample. Inputs are resident on the device before the timed region.
"""
import json
import os
import time

import numpy as np

import bench

NODE_BYTES, TRI_BYTES, RAY_BYTES, HIT_BYTES = bench.NODE_BYTES, bench.TRI_BYTES, bench.RAY_BYTES, bench.HIT_BYTES


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


TRACE_KERNEL = "mtxd::k_trace_closest<false>"


def _trace_roofline(cnt, trace_ms_per_unit, units_label, timed_launches=None, args=None):
    """The headline's roofline definition (bench.py) for a workload's
    closest-hit launches: algorithmic bytes over HIP-event time against the
    vector-memory byte peak, with the PMC traffic (HBM side) and unit
    occupancy of the committed profiles/*_pmc_{traffic,units}.json whose
    source hash and bench key (bench.traffic_key: workload, spp, iterations)
    match this build and run, else null.

    `cnt`: visit counters of one untimed run. When that run is shorter than
    the timed unit (PSSMLT: 20 of 200 iterations), `timed_launches` is the
    timed unit's launch count: the bytes per launch come from the counter run
    and are scaled to the timed launches."""
    alg = (cnt["rays_closest"] * (RAY_BYTES + HIT_BYTES) + cnt["nodes_closest"] * NODE_BYTES
           + cnt["tris_closest"] * TRI_BYTES)
    launches = max(1, cnt["trace_launches"])
    if timed_launches:
        alg = alg / launches * timed_launches
        launches = max(1, int(round(timed_launches)))
    s = trace_ms_per_unit / 1e3
    ach = alg / s / 1e9 if s > 0 else 0.0
    if args is not None:
        key = bench.traffic_key(args)
        tr, tsrc = bench.measured_traffic([TRACE_KERNEL], key)
        un, usrc = bench.measured_units([TRACE_KERNEL], key)
    else:
        tr, tsrc, un, usrc = {TRACE_KERNEL: None}, "no bench key", {TRACE_KERNEL: None}, "no bench key"
    tc, uc = tr[TRACE_KERNEL], un[TRACE_KERNEL]
    launch_s = s / launches
    hbm = None
    if tc is not None and launch_s > 0:
        hb = tc / launch_s / 1e9
        hbm = {"achieved": round(hb, 1), "peak": bench.HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hb / bench.HBM_PEAK_GBS, 4), "bytes_per_launch": tc,
               "definition": "PMC FETCH_SIZE x2 + WRITE_SIZE per launch / avg launch time"}
    return {"bound": "vmem" if (uc is None or uc["ta_busy"] >= uc["valu_busy"]) else "valu",
            "kernel": "k_trace_closest (closest hit)",
            "achieved": round(ach, 1), "peak": bench.VMEM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / bench.VMEM_PEAK_GBS, 4), "traffic": tc, "traffic_source": tsrc,
            "units": uc, "units_source": usrc, "hbm": hbm,
            "peak_source": "vector-memory (TA/TCP) byte path, as bench.py's headline roofline",
            "avg_launch_ms": round(trace_ms_per_unit / launches, 4), "launches_per_" + units_label: int(launches),
            "alg_bytes_per_launch": int(alg / launches),
            "node_visits_per_ray": round(cnt["nodes_closest"] / max(1, cnt["rays_closest"]), 2),
            "tri_visits_per_ray": round(cnt["tris_closest"] / max(1, cnt["rays_closest"]), 2)}


def _line(metric, value, unit, steps, warmup, ms, config, roofline, cpu, extra=None, dtype="f32"):
    if isinstance(cpu, dict) and "cpu_model" not in cpu:
        cpu = dict(cpu, cpu_model=bench.cpu_model())
    out = {"metric": metric, "value": round(value, 4), "unit": unit, "n_gpus": 1, "steps": steps, "warmup": warmup,
           "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": dtype, "data": "synthetic: deterministic bedroom proxy / seeded PCG32 inputs",
           "config": config, "roofline": roofline, "cpu_baseline": cpu}
    if extra:
        out.update(extra)
    print(json.dumps(out), flush=True)


def _sync():
    import torch

    torch.cuda.synchronize()


# ------------------------------------------------------- ranks (C3, C4) --
class Ranks:
    """One process per GPU (torchrun env) or a single process. C3 and C4 are
    strong-scaling row bands of one film: each rank owns rows
    [y0, y1); the timed region is bracketed by barrier + synchronize and the
    elapsed time is the max over ranks. backend "nccl" is RCCL; "gloo"
    (--backend gloo) stages device tensors through the host so that several
    ranks can share one GPU in a rehearsal."""

    def __init__(self, args, height):
        import torch
        import torch.distributed as dist

        from mtx import distributed

        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.dev)
        if self.world > 1:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.dev))
            else:
                dist.init_process_group(args.backend)
        self.y0, self.y1 = distributed.row_bands(height, self.world)[self.rank]

    def barrier(self):
        import torch
        import torch.distributed as dist

        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_elapsed(self, t):
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return t
        x = torch.tensor([t], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            x = x.cuda()
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return float(x.item())

    def gather(self, band, height):
        from mtx import distributed

        if self.world > 1:
            distributed.gather_bands(band, self.y0, self.y1, height)

    def parallelism(self):
        return f"row bands x{self.world}" + (", RCCL all_gather of band films" if self.world > 1 else "")

    def close(self):
        import torch.distributed as dist

        if self.world > 1:
            dist.destroy_process_group()


def _sum_stats(a, b):
    return dict(b) if a is None else {x: a[x] + b[x] for x in b}


# --------------------------------------------------------------- PSSMLT (C3) --
def pssmlt(args, with_nee=False):
    """Pssmlt.render (pssmlt.py:167-228) on the reference's own schedule: 200
    iterations by default (large step every 50, aggregation + block.put when
    i % 50 > 40, :206-219), so the splat phase is inside the timed region.
    N > 1: every rank runs the chain range [r*spp/N, (r+1)*spp/N) of every
    pixel (chains never leave their pixel, pssmlt.py:250-254; global-lane
    seeding keeps each chain identical to the one-GPU render), films are
    gathered to rank 0 and summed in rank order: the same work split as the
    headline's sample shards, balanced whatever the scene's row costs."""
    import binding as oracle
    import torch
    from mtx import PssmltPath, PssmltSimple, distributed, scene

    sc = scene.bedroom(1280, 720)
    rk = Ranks(args, sc.height)
    spp, it = args.spp, args.iterations
    s0, s1 = distributed.sample_range(spp, rk.world, rk.rank)
    cls = PssmltPath if with_nee else PssmltSimple
    integ = cls({"iterations": it})
    film = torch.empty((sc.height + 2, sc.width + 2, 4), dtype=torch.float32, device=f"cuda:{rk.dev}")
    shard = dict(spp=s1 - s0, spp_total=spp, sample_offset=s0, out=film, device=rk.dev)
    cls({"iterations": 1}).render_film(sc, seed=99, **shard)  # warm-up
    rk.barrier()
    t0 = time.perf_counter()
    st = None
    for k in range(args.steps):
        st = _sum_stats(st, integ.render_film(sc, seed=k, stats=True, **shard)[1])
        if rk.world > 1:
            distributed.reduce_sum(film)
    rk.barrier()
    dt = rk.max_elapsed(time.perf_counter() - t0) / args.steps
    st = {x: v / args.steps for x, v in st.items()}
    # visit counters (untimed): one short render of the same chains
    cnt = cls({"iterations": min(it, 20)}).render_film(sc, seed=0, stats=True, counters=True, **shard)[1]
    chains = sc.width * sc.height * spp
    cpu = None
    if rk.world == 1 and not args.no_cpu_baseline:
        # CPU: the oracle on whole film rows at 16 chains per pixel (the cost
        # per chain-iteration does not depend on the chain count), same
        # iterations, rows sized to the CPU budget
        oracle.build()
        cs = min(spp, 16)
        a1 = integ.render_args(sc, 0, cs, 0, 1)
        t1 = time.perf_counter()
        oracle.pssmlt_render(sc, a1, it)
        c1 = time.perf_counter() - t1
        rows = max(1, min(sc.height, int(args.cpu_seconds / max(c1, 1e-3))))
        a = integ.render_args(sc, 0, cs, 0, rows)
        t1 = time.perf_counter()
        oracle.pssmlt_render(sc, a, it)
        c = time.perf_counter() - t1
        cpu = {"value": round(sc.width * rows * cs * it / c / 1e6, 4), "unit": "Mchain-iterations/s",
               "cores": _threads(), "kind": "port",
               "sample": f"{rows} of {sc.height} rows x {sc.width} px x {cs} chains x {it} iterations ({c:.1f} s); "
                         "oracle/oracle.cpp orc_pssmlt_render (OpenMP)"}
    if rk.rank == 0:
        script = "pssmltpath.py (NEE + MIS)" if with_nee else "pssmltsimple.py"
        par = f"chain-range shards x{rk.world}" + (", RCCL gather of films to rank 0" if rk.world > 1 else "")
        _line(f"PSSMLT{'-path' if with_nee else ''} Mchain-iterations/sec on bedroom@1280x720, {spp} chains/pixel (C3)",
              chains * it / dt / 1e6, "Mchain-iterations/s", args.steps, 1, dt * 1e3,
              {"workload": f"{script} + pssmlt.py render, {it} iterations (large step every 50, aggregate "
                           f"i%50>40), max_depth 16, rr_depth 4, {chains} chains", "chains": chains,
               "iterations": it, "aggregation_iterations": sum(1 for i in range(it) if i % 50 > 40),
               "chains_per_rank": sc.width * sc.height * (s1 - s0), "parallelism": par},
              _trace_roofline(cnt, st["trace_ms"], "step", st["trace_launches"], args), cpu,
              {"kernels_ms_per_step": {"trace_closest": round(st["trace_ms"], 3), "shade": round(st["shade_ms"], 3),
                                       "trace_shadow": round(st["shadow_ms"], 3), "other": round(st["other_ms"], 3)},
               "n_gpus": rk.world, "scaling": "strong" if rk.world > 1 else "weak"})
    rk.close()


# -------------------------------------------------------------- ReSTIR (C4) --
RESTIR_C4 = {"jacobian": False, "bias_correction": False, "bsdf_sampling": True, "max_M_spatial": 500,
             "max_M_temporal": 30, "initial_search_radius": 10}


def restir(args):
    import binding as oracle
    import torch
    from mtx import RestirIntegrator, distributed, scene
    from mtx._lib import context

    sc = scene.bedroom(1920, 1080)
    rk = Ranks(args, sc.height)
    y0, y1 = rk.y0, rk.y1
    integ = RestirIntegrator(RESTIR_C4)
    film = torch.empty((y1 - y0 + 2, sc.width + 2, 4), dtype=torch.float32, device=f"cuda:{rk.dev}")
    halo = distributed.restir_halo(integ)
    ctx = context(rk.dev)
    ex, im = distributed.device_row_io(integ, sc, 1, ctx)

    def frame(seed, stats=False, counters=False):
        """One frame of this rank's band: stage A, halo swap, stage B, film
        gather (a single-rank frame is one call)."""
        if rk.world == 1:
            r = integ.render_film(sc, seed=seed, spp=1, out=film, stats=stats, counters=counters, ctx=ctx)
            return r[1] if stats else None
        a = integ.render_film(sc, seed=seed, spp=1, y0=y0, y1=y1, stage="A", stats=stats, counters=counters,
                              ctx=ctx)
        distributed.exchange_halos(ex, im, y0, y1, sc.height, halo)
        b = integ.render_film(sc, seed=seed, spp=1, y0=y0, y1=y1, stage="B", out=film, stats=stats,
                              counters=counters, ctx=ctx)
        rk.gather(film, sc.height)
        return _sum_stats(a[1], b[1]) if stats else None

    W = max(1, args.warmup)
    for k in range(W):
        frame(k)
    rk.barrier()
    agg = None
    t0 = time.perf_counter()
    for k in range(args.frames):
        agg = _sum_stats(agg, frame(W + k, stats=True))
    rk.barrier()
    dt = rk.max_elapsed(time.perf_counter() - t0) / args.frames
    cnt = frame(W + args.frames, stats=True, counters=True)
    px = sc.width * sc.height
    cpu = None
    if rk.world == 1 and not args.no_cpu_baseline:
        # CPU: the oracle's frame loop on the same 1920x1080 film (frame 0,
        # then as many frames as fit the CPU budget, at most 3)
        oracle.build()
        orc = oracle.RestirOracle(sc)
        ci = RestirIntegrator(RESTIR_C4)
        t1 = time.perf_counter()
        nf = 0
        while nf < 3 and (nf == 0 or time.perf_counter() - t1 < args.cpu_seconds):
            ci.n = nf
            orc.frame(sc, ci.render_args(sc, nf, 1))
            nf += 1
        c = time.perf_counter() - t1
        cpu = {"value": round(sc.width * sc.height * nf / c / 1e6, 4), "unit": "Mpixel-frames/s", "cores": _threads(),
               "kind": "port", "sample": f"{nf} frames at {sc.width}x{sc.height} ({c:.1f} s), same properties; "
                                         "oracle/oracle.cpp orc_restir_frame (OpenMP)"}
    if rk.rank == 0:
        _line(f"ReSTIR GI Mpixel-frames/sec on bedroom@1920x1080 (C4, {rk.world} GPU)", px / dt / 1e6,
              "Mpixel-frames/s", args.frames, W, dt * 1e3,
              {"workload": "restirgi.py render per frame: initial sample + path-mis secondary path (max_depth 8), "
                           "temporal + 9-tap spatial reuse with visibility, props restirgi.py:610-620",
               "frames_per_s": round(1.0 / dt, 2), "pixels": px,
               "parallelism": rk.parallelism() + (f", P2P halo of {halo} rows (samples + temporal reservoirs)"
                                                  if rk.world > 1 else "")},
              _trace_roofline(cnt, agg["trace_ms"] / args.frames, "frame", args=args), cpu,
              {"kernels_ms_per_frame": {"trace_closest": round(agg["trace_ms"] / args.frames, 3),
                                        "trace_shadow_and_visibility": round(agg["shadow_ms"] / args.frames, 3),
                                        "shade": round(agg["shade_ms"] / args.frames, 3),
                                        "other": round(agg["other_ms"] / args.frames, 3)},
               "n_gpus": rk.world, "scaling": "strong" if rk.world > 1 else "weak"})
    rk.close()


# ----------------------------------------------------------------- NRC (C5) --
def nrc(args):
    import torch
    from mtx import NRCIntegrator, scene

    torch.cuda.set_device(0)
    sc = scene.bedroom(1280, 720)
    integ = NRCIntegrator({})
    spp = 4
    film = torch.empty((sc.height + 2, sc.width + 2, 4), dtype=torch.float32, device="cuda:0")
    integ.render_film(sc, seed=99, spp=spp, out=film)
    _sync()
    reps = max(args.steps, 5)
    agg = None
    t0 = time.perf_counter()
    for k in range(reps):
        st = integ.render_film(sc, seed=k, spp=spp, out=film, stats=True)[1]
        agg = dict(st) if agg is None else {x: agg[x] + st[x] for x in st}
    _sync()
    dt = (time.perf_counter() - t0) / reps
    cnt = integ.render_film(sc, seed=0, spp=spp, out=film, stats=True, counters=True)[1]
    n = sc.width * sc.height * spp

    class A:  # cpu_baseline wants args.cpu_seconds only
        cpu_seconds = args.cpu_seconds

    cpu = None if args.no_cpu_baseline else bench.cpu_baseline(sc, integ, A)
    _line("NRC Mpaths/sec on bedroom@1280x720 spp=4 (C5)", n / dt / 1e6, "Mpaths/s", reps, 1, dt * 1e3,
          {"workload": "nrc.py NRCIntegrator.sample: NEE+MIS segments, spread heuristic c=0.01, max_depth 10",
           "paths_per_step": n}, _trace_roofline(cnt, agg["trace_ms"] / reps, "step", args=args), cpu)
    # the same with the radiance cache: stopped segments
    # trace one more segment and query the fused fp16 MFMA field there
    from mtx.field import Field

    cached = NRCIntegrator({"field": Field(sc)})
    cached.render_film(sc, seed=99, spp=spp, out=film)
    _sync()
    agg = None
    t0 = time.perf_counter()
    for k in range(reps):
        st = cached.render_film(sc, seed=k, spp=spp, out=film, stats=True)[1]
        agg = dict(st) if agg is None else {x: agg[x] + st[x] for x in st}
    _sync()
    dtc = (time.perf_counter() - t0) / reps
    cnt = cached.render_film(sc, seed=0, spp=spp, out=film, stats=True, counters=True)[1]
    _line("NRC + radiance cache Mpaths/sec on bedroom@1280x720 spp=4 (C5, nerad.py Field queries)", n / dtc / 1e6,
          "Mpaths/s", reps, 1, dtc * 1e3,
          {"workload": "nrc.py segments + one cache query per stopped segment: hash-grid/SH encode + fused "
                       "54->64x5->3 fp16 MLP (v_mfma_f32_32x32x16_f16) + L += T * out",
           "paths_per_step": n, "extra_ms_per_step": round((dtc - dt) * 1e3, 3),
           "cache_queries_per_step": int(agg["cache_queries"] / reps),
           "cache_encode_ms": round(agg["cache_encode_ms"] / reps, 3),
           "cache_mlp_ms": round(agg["cache_mlp_ms"] / reps, 3),
           "trace_ms": round(agg["trace_ms"] / reps, 3), "shadow_ms": round(agg["shadow_ms"] / reps, 3),
           "shade_ms": round(agg["shade_ms"] / reps, 3)},
          _trace_roofline(cnt, agg["trace_ms"] / reps, "step", args=args), cpu)


# ------------------------------------------------------------- primitives --
def prims(args):
    import binding as oracle
    from mtx import primitives
    from mtx._lib import context, lib

    ctx = context(0)
    dev_ms = lambda: lib().mtx_last_device_ms(ctx.handle)  # noqa: E731
    oracle.build()

    def best(fn, reps=3):
        t = []
        for _ in range(reps):
            fn()
            t.append(dev_ms())
        return min(t)

    def cpu_time(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    import torch

    def api_ms(fn, reps=3):
        """End-to-end wall time of one API call (the call returns with its
        results complete), best of reps: the device-tensor form (inputs and
        outputs in HBM, *_dev entry points) and the numpy form (host copies
        both ways) -- beside the kernels' HIP-event time."""
        fn()
        t = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            t.append((time.perf_counter() - t0) * 1e3)
        return round(min(t), 3)

    def api_extra(dev_fn, host_fn, kernel_ms):
        return {"api_ms_device_tensors": api_ms(dev_fn), "api_ms_host_arrays": api_ms(host_fn, reps=2),
                "kernel_ms": round(kernel_ms, 4),
                "api_note": "end-to-end wall time of the Python call: device tensors (mtx_*_dev, no host copy) "
                            "and numpy arrays (host<->device copies); kernel_ms is the HIP-event time of the "
                            "device work alone (the line's value)"}

    rng = np.random.default_rng(0)
    # prefix_sum u32, n = 2^28: 8 B/element
    n = 1 << 28
    x = rng.integers(0, 1 << 16, n, dtype=np.uint32)
    ms = best(lambda: primitives.prefix_sum(x))
    xt = torch.as_tensor(x.view(np.int32), device="cuda")
    ext = api_extra(lambda: primitives.prefix_sum(xt), lambda: primitives.prefix_sum(x), ms)
    del xt
    nc = 1 << 28
    c = cpu_time(lambda: oracle.prefix_sum_u32_mt(x[:nc]))
    ach = 8 * n / (ms / 1e3) / 1e9
    _line("prefix_sum u32 Gelem/sec (prefix_sum.py:9-36), n=2^28", n / (ms / 1e3) / 1e9, "Gelem/s", 3, 1, ms,
          {"workload": "inclusive scan of 2^28 u32, decoupled look-back", "n": n},
          {"bound": "hbm", "kernel": "scan_u32 (decoupled look-back)", "achieved": round(ach, 1),
           "peak": bench.HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / bench.HBM_PEAK_GBS, 4), "traffic": None,
           "alg_bytes_per_launch": 8 * n},
          {"value": round(nc / c / 1e9, 4), "unit": "Gelem/s", "cores": _threads(), "kind": "port",
           "sample": f"same 2^28 elements ({c:.2f} s), oracle orc_prefix_sum_u32_mt (OpenMP, equal to the "
                     "sequential restatement)"}, extra=ext, dtype="u32")
    del x
    # prefix_sum f32 in Hillis-Steele order, n = 2^24
    n = 1 << 24
    xf = rng.random(n, dtype=np.float32)
    ms = best(lambda: primitives.prefix_sum(xf))
    xft = torch.as_tensor(xf, device="cuda")
    ext = api_extra(lambda: primitives.prefix_sum(xft), lambda: primitives.prefix_sum(xf), ms)
    c = cpu_time(lambda: oracle.prefix_sum_f32_hs_mt(xf))
    passes = int(np.floor(np.log2(n))) + 1
    ach = 8 * n / (ms / 1e3) / 1e9
    hs_bytes = 12 * n * (1 + max(0, passes - 11))
    _line("prefix_sum f32 Hillis-Steele Gelem/sec (prefix_sum.py:9-36), n=2^24", n / (ms / 1e3) / 1e9, "Gelem/s", 3,
          1, ms, {"workload": f"{passes} Hillis-Steele passes in the reference's summation order (bit-exact)",
                  "n": n},
          {"bound": "hbm", "kernel": "scan_f32_hs (LDS passes + global passes)", "achieved": round(ach, 1),
           "peak": bench.HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / bench.HBM_PEAK_GBS, 4), "traffic": None,
           "alg_bytes_per_launch": 8 * n, "note": "algorithmic bytes = one read + one write per element",
           "hs_pass_bytes_per_launch": hs_bytes, "hs_pass_GBs": round(hs_bytes / (ms / 1e3) / 1e9, 1),
           "hs_note": "bytes the reference's Hillis-Steele order needs with 11 passes fused in LDS "
                      "(12 B/element) + one 2-read/1-write pass per remaining level (12 B/element each)"},
          {"value": round(n / c / 1e9, 4), "unit": "Gelem/s", "cores": _threads(), "kind": "port",
           "sample": f"same 2^24 elements ({c:.2f} s), oracle orc_prefix_sum_f32_hs_mt (OpenMP passes)"}, extra=ext)
    # hash grid, n = 2^24 points, res 100, n_cells = n (hashgrid.py:16-84)
    n = 1 << 24
    p = rng.random((3, n), dtype=np.float32)
    ms = best(lambda: primitives.HashGrid(p, 100, n))
    pt = torch.as_tensor(p, device="cuda")
    ext = api_extra(lambda: primitives.HashGrid(pt, 100, n), lambda: primitives.HashGrid(p, 100, n), ms)
    del pt
    nc = n
    c = cpu_time(lambda: oracle.hashgrid_mt(p, 100, nc))
    ach = 32 * n / (ms / 1e3) / 1e9
    _line("hashgrid build Msamples/sec (hashgrid.py:16-84), n=2^24", n / (ms / 1e3) / 1e6, "Msamples/s", 3, 1, ms,
          {"workload": "bbox reduce, cell hash, per-tile LDS split by the top 12 cell bits, per-bucket LDS sort "
                       "of the low 12 bits (cell_size / cell_offset / sample_idx); res 100, n_cells = n", "n": n},
          {"bound": "hbm", "kernel": "hashgrid_build (k_minmax, k_hash_cells, k_tile_split, k_bucket_fast)", "achieved": round(ach, 1),
           "peak": bench.HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / bench.HBM_PEAK_GBS, 4), "traffic": None,
           "alg_bytes_per_launch": 32 * n, "note": "SURVEY §8d: ~32 B/sample"},
          {"value": round(nc / c / 1e6, 4), "unit": "Msamples/s", "cores": _threads(), "kind": "port",
           "sample": f"same 2^24 points ({c:.2f} s), oracle orc_hashgrid_mt (OpenMP, parallel sort)"}, extra=ext,
          dtype="u32")
    del p
    # scatter_reduce add, nv = 2^24, nt = 2^20 (reductions.py:12-54)
    nv, nt = 1 << 24, 1 << 20
    idx = rng.integers(0, nt, nv, dtype=np.uint32)
    val = rng.random(nv, dtype=np.float32)
    tgt = np.zeros(nt, np.float32)
    ms = best(lambda: primitives.scatter_reduce_with("add", tgt, val, idx))
    tt, vt, it = (torch.as_tensor(a, device="cuda") for a in (tgt, val, idx.view(np.int32)))
    ext = api_extra(lambda: primitives.scatter_reduce_with("add", tt, vt, it),
                    lambda: primitives.scatter_reduce_with("add", tgt, val, idx), ms)
    c = cpu_time(lambda: oracle.scatter_reduce_mt(0, tgt, val, idx))
    ach = 16 * nv / (ms / 1e3) / 1e9
    _line("scatter_reduce add Gvalues/sec (reductions.py:12-54), nv=2^24 nt=2^20", nv / (ms / 1e3) / 1e9,
          "Gvalues/s", 3, 1, ms,
          {"workload": "stable group-by target (per-tile LDS split by the top 12 target bits, per-bucket LDS sort "
                       "of the low 8 bits), ordered fold per target (ascending index)", "n_value": nv,
           "n_target": nt},
          {"bound": "hbm", "kernel": "scatter_reduce (k_tile_split, k_bucket_fast)", "achieved": round(ach, 1), "peak": bench.HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(ach / bench.HBM_PEAK_GBS, 4), "traffic": None, "alg_bytes_per_launch": 16 * nv,
           "note": "SURVEY §8d: 16 B/value"},
          {"value": round(nv / c / 1e9, 4), "unit": "Gvalues/s", "cores": _threads(), "kind": "port",
           "sample": f"same {nv} values ({c:.2f} s), oracle orc_scatter_reduce_f32_mt (OpenMP, parallel sort)"},
          extra=ext)


# ------------------------------------------------- radiance field (MFMA) --
MFMA_F16_PEAK_TFS = 2500.0  # MI355X dense fp16 (MI355X_MICROARCH.md; 2:1-sparse figure excluded)


def field(args):
    from mtx.field import Field
    from mtx._lib import context, lib

    ctx = context(0)
    f = Field(bbox=([-3.0, 0.0, -2.0], [4.0, 3.0, 4.0]))
    f.upload(ctx)
    n = 1 << 22
    rng = np.random.default_rng(0)
    p = rng.uniform([-3, 0, -2], [4, 3, 4], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    feat = f.features(p, d, ctx)
    enc_ms = min(lib().mtx_last_device_ms(ctx.handle), (f.features(p, d, ctx), lib().mtx_last_device_ms(ctx.handle))[1])
    # the same queries in Morton order: hash-grid gathers of neighbouring
    # lanes then share cache lines (the locality the table's L2/MALL sees)
    g = np.clip(((p - p.min(0)) / (p.max(0) - p.min(0)) * 1023).astype(np.uint64), 0, 1023)

    def spread3(x):
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        return (x | (x << 2)) & 0x09249249

    order = np.argsort(spread3(g[:, 0]) | (spread3(g[:, 1]) << 1) | (spread3(g[:, 2]) << 2), kind="stable")
    ps, ds = np.ascontiguousarray(p[order]), np.ascontiguousarray(d[order])
    f.features(ps, ds, ctx)
    enc_sorted_ms = min(lib().mtx_last_device_ms(ctx.handle),
                        (f.features(ps, ds, ctx), lib().mtx_last_device_ms(ctx.handle))[1])
    ms = []
    for _ in range(5):
        f.mlp(feat, ctx)
        ms.append(lib().mtx_last_device_ms(ctx.handle))
    ms = min(ms)
    flops = f.flops_per_query() * n
    tfs = flops / (ms / 1e3) / 1e12
    # CPU: the fp32 numpy reference network on a sample (plain BLAS threads)
    nc = 1 << 16
    t0 = time.perf_counter()
    f.mlp_reference(feat[:nc])
    c = time.perf_counter() - t0
    _line("Field MLP inference Mqueries/sec (nerad.py:54-106: 54->64x5->3 fp16, MFMA)", n / (ms / 1e3) / 1e6,
          "Mqueries/s", 5, 1, ms,
          {"workload": f"fused 6-layer MLP, {n} queries, v_mfma_f32_32x32x16_f16, f32 accumulate",
           "flops_per_query": f.flops_per_query(), "encode_ms": round(enc_ms, 3),
           "encode_Mqueries_s": round(n / (enc_ms / 1e3) / 1e6, 1), "encode_morton_ms": round(enc_sorted_ms, 3),
           "encode_morton_Mqueries_s": round(n / (enc_sorted_ms / 1e3) / 1e6, 1)},
          {"bound": "mfma", "kernel": "k_field_mlp", "achieved": round(tfs, 2), "peak": MFMA_F16_PEAK_TFS,
           "unit": "TFLOP/s", "frac": round(tfs / MFMA_F16_PEAK_TFS, 4), "traffic": None,
           "alg_bytes_per_launch": int(n * (128 + 12))},
          {"value": round(nc / c / 1e6, 4), "unit": "Mqueries/s", "cores": _threads(), "kind": "port",
           "sample": f"{nc} queries, numpy fp32 reference network ({c:.2f} s)"}, dtype="f16")


# ---------------------------------------------------- nerad training (f3) --
def nerad(args):
    """nerad.py training_step on the bedroom proxy at the script's sizes
    (batch_size 2^14 LHS points, M = 32 RHS samples each, :244-245)."""
    import binding as oracle
    import torch
    from mtx import scene
    from mtx.field import Field
    from mtx.nerad import FieldTrainer

    torch.cuda.set_device(0)
    sc = scene.bedroom(1280, 720)
    field = Field(sc)
    batch, M = 2 ** 14, 32
    tr = FieldTrainer(sc, field, batch_size=batch, M=M)
    for _ in range(max(1, args.warmup)):
        tr.step()
    _sync()
    reps = max(args.steps, 10)
    agg = None
    t0 = time.perf_counter()
    for _ in range(reps):
        st = tr.step()
        agg = _sum_stats(agg, st)
    _sync()
    dt = (time.perf_counter() - t0) / reps
    lanes = batch * M
    cnt = tr.step(counters=True)  # untimed: RHS visit counts
    alg = (cnt["rays_closest"] * (RAY_BYTES + HIT_BYTES) + cnt["nodes_closest"] * NODE_BYTES
           + cnt["tris_closest"] * TRI_BYTES)
    tms = agg["ms_trace"] / reps
    ach = alg / (tms / 1e3) / 1e9 if tms > 0 else 0.0
    roof = {"bound": "vmem", "kernel": "k_trace_closest (RHS BSDF rays + next_smooth_si chain)",
            "achieved": round(ach, 1), "peak": bench.VMEM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / bench.VMEM_PEAK_GBS, 4), "traffic": None,
            "peak_source": "vector-memory (TA/TCP) byte path, as bench.py's headline roofline",
            "trace_ms_per_step": round(tms, 3),
            "alg_bytes_per_step": int(alg), "rays_per_step": int(cnt["rays_closest"]),
            "node_visits_per_ray": round(cnt["nodes_closest"] / max(1, cnt["rays_closest"]), 2),
            "tri_visits_per_ray": round(cnt["tris_closest"] / max(1, cnt["rays_closest"]), 2)}
    # CPU: the oracle's RHS lanes (the dominant part) on a reduced batch
    oracle.build()
    nb = 64
    t1 = time.perf_counter()
    oracle.nerad_rhs(sc, tr.isampler.tables, 1, 2, nb, M)
    c = time.perf_counter() - t1
    nb = max(nb, min(2 ** 20, int(nb * args.cpu_seconds / max(c, 1e-3))))
    t1 = time.perf_counter()
    oracle.nerad_rhs(sc, tr.isampler.tables, 1, 2, nb, M)
    c = time.perf_counter() - t1
    cpu = {"value": round(nb * M / c / 1e6, 4), "unit": "M RHS samples/s", "cores": _threads(), "kind": "port",
           "sample": f"{nb} points x {M} RHS samples without the field term ({c:.1f} s); oracle/oracle.cpp "
                     "orc_nerad_rhs (OpenMP)"}
    ms = {k: round(agg[k] / reps, 3) for k in ("ms_lhs", "ms_rhs", "ms_trace", "ms_train", "ms_total")}
    _line("nerad training steps/sec on bedroom (batch 2^14 x M=32, f3)", 1.0 / dt, "steps/s", reps,
          max(1, args.warmup), dt * 1e3,
          {"workload": "nerad.py training_step: IntersectionSampler LHS, sample_rhs (NEE + BSDF sample + "
                       "next_smooth_si + field query) on the wavefront, fp16 field forward/backward, hash-grid "
                       "gradient scatter, GradScaler + Adam", "batch_size": batch, "M": M,
           "rhs_samples_per_s": round(lanes / dt / 1e6, 3), "phase_ms": ms,
           "rhs_field_queries_per_step": int(agg["rhs_queries"] / reps), "final_loss": round(st["loss"], 6)},
          roof, cpu)


def run(args):
    {"pssmlt": pssmlt, "pssmltpath": lambda a: pssmlt(a, with_nee=True), "restir": restir, "nrc": nrc,
     "prims": prims, "field": field, "nerad": nerad}[args.workload](args)
