// kernels.hip — gfx950 wavefront path-tracing kernels.
//
// Replaces the Dr.Jit-traced megakernel that mi.render() builds from the
// reference sample() loops (path.py:194-302, path-mis.py:24-155,
// nrc.py:25-125) with explicit kernels over SoA state in HBM:
//
//   raygen   camera rays for a chunk of (pixel, sample) lanes
//            (transcribed render_sample, path.py:27-101)
//   trace    persistent closest-hit BVH2 traversal, LDS stack per lane,
//            rays fetched 64 at a time per wave from an atomic counter
//            (Scene.ray_intersect, path-mis.py:69-71)
//   shade    one bounce of the integrator: emission + MIS, NEE sampling,
//            BSDF eval/sample, Russian roulette; survivors and shadow rays are
//            stream-compacted with wave64 ballot + mbcnt and one atomic/wave
//   shadow   persistent any-hit traversal of the NEE rays; visible ones add
//            their contribution to L (Scene.ray_test inside
//            sample_emitter_direction(..., test_visibility=True), path.py:247)
//   film     deterministic gather-form tent splat (ImageBlock.put, path.py:101)
//
// All arithmetic is IEEE fp32 with -ffp-contract=off; the per-lane
// primitives are the shared mtx_core headers, so every lane reproduces the
// CPU restatement in oracle/ bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.h"
#include "restir_dev.h"

using namespace mtx;

// Minimum resident shade blocks per CU (caps the shade kernels' VGPRs: 3
// blocks of 256 threads = 3 waves/SIMD at <= 168 VGPRs). 4 blocks (<= 128
// VGPRs) spill 26 VGPRs of k_shade<2>: shade 63.4 -> 74.6 ms per step, and
// 69.4 ms with the NEE record staged in LDS (13 spilled); the record in LDS
// at 3 blocks (149 VGPRs): 64.4 ms (profiles/r6e_ab_shade_vgpr_budget.jsonl).
#ifndef MTX_SHADE_MIN_BLOCKS
#define MTX_SHADE_MIN_BLOCKS 3
#endif
constexpr int kShadeMinBlocks = MTX_SHADE_MIN_BLOCKS;

namespace mtxd {

// Closest-hit queries of bounce `bounce`: queue entries are path indices.
// The hit record goes to the queue position k (not the path): the shade
// kernel, which walks the same queue, then reads it coalesced and without
// waiting for its queue entry.
struct ClosestSrc {
  using Payload = uint32_t;  // the queue position
  WaveBuffers b;
  const uint32_t *queue;
  const float4 *ro, *rd;  // this bounce's ray planes, by queue position
  __device__ __forceinline__ void load(uint32_t k, TraceRay &r, float &tmax, uint32_t &payload) const {
    const float4 o4 = ld_stream<kNtTrace>(ro + k), d4 = ld_stream<kNtTrace>(rd + k);
    r = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
    tmax = o4.w;
    payload = k;
  }
  __device__ __forceinline__ void finish(uint32_t slot, bool, float t, uint32_t prim, float u, float v) const {
    st_stream<kNtTraceSt>(b.hit + slot, make_float4(prim == 0xffffffffu ? kInf : t, __uint_as_float(prim), u, v));
  }
};

// 8 waves/SIMD for the trace kernels (their grid is sized for 8): left alone
// the compiler took 66 VGPRs for the any-hit kernel (7 waves); asked for 8 it
// fits without spills. Shadow 56.4 -> 55.6 ms per step (A/B, one box, 3
// rounds, round 2).
#define MTX_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(8)))
#ifndef MTX_CLOSEST_WAVES
#define MTX_CLOSEST_WAVES 8  // closest hit: waves/SIMD the register budget is sized for
#endif
template <bool STATS>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(MTX_CLOSEST_WAVES))) void k_trace_closest(DevScene s, WaveBuffers b, uint32_t bounce) {
  // dynamic LDS: stack columns + tree top (device_common.h trace_loop)
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  const ClosestSrc src{b, b.queue[bounce & 1], b.ray_o[rp], b.ray_d[rp]};
  uint32_t nv = 0, tv = 0, nr = 0, wi[2] = {0, 0};
  trace_loop<false, STATS>(s, src, b.counters[4 * bounce + 0], b.xheads + (2 * bounce) * kXSlotWords, nv, tv, nr,
                           wi);
  if (STATS) {
    unsigned long long a = wave_sum_u64(nv), c = wave_sum_u64(tv), n = wave_sum_u64(nr);
    unsigned long long w0 = wave_sum_u64(wi[0]), w1 = wave_sum_u64(wi[1]);
    if ((threadIdx.x & 63) == 0 && n) {
      atomicAdd(&b.stats[0], a);
      atomicAdd(&b.stats[1], c);
      atomicAdd(&b.stats[4], n);
      atomicAdd(&b.stats[6], w0);
      atomicAdd(&b.stats[7], w1);
    }
  }
}

// A shadow record's contribution to its path's L (T, X and flags of
// make_shadow): fma(T, X, L) or L + X when the ray is unoccluded, the
// flagged channels NaN when it is occluded.
__device__ __forceinline__ void apply_shadow(float4 &L, float4 rt, float4 rx, bool occluded) {
  const uint32_t fl = __float_as_uint(rt.w);
  if (!occluded) {
    if (fl & 1u) {
      L.x = fmaf(rt.x, rx.x, L.x);
      L.y = fmaf(rt.y, rx.y, L.y);
      L.z = fmaf(rt.z, rx.z, L.z);
    } else {
      L.x = L.x + rx.x;
      L.y = L.y + rx.y;
      L.z = L.z + rx.z;
    }
  } else {
    const float qnan = __uint_as_float(0x7fc00000u);
    if (fl & 2u) L.x = qnan;
    if (fl & 4u) L.y = qnan;
    if (fl & 8u) L.z = qnan;
  }
}

// Any-hit traversal of the NEE shadow rays. k_shade stores each record of
// the integrators whose L it stores itself (path-mis, path, nrc, pssmltpath)
// in its final-value form (make_shadow with Lcur, flag kShadowFinal): t = the path's L after an unoccluded
// ray (fma(T, X, L), path-mis.py:117, or L + X, path.py:259 / nrc.py:62) with
// the flags in t.w, x = the path's L before it. The finish is one store -- no
// read of L: t.xyz with x.w when unoccluded; when occluded, nothing unless a
// flagged channel must become NaN (then x, read from the record, with those
// channels NaN).
constexpr uint32_t kShadowFinal = 16u;  // record flag: final-value form

struct ShadowSrc {
  struct Payload {
    uint32_t k, li;  // record, L index of the target (plane * capacity + position)
    float4 t;        // L after an unoccluded ray | flags
    float lw;        // L.w (unchanged by the update)
  };
  WaveBuffers b;
  __device__ __forceinline__ void load(uint32_t k, TraceRay &r, float &tmax, Payload &pl) const {
    const float4 o4 = ld_stream<kNtTrace>(&b.shadow[k].o), d4 = ld_stream<kNtTrace>(&b.shadow[k].d);
    r = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
    tmax = o4.w;
    pl.k = k;
    pl.li = __float_as_uint(d4.w);
    pl.t = ld_stream<kNtTrace>(&b.shadow[k].t);
    pl.lw = b.shadow[k].x.w;
  }
  __device__ __forceinline__ void finish(const Payload &pl, bool occluded, float, uint32_t, float, float) const {
    const uint32_t fl = __float_as_uint(pl.t.w);
    if (!(fl & kShadowFinal)) {
      // make_shadow's form (the nerad integrators keep L by path outside
      // k_shade's stores): read-modify-write of L
      if (occluded && (fl & 14u) == 0u) return;
      float4 L = b.L[0][pl.li];
      apply_shadow(L, pl.t, b.shadow[pl.k].x, occluded);
      b.L[0][pl.li] = L;
      return;
    }
    if (!occluded) {
      st_stream<kNtTraceSt>(b.L[0] + pl.li, make_float4(pl.t.x, pl.t.y, pl.t.z, pl.lw));
    } else if (fl & 14u) {
      float4 L = b.shadow[pl.k].x;
      const float qnan = __uint_as_float(0x7fc00000u);
      if (fl & 2u) L.x = qnan;
      if (fl & 4u) L.y = qnan;
      if (fl & 8u) L.z = qnan;
      b.L[0][pl.li] = L;
    }
    // occluded without flags: L unchanged, nothing to store
  }
};

template <bool STATS>
__global__ __launch_bounds__(kTraceBlock) MTX_TRACE_ATTR void k_trace_shadow(DevScene s, WaveBuffers b, uint32_t bounce) {
  // dynamic LDS: stack columns + tree top (device_common.h trace_loop)
  const ShadowSrc src{b};
  uint32_t nv = 0, tv = 0, nr = 0;
  trace_loop<true>(s, src, b.counters[4 * (bounce + 1) + 1], b.xheads + (2 * bounce + 1) * kXSlotWords, nv, tv, nr);
  if (STATS) {
    unsigned long long a = wave_sum_u64(nv), c = wave_sum_u64(tv), n = wave_sum_u64(nr);
    if ((threadIdx.x & 63) == 0 && n) {
      atomicAdd(&b.stats[2], a);
      atomicAdd(&b.stats[3], c);
      atomicAdd(&b.stats[5], n);
    }
  }
}

// ---------------------------------------------------------------------------
// Ray generation
// ---------------------------------------------------------------------------
__device__ __forceinline__ void init_path(const WaveBuffers &b, const ChunkParams &p, uint32_t i, const Ray &ray,
                                          const Pcg32 &rng, float2 pos, bool env) {
  uint32_t depth = 0, flags = 0;
  if (p.integrator == MTX_INT_PATH_MIS) {
    depth = 0;
    // prev_bsdf_delta = True (path-mis.py:46); valid_ray = scene.environment() is not None (:41)
    flags = PF_PREV_DELTA | (env ? PF_VALID_RAY : 0u);
  } else if (p.integrator == MTX_INT_SIMPLE) {
    depth = 0;  // simple.py:27
  } else {
    depth = 1;  // path.py:230, nrc.py:39
  }
  // throughput = 1, eta = 1, L = 0, prev_bsdf_pdf = 1 (path-mis.py:45), prev_p = 0 are
  // not stored: the bounce-0 shade uses these constants (kInitThr / kInitL / kInitPrev)
  st_stream<kNtRaygen>(b.ray_o[0] + i, make_float4(ray.o.x, ray.o.y, ray.o.z, ray.maxt));  // queue position i (identity)
  st_stream<kNtRaygen>(b.ray_d[0] + i, make_float4(ray.d.x, ray.d.y, ray.d.z, 0.f));
  st_stream<kNtRaygen>(b.misc[0] + i,
                       make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16)));
  b.pos[i] = pos;
  if (!p.ident0) b.queue[0][i] = i;
}

__global__ void k_raygen_camera(DevScene s, WaveBuffers b, ChunkParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) b.counters[0] = p.n_paths;
  if (i >= p.n_paths) return;
  // path order within the chunk: pixel-major keeps the samples of one pixel
  // in one wave (coherent traversal)
  const uint32_t px_local = i / p.spp, smp = i - px_local * p.spp;
  const uint32_t pix = p.px0 + px_local;
  const uint32_t y = pix / p.width, x = pix - y * p.width;
  const uint32_t lane = pix * p.spp_total + p.sample_offset + smp;
  Pcg32 rng = sampler_lane(p.seed, lane);
  const V2 u = rng.next_2d();  // film jitter (path.py:45)
  const float sx = (float)x + u.x, sy = (float)y + u.y;
  const V2 adj = V2{sx / (float)p.width, sy / (float)p.height};
  const Ray ray = camera_ray(s.camera, adj);  // path.py:60-62
  init_path(b, p, i, ray, rng, make_float2(sx, sy), s.has_env != 0);
}

__global__ void k_raygen_rays(DevScene s, WaveBuffers b, ChunkParams p, const float *rays, const uint32_t *lanes,
                              uint32_t rng_skip) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) b.counters[0] = p.n_paths;
  if (i >= p.n_paths) return;
  Pcg32 rng = sampler_lane(p.seed, lanes[i]);
  for (uint32_t k = 0; k < rng_skip; ++k) rng.next_u32();
  const float *r = rays + 6 * (size_t)i;
  Ray ray{V3{r[0], r[1], r[2]}, V3{r[3], r[4], r[5]}, kLargest};
  init_path(b, p, i, ray, rng, make_float2(0.f, 0.f), s.has_env != 0);
}

// ---------------------------------------------------------------------------
// Shading: one bounce of the integrator for one path.
// ---------------------------------------------------------------------------
// Initial path state (init_path, k_rs_begin): throughput 1 / eta 1, L 0 /
// prev_bsdf_pdf 1, prev_p 0 / spread 0. Never stored: bounce-0 shades use it.
// (register constants: a select between a __device__ constant and the state
// plane compiled to a pointer select + flat load per plane)
#define kInitThr make_float4(1.f, 1.f, 1.f, 1.f)
#define kInitL make_float4(0.f, 0.f, 0.f, 1.f)
#define kInitPrev make_float4(0.f, 0.f, 0.f, 0.f)

// Diagnostic build only (MTX_DIAG_STAMPS=1, tools/shade_stamps.py): s_memtime
// stamps between the phases of a shade step, summed per wave in scalar
// registers and added to g_shade_stamps at the kernel's end. Read shares, not
// the build's run time (cdna_hip_programming.md "In-kernel stamps").
#ifndef MTX_DIAG_STAMPS
#define MTX_DIAG_STAMPS 0
#endif
constexpr int kStampSegs = 8;
struct Stamps {
  unsigned long long prev, acc[kStampSegs];
};
#if MTX_DIAG_STAMPS
__device__ unsigned long long g_shade_stamps[kStampSegs + 2];
#define MTX_STAMP(st, i)                                                                  \
  do {                                                                                    \
    unsigned long long t_;                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    (st).acc[i] += t_ - (st).prev;                                                        \
    (st).prev = t_;                                                                       \
  } while (0)
#endif

struct ShadeIO {
  ShadowRec rec;
  bool emit;
  bool em_hi;  // the shadow ray's emitter index is odd (block append: even emitters' rays first)
  bool query;  // NRC radiance-cache query at this hit (field.hip)
  float4 qp, qd, qt;
  float4 nro, nrd, nthr, nprev;  // the next ray and state: k_shade stores them at the path's append slot
  float4 nL;                     // result and sampler state: at the append slot, or by path once the path ends
  uint4 nmisc;
  float warm;                    // MTX_SHADE_WARM: the next entry's shading-record word (L2 warm-up)
#if MTX_DIAG_STAMPS
  Stamps st;
#endif
};

// Which shadow-record form an integrator's NEE must use (ShadowSrc::finish
// reads it from flag bit 4, kShadowFinal): true where k_shade itself stores
// the path's L at the queue slot / final plane after the bounce, so the L the
// record is built from is final for the bounce and the any-hit finish may
// overwrite L without reading it (final-value form); false where L lives by
// path outside k_shade's stores (the neural-radiosity RHS: k_nerad_apply adds
// to it), so the finish must read-modify-write L. make_shadow<INT> checks the
// choice at compile time: a new integrator that emits shadow rays must be
// listed here (the round-5 nerad regression was this choice made wrongly).
constexpr bool shadow_final_form(int INT) {
  return INT == MTX_INT_PATH || INT == MTX_INT_PATH_MIS || INT == MTX_INT_NRC || INT == MTX_INT_PSSMLT_PATH;
}
constexpr bool shadow_rmw_form(int INT) { return INT == MTX_INT_NERAD_RHS; }

// Builds the shadow record for an NEE contribution. fma_form: value = (T, X)
// applied as fma(T, X, L); otherwise X is added. Xo is the contribution the
// reference forms when the shadow ray is occluded (em_weight = 0). With Lcur
// (the path's L, final for this bounce: the integrators that k_shade stores
// L for add nothing to L after their NEE) the record is built in its
// final-value form (see ShadowSrc; k_shade completes x.w with L.w).
template <int INT, bool FINAL>
__device__ __forceinline__ void make_shadow(ShadeIO &io, const SurfaceInteraction &si, const DirectionSample &ds,
                                            V3 T, V3 X, V3 Xo, bool fma_form, const V3 *Lcur = nullptr) {
  static_assert(FINAL ? shadow_final_form(INT) : shadow_rmw_form(INT),
                "shadow record form does not match where this integrator's L is stored (shadow_final_form)");
  uint32_t fl = fma_form ? 1u : 0u;
  bool vis_noop, occ_noop;
  if (fma_form) {
    fl |= (Xo.x == 0.f && isfinite_(T.x)) ? 0u : 2u;
    fl |= (Xo.y == 0.f && isfinite_(T.y)) ? 0u : 4u;
    fl |= (Xo.z == 0.f && isfinite_(T.z)) ? 0u : 8u;
    vis_noop = X.x == 0.f && X.y == 0.f && X.z == 0.f && isfinite_(T.x) && isfinite_(T.y) && isfinite_(T.z);
  } else {
    fl |= (Xo.x == 0.f) ? 0u : 2u;
    fl |= (Xo.y == 0.f) ? 0u : 4u;
    fl |= (Xo.z == 0.f) ? 0u : 8u;
    vis_noop = X.x == 0.f && X.y == 0.f && X.z == 0.f;
  }
  occ_noop = (fl & 14u) == 0u;
  io.emit = !(vis_noop && occ_noop);
  if (!io.emit) return;
  io.em_hi = (ds.emitter & 1) != 0;
  const Ray sr = spawn_ray_to(si.p, si.n, ds.p);
  io.rec.o = make_float4(sr.o.x, sr.o.y, sr.o.z, sr.maxt);
  io.rec.d = make_float4(sr.d.x, sr.d.y, sr.d.z, 0.f);  // .w: the L index, set by k_shade after its append
  if constexpr (FINAL) {
    float4 lv = make_float4(Lcur->x, Lcur->y, Lcur->z, 0.f);
    apply_shadow(lv, make_float4(T.x, T.y, T.z, __uint_as_float(fl)), make_float4(X.x, X.y, X.z, 0.f), false);
    io.rec.t = make_float4(lv.x, lv.y, lv.z, __uint_as_float(fl | kShadowFinal));
    io.rec.x = make_float4(Lcur->x, Lcur->y, Lcur->z, 0.f);
  } else {
    io.rec.t = make_float4(T.x, T.y, T.z, __uint_as_float(fl));
    io.rec.x = make_float4(X.x, X.y, X.z, 0.f);
  }
}

// A shadow record applied to its path's L in registers (the path megakernels:
// the record of make_shadow, in either form).
__device__ __forceinline__ void apply_shadow_rec(float4 &L, const ShadowRec &rec, bool occluded) {
  const uint32_t fl = __float_as_uint(rec.t.w);
  if (!(fl & kShadowFinal)) {
    apply_shadow(L, rec.t, rec.x, occluded);
  } else if (!occluded) {
    L = make_float4(rec.t.x, rec.t.y, rec.t.z, L.w);
  } else {
    const float qnan = __uint_as_float(0x7fc00000u);
    if (fl & 2u) L.x = qnan;
    if (fl & 4u) L.y = qnan;
    if (fl & 8u) L.z = qnan;
  }
}

// BSDF data for one shading point: the textured colour of the diffuse and
// roughplastic lobes fetched once (and early: its latency overlaps the work
// before the first BSDF call), read by every BSDF call at this point.
__device__ __forceinline__ BsdfData bsdf_at(const SceneView &sv, const mtx_material &mat, V2 uv) {
  BsdfData bd = sv.bsdf;
  if (mat.tex >= 0 && (mat.type == MTX_MAT_DIFFUSE || mat.type == MTX_MAT_ROUGHPLASTIC)) {
    bd.col = texture_eval(sv.bsdf, mat.tex, uv);
    bd.has_col = true;
  }
  return bd;
}
// path-mis: once a path ends, L.w (its prev_bsdf_pdf until then) holds
// valid_ray as 1 / 0 (path-mis.py:155), so the film reads L and pos only,
// not the 16-B misc record for one flag.
__device__ __forceinline__ float end_w(uint32_t flags, float prev_pdf) {
  (void)prev_pdf;
  return (flags & PF_VALID_RAY) ? 1.f : 0.f;
}
__device__ __forceinline__ bool end_valid(const WaveBuffers &b, uint32_t path, float lw) {
  (void)b;
  (void)path;
  return lw != 0.f;
}
template <int INT>
__device__ __forceinline__ bool shade_path(const DevScene &s, const SceneView &sv, const WaveBuffers &b,
                                           const ChunkParams &p, uint32_t bounce, uint32_t path, uint32_t qi,
                                           const float4 h, ShadeIO &io, const float4 *warm = nullptr) {
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  const float4 ro = ld_stream<kNtShade>(b.ray_o[rp] + qi), rd = ld_stream<kNtShade>(b.ray_d[rp] + qi);
  // bounce 0: the state init_path / k_rs_begin would have stored (not read)
  const float4 th = bounce == 0 ? kInitThr : ld_stream<kNtShade>(b.thr[rp] + qi),
               Lr = bounce == 0 ? kInitL : ld_stream<kNtShade>(b.L[rp] + qi);
  // prev (previous vertex, NRC spread): path-mis / path read it only for the
  // emission MIS of an emitter hit (pdf_emitter_direction is 0 otherwise), so
  // they load it below once the hit's emitter is known
  constexpr bool kPrevOnEmitter = INT == MTX_INT_PATH_MIS || INT == MTX_INT_PATH;
  float4 pv = kInitPrev;
  if (!kPrevOnEmitter && bounce != 0) pv = ld_stream<kNtShade>(b.prev[rp] + qi);
  const uint4 mi = ld_stream<kNtShade>(b.misc[rp] + qi);
  io.nL = Lr;  // an exit that changes neither keeps them
  io.nmisc = mi;
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  uint32_t depth = mi.w & 0xffffu, flags = mi.w >> 16;
  V3 T = V3{th.x, th.y, th.z};
  float eta = th.w;
  V3 L = V3{Lr.x, Lr.y, Lr.z};
  float prev_pdf = Lr.w;
  const V3 ray_d = V3{rd.x, rd.y, rd.z};
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, ray_d);
#if MTX_DIAG_STAMPS
  MTX_STAMP(io.st, 1);
#endif
  // the next queue entry's shading record, one word: its line is in L2 when
  // the next iteration reads the record (k_shade, MTX_SHADE_WARM)
  if (warm) io.warm = warm->x;
  if (kPrevOnEmitter && bounce != 0 && si.emitter >= 0) pv = b.prev[rp][qi];
  V3 prev_p = V3{pv.x, pv.y, pv.z};
  float spread = pv.w, a0 = rd.w;
  io.emit = false;
  io.query = false;

  // ------------------------------ head ------------------------------------
  bool active_next = true;
  if (INT == MTX_INT_PATH_MIS) {
    // Direct emission with MIS against the previous BSDF sample (:75-86)
    const bool prev_delta = (flags & PF_PREV_DELTA) != 0;
    float em_pdf = 0.f;
    if (!prev_delta && si.emitter >= 0) {
      const V3 rel = si.p - prev_p;
      const float dist = norm(rel);
      em_pdf = pdf_emitter_direction(sv, si.emitter, rel / dist, dist, si.sh.n);
    }
    const float mis_bsdf = mis_weight_b(prev_pdf, em_pdf);
    const V3 le = (prev_pdf > 0.f) ? emitter_eval(sv, si.emitter, si.wi) : v3s(0.f);
    L = fma3v(T, le * mis_bsdf, L);
    active_next = (depth + 1 < p.max_depth) && si.valid;  // :88
  } else if (bounce == 0) {
    if (INT == MTX_INT_PATH) {
      L = L + emitter_eval(sv, si.emitter, si.wi);  // path.py:239
      if (!(depth < p.max_depth)) {                // path.py:235
        io.nL = make_float4(L.x, L.y, L.z, prev_pdf);
        return false;
      }
    } else {  // NRC primary (nrc.py:117-121)
      if (si.valid) flags |= PF_PRIMARY_VALID;
      a0 = squared_norm(V3{ro.x, ro.y, ro.z} - si.p) / (kFourPi * fabsf(si.wi.z));
      spread = 0.f;
    }
  } else {
    if (INT == MTX_INT_NRC && (flags & PF_CACHE_QUERY)) {
      // the segment ended by the spread criterion (nrc.py:70-71): the radiance
      // cache replaces the rest of the path, queried at the next hit with the
      // direction back to the previous vertex (nerad.py:86-106 Field(si))
      if (si.valid) {
        io.query = true;
        io.qp = make_float4(si.p.x, si.p.y, si.p.z, 0.f);
        io.qd = make_float4(-ray_d.x, -ray_d.y, -ray_d.z, 0.f);
        io.qt = make_float4(T.x, T.y, T.z, __uint_as_float(path));
      }
      return false;
    }
    // path.py:283-300 / nrc.py:79-100: emission of the BSDF-sampled hit
    const bool bsdf_delta = (flags & PF_PREV_DELTA) != 0;
    float em_pdf = 0.f;
    if (!bsdf_delta && si.emitter >= 0) {
      const V3 rel = si.p - prev_p;
      const float dist = norm(rel);
      em_pdf = pdf_emitter_direction(sv, si.emitter, rel / dist, dist, si.sh.n);
    }
    const float mis_bsdf =
        INT == MTX_INT_PATH ? mis_weight_a(prev_pdf, em_pdf) : mis_weight_b(prev_pdf, em_pdf);
    const V3 le = (prev_pdf > 0.f) ? emitter_eval(sv, si.emitter, si.wi) : v3s(0.f);
    L = L + T * le * mis_bsdf;
    if (INT == MTX_INT_NRC) spread += sqrtf(squared_norm(si.p - prev_p) / (prev_pdf * fabsf(si.wi.z)));
    depth += 1;
  }
  // path.py:235,299-300 / nrc.py:119,272-273: the NRC primary bounce only
  // requires a valid hit (its depth test runs at the end of an iteration).
  const bool head_ok =
      (INT == MTX_INT_NRC && bounce == 0) ? si.valid : (depth < p.max_depth && si.valid);
  if (INT != MTX_INT_PATH_MIS && !head_ok) {
    io.nL = make_float4(L.x, L.y, L.z, prev_pdf);
    if (INT == MTX_INT_NRC) io.nmisc = make_uint4(mi.x, mi.y, mi.z, depth | (flags << 16));
    return false;
  }
  if (INT == MTX_INT_PATH_MIS && p.restir && bounce == 0) {
    // restirgi.py:452-455: x_s, n_s of the secondary ray's first hit
    b.rs_xs[path] = si.valid ? make_float4(si.p.x, si.p.y, si.p.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    b.rs_ns[path] = si.valid ? make_float4(si.n.x, si.n.y, si.n.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (INT == MTX_INT_PATH_MIS && !si.valid) {
    // escaped path: nothing after this point is observable (valid_ray,
    // result unchanged; throughput becomes 0 -> inactive) -- except the
    // sampler position, which ReSTIR keeps using (6 draws per iteration)
    io.nL = make_float4(L.x, L.y, L.z, end_w(flags, prev_pdf));
    if (p.restir) {
      rng.advance(6);
      io.nmisc = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16));
    }
    return false;
  }

  // ------------------------------ body ------------------------------------
  const mtx_material mat = sv.materials[si.material];
  // before the emitter sample; the NEE eval and the BSDF sample both read it
  const BsdfData bd = bsdf_at(sv, mat, si.uv);
#if MTX_DIAG_STAMPS
  MTX_STAMP(io.st, 2);
#endif
  const bool smooth = (bsdf_flags(mat) & BF_SMOOTH) != 0;
  bool active_em = (INT == MTX_INT_PATH_MIS ? active_next : true) && smooth;
  const V2 u_em = rng.next_2d();
  DirectionSample ds;
  ds.p = v3s(0.f);
  ds.n = v3s(0.f);
  ds.d = v3s(0.f);
  ds.dist = 0.f;
  ds.pdf = 0.f;
  ds.emitter = -1;
  V3 em_weight = v3s(0.f);
  const bool do_nee = (INT == MTX_INT_NRC) ? true : active_em;  // nrc.py:51-53 samples with `active`
  if (do_nee) em_weight = sample_emitter_direction(sv, si.p, u_em, &ds);
#if MTX_DIAG_STAMPS
  MTX_STAMP(io.st, 3);
#endif
  if (INT != MTX_INT_PATH_MIS) active_em = active_em && ds.pdf != 0.f;
  const V3 wo = to_local(si.sh, ds.d);
  const float s1 = rng.next_1d();
  const V2 s2 = rng.next_2d();
  V3 bsdf_val = v3s(0.f);
  float bsdf_pdf = 0.f;
  BSDFSample bs;
  // eval / pdf only feed the NEE contribution (no draws, no side effects)
  if (active_em) bsdf_eval_pdf(bd, mat, si.uv, si.wi, wo, &bsdf_val, &bsdf_pdf);
  const V3 bsdf_weight = bsdf_sample(bd, mat, si.uv, si.wi, s1, s2, &bs);
#if MTX_DIAG_STAMPS
  MTX_STAMP(io.st, 4);
#endif

  if (INT == MTX_INT_PATH_MIS) {
    const float mi_em = mis_weight_b(ds.pdf, bsdf_pdf);
    if (active_em) {
      const V3 X = bsdf_val * em_weight * mi_em;
      const V3 Xo = bsdf_val * v3s(0.f) * mi_em;
      make_shadow<INT, true>(io, si, ds, T, X, Xo, true, &L);
    }
  } else {
    const float mis_em = INT == MTX_INT_PATH ? mis_weight_a(ds.pdf, bsdf_pdf) : mis_weight_b(ds.pdf, bsdf_pdf);
    if (active_em) {
      const V3 P = T * bsdf_val * em_weight * mis_em;
      const V3 Po = T * bsdf_val * v3s(0.f) * mis_em;
      make_shadow<INT, true>(io, si, ds, T, P, Po, false, &L);
    }
  }

  bool active;
  const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));
  if (INT == MTX_INT_PATH_MIS) {
    T = T * bsdf_weight;
    eta *= bs.eta;
    if (!(bs.type & BF_NULL)) flags |= PF_VALID_RAY;  // :129-133 (active & si.valid hold here)
    prev_p = si.p;
    prev_pdf = bs.pdf;
    flags = (bs.type & BF_DELTA) ? (flags | PF_PREV_DELTA) : (flags & ~PF_PREV_DELTA);
    depth += 1;  // :141 (si valid here)
    const float throughput_max = hmax(T);
    const float rr_prop = fminf(throughput_max * sqr(eta), 0.95f);
    const bool rr_active = depth >= p.rr_depth;
    const bool rr_continue = rng.next_1d() < rr_prop;
    if (rr_active) T = T * rcp(rr_prop);
    active = active_next && (!rr_active || rr_continue) && (throughput_max != 0.f);
  } else if (INT == MTX_INT_PATH) {
    T = T * bsdf_weight;  // path.py:263
    eta *= bs.eta;
    const float fmax_ = hmax(T);
    const float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
    const bool rr_active = depth >= p.rr_depth;
    const bool rr_continue = rng.next_1d() < rr_prob;
    if (rr_active) T = T * rcp(rr_prob);
    active = (fmax_ != 0.f) && (!rr_active || rr_continue);
    prev_p = si.p;
    prev_pdf = bs.pdf;
    flags = (bs.type & BF_DELTA) ? (flags | PF_PREV_DELTA) : (flags & ~PF_PREV_DELTA);
  } else {  // NRC
    T = T * bsdf_weight;
    eta *= bs.eta;
    const float a = sqr(spread);  // nrc.py:70-71
    active = a < p.nrc_c * a0;
    if (!active && p.nrc_cache) {  // trace one more segment to the cache query
      flags |= PF_CACHE_QUERY;
      active = true;
    }
    prev_p = si.p;
    prev_pdf = bs.pdf;
    flags = (bs.type & BF_DELTA) ? (flags | PF_PREV_DELTA) : (flags & ~PF_PREV_DELTA);
  }

  // ray, throughput and previous vertex travel with the queue entry (k_shade
  // stores them at the append slot, coalesced, for continuing paths only);
  // a path that ends is read afterwards through L and misc alone
  io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
  io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, a0);
  io.nthr = make_float4(T.x, T.y, T.z, eta);
  io.nprev = make_float4(prev_p.x, prev_p.y, prev_p.z, spread);
  io.nL = make_float4(L.x, L.y, L.z, (INT == MTX_INT_PATH_MIS && !active) ? end_w(flags, prev_pdf) : prev_pdf);
  io.nmisc = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16));
#if MTX_DIAG_STAMPS
  MTX_STAMP(io.st, 5);
#endif
  return active;
}

// Dr.Jit clamp(x, lo, hi) = maximum(minimum(x, hi), lo), NaN-ignoring (App. A).
__device__ __forceinline__ float dr_clamp(float x, float lo, float hi) { return fmaxf(fminf(x, hi), lo); }

// pssmltsimple.py:60-131 — one bounce of a PSSMLT proposal: emission without
// MIS (:74), BSDF sample masked by active_next (:84), mutation of the local
// direction against the current path's vertex (:88, mutate :135-142),
// re-evaluation (:93-96), proposed vertex write (:99), spawn, RR. Every
// executed bounce consumes 4 draws: the chain's RNG stream continues across
// the Metropolis iterations.
__device__ __forceinline__ bool shade_pssmlt(const DevScene &s, const SceneView &sv, const WaveBuffers &b,
                                             const ChunkParams &p, uint32_t bounce, uint32_t path, uint32_t qi,
                                             const float4 h, ShadeIO &io) {
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  const float4 rd = b.ray_d[rp][qi], th = b.thr[rp][qi], Lr = b.L[rp][qi];
  const uint4 mi = b.misc[rp][qi];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  uint32_t depth = mi.w & 0xffffu;
  const uint32_t flags = mi.w >> 16;
  V3 T = V3{th.x, th.y, th.z};
  float eta = th.w;
  V3 L = V3{Lr.x, Lr.y, Lr.z};
  float prev_pdf = Lr.w;
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{rd.x, rd.y, rd.z});
  const V3 le = (prev_pdf > 0.f) ? emitter_eval(sv, si.emitter, si.wi) : v3s(0.f);
  L = fma3v(T, le, L);
  const bool active_next = (depth + 1 < p.max_depth) && si.valid;
  const float s1 = rng.next_1d();
  const V2 s2 = rng.next_2d();
  BSDFSample bs;
  bs.wo = v3s(0.f);
  bs.pdf = 0.f;
  bs.eta = 0.f;
  bs.type = 0;
  V3 w = v3s(0.f);
  mtx_material mat;
  BsdfData bd = sv.bsdf;
  if (si.valid) {
    mat = sv.materials[si.material];
    bd = bsdf_at(sv, mat, si.uv);
    w = bsdf_sample(bd, mat, si.uv, si.wi, s1, s2, &bs);
  }
  if (!active_next) w = v3s(0.f);
  const float4 o4 = b.vpath[(size_t)depth * b.capacity + path];
  const V3 old = V3{o4.x, o4.y, o4.z};
  V3 vwo = p.large_step ? bs.wo : normalize(old * 0.9f + bs.wo * 0.1f);
  V3 val = v3s(0.f);
  float pdf = 0.f;
  if (si.valid) bsdf_eval_pdf(bd, mat, si.uv, si.wi, vwo, &val, &pdf);
  if (pdf <= 0.f) vwo = bs.wo;
  if (pdf > 0.f) w = val / pdf;
  b.vprop[(size_t)depth * b.capacity + path] = make_float4(vwo.x, vwo.y, vwo.z, 0.f);
  const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, vwo));
  T = T * w;
  eta *= bs.eta;
  prev_pdf = bs.pdf;
  if (si.valid) depth += 1;
  const float fmax_ = hmax(T);
  const float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
  const bool rr_active = depth >= p.rr_depth;
  const bool rr_continue = rng.next_1d() < rr_prob;
  if (rr_active) T = T * rcp(rr_prob);
  const bool active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);
  io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
  io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, 0.f);
  io.nthr = make_float4(T.x, T.y, T.z, eta);
  io.nL = make_float4(L.x, L.y, L.z, prev_pdf);
  io.nmisc = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16));
  return active;
}

// simple.py:55-113 — one bounce of the BSDF-only path tracer: emission at
// the hit without MIS (:69-70, masked by prev_bsdf_pdf > 0), BSDF sample
// masked by active_next (:79), spawn (:84), depth on a valid hit (:102), RR
// (:104-111). 4 draws per executed bounce. The same loop as
// pssmltsimple.py:60-131 without the mutation; bounce 0 starts from the
// constant initial state (f = 1, eta = 1, L = 0, prev_bsdf_pdf = 1).
__device__ __forceinline__ bool shade_simple(const DevScene &s, const SceneView &sv, const WaveBuffers &b,
                                             const ChunkParams &p, uint32_t bounce, uint32_t path, uint32_t qi,
                                             const float4 h, ShadeIO &io) {
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  const float4 rd = b.ray_d[rp][qi];
  const float4 th = bounce == 0 ? kInitThr : b.thr[rp][qi], Lr = bounce == 0 ? kInitL : b.L[rp][qi];
  const uint4 mi = b.misc[rp][qi];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  uint32_t depth = mi.w & 0xffffu;
  const uint32_t flags = mi.w >> 16;
  V3 T = V3{th.x, th.y, th.z};
  float eta = th.w;
  V3 L = V3{Lr.x, Lr.y, Lr.z};
  const float prev_pdf = Lr.w;
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{rd.x, rd.y, rd.z});
  const V3 le = (prev_pdf > 0.f) ? emitter_eval(sv, si.emitter, si.wi) : v3s(0.f);
  L = fma3v(T, le, L);
  const bool active_next = (depth + 1 < p.max_depth) && si.valid;
  const float s1 = rng.next_1d();
  const V2 s2 = rng.next_2d();
  BSDFSample bs;
  bs.wo = v3s(0.f);
  bs.pdf = 0.f;
  bs.eta = 0.f;
  bs.type = 0;
  V3 w = v3s(0.f);
  if (active_next) w = bsdf_sample(sv.bsdf, sv.materials[si.material], si.uv, si.wi, s1, s2, &bs);
  const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));
  T = T * w;
  eta *= bs.eta;
  if (si.valid) depth += 1;
  const float fmax_ = hmax(T);
  const float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
  const bool rr_active = depth >= p.rr_depth;
  const bool rr_continue = rng.next_1d() < rr_prob;
  if (rr_active) T = T * rcp(rr_prob);
  const bool active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);
  io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
  io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, 0.f);
  io.nthr = make_float4(T.x, T.y, T.z, eta);
  io.nL = make_float4(L.x, L.y, L.z, bs.pdf);
  io.nmisc = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16));
  return active;
}

// pssmltpath.py:17-168 — one bounce of a PSSMLT proposal with NEE + MIS:
// emission at the hit weighted against the previous BSDF sample (:71-82),
// unmasked BSDF sample (:99-101), mutation of the local direction AND of the
// emitter sample against the current path's vertex (:103-105, mutate
// :170-190), re-evaluation (:107-110), NEE from the mutated emitter sample
// (:118-134, shadow ray), proposed vertex write (:138), RR (:154-166).
// Draws per bounce: 1 + 2 (BSDF) + 2 (mutation) + 1 (RR).
__device__ __forceinline__ bool shade_pssmlt_path(const DevScene &s, const SceneView &sv, const WaveBuffers &b,
                                                  const ChunkParams &p, uint32_t bounce, uint32_t path, uint32_t qi,
                                                  const float4 h, ShadeIO &io) {
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  const float4 rd = b.ray_d[rp][qi], th = b.thr[rp][qi], Lr = b.L[rp][qi], pv = b.prev[rp][qi];
  const uint4 mi = b.misc[rp][qi];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  uint32_t depth = mi.w & 0xffffu, flags = mi.w >> 16;
  V3 T = V3{th.x, th.y, th.z};
  float eta = th.w;
  V3 L = V3{Lr.x, Lr.y, Lr.z};
  float prev_pdf = Lr.w;
  const V3 prev_p = V3{pv.x, pv.y, pv.z};
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{rd.x, rd.y, rd.z});
  io.emit = false;
  io.query = false;
  // direct emission (:71-82)
  const bool prev_delta = (flags & PF_PREV_DELTA) != 0;
  const V3 rel = si.p - prev_p;
  const float dist = norm(rel);
  const float em_pdf = prev_delta ? 0.f : pdf_emitter_direction(sv, si.emitter, rel / dist, dist, si.sh.n);
  const float mis_bsdf = mis_weight_b(prev_pdf, em_pdf);
  const V3 le = (prev_pdf > 0.f) ? emitter_eval(sv, si.emitter, si.wi) : v3s(0.f);
  L = fma3v(T, le * mis_bsdf, L);
  const bool active_next = (depth + 1 < p.max_depth) && si.valid;  // :84
  // BSDF sampling (:99-101), not masked
  const float s1 = rng.next_1d();
  const V2 s2 = rng.next_2d();
  BSDFSample bs;
  bs.wo = v3s(0.f);
  bs.pdf = 0.f;
  bs.eta = 0.f;
  bs.type = 0;
  V3 w = v3s(0.f);
  mtx_material mat;
  BsdfData bd = sv.bsdf;
  if (si.valid) {
    mat = sv.materials[si.material];
    bd = bsdf_at(sv, mat, si.uv);
    w = bsdf_sample(bd, mat, si.uv, si.wi, s1, s2, &bs);
  }
  // mutate (:170-190): a = 0.01 on the direction, sqrt(0.01) on the emitter sample
  const V2 um = rng.next_2d();
  const size_t vi = (size_t)depth * b.capacity + path;
  const float4 o4 = b.vpath[vi];
  const float2 oes = b.vpath_es[vi];
  V3 vwo;
  V2 es;
  if (p.large_step) {
    vwo = bs.wo;
    es = um;
  } else {
    vwo = normalize(V3{o4.x, o4.y, o4.z} * 0.99f + bs.wo * 0.01f);
    const V2 g = square_to_std_normal(um);
    es = V2{dr_clamp(g.x * 0.1f + oes.x, 0.f, 1.f), dr_clamp(g.y * 0.1f + oes.y, 0.f, 1.f)};
  }
  V3 val = v3s(0.f);
  float pdf = 0.f;
  if (si.valid) bsdf_eval_pdf(bd, mat, si.uv, si.wi, vwo, &val, &pdf);  // :107
  if (pdf <= 0.f) vwo = bs.wo;                                                // :109
  if (pdf > 0.f) w = val / pdf;                                               // :110
  const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, vwo));               // :114
  // emitter sampling from the mutated sample (:118-134)
  const bool active_em = active_next && (bsdf_flags(mat) & BF_SMOOTH) != 0;
  if (active_em) {
    DirectionSample ds;
    const V3 em_weight = sample_emitter_direction(sv, si.p, es, &ds);
    const V3 wo = to_local(si.sh, ds.d);
    V3 ev;
    float epdf;
    bsdf_eval_pdf(bd, mat, si.uv, si.wi, wo, &ev, &epdf);
    const float mi_em = mis_weight_b(ds.pdf, epdf);
    make_shadow<MTX_INT_PSSMLT_PATH, true>(io, si, ds, T, ev * em_weight * mi_em, ev * v3s(0.f) * mi_em, true, &L);
  }
  b.vprop[vi] = make_float4(vwo.x, vwo.y, vwo.z, 0.f);  // :138
  b.vprop_es[vi] = make_float2(es.x, es.y);
  T = T * w;
  eta *= bs.eta;
  prev_pdf = bs.pdf;
  flags = (bs.type & BF_DELTA) ? (flags | PF_PREV_DELTA) : (flags & ~PF_PREV_DELTA);
  if (si.valid) depth += 1;  // :154
  const float fmax_ = hmax(T);
  const float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
  const bool rr_active = depth >= p.rr_depth;
  const bool rr_continue = rng.next_1d() < rr_prob;
  if (rr_active) T = T * rcp(rr_prob);
  const bool active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);
  io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
  io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, 0.f);
  io.nthr = make_float4(T.x, T.y, T.z, eta);
  io.nL = make_float4(L.x, L.y, L.z, prev_pdf);
  io.nprev = make_float4(si.p.x, si.p.y, si.p.z, 0.f);
  io.nmisc = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth | (flags << 16));
  return active;
}

// nerad.py:174-233 Integrator.sample_rhs, one lane = one of the M samples of a
// training point (nerad.py:182-184 dr.repeat). Bounce 0 is the sampled
// surface point itself (hit record written by k_nerad_raygen): NEE with a
// visibility test (:197-200, mis_weight of mitsuba.ad.integrators.common =
// variant B) and a BSDF sample (:204-206). Bounce 1 is the BSDF ray's hit:
// f = mis_weight(bs.pdf, emitter pdf) * bsdf_weight (:208-217), then
// next_smooth_si (:124-164) follows delta / null vertices (bounces 2..11,
// f2 in prev.xyz). At the stop vertex: f *= f2, zero if invalid (:219-222);
// a valid vertex becomes a field query (Le kept in prev.xyz), L += f * (Le +
// field) is applied after the field evaluation (k_nerad_apply, :226-229).
// State: thr.xyz = f, L.w = bs.pdf of bounce 0, prev.xyz = si.p (bounce 0)
// then f2, misc.w = chain depth.
// RENDER: Integrator.sample (nerad.py:235-254) -- a camera lane runs
// next_smooth_si from its first hit (bounce 0 = chain start, no NEE), then
// L = Field(si) * f + Le(si) (applied by k_nerad_apply after the field).
template <bool RENDER>
__device__ __forceinline__ bool shade_nerad(const DevScene &s, const SceneView &sv, const WaveBuffers &b,
                                            uint32_t bounce, uint32_t path, uint32_t qi, const float4 h,
                                            ShadeIO &io) {
  const float4 rd = b.ray_d[(bounce + b.ray_par) & 1u][qi];
  // a rendered lane's bounce-0 state is the camera raygen's (nothing stored)
  const float4 Lr = (RENDER && bounce == 0) ? kInitL : b.L[kFinal][path];
  // thr / prev path-indexed in plane 0 (k_nerad_apply reads prev by path)
  const float4 pv = (RENDER && bounce == 0) ? kInitPrev : b.prev[0][path];
  const float4 th = (RENDER && bounce == 0) ? kInitThr : b.thr[0][path];
  // a rendered lane's bounce-0 sampler state is the camera raygen's (queue plane 0, identity)
  const uint4 mi = (RENDER && bounce == 0) ? b.misc[0][path] : b.misc[kFinal][path];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  uint32_t depth = mi.w & 0xffffu;
  const V3 ray_d = V3{rd.x, rd.y, rd.z};
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, ray_d);
  io.emit = false;
  io.query = false;
  V3 L = V3{Lr.x, Lr.y, Lr.z};
  V3 f = V3{th.x, th.y, th.z};
  V3 f2 = V3{pv.x, pv.y, pv.z};
  if (RENDER && bounce == 0) {  // next_smooth_si's f = Spectrum(1) (:135)
    f = v3s(1.f);
    f2 = v3s(1.f);
    depth = 0;
  }
  if (!RENDER && bounce == 0) {
    const mtx_material mat = sv.materials[si.material];
    DirectionSample ds;
    const V3 em = sample_emitter_direction(sv, si.p, rng.next_2d(), &ds);  // :197
    V3 val;
    float pdf;
    bsdf_eval_pdf(sv.bsdf, mat, si.uv, si.wi, to_local(si.sh, ds.d), &val, &pdf);  // :198
    const float mis = mis_weight_b(ds.pdf, pdf);
    make_shadow<MTX_INT_NERAD_RHS, false>(io, si, ds, v3s(1.f), val * mis * em, val * mis * v3s(0.f), false);  // :200
    const float s1 = rng.next_1d();
    const V2 s2 = rng.next_2d();
    BSDFSample bs;
    const V3 w = bsdf_sample(sv.bsdf, mat, si.uv, si.wi, s1, s2, &bs);  // :204-206
    const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));   // :208
    io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
    io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, 0.f);
    b.thr[0][path] = make_float4(w.x, w.y, w.z, 1.f);
    b.L[kFinal][path] = make_float4(L.x, L.y, L.z, bs.pdf);
    b.prev[0][path] = make_float4(si.p.x, si.p.y, si.p.z, 0.f);
    b.misc[kFinal][path] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, 0u);
    return true;  // traced unconditionally (:209)
  }
  if (!RENDER && bounce == 1) {
    // emitter pdf of the BSDF-sampled hit (:213-216), f (:217)
    const V3 prev_p = f2;
    const V3 rel = si.p - prev_p;
    const float dist = norm(rel);
    const float em_pdf = pdf_emitter_direction(sv, si.emitter, rel / dist, dist, si.sh.n);
    f = f * mis_weight_b(Lr.w, em_pdf);
    f2 = v3s(1.f);
  }
  // next_smooth_si (:124-164): sample at this vertex; continue while delta
  BSDFSample bs;
  bs.type = 0;
  V3 w = v3s(0.f);
  const float s1 = rng.next_1d();
  const V2 s2 = rng.next_2d();
  if (si.valid) {
    const mtx_material mat = sv.materials[si.material];
    w = bsdf_sample(sv.bsdf, mat, si.uv, si.wi, s1, s2, &bs);
  }
  if (bounce > (RENDER ? 0u : 1u)) depth += 1;  // :160
  const bool chain = (bs.type & BF_DELTA) != 0 && depth < 10;
  if (chain) {
    f2 = f2 * w;  // :150
    const Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));
    io.nro = make_float4(nray.o.x, nray.o.y, nray.o.z, nray.maxt);
    io.nrd = make_float4(nray.d.x, nray.d.y, nray.d.z, 0.f);
    b.thr[0][path] = make_float4(f.x, f.y, f.z, 1.f);
    b.prev[0][path] = make_float4(f2.x, f2.y, f2.z, 0.f);
    b.misc[kFinal][path] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, depth);
    return true;
  }
  // stop vertex (:219-229; render: :250-252)
  f = f * f2;
  if (!si.valid) f = f * 0.f;
  const V3 le = emitter_eval(sv, si.emitter, si.wi);
  if (RENDER && !si.valid) {
    L = v3s(0.f) * f + le;
    b.L[kFinal][path] = make_float4(L.x, L.y, L.z, Lr.w);
  } else if (si.valid) {
    io.query = true;
    const V3 wi = to_world(si.sh, si.wi);  // Field.__call__ wi (nerad.py:100)
    io.qp = make_float4(si.p.x, si.p.y, si.p.z, 0.f);
    io.qd = make_float4(wi.x, wi.y, wi.z, 0.f);
    io.qt = make_float4(f.x, f.y, f.z, __uint_as_float(path));
    b.prev[0][path] = make_float4(le.x, le.y, le.z, 0.f);
  } else {
    L = L + f * (le + v3s(0.f));
    b.L[kFinal][path] = make_float4(L.x, L.y, L.z, Lr.w);
  }
  return false;
}

// blocks per CU the shade kernels are built for (their register budget):
// kShadeMinBlocks for every integrator (pssmltpath.py's shade at 2 blocks,
// without its spills, measured slower: DESIGN.md §7)
template <int INT>
__global__ __launch_bounds__(kShadeBlock, kShadeMinBlocks) void k_shade(DevScene s, WaveBuffers b, ChunkParams p, uint32_t bounce) {
  const SceneView sv = make_view(s);
  const uint32_t count = b.counters[4 * bounce + 0];
  const uint32_t *in_q = b.queue[bounce & 1];
  uint32_t *out_q = b.queue[(bounce + 1) & 1];
  // [4(bounce+1)] next queue count, [4(bounce+1)+1] this bounce's shadow
  // rays: one 64-bit pair, reserved by one atomic per block step
  uint32_t *out_cnt = &b.counters[4 * (bounce + 1) + 0];
  const uint32_t rp = (bounce + b.ray_par) & 1u;  // this bounce's ray planes; the next ray goes to rp ^ 1
  // the nerad integrators keep thr / prev / L / misc by path (plane 0 / kFinal)
  constexpr bool kNerad = INT == MTX_INT_NERAD_RHS || INT == MTX_INT_NERAD;
  const uint32_t stride = gridDim.x * kShadeBlock;
  uint32_t parity = 0;
  // software pipeline over the persistent loop: the next step's queue entry
  // loads during this step, its hit record before this step's appends. Hit
  // records are stored by queue position (ClosestSrc), so they load
  // coalesced and in parallel with the queue entry.
  uint32_t path = 0;
  float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
  // an identity bounce-0 queue is not stored: position i is path i
  const bool ident = bounce == 0 && p.ident0;
  if (blockIdx.x * kShadeBlock + threadIdx.x < count) {
    const uint32_t i0 = blockIdx.x * kShadeBlock + threadIdx.x;
    path = ident ? i0 : ld_stream<kNtQueue>(in_q + i0);
    h = ld_stream<kNtShade>(b.hit + i0);
  }

#if MTX_DIAG_STAMPS
  Stamps stp{};
  unsigned long long steps = 0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stp.prev)::"memory");
#endif
  for (uint32_t base = blockIdx.x * kShadeBlock; base < count; base += stride, parity ^= 1u) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t inext = i + stride;
    uint32_t path_n = 0;
    if (inext < count) path_n = ident ? inext : ld_stream<kNtQueue>(in_q + inext);
#if MTX_SHADE_WARM
    float4 hn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (inext < count) hn = b.hit[inext];
    const uint32_t pn = __float_as_uint(hn.y);
    const float4 *wp = (inext < count && pn != 0xffffffffu) ? s.shade_rec + 8 * (size_t)pn : nullptr;
#else
    const float4 *wp = nullptr;
#endif
    ShadeIO io;
    io.emit = false;
    io.em_hi = false;
    io.query = false;
    io.warm = 0.f;
#if MTX_DIAG_STAMPS
    ++steps;
    MTX_STAMP(stp, 0);
    io.st = stp;
#endif
    bool cont = false;
    const bool valid = i < count;
    if (valid) {
      if constexpr (INT == MTX_INT_PSSMLT_SIMPLE)
        cont = shade_pssmlt(s, sv, b, p, bounce, path, i, h, io);
      else if constexpr (INT == MTX_INT_SIMPLE)
        cont = shade_simple(s, sv, b, p, bounce, path, i, h, io);
      else if constexpr (INT == MTX_INT_PSSMLT_PATH)
        cont = shade_pssmlt_path(s, sv, b, p, bounce, path, i, h, io);
      else if constexpr (INT == MTX_INT_NERAD_RHS)
        cont = shade_nerad<false>(s, sv, b, bounce, path, i, h, io);
      else if constexpr (INT == MTX_INT_NERAD)
        cont = shade_nerad<true>(s, sv, b, bounce, path, i, h, io);
      else
        cont = shade_path<INT>(s, sv, b, p, bounce, path, i, h, io, wp);
    }
    (void)wp;
    const uint32_t path_c = path;
    path = path_n;
#if MTX_SHADE_WARM
    h = hn;
    asm volatile("" ::"v"(io.warm));  // the warm-up load completes in this iteration
#else
    if (inext < count) h = ld_stream<kNtShade>(b.hit + inext);
#endif

#if MTX_DIAG_STAMPS
    stp = io.st;
#endif
    uint32_t slot, sslot;
    block_append2<kShadeBlock>(cont, io.emit, io.emit && io.em_hi, out_cnt, parity, slot, sslot);
    if (cont) {
      st_stream<kNtQueue>(out_q + slot, path_c);
      st_stream<kNtShadeSt>(b.ray_o[rp ^ 1u] + slot, io.nro);
      st_stream<kNtShadeSt>(b.ray_d[rp ^ 1u] + slot, io.nrd);
      if constexpr (!kNerad) st_stream<kNtShadeSt>(b.thr[rp ^ 1u] + slot, io.nthr);
      if constexpr (INT == MTX_INT_PATH_MIS || INT == MTX_INT_PATH || INT == MTX_INT_NRC || INT == MTX_INT_PSSMLT_PATH)
        st_stream<kNtShadeSt>(b.prev[rp ^ 1u] + slot, io.nprev);
      if constexpr (!kNerad) {
        st_stream<kNtShadeSt>(b.L[rp ^ 1u] + slot, io.nL);
        st_stream<kNtShadeSt>(b.misc[rp ^ 1u] + slot, io.nmisc);
      }
    } else if (!kNerad && valid) {
      st_stream<kNtShadeSt>(b.L[kFinal] + path_c, io.nL);
      if (!p.drop_end_misc) st_stream<kNtShadeSt>(b.misc[kFinal] + path_c, io.nmisc);
    }
    if (io.emit) {
      // the contribution goes to the path's L where the next shade (or the
      // film) reads it; the integrators that emit shadow rays (path-mis,
      // path, nrc, pssmltpath; not the nerad ones) store io.nL there
      const uint32_t li = (kNerad || !cont) ? kFinal * b.capacity + path_c : (rp ^ 1u) * b.capacity + slot;
      io.rec.d.w = __uint_as_float(li);
      if constexpr (!kNerad) io.rec.x.w = io.nL.w;  // final-value form: L.w (set after the NEE)
      ShadowRec *sr = b.shadow + sslot;
      st_stream<kNtShadeSt>(&sr->o, io.rec.o);
      st_stream<kNtShadeSt>(&sr->d, io.rec.d);
      st_stream<kNtShadeSt>(&sr->t, io.rec.t);
      st_stream<kNtShadeSt>(&sr->x, io.rec.x);
    }
#if MTX_DIAG_STAMPS
    MTX_STAMP(stp, 6);
#endif
    if constexpr (INT == MTX_INT_NRC || INT == MTX_INT_NERAD_RHS || INT == MTX_INT_NERAD) {
      if (INT != MTX_INT_NRC || p.nrc_cache) {
        const uint32_t q = block_reserve<kShadeBlock>(io.query ? 1u : 0u, b.cq_count);
        if (io.query) {
          b.cq_p[q] = io.qp;
          b.cq_d[q] = io.qd;
          b.cq_t[q] = io.qt;
        }
      }
    }
#if MTX_DIAG_STAMPS
    MTX_STAMP(stp, 7);
#endif
  }
#if MTX_DIAG_STAMPS
  if ((threadIdx.x & 63u) == 0) {
    for (int k = 0; k < kStampSegs; ++k) atomicAdd(&g_shade_stamps[k], stp.acc[k]);
    atomicAdd(&g_shade_stamps[kStampSegs], steps);
    atomicAdd(&g_shade_stamps[kStampSegs + 1], 1ull);
  }
#endif
}

// Paths still queued after a chunk's last bounce (its depth limit stops
// every integrator's paths first; kept so that no loop bound can leave a
// result in a queue plane): their L / misc move to the per-path plane.
// A path-mis path's final L.w holds valid_ray (end_w), not its prev_bsdf_pdf.
__global__ void k_flush_tail(WaveBuffers b, uint32_t bounce, uint32_t integrator) {
  const uint32_t n = b.counters[4 * bounce];
  const uint32_t *q = b.queue[bounce & 1];
  const uint32_t rp = (bounce + b.ray_par) & 1u;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t path = q[k];
    float4 L = b.L[rp][k];
    const uint4 m = b.misc[rp][k];
    // decided by the shade variant: ReSTIR GI's secondary paths are shaded by
    // the path-mis kernel (launch_shade), so their final L.w is valid_ray too,
    // the bits k_path_mega<PATH_MIS> stores for the same path
    if (integrator == MTX_INT_PATH_MIS || integrator == MTX_INT_RESTIR_GI) L.w = end_w(m.w >> 16, L.w);
    b.L[kFinal][path] = L;
    b.misc[kFinal][path] = m;
  }
}

// Path megakernel for short wavefronts (ReSTIR GI's secondary paths of a
// row band): each thread takes one queued path and runs all of its bounces
// -- closest hit (traverse_closest), shade_path, the NEE shadow ray
// (traverse_occ) applied to its L at once -- with its state kept at its own
// queue position (no compaction). A short queue leaves most lanes of the
// wavefront kernels idle and each launch waits for its slowest ray, once per
// bounce and kernel; here a path waits only on its own chain. Same operations
// per path as the wavefront kernels (same hits: the closest hit does not
// depend on the visit order; same shading code), so the same bits. The block's
// dynamic LDS holds one traversal stack column per thread (stack_bytes).
#ifndef MTX_MEGA_MIN_BLOCKS
#define MTX_MEGA_MIN_BLOCKS 3  // A/B: 4 = <= 128 VGPRs (spills), every band path resident at once
#endif
// The traversals index their LDS stack columns with the stride kTraceBlock and
// stack_bytes() sizes the allocation with it: a megakernel block of another
// width would let threads share stack words.
static_assert(kShadeBlock == kTraceBlock, "k_path_mega: stack column stride must equal the block width");
// Round 5: lanes, not waves, take paths. Each iteration a lane runs ONE
// bounce of its path; a lane whose path has ended takes the next queued path
// as soon as kMegaRefill lanes of its wave are idle (one claim atomic per
// refill for all of them, consecutive queue positions), so a wave no longer
// waits for the longest of its 64 paths before any lane starts another (the
// round-4 form claimed 64 paths per wave and ran them to completion).
#ifndef MTX_MEGA_REFILL
#define MTX_MEGA_REFILL 16  // idle lanes of a wave that trigger a claim (64: the round-4 whole-wave batches)
#endif
template <int INT>
__global__ __launch_bounds__(kShadeBlock, MTX_MEGA_MIN_BLOCKS) void k_path_mega(DevScene s, WaveBuffers b, ChunkParams p) {
  static_assert(INT == MTX_INT_PATH_MIS || INT == MTX_INT_PATH, "megakernel: path / path-mis only");
  extern __shared__ int4 mega_lds[];
  const SceneView sv = make_view(s);
  const uint32_t count = b.counters[0];
  const uint32_t iters = p.max_depth > 1u ? p.max_depth : 1u;
  int32_t *stk = reinterpret_cast<int32_t *>(mega_lds) + threadIdx.x;
  uint32_t *ostk = reinterpret_cast<uint32_t *>(mega_lds) + threadIdx.x;  // the same column
  const uint32_t lane = threadIdx.x & 63u;
  bool has = false, drained = false;
  uint32_t qi = 0, path = 0, bounce = 0;
  while (true) {
    // ---- refill: the idle lanes of the wave claim consecutive queue positions
    if (!drained) {
      const uint64_t idle = __ballot(!has);
      const uint32_t n_idle = (uint32_t)__popcll(idle);
      if (n_idle >= MTX_MEGA_REFILL || idle == ~0ull) {
        const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)idle) - 1);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&b.counters[2], n_idle);
        base = __builtin_amdgcn_readlane(base, leader);
        if (base + n_idle >= count) drained = true;
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (!has && base + rk < count) {
          has = true;
          qi = base + rk;
          path = p.ident0 ? qi : b.queue[0][qi];
          bounce = 0;
        }
      }
    }
    if (__ballot(has) == 0) break;
    if (has) {
      // ---- one bounce of the lane's path
      const uint32_t rp = (bounce + b.ray_par) & 1u;
      const float4 o4 = b.ray_o[rp][qi], d4 = b.ray_d[rp][qi];
      const TraceRay r = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
      float tbest = o4.w, bu = 0.f, bv = 0.f;
      uint32_t prim = 0xffffffffu, nv = 0, tv = 0;
      traverse_closest(s, stk, r, tbest, prim, bu, bv, nv, tv);
      const float4 h = make_float4(prim == 0xffffffffu ? kInf : tbest, __uint_as_float(prim), bu, bv);
      ShadeIO io;
      io.emit = false;
      io.em_hi = false;
      io.query = false;
      const bool cont = shade_path<INT>(s, sv, b, p, bounce, path, qi, h, io);
      if (io.emit) {
        const float4 so = io.rec.o, sd = io.rec.d;
        const TraceRay sr = make_trace_ray(V3{so.x, so.y, so.z}, V3{sd.x, sd.y, sd.z}, so.w);
        apply_shadow_rec(io.nL, io.rec, traverse_occ(s, ostk, sr, so.w, nv, tv));
      }
      ++bounce;
      if (cont && bounce < iters) {
        b.ray_o[rp ^ 1u][qi] = io.nro;
        b.ray_d[rp ^ 1u][qi] = io.nrd;
        b.thr[rp ^ 1u][qi] = io.nthr;
        b.prev[rp ^ 1u][qi] = io.nprev;
        b.L[rp ^ 1u][qi] = io.nL;
        b.misc[rp ^ 1u][qi] = io.nmisc;
      } else {
        // ended, or still queued after the last bounce (k_flush_tail's move:
        // a path-mis path's final L.w holds valid_ray)
        float4 L = io.nL;
        if (cont && INT == MTX_INT_PATH_MIS) L.w = end_w(io.nmisc.w >> 16, L.w);
        b.L[kFinal][path] = L;
        if (!p.drop_end_misc || cont) b.misc[kFinal][path] = io.nmisc;
        has = false;
      }
    }
  }
}

// ReSTIR GI stage A of a short band in ONE launch (round 5): a lane takes a
// pixel sample t of the band and runs restirgi.py's sample_initial for it --
// the camera ray (k_raygen_camera), the primary closest hit, k_rs_begin's
// emittance and BSDF / hemisphere sample (:419-448), then the secondary
// path's bounces (the path megakernel's body, :459-588) and k_rs_collect's
// L_o / sampler store -- with its path state at its own position t, then
// takes the next sample (lanes refill as in k_path_mega). The same per-lane
// operations as the five launches it replaces (hits do not depend on the
// traversal order), so the same reservoirs and films; k_rs_temporal follows
// as its own launch (it reads other pixels' samples).
__global__ __launch_bounds__(kShadeBlock, MTX_MEGA_MIN_BLOCKS) void k_rs_stage_a(DevScene s, WaveBuffers b,
                                                                                  ChunkParams p, RestirBuffers r) {
  extern __shared__ int4 mega_lds[];
  const SceneView sv = make_view(s);
  const uint32_t count = r.nb;
  const uint32_t iters = p.max_depth > 1u ? p.max_depth : 1u;
  int32_t *stk = reinterpret_cast<int32_t *>(mega_lds) + threadIdx.x;
  uint32_t *ostk = reinterpret_cast<uint32_t *>(mega_lds) + threadIdx.x;
  // b.ray_par == 1 (launch_rs_stage_a): the secondary loop's bounce-0 rays are parity 1
  const uint32_t lane = threadIdx.x & 63u;
  const size_t n = r.n;
  bool has = false, drained = false, started = false;
  uint32_t t = 0, bounce = 0;
  while (true) {
    if (!drained) {
      const uint64_t idle = __ballot(!has);
      const uint32_t n_idle = (uint32_t)__popcll(idle);
      if (n_idle >= MTX_MEGA_REFILL || idle == ~0ull) {
        const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)idle) - 1);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&b.counters[2], n_idle);
        base = __builtin_amdgcn_readlane(base, leader);
        if (base + n_idle >= count) drained = true;
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (!has && base + rk < count) {
          has = true;
          started = false;
          t = base + rk;
        }
      }
    }
    if (__ballot(has) == 0) break;
    if (has) {
      const uint32_t i = r.lane0 + t;
      float4 o4, d4;
      Pcg32 rng;
      if (!started) {
        // the camera ray of sample t (k_raygen_camera; init_path's sampler state)
        const uint32_t px_local = t / p.spp, smp = t - px_local * p.spp;
        const uint32_t pix = p.px0 + px_local;
        const uint32_t y = pix / p.width, x = pix - y * p.width;
        rng = sampler_lane(p.seed, pix * p.spp_total + p.sample_offset + smp);
        const V2 u = rng.next_2d();  // film jitter (path.py:45)
        const Ray ray = camera_ray(s.camera, V2{((float)x + u.x) / (float)p.width, ((float)y + u.y) / (float)p.height});
        o4 = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.maxt);
        d4 = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.f);
      } else {
        const uint32_t rp = (bounce + 1u) & 1u;
        o4 = b.ray_o[rp][t];
        d4 = b.ray_d[rp][t];
      }
      const TraceRay tr = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
      float tbest = o4.w, bu = 0.f, bv = 0.f;
      uint32_t prim = 0xffffffffu, nv = 0, tv = 0;
      traverse_closest(s, stk, tr, tbest, prim, bu, bv, nv, tv);
      const float4 h = make_float4(prim == 0xffffffffu ? kInf : tbest, __uint_as_float(prim), bu, bv);
      float4 Lf;
      uint4 mf;
      bool done = false;
      if (!started) {
        // k_rs_begin (:419-448)
        r.prim_hit[i] = h;
        r.prim_dir[i] = d4;
        const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{d4.x, d4.y, d4.z});
        r.emit[i] = f4(emitter_eval(sv, si.emitter, si.wi), 0.f);
        V3 wo;
        float pdf;
        if (r.flags & MTX_RESTIR_BSDF_SAMPLING) {
          const float s1 = rng.next_1d();
          const V2 s2 = rng.next_2d();
          BSDFSample bs;
          bs.wo = v3s(0.f);
          bs.pdf = 0.f;
          if (si.valid) bsdf_sample(sv.bsdf, sv.materials[si.material], si.uv, si.wi, s1, s2, &bs);
          wo = bs.wo;
          pdf = bs.pdf;
        } else {
          wo = square_to_uniform_hemisphere(rng.next_2d());
          pdf = square_to_uniform_hemisphere_pdf(wo);
        }
        r.cur[i] = si.valid ? f4(si.p, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
        r.cur[n + i] = si.valid ? f4(si.n, pdf) : make_float4(0.f, 0.f, 0.f, pdf);
        if (si.valid) {
          const Ray nr = spawn_ray(si.p, si.n, to_world(si.sh, wo));
          b.ray_o[1][t] = make_float4(nr.o.x, nr.o.y, nr.o.z, nr.maxt);
          b.ray_d[1][t] = make_float4(nr.d.x, nr.d.y, nr.d.z, 0.f);
          b.misc[1][t] = st_rng(rng, PF_PREV_DELTA << 16);  // depth 0, prev_bsdf_delta
          started = true;
          bounce = 0;
        } else {
          rng.advance(6);
          Lf = make_float4(0.f, 0.f, 0.f, 1.f);
          mf = st_rng(rng, 0u);
          b.rs_xs[t] = make_float4(0.f, 0.f, 0.f, 0.f);
          b.rs_ns[t] = make_float4(0.f, 0.f, 0.f, 0.f);
          done = true;
        }
      } else {
        // one bounce of the secondary path (k_path_mega's body)
        const uint32_t rp = (bounce + 1u) & 1u;
        ShadeIO io;
        io.emit = false;
        io.em_hi = false;
        io.query = false;
        const bool cont = shade_path<MTX_INT_PATH_MIS>(s, sv, b, p, bounce, t, t, h, io);
        if (io.emit) {
          const float4 so = io.rec.o, sd = io.rec.d;
          const TraceRay sr = make_trace_ray(V3{so.x, so.y, so.z}, V3{sd.x, sd.y, sd.z}, so.w);
          apply_shadow_rec(io.nL, io.rec, traverse_occ(s, ostk, sr, so.w, nv, tv));
        }
        ++bounce;
        if (cont && bounce < iters) {
          b.ray_o[rp ^ 1u][t] = io.nro;
          b.ray_d[rp ^ 1u][t] = io.nrd;
          b.thr[rp ^ 1u][t] = io.nthr;
          b.prev[rp ^ 1u][t] = io.nprev;
          b.L[rp ^ 1u][t] = io.nL;
          b.misc[rp ^ 1u][t] = io.nmisc;
        } else {
          Lf = io.nL;
          if (cont) Lf.w = end_w(io.nmisc.w >> 16, Lf.w);
          mf = io.nmisc;
          done = true;
        }
      }
      if (done) {
        // k_rs_collect: L_o = select(valid_ray, result, 0) (:588), x_s / n_s of
        // the first secondary hit (written by the bounce-0 shade), sampler state
        const bool valid_ray = ((mf.w >> 16) & PF_VALID_RAY) != 0;
        r.cur[2 * n + i] = b.rs_xs[t];
        r.cur[3 * n + i] = b.rs_ns[t];
        r.cur[4 * n + i] = valid_ray ? make_float4(Lf.x, Lf.y, Lf.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
        r.rng[i] = mf;
        has = false;
      }
    }
  }
}
void launch_rs_stage_a(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                       int grid, hipStream_t st) {
  WaveBuffers b1 = b;
  b1.ray_par = 1;
  hipLaunchKernelGGL(k_rs_stage_a, dim3(grid), dim3(kShadeBlock), stack_bytes(s), st, s, b1, p, r);
}

// L += T * Field(query) for the NRC cache queries of a chunk (nrc.py L is a
// plain sum: L = L + T * out, as the oracle-side composition in the tests).
__global__ void k_cache_apply(WaveBuffers b, const float *out, const uint32_t *perm) {
  const uint32_t n = *b.cq_count;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const float4 t = b.cq_t[perm ? perm[q] : q];  // out row q belongs to query perm[q]
    const uint32_t path = __float_as_uint(t.w);
    float4 L = b.L[kFinal][path];
    L.x = L.x + t.x * out[3 * (size_t)q];
    L.y = L.y + t.y * out[3 * (size_t)q + 1];
    L.z = L.z + t.z * out[3 * (size_t)q + 2];
    b.L[kFinal][path] = L;
  }
}

// ---------------------------------------------------------------------------
// Film: stage 1 per source pixel (3x3 tent footprint, samples in order),
// stage 2 per film pixel (9 neighbours in fixed order). See DESIGN.md.
// ---------------------------------------------------------------------------
__device__ __forceinline__ V3 final_L(const WaveBuffers &b, const ChunkParams &p, uint32_t path) {
  const float4 l = b.L[kFinal][path];
  V3 L = V3{l.x, l.y, l.z};
  if (p.integrator == MTX_INT_PATH_MIS && !end_valid(b, path, l.w)) L = v3s(0.f);  // path-mis.py:155
  return L;
}

// Pixel-major chunks: a pixel's samples are contiguous, so one wave stages
// 64 pixels x kFilmStage samples through LDS with coalesced loads, then each
// lane accumulates its own pixel in sample order (same order as below).
constexpr int kFilmStage = 8;  // 8 (11.5 KB of LDS per wave, twice the waves per CU) beat 16 by 0.8 ms, and 4

__device__ __forceinline__ void film_accumulate(float4 acc[9], int x, int y, float2 ps, V3 L) {
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const float wy = fmaxf(0.f, 1.f - fabsf(ps.y - ((float)(y + dy - 1) + 0.5f)));
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const float wx = fmaxf(0.f, 1.f - fabsf(ps.x - ((float)(x + dx - 1) + 0.5f)));
      const float w = wx * wy;
      float4 &c = acc[dy * 3 + dx];
      c.x = c.x + L.x * w;
      c.y = c.y + L.y * w;
      c.z = c.z + L.z * w;
      c.w = c.w + w;
    }
  }
}

// Partial film slots (mtx_core/common.h film_slot): with p.film_slots == 8
// a lane moves on to the next slot's contribution planes whenever its sample
// index passes a slot end (the same for every lane of the launch: no
// divergence) and writes all 8 slots (zeros for slots without samples);
// otherwise one slot. contrib: [slot][9][band_px].
struct FilmSlots {
  uint32_t cur, end, T, mask;
  bool eight;
  __device__ __forceinline__ void init(const ChunkParams &p) {
    eight = p.film_slots == 8;
    mask = eight ? p.slot_mask : 1u;
    T = p.spp_total;
    cur = 0;
    end = eight ? film_slot_end(0, T) : 0xffffffffu;
  }
  __device__ __forceinline__ void flush(float4 acc[9], float4 *contrib, const ChunkParams &p, size_t o) {
    const bool used = (mask >> cur) & 1u;  // a slot without samples of this render stays unwritten
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (used) contrib[((size_t)cur * 9 + k) * p.band_px + o] = acc[k];
      acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    ++cur;
    end = cur < 7 ? film_slot_end(cur, T) : 0xffffffffu;
  }
  // before accumulating global sample g
  __device__ __forceinline__ void advance(uint32_t g, float4 acc[9], float4 *contrib, const ChunkParams &p, size_t o,
                                          bool write) {
    while (g >= end) {
      if (write) {
        flush(acc, contrib, p, o);
      } else {
        ++cur;
        end = cur < 7 ? film_slot_end(cur, T) : 0xffffffffu;
      }
    }
  }
  __device__ __forceinline__ void finish(float4 acc[9], float4 *contrib, const ChunkParams &p, size_t o) {
    const uint32_t n = eight ? 8u : 1u;
    while (cur < n) flush(acc, contrib, p, o);
  }
};

__global__ __launch_bounds__(64) void k_film_src_staged(WaveBuffers b, ChunkParams p, float4 *contrib) {
  constexpr int S = kFilmStage;
  __shared__ float sv[5][64][S + 1];  // L.xyz, pos.xy
  const uint32_t q0 = blockIdx.x * 64, lane = threadIdx.x, q = q0 + lane;
  const uint32_t pix = p.px0 + q;
  const int y = (int)(pix / p.width), x = (int)(pix - (uint32_t)y * p.width);
  const bool mask_valid = p.integrator == MTX_INT_PATH_MIS;
  const bool live = q < p.n_px;
  const size_t o = (size_t)(pix - p.band_y0 * p.width);  // contrib: [slot][9][band_px]
  FilmSlots fs;
  fs.init(p);
  float4 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t s0 = 0; s0 < p.spp; s0 += S) {
    const uint32_t ns = min((uint32_t)S, p.spp - s0);
#pragma unroll 4
    for (int it = 0; it < S; ++it) {
      const uint32_t e = (uint32_t)it * 64 + lane, j = e / S, sm = e % S;
      if (q0 + j < p.n_px && sm < ns) {
        const uint32_t path = (q0 + j) * p.spp + s0 + sm;
        float4 l = ld_stream<kNtQueue>(b.L[kFinal] + path);
        if (mask_valid && !end_valid(b, path, l.w)) l = make_float4(0.f, 0.f, 0.f, 0.f);
        const float2 ps = ld_stream<kNtQueue>(b.pos + path);
        sv[0][j][sm] = l.x;
        sv[1][j][sm] = l.y;
        sv[2][j][sm] = l.z;
        sv[3][j][sm] = ps.x;
        sv[4][j][sm] = ps.y;
      }
    }
    __syncthreads();
    for (uint32_t sm = 0; sm < ns; ++sm) {
      fs.advance(p.sample_offset + s0 + sm, acc, contrib, p, o, live);
      if (live)
        film_accumulate(acc, x, y, make_float2(sv[3][lane][sm], sv[4][lane][sm]),
                        V3{sv[0][lane][sm], sv[1][lane][sm], sv[2][lane][sm]});
    }
    __syncthreads();
  }
  if (!live) return;
  fs.finish(acc, contrib, p, o);
}

__global__ void k_film_src(WaveBuffers b, ChunkParams p, float4 *contrib) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.n_px) return;
  const uint32_t pix = p.px0 + q;
  const int y = (int)(pix / p.width), x = (int)(pix - (uint32_t)y * p.width);
  const size_t o = (size_t)(pix - p.band_y0 * p.width);  // contrib: [slot][9][band_px]
  FilmSlots fs;
  fs.init(p);
  float4 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t sidx = 0; sidx < p.spp; ++sidx) {
    fs.advance(p.sample_offset + sidx, acc, contrib, p, o, true);
    const uint32_t path = q * p.spp + sidx;
    film_accumulate(acc, x, y, b.pos[path], final_L(b, p, path));
  }
  fs.finish(acc, contrib, p, o);
}

// Stage 2: per film pixel and slot the 9 neighbours in (dy, dx) order, then
// the slots' fixed binary tree (film_tree8) when nslots == 8. Slots outside
// slot_mask hold no sample of the render: they are zero, not read (a sum
// that starts at +0 never becomes -0, so adding their +0 changes nothing).
__global__ void k_film_gather(const float4 *contrib, float4 *film, uint32_t W, uint32_t y0, uint32_t y1,
                              uint32_t nslots, uint32_t slot_mask) {
  const uint32_t FW = W + 2, FH = (y1 - y0) + 2;
  const size_t P = (size_t)(y1 - y0) * W;  // contrib: [slot][9][band pixels]
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= FW * FH) return;
  const int px = (int)(q % FW) - 1, py = (int)(y0 + q / FW) - 1;
  V4 sl[8];
  const uint32_t ns = nslots == 8 ? 8u : 1u;
  for (uint32_t k = 0; k < ns; ++k) {
    float r = 0.f, g = 0.f, bl = 0.f, w = 0.f;
    if (ns == 8 && !((slot_mask >> k) & 1u)) {
      sl[k] = V4{r, g, bl, w};
      continue;
    }
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int sxp = px - dx + 1, syp = py - dy + 1;
        if (sxp < 0 || sxp >= (int)W || syp < (int)y0 || syp >= (int)y1) continue;
        const float4 c = contrib[((size_t)k * 9 + (size_t)(dy * 3 + dx)) * P + (size_t)(syp - (int)y0) * W + sxp];
        r = r + c.x;
        g = g + c.y;
        bl = bl + c.z;
        w = w + c.w;
      }
    sl[k] = V4{r, g, bl, w};
  }
  const V4 f = ns == 8 ? film_tree8(sl) : sl[0];
  film[q] = make_float4(f.x, f.y, f.z, f.w);
}

__global__ void k_collect(WaveBuffers b, ChunkParams p, float *L_out, uint8_t *valid_out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_paths) return;
  const V3 L = final_L(b, p, i);
  L_out[3 * (size_t)i] = L.x;
  L_out[3 * (size_t)i + 1] = L.y;
  L_out[3 * (size_t)i + 2] = L.z;
  const uint32_t flags = b.misc[kFinal][i].w >> 16;
  uint8_t v = 1;
  if (p.integrator == MTX_INT_PATH_MIS) v = (flags & PF_VALID_RAY) ? 1 : 0;
  if (p.integrator == MTX_INT_NRC) v = (flags & PF_PRIMARY_VALID) ? 1 : 0;
  if (p.integrator == MTX_INT_SIMPLE) v = (b.misc[kFinal][i].w & 0xffffu) != 0 ? 1 : 0;  // simple.py:118
  valid_out[i] = v;
}

// Raw traversal for mtx_trace: rays as (o.xyz, maxt), (d.xyz, 0). mode 0
// closest hit (4-wide tree), 1 any hit (8-wide occlusion tree).
__device__ __forceinline__ void trace_raw_one(const DevScene &s, const float4 *rays, uint32_t i, int any_hit,
                                              uint32_t *hits, uint32_t *visits, int4 *raw_lds) {
  const float4 o4 = rays[2 * (size_t)i], d4 = rays[2 * (size_t)i + 1];
  TraceRay r = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
  float tbest = o4.w, bu = 0.f, bv = 0.f;
  uint32_t prim = 0xffffffffu, nv = 0, tv = 0;
  if (any_hit == 1) {
    hits[i] = traverse_occ(s, reinterpret_cast<uint32_t *>(raw_lds) + threadIdx.x, r, o4.w, nv, tv) ? 1u : 0u;
  } else {
    traverse_closest(s, reinterpret_cast<int32_t *>(raw_lds) + threadIdx.x, r, tbest, prim, bu, bv, nv, tv);
    if (prim == 0xffffffffu) tbest = kInf;
    hits[4 * (size_t)i + 0] = __float_as_uint(tbest);
    hits[4 * (size_t)i + 1] = prim;
    hits[4 * (size_t)i + 2] = __float_as_uint(bu);
    hits[4 * (size_t)i + 3] = __float_as_uint(bv);
  }
  if (visits) {
    visits[2 * (size_t)i] = nv;
    visits[2 * (size_t)i + 1] = tv;
  }
}

__global__ __launch_bounds__(kTraceBlock) void k_trace_raw(DevScene s, const float4 *rays, uint32_t n, int any_hit,
                                                           uint32_t *hits, uint32_t *visits) {
  extern __shared__ int4 raw_lds[];  // one stack column per thread (device_common.h stack_bytes)
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    trace_raw_one(s, rays, i, any_hit, hits, visits, raw_lds);
}

// ---------------------------------------------------------------------------
// PSSMLT chain kernels (pssmlt.py:167-228). Chains of a chunk keep their
// state in HBM across all Metropolis iterations; chain i of the chunk is
// chain s = sample_offset + i % spp of pixel px0 + i / spp, sampler lane
// pixel * spp_total + s (pssmlt.py:188-193 with wavefront W*H*spp_total): a
// chain range [sample_offset, sample_offset + spp) of every pixel is a shard
// of the spp_total-chain render (multi-GPU, chains never leave their pixel).
// ---------------------------------------------------------------------------
__global__ void k_mlt_init(WaveBuffers b, ChunkParams p, uint32_t max_depth) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_paths) return;
  const uint32_t q = i / p.spp;
  const Pcg32 rng = sampler_lane(p.seed, (p.px0 + q) * p.spp_total + p.sample_offset + (i - q * p.spp));
  b.misc[kFinal][i] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, 0u);
  // offset = 0.5, cumulative_weight = 0 (:198-200); w: vertex depths that may
  // differ between the proposed and current buffers (k_mlt_end)
  b.mlt_cur[i] = make_float4(0.5f, 0.5f, 0.f, 0.f);
  b.mlt_L[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t d = 0; d < max_depth; ++d) {
    b.vpath[(size_t)d * b.capacity + i] = make_float4(0.f, 0.f, 0.f, 0.f);
    b.vprop[(size_t)d * b.capacity + i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.integrator == MTX_INT_PSSMLT_PATH) {
      b.vpath_es[(size_t)d * b.capacity + i] = make_float2(0.f, 0.f);
      b.vprop_es[(size_t)d * b.capacity + i] = make_float2(0.f, 0.f);
    }
  }
}

// render_sample head (:122-129): offset mutation, camera ray, path state.
__global__ void k_mlt_begin(DevScene s, WaveBuffers b, ChunkParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) b.counters[0] = p.n_paths;
  if (i >= p.n_paths) return;
  const uint4 mi = b.misc[kFinal][i];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  const V2 u = rng.next_2d();
  V2 po;
  if (p.large_step) {
    po = u;
  } else {  // mutate_offset (:245-255)
    const float4 cur = b.mlt_cur[i];
    const V2 g = square_to_std_normal(u);
    const float k = 0.31622776601683794f;  // sqrt(0.1)
    po = V2{dr_clamp(g.x * k + cur.x, 0.f, 1.f), dr_clamp(g.y * k + cur.y, 0.f, 1.f)};
  }
  const uint32_t pix = p.px0 + i / p.spp;
  const uint32_t y = pix / p.width, x = pix - y * p.width;
  const V2 sp = V2{((float)x + po.x) / (float)p.width, ((float)y + po.y) / (float)p.height};
  const Ray ray = camera_ray(s.camera, sp);
  b.mlt_prop[i] = make_float2(po.x, po.y);
  b.ray_o[0][i] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.maxt);  // queue position i (identity)
  b.ray_d[0][i] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.f);
  b.thr[0][i] = make_float4(1.f, 1.f, 1.f, 1.f);
  b.L[0][i] = make_float4(0.f, 0.f, 0.f, 1.f);  // prev_bsdf_pdf = 1 (queue position i)
  // pssmltpath.py:39-44: prev_si zero, prev_bsdf_delta = True, valid_ray = scene.environment() is not None
  const uint32_t fl =
      p.integrator == MTX_INT_PSSMLT_PATH ? ((PF_PREV_DELTA | (s.has_env ? PF_VALID_RAY : 0u)) << 16) : 0u;
  if (p.integrator == MTX_INT_PSSMLT_PATH) b.prev[0][i] = make_float4(0.f, 0.f, 0.f, 0.f);
  b.misc[0][i] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, fl);
  if (!p.ident0) b.queue[0][i] = i;
}

// render_sample tail (:137-159): acceptance, cumulative weights, state swap.
__global__ void k_mlt_end(WaveBuffers b, ChunkParams p, uint32_t max_depth) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_paths) return;
  const uint4 mi = b.misc[kFinal][i];
  Pcg32 rng;
  rng.state = ((uint64_t)mi.y << 32) | (uint64_t)mi.x;
  rng.seq = mi.z;
  const float4 lp4 = b.L[kFinal][i];
  const V3 Lp = V3{lp4.x, lp4.y, lp4.z};
  float4 cur = b.mlt_cur[i];
  const float4 lc4 = b.mlt_L[i];
  const float a = dr_clamp(luminance(Lp) / luminance(V3{lc4.x, lc4.y, lc4.z}), 0.f, 1.f);
  const bool accept = rng.next_1d() < a;
  if (accept) {
    cur.z = a;
  } else {
    cur.z += 1.f - a;
  }
  // The reference copies all max_depth proposed vertices on acceptance
  // (dr.tile(accept, max_depth), :155-158). A proposal writes depths
  // 0..depth only (its final depth is in misc), so the two vertex buffers can
  // differ only below the largest such bound since the chain's last
  // acceptance (cur.w): copying those depths gives the same current path.
  uint32_t dirty = max((uint32_t)cur.w, min(max_depth, (mi.w & 0xffffu) + 1u));
  if (accept) {
    const float2 po = b.mlt_prop[i];
    cur.x = po.x;
    cur.y = po.y;
    b.mlt_L[i] = make_float4(Lp.x, Lp.y, Lp.z, 0.f);
    for (uint32_t d = 0; d < dirty; ++d)
      b.vpath[(size_t)d * b.capacity + i] = b.vprop[(size_t)d * b.capacity + i];
    if (p.integrator == MTX_INT_PSSMLT_PATH)
      for (uint32_t d = 0; d < dirty; ++d)
        b.vpath_es[(size_t)d * b.capacity + i] = b.vprop_es[(size_t)d * b.capacity + i];
    dirty = 0;
  }
  cur.w = (float)dirty;
  b.mlt_cur[i] = cur;
  b.misc[kFinal][i] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, 0u);
}

// block.put(pos, L / cw) at the integer pixel position (:161-165), running
// accumulation per source pixel: iteration, then chain order.
__global__ void k_mlt_film(WaveBuffers b, ChunkParams p, float4 *contrib) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.n_px) return;
  const uint32_t pix = p.px0 + q;
  const int y = (int)(pix / p.width), x = (int)(pix - (uint32_t)y * p.width);
  const size_t o = (size_t)(pix - p.band_y0 * p.width);  // contrib: 9 planes of band_px
  float4 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = contrib[(size_t)k * p.band_px + o];
  for (uint32_t sidx = 0; sidx < p.spp; ++sidx) {
    const uint32_t c = q * p.spp + sidx;
    const float4 lc = b.mlt_L[c];
    const float cw = b.mlt_cur[c].z;
    const V3 res = V3{lc.x, lc.y, lc.z} / cw;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float wy = fmaxf(0.f, 1.f - fabsf((float)y - ((float)(y + dy - 1) + 0.5f)));
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float wx = fmaxf(0.f, 1.f - fabsf((float)x - ((float)(x + dx - 1) + 0.5f)));
        const float w = wx * wy;
        float4 &a = acc[dy * 3 + dx];
        a.x = a.x + res.x * w;
        a.y = a.y + res.y * w;
        a.z = a.z + res.z * w;
        a.w = a.w + w;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) contrib[(size_t)k * p.band_px + o] = acc[k];
}

// ---------------------------------------------------------------------------
// Launch wrappers
// ---------------------------------------------------------------------------
static inline unsigned blocks_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_raygen_camera(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_raygen_camera, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, s, b, p);
}
void launch_raygen_rays(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const float *rays,
                        const uint32_t *lanes, uint32_t rng_skip, hipStream_t st) {
  hipLaunchKernelGGL(k_raygen_rays, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, s, b, p, rays, lanes,
                     rng_skip);
}
void launch_trace_closest(const DevScene &s, const WaveBuffers &b, uint32_t bounce, uint32_t stats, int grid,
                          hipStream_t st) {
  const size_t lds = persistent_stack_bytes(s, false);
  if (stats)
    hipLaunchKernelGGL(k_trace_closest<true>, dim3(grid), dim3(kTraceBlock), lds, st, s, b, bounce);
  else
    hipLaunchKernelGGL(k_trace_closest<false>, dim3(grid), dim3(kTraceBlock), lds, st, s, b, bounce);
}
void launch_trace_shadow(const DevScene &s, const WaveBuffers &b, uint32_t bounce, uint32_t stats, int grid,
                         hipStream_t st) {
  if (stats)
    hipLaunchKernelGGL(k_trace_shadow<true>, dim3(grid), dim3(kTraceBlock), persistent_stack_bytes(s, true), st, s, b, bounce);
  else
    hipLaunchKernelGGL(k_trace_shadow<false>, dim3(grid), dim3(kTraceBlock), persistent_stack_bytes(s, true), st, s, b, bounce);
}
void launch_shade(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, uint32_t bounce, int grid,
                  hipStream_t st) {
  switch (p.integrator) {
    case MTX_INT_PATH:
      hipLaunchKernelGGL(k_shade<MTX_INT_PATH>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_NRC:
      hipLaunchKernelGGL(k_shade<MTX_INT_NRC>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_PSSMLT_SIMPLE:
      hipLaunchKernelGGL(k_shade<MTX_INT_PSSMLT_SIMPLE>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_SIMPLE:
      hipLaunchKernelGGL(k_shade<MTX_INT_SIMPLE>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_PSSMLT_PATH:
      hipLaunchKernelGGL(k_shade<MTX_INT_PSSMLT_PATH>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_NERAD_RHS:
      hipLaunchKernelGGL(k_shade<MTX_INT_NERAD_RHS>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    case MTX_INT_NERAD:
      hipLaunchKernelGGL(k_shade<MTX_INT_NERAD>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
      break;
    default:
      hipLaunchKernelGGL(k_shade<MTX_INT_PATH_MIS>, dim3(grid), dim3(kShadeBlock), 0, st, s, b, p, bounce);
  }
}
// Resident blocks per CU of the persistent kernels (grid = n_cu x this):
// the any-hit kernels (shadow, ReSTIR visibility) and the closest-hit kernel.
int trace_blocks_per_cu(const DevScene &s) {
  int na = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&na, k_trace_shadow<false>, kTraceBlock,
                                                   persistent_stack_bytes(s, true)) != hipSuccess ||
      na <= 0)
    na = 4;
  return na;
}
int closest_blocks_per_cu(const DevScene &s) {
  int nc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nc, k_trace_closest<false>, kTraceBlock,
                                                   persistent_stack_bytes(s, false)) != hipSuccess ||
      nc <= 0)
    nc = 4;
  return nc;
}
// MTX_DIAG_STAMPS builds: read (and zero) the shade stamp sums; -1 otherwise.
int shade_stamps(unsigned long long *out) {
#if MTX_DIAG_STAMPS
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_shade_stamps), sizeof(unsigned long long) * (kStampSegs + 2)) !=
      hipSuccess)
    return -1;
  unsigned long long z[kStampSegs + 2] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_shade_stamps), z, sizeof(z)) != hipSuccess) return -1;
  return kStampSegs;
#else
  (void)out;
  return -1;
#endif
}
int shade_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_shade<MTX_INT_PATH_MIS>, kShadeBlock, 0) != hipSuccess ||
      nb <= 0)
    nb = 2;
  return nb;
}
void launch_cache_apply(const WaveBuffers &b, const float *out, uint32_t capacity, hipStream_t st,
                        const uint32_t *perm) {
  const unsigned blocks = (unsigned)std::min<uint64_t>((capacity + 255) / 256, 16384);
  hipLaunchKernelGGL(k_cache_apply, dim3(std::max(1u, blocks)), dim3(256), 0, st, b, out, perm);
}
// Resident blocks per CU of the path megakernel (its LDS stacks and the shade
// register budget).
int mega_blocks_per_cu(const DevScene &s) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_path_mega<MTX_INT_PATH_MIS>, kShadeBlock, stack_bytes(s)) !=
          hipSuccess ||
      nb <= 0)
    nb = 1;
  return nb;
}
void launch_path_mega(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, int grid, hipStream_t st) {
  if (p.integrator == MTX_INT_PATH)
    hipLaunchKernelGGL(k_path_mega<MTX_INT_PATH>, dim3(grid), dim3(kShadeBlock), stack_bytes(s), st, s, b, p);
  else
    hipLaunchKernelGGL(k_path_mega<MTX_INT_PATH_MIS>, dim3(grid), dim3(kShadeBlock), stack_bytes(s), st, s, b, p);
}
void launch_flush_tail(const WaveBuffers &b, uint32_t bounce, uint32_t capacity, uint32_t integrator,
                       hipStream_t st) {
  const unsigned blocks = (unsigned)std::min<uint64_t>((capacity + 255) / 256, 1024);
  hipLaunchKernelGGL(k_flush_tail, dim3(std::max(1u, blocks)), dim3(256), 0, st, b, bounce, integrator);
}
void launch_mlt_init(const WaveBuffers &b, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_mlt_init, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, b, p, p.max_depth);
}
void launch_mlt_begin(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_mlt_begin, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, s, b, p);
}
void launch_mlt_end(const WaveBuffers &b, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_mlt_end, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, b, p, p.max_depth);
}
void launch_mlt_film(const WaveBuffers &b, const ChunkParams &p, float4 *contrib, hipStream_t st) {
  hipLaunchKernelGGL(k_mlt_film, dim3(blocks_for(p.n_px, 128)), dim3(128), 0, st, b, p, contrib);
}
void launch_film_src(const WaveBuffers &b, const ChunkParams &p, float4 *contrib, hipStream_t st) {
  if (p.spp < 4)
    hipLaunchKernelGGL(k_film_src, dim3(blocks_for(p.n_px, 128)), dim3(128), 0, st, b, p, contrib);
  else
    hipLaunchKernelGGL(k_film_src_staged, dim3(blocks_for(p.n_px, 64)), dim3(64), 0, st, b, p, contrib);
}
void launch_film_gather(const float4 *contrib, float4 *film, uint32_t width, uint32_t y0, uint32_t y1,
                        uint32_t nslots, uint32_t slot_mask, hipStream_t st) {
  const uint64_t n = (uint64_t)(width + 2) * (y1 - y0 + 2);
  hipLaunchKernelGGL(k_film_gather, dim3(blocks_for(n, 256)), dim3(256), 0, st, contrib, film, width, y0, y1, nslots,
                     slot_mask);
}
void launch_collect(const WaveBuffers &b, const ChunkParams &p, float *L_out, uint8_t *valid_out, hipStream_t st) {
  hipLaunchKernelGGL(k_collect, dim3(blocks_for(p.n_paths, 256)), dim3(256), 0, st, b, p, L_out, valid_out);
}
void launch_trace_raw(const DevScene &s, const float4 *rays, uint32_t n, int any_hit, uint32_t *hits,
                      uint32_t *visits, hipStream_t st) {
  // at most the persistent grid's threads: mode 2 indexes the spill area by thread
  const unsigned grid = std::min<unsigned>(blocks_for(n, kTraceBlock), s.ovf_threads / kTraceBlock);
  hipLaunchKernelGGL(k_trace_raw, dim3(std::max(1u, grid)), dim3(kTraceBlock), stack_bytes(s), st, s, rays, n, any_hit,
                     hits, visits);
}

}  // namespace mtxd

#ifdef MTX_TEST_BAD_SHADOW_FORM
// tests/test_abi.py::test_shadow_record_form_is_checked: an integrator whose L
// lives outside k_shade's stores asking for the final-value form must not compile.
__device__ void mtx_bad_shadow_form(mtxd::ShadeIO &io, const mtx::SurfaceInteraction &si,
                                    const mtx::DirectionSample &ds) {
  const mtx::V3 L = mtx::v3s(0.f);
  mtxd::make_shadow<MTX_INT_NERAD_RHS, true>(io, si, ds, L, L, L, true, &L);
}
#endif
