// restir.hip — gfx950 kernels of one ReSTIR GI frame (restirgi.py:182-588).
//
// The reference evaluates a frame as four whole-film phases (sample_initial,
// temporal_resampling, spatial_resampling, render_final); each phase reads
// other pixels' results of the previous phase, so each becomes one or more
// kernels over all W*H*spp lanes:
//
//   raygen + trace_closest   primary rays (kernels.hip, bounce 0)
//   k_rs_begin               emittance, BSDF/hemisphere sample, secondary ray
//   [trace, shade, shadow]*  the path-mis loop of sample_ray (:459-588) on the
//                            wavefront machinery; shade bounce 0 records x_s,n_s
//   k_rs_collect             L_o, sampler state
//   k_rs_temporal            reprojection into the previous camera, merge
//   k_rs_spatial_rays        9 neighbour candidates -> visibility test rays
//   k_trace_test             any-hit traversal of the compacted tests
//   k_rs_spatial_merge       replays the same draws, merges the neighbours
//   (k_trace_test, k_rs_bias_finish)   bias correction (:334-348) when enabled
//   k_rs_final               bsdf.eval * L_o * W + emittance, film position
//
// The sampler stream of every lane is consumed in the reference order; the
// per-lane arithmetic is mtx_core/restir.h, shared with oracle/oracle.cpp.
#include "device_common.h"
#include "mtx_core/restir.h"
#include "restir_dev.h"

namespace mtxd {

namespace {

constexpr int kRsBlock = 256;  // block size of the k_rs_* kernels (block_reserve)

// Lane of this thread with the grid's blocks regrouped so that the blocks
// sharing an XCD (b, b+8, ...) take one contiguous band of pixels: the
// neighbour reads of the temporal / spatial passes then hit that XCD's L2.
// A bijection for any grid size (speed only).
__device__ __forceinline__ uint32_t rs_thread(const RestirBuffers &r) {
  uint32_t b = blockIdx.x;
  if (r.xcd_remap) {
    const uint32_t n = gridDim.x, q = n / 8u, rem = n % 8u, x = b % 8u, k = b / 8u;
    b = x * q + min(x, rem) + k;
  }
  return b * blockDim.x + threadIdx.x;
}

// band-local lane t = q * spp + s (pixel-major, the sampler lane order) ->
// wavefront path index (the same: chunks are pixel-major); global lane =
// r.lane0 + t
__device__ __forceinline__ uint32_t path_of(uint32_t i, const ChunkParams &p) {
  (void)p;
  return i;
}

}  // namespace

// sample_initial after the primary intersection (:419-448). Lanes with a
// valid primary hit start the path-mis loop on the secondary ray; the others
// consume the draws of one missed loop iteration.
__global__ void k_rs_begin(DevScene s, WaveBuffers b, ChunkParams p, RestirBuffers r) {
  const SceneView sv = make_view(s);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = r.lane0 + t;
  bool enq = false;
  float4 nro = make_float4(0.f, 0.f, 0.f, 0.f), nrd = nro;
  uint4 nmi = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t path = t < r.nb ? path_of(t, p) : 0u;
  if (t < r.nb) {
    const float4 h = b.hit[path], d4 = b.ray_d[0][path];  // bounce-0 queue is the identity
    r.prim_hit[i] = h;
    r.prim_dir[i] = d4;
    const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{d4.x, d4.y, d4.z});
    r.emit[i] = f4(emitter_eval(sv, si.emitter, si.wi), 0.f);
    Pcg32 rng = ld_rng(b.misc[0][path]);
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
    const size_t n = r.n;
    r.cur[i] = si.valid ? f4(si.p, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    r.cur[n + i] = si.valid ? f4(si.n, pdf) : make_float4(0.f, 0.f, 0.f, pdf);
    if (si.valid) {
      const Ray nr = spawn_ray(si.p, si.n, to_world(si.sh, wo));
      nro = make_float4(nr.o.x, nr.o.y, nr.o.z, nr.maxt);
      nrd = make_float4(nr.d.x, nr.d.y, nr.d.z, 0.f);
      // throughput 1, L 0, prev_bsdf_pdf 1, prev_p 0: the bounce-0 shade's constants
      nmi = st_rng(rng, PF_PREV_DELTA << 16);  // depth 0, prev_bsdf_delta
      enq = true;
    } else {
      rng.advance(6);
      b.L[kFinal][path] = make_float4(0.f, 0.f, 0.f, 1.f);
      b.misc[kFinal][path] = st_rng(rng, 0u);
      b.rs_xs[path] = make_float4(0.f, 0.f, 0.f, 0.f);
      b.rs_ns[path] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const uint32_t slot = block_reserve<kRsBlock>(enq ? 1u : 0u, &b.counters[0]);
  if (enq) {
    // the secondary loop runs with ray_par = 1: its bounce-0 rays are the
    // parity-1 planes (the primary rays, still read above, are parity 0)
    b.queue[0][slot] = path;
    b.ray_o[1][slot] = nro;
    b.ray_d[1][slot] = nrd;
    b.misc[1][slot] = nmi;
  }
}

// L_o = select(valid_ray, result, 0) (:588) and the sampler position.
__global__ void k_rs_collect(WaveBuffers b, ChunkParams p, RestirBuffers r) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= r.nb) return;
  const uint32_t i = r.lane0 + t, path = path_of(t, p);
  const float4 l = b.L[kFinal][path];
  const uint4 m = b.misc[kFinal][path];
  const bool valid_ray = ((m.w >> 16) & PF_VALID_RAY) != 0;
  r.cur[2 * (size_t)r.n + i] = b.rs_xs[path];
  r.cur[3 * (size_t)r.n + i] = b.rs_ns[path];
  r.cur[4 * (size_t)r.n + i] = valid_ray ? make_float4(l.x, l.y, l.z, 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
  r.rng[i] = m;
}

// temporal_resampling (:365-410)
__global__ void k_rs_temporal(RestirBuffers r, ChunkParams p) {
  const uint32_t t = rs_thread(r);
  if (t >= r.nb) return;
  const uint32_t i = r.lane0 + t;
  const uint32_t smp = i % p.spp;
  Pcg32 rng = ld_rng(r.rng[i]);
  const RSample S = ld_sample(r.cur, r.n, i);
  float ux = 0.f, uy = 0.f;
  bool valid = project_prev(r.prev_cam, S.x_v, &ux, &uy);
  RSample Sprev = rsample_zero();
  if (valid) Sprev = ld_sample(r.prev, r.n, pixel_index((int64_t)ux, (int64_t)uy, p.width, p.height, p.spp, smp));
  valid = valid && similar(S, Sprev);
  const RReservoir R = valid ? ld_res(r.tres, r.n, i) : rres_zero();
  RReservoir Rn = rres_zero();
  float phat = p_hat(S.L_o);
  const float w = S.p_q > 0.f ? phat / S.p_q : 0.f;
  res_update(Rn, S, w, true, rng.next_1d());
  res_merge(Rn, R, p_hat(R.z.L_o), true, rng.next_1d());
  phat = p_hat(Rn.z.L_o);
  Rn.W = (phat * (float)Rn.M > 0.f) ? Rn.w / ((float)Rn.M * phat) : 0.f;
  if (r.max_M_temporal) Rn.M = min(Rn.M, r.max_M_temporal);
  st_res(r.tres, r.n, i, Rn);
  r.rng[i] = st_rng(rng, 0u);
}

// Neighbour k of lane i in spatial_resampling (:300-313): the disk offset
// draw, clamped pixel, candidate similarity. Consumes 2 draws.
struct Neighbour {
  uint32_t idx;
  bool active;
};

__device__ __forceinline__ Neighbour neighbour(const RestirBuffers &r, const ChunkParams &p, Pcg32 &rng, int k,
                                               int max_iter, float rad, int64_t x, int64_t y, uint32_t smp,
                                               const RSample &q) {
  const V2 d2 = square_to_uniform_disk(rng.next_2d());
  const V2 off = V2{d2.x * rad, d2.y * rad};
  Neighbour nb;
  nb.idx = pixel_index(x + (int32_t)off.x, y + (int32_t)off.y, p.width, p.height, p.spp, smp);
  const RSample qn = ld_sample(r.cur, r.n, nb.idx);
  nb.active = (k < max_iter) && similar(qn, q);
  return nb;
}

__device__ __forceinline__ int spatial_max_iter(const RestirBuffers &r, uint32_t M) {
  return (r.max_M_spatial == 0 || (double)M < (double)r.max_M_spatial / 2.0) ? 9 : 3;  // :297
}

__device__ __forceinline__ void put_test(const RestirBuffers &r, uint32_t o, const Ray &ray, uint32_t slot) {
  r.test_rays[2 * (size_t)o] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.maxt);
  r.test_rays[2 * (size_t)o + 1] = make_float4(ray.d.x, ray.d.y, ray.d.z, __uint_as_float(slot));
}

// spatial_resampling, pass 1: the visibility rays of :316-318.
__global__ void k_rs_spatial_rays(RestirBuffers r, ChunkParams p) {
  const uint32_t t = rs_thread(r);
  const bool live = t < r.nb;
  const uint32_t ii = r.lane0 + (live ? t : 0u);
  const uint32_t smp = ii % p.spp;
  const int64_t x = (int64_t)(ii / p.spp % p.width), y = (int64_t)(ii / p.width / p.spp);
  Pcg32 rng = ld_rng(r.rng[ii]);
  const uint32_t Ms = __float_as_uint(r.sres[5 * (size_t)r.n + ii].z);
  if (r.flags & MTX_RESTIR_SPATIAL_SPATIAL) rng.next_1d();  // merge draw (:291-293)
  const int max_iter = spatial_max_iter(r, Ms);
  const RSample q = ld_sample(r.cur, r.n, ii);
  const float rad = r.radius[ii];
  // candidates first, then one block-wide reservation for all of the lane's
  // tests (test order is irrelevant: results are addressed by slot)
  uint32_t idx[9], mask = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const Neighbour nb = neighbour(r, p, rng, k, max_iter, rad, x, y, smp, q);
    idx[k] = nb.idx;
    if (live && nb.active) mask |= 1u << k;
    rng.next_1d();  // merge draw (:328)
  }
  if (live) {  // the candidates, for k_rs_spatial_merge (instead of re-deriving them)
#pragma unroll
    for (int k = 0; k < 9; ++k) r.nbr[10 * (size_t)ii + k] = idx[k];
    r.nbr[10 * (size_t)ii + 9] = mask;
  }
  uint32_t o = block_reserve<kRsBlock>((uint32_t)__popc(mask), &r.test_count[0]);
#pragma unroll
  for (int k = 0; k < 9; ++k)
    if ((mask >> k) & 1u) {
      const float4 xs = r.tres[2 * (size_t)r.n + idx[k]];
      put_test(r, o++, spawn_ray_to(q.x_v, q.n_v, V3{xs.x, xs.y, xs.z}), 9 * ii + (uint32_t)k);
    }
}

// spatial_resampling, pass 2: replays the lane's draws with the visibility
// results, merges (:320-332), and either finishes W (:350) or emits the
// bias-correction rays (:334-346).
__global__ void k_rs_spatial_merge(RestirBuffers r, ChunkParams p) {
  const uint32_t t = rs_thread(r);
  const bool live = t < r.nb;
  const uint32_t ii = r.lane0 + (live ? t : 0u);
  const bool bias = (r.flags & MTX_RESTIR_BIAS_CORRECTION) != 0;
  const bool jac = (r.flags & MTX_RESTIR_JACOBIAN) != 0;
  Pcg32 rng = ld_rng(r.rng[ii]);
  const RReservoir Rs = ld_res(r.sres, r.n, ii);
  RReservoir Rn = rres_zero();
  const RSample q = ld_sample(r.cur, r.n, ii);
  uint32_t Z = 0;
  if (r.flags & MTX_RESTIR_SPATIAL_SPATIAL) {
    res_merge(Rn, Rs, p_hat(Rs.z.L_o), true, rng.next_1d());
    Z += Rs.M;
  }
  const float rad = r.radius[ii];
  bool any_reused = false;
  // the 9 candidates k_rs_spatial_rays drew (same draws: each disk sample's
  // two draws are consumed unused)
  const uint32_t nmask = live ? r.nbr[10 * (size_t)ii + 9] : 0u;
  uint32_t qM[9];
  V3 qp[9];
  uint32_t qa = 0;
  // Neighbour reservoirs: per candidate only the planes the merge weight
  // reads (L_o, then W and M; x_v / x_s / n_s with bias correction or the
  // Jacobian); the sample planes of the one that ends up selected are read
  // once after the loop (res_merge_w: same arithmetic as res_merge).
  uint32_t sel = 0xffffffffu;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    rng.next_u32();  // the candidate's disk sample (next_2d)
    rng.next_u32();
    Neighbour nb;
    nb.idx = live ? r.nbr[10 * (size_t)ii + k] : 0u;
    nb.active = ((nmask >> k) & 1u) != 0;
    const bool active = nb.active;
    RReservoir Rk = rres_zero();
    if (active) {
      const float4 p4 = r.tres[4 * (size_t)r.n + nb.idx], p5 = r.tres[5 * (size_t)r.n + nb.idx];
      Rk.z.L_o = V3{p4.x, p4.y, p4.z};
      Rk.w = p5.x;
      Rk.W = p5.y;
      Rk.M = __float_as_uint(p5.z);
      if (bias || jac) {
        const float4 p0 = r.tres[nb.idx];
        Rk.z.x_v = V3{p0.x, p0.y, p0.z};
      }
      if (jac) {
        const float4 p2 = r.tres[2 * (size_t)r.n + nb.idx], p3 = r.tres[3 * (size_t)r.n + nb.idx];
        Rk.z.x_s = V3{p2.x, p2.y, p2.z};
        Rk.z.n_s = V3{p3.x, p3.y, p3.z};
      }
    }
    const bool shadowed = active && r.occ[9 * (size_t)ii + k] != 0;
    const float jf = jac ? dr_clampf(jacobian_J(q.x_v, Rk), 0.f, 1000.f) : 1.0f;
    const float phat = (!active || shadowed) ? 0.f : p_hat(Rk.z.L_o) * jf;
    if (res_merge_w(Rn, Rk.W, Rk.M, phat, active, rng.next_1d())) sel = nb.idx;
    qM[k] = Rk.M;
    qp[k] = Rk.z.x_v;
    qa |= active ? (1u << k) : 0u;
    any_reused = any_reused || active;
  }
  if (sel != 0xffffffffu) Rn.z = ld_sample(r.tres, r.n, sel);
  const float phat = p_hat(Rn.z.L_o);
  if (!bias) Rn.W = (phat * (float)Rn.M > 0.f) ? Rn.w / ((float)Rn.M * phat) : 0.f;
  if (live) {
    r.radius[ii] = fmaxf(any_reused ? rad : rad / 2.f, r.minimal_radius);  // :353-356
    if (!bias && r.max_M_spatial) Rn.M = min(Rn.M, r.max_M_spatial);
    st_res(r.sres, r.n, ii, Rn);
  }
  if (bias) {
    if (live) {
#pragma unroll
      for (int k = 0; k < 9; ++k) r.qM[10 * (size_t)ii + k] = qM[k] | (((qa >> k) & 1u) << 31);
      r.qM[10 * (size_t)ii + 9] = Z;
    }
    const uint32_t m = live ? (qa & 0x1ffu) : 0u;
    uint32_t o = block_reserve<kRsBlock>((uint32_t)__popc(m), &r.test_count[0]);
#pragma unroll
    for (int k = 0; k < 9; ++k)
      if ((m >> k) & 1u) put_test(r, o++, spawn_ray_to(Rn.z.x_s, Rn.z.n_s, qp[k]), 9 * ii + (uint32_t)k);
  }
}

// bias correction tail (:340-348)
__global__ void k_rs_bias_finish(RestirBuffers r, ChunkParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= r.nb) return;
  const uint32_t i = r.lane0 + t;
  uint32_t Z = r.qM[10 * (size_t)i + 9];
  for (int k = 0; k < 9; ++k) {
    const uint32_t e = r.qM[10 * (size_t)i + k];
    const bool active = (e >> 31) && r.occ[9 * (size_t)r.n + 9 * (size_t)i + k] == 0;
    Z += active ? (e & 0x7fffffffu) : 0u;
  }
  const float4 lo = r.sres[4 * (size_t)r.n + i];
  const float phat = p_hat(V3{lo.x, lo.y, lo.z});
  float4 p5 = r.sres[5 * (size_t)r.n + i];
  uint32_t M = __float_as_uint(p5.z);
  p5.y = ((float)Z * phat > 0.f) ? p5.x / ((float)Z * phat) : 0.f;
  if (r.max_M_spatial) M = min(M, r.max_M_spatial);
  p5.z = __uint_as_float(M);
  r.sres[5 * (size_t)r.n + i] = p5;
}

// render_final (:261-272) and the block.put position (:236-242)
__global__ void k_rs_final(DevScene s, WaveBuffers b, ChunkParams p, RestirBuffers r) {
  const SceneView sv = make_view(s);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= r.nb) return;
  const uint32_t i = r.lane0 + t;
  const RReservoir R = ld_res(r.sres, r.n, i);
  const float4 h = r.prim_hit[i], d4 = r.prim_dir[i];
  const SurfaceInteraction si = compute_si_dev(s, h.x, __float_as_uint(h.y), h.z, h.w, V3{d4.x, d4.y, d4.z});
  V3 beta = v3s(0.f);
  if (si.valid) {
    float pdf_unused;
    const V3 wo = to_local(si.sh, normalize(R.z.x_s - si.p));
    bsdf_eval_pdf(sv.bsdf, sv.materials[si.material], si.uv, si.wi, wo, &beta, &pdf_unused);
  }
  const float4 em = r.emit[i];
  const V3 res = beta * R.z.L_o * R.W + V3{em.x, em.y, em.z};
  const uint32_t path = path_of(t, p);
  b.L[kFinal][path] = make_float4(res.x, res.y, res.z, 0.f);
  const uint32_t x = i / p.spp % p.width, y = i / p.width / p.spp;
  b.pos[path] = make_float2((float)x, (float)y);
}

// Any-hit traversal of the compacted visibility tests; occ[base + slot].
struct TestSrc {
  using Payload = uint32_t;  // the test slot
  RestirBuffers r;
  uint32_t occ_base;
  __device__ __forceinline__ void load(uint32_t k, TraceRay &tr, float &tmax, uint32_t &payload) const {
    const float4 o4 = r.test_rays[2 * (size_t)k], d4 = r.test_rays[2 * (size_t)k + 1];
    tr = make_trace_ray(V3{o4.x, o4.y, o4.z}, V3{d4.x, d4.y, d4.z}, o4.w);
    tmax = o4.w;
    payload = __float_as_uint(d4.w);
  }
  __device__ __forceinline__ void finish(uint32_t slot, bool occluded, float, uint32_t, float, float) const {
    r.occ[occ_base + slot] = occluded ? 1 : 0;
  }
};

__global__ __launch_bounds__(kTraceBlock) void k_trace_test(DevScene s, RestirBuffers r, uint32_t occ_base) {
  // dynamic LDS: stack columns + tree top (device_common.h trace_loop)
  const TestSrc src{r, occ_base};
  uint32_t nv = 0, tv = 0, nr = 0;
  trace_loop<true>(s, src, r.test_count[0], r.test_heads, nv, tv, nr);
}

static inline unsigned rs_blocks(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_restir_begin(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_rs_begin, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, s, b, p, r);
}
void launch_restir_collect(const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r, hipStream_t st) {
  hipLaunchKernelGGL(k_rs_collect, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, b, p, r);
}
void launch_restir_temporal(const RestirBuffers &r, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_rs_temporal, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, r, p);
}
void launch_restir_spatial_rays(const RestirBuffers &r, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_rs_spatial_rays, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, r, p);
}
void launch_restir_spatial_merge(const RestirBuffers &r, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_rs_spatial_merge, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, r, p);
}
void launch_restir_bias_finish(const RestirBuffers &r, const ChunkParams &p, hipStream_t st) {
  hipLaunchKernelGGL(k_rs_bias_finish, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, r, p);
}
void launch_restir_final(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_rs_final, dim3(rs_blocks(r.nb, 256)), dim3(256), 0, st, s, b, p, r);
}
void launch_trace_test(const DevScene &s, const RestirBuffers &r, uint32_t occ_base, int grid, hipStream_t st) {
  hipLaunchKernelGGL(k_trace_test, dim3(grid), dim3(kTraceBlock), persistent_stack_bytes(s, true), st, s, r, occ_base);
}

}  // namespace mtxd
