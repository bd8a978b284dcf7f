// nerad.hip — training samples of the neural radiosity field (nerad.py,
// SURVEY §8f item 3): the left-hand side points (IntersectionSampler.sample,
// nerad.py:291-310) and the right-hand side estimate (Integrator.sample_rhs,
// nerad.py:174-233) on the wavefront. The RHS lanes (M per point, dr.repeat
// at :182) run k_shade<MTX_INT_NERAD_RHS> (kernels.hip, shade_nerad) over
// the same persistent trace kernels as the path tracers; their stop
// vertices query the fp16 MFMA field (field.hip) through the NRC cache
// queue, then k_nerad_apply and k_nerad_mean form L_rhs.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "mtx_core/nerad.h"

namespace mtxd {

// One thread per training point: surface sample, its shading frame, the
// world incident direction Field(si) sees (si.to_world(si.wi), :100).
// lhs: 3 float4 per point: (p, prim bits), (wi_world, b1), (b2, 0, 0, 0);
// qp / qd: the field query (p, wi_world).
__global__ void k_nerad_lhs(DevScene s, NeradTables t, uint32_t seed, uint32_t n, float4 *lhs, float4 *qp,
                            float4 *qd) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pcg32 rng = sampler_lane(seed, i);
  const SurfaceSample ss = nerad_surface_sample(t, s.shapes, s.materials, rng);
  const SurfaceInteraction si = compute_si_dev(s, 1.f, ss.prim, ss.b1, ss.b2, V3{0.f, 0.f, 1.f});
  const V3 wi = to_world(si.sh, ss.wi_local);
  lhs[3 * (size_t)i + 0] = make_float4(si.p.x, si.p.y, si.p.z, __uint_as_float(ss.prim));
  lhs[3 * (size_t)i + 1] = make_float4(wi.x, wi.y, wi.z, ss.b1);
  lhs[3 * (size_t)i + 2] = make_float4(ss.b2, 0.f, 0.f, 0.f);
  qp[i] = make_float4(si.p.x, si.p.y, si.p.z, 0.f);
  qd[i] = make_float4(wi.x, wi.y, wi.z, 0.f);
}

// RHS lane i = point * M + j (sampler lane i, nerad.py:182-189): the hit
// record is the point itself, seen from the ray direction -wi_world.
__global__ void k_nerad_raygen(WaveBuffers b, ChunkParams p, const float4 *lhs, uint32_t M) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) b.counters[0] = p.n_paths;
  if (i >= p.n_paths) return;
  const uint32_t pt = i / M;
  const float4 a = lhs[3 * (size_t)pt], c = lhs[3 * (size_t)pt + 1], d = lhs[3 * (size_t)pt + 2];
  const Pcg32 rng = sampler_lane(p.seed, i);
  b.hit[i] = make_float4(1.f, a.w, c.w, d.x);
  b.ray_o[0][i] = make_float4(a.x, a.y, a.z, 0.f);  // queue position i (identity)
  b.ray_d[0][i] = make_float4(-c.x, -c.y, -c.z, 0.f);
  b.thr[0][i] = make_float4(1.f, 1.f, 1.f, 1.f);
  b.L[kFinal][i] = make_float4(0.f, 0.f, 0.f, 0.f);
  b.prev[0][i] = make_float4(0.f, 0.f, 0.f, 0.f);
  b.misc[kFinal][i] = make_uint4((uint32_t)rng.state, (uint32_t)(rng.state >> 32), rng.seq, 0u);
  b.queue[0][i] = i;
}

// L += f * (Le + Field(si)) at the stop vertices (nerad.py:226-229), or for
// a rendered lane L = Field(si) * f + Le(si) (:251-252).
__global__ void k_nerad_apply(WaveBuffers b, const float *out, uint32_t render) {
  const uint32_t n = *b.cq_count;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const float4 t = b.cq_t[q];
    const uint32_t path = __float_as_uint(t.w);
    const float4 le = b.prev[0][path];
    float4 L = b.L[kFinal][path];
    if (render) {
      L.x = out[3 * (size_t)q] * t.x + le.x;
      L.y = out[3 * (size_t)q + 1] * t.y + le.y;
      L.z = out[3 * (size_t)q + 2] * t.z + le.z;
    } else {
      L.x = L.x + t.x * (le.x + out[3 * (size_t)q]);
      L.y = L.y + t.y * (le.y + out[3 * (size_t)q + 1]);
      L.z = L.z + t.z * (le.z + out[3 * (size_t)q + 2]);
    }
    b.L[kFinal][path] = L;
  }
}

// dr.block_sum(L, M) / M (nerad.py:231), samples summed in order.
__global__ void k_nerad_mean(WaveBuffers b, uint32_t n, uint32_t M, float *L_rhs, float *lanes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = 0.f, y = 0.f, z = 0.f;
  for (uint32_t j = 0; j < M; ++j) {
    const uint32_t k = i * M + j;
    const float4 L = b.L[kFinal][k];
    x = x + L.x;
    y = y + L.y;
    z = z + L.z;
    if (lanes) {
      lanes[3 * (size_t)k] = L.x;
      lanes[3 * (size_t)k + 1] = L.y;
      lanes[3 * (size_t)k + 2] = L.z;
    }
  }
  const float m = (float)M;
  L_rhs[3 * (size_t)i] = x / m;
  L_rhs[3 * (size_t)i + 1] = y / m;
  L_rhs[3 * (size_t)i + 2] = z / m;
}

static inline unsigned nblocks(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_nerad_lhs(const DevScene &s, const NeradTables &t, uint32_t seed, uint32_t n, float4 *lhs, float4 *qp,
                      float4 *qd, hipStream_t st) {
  hipLaunchKernelGGL(k_nerad_lhs, dim3(nblocks(n, 256)), dim3(256), 0, st, s, t, seed, n, lhs, qp, qd);
}
void launch_nerad_raygen(const WaveBuffers &b, const ChunkParams &p, const float4 *lhs, uint32_t M,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_nerad_raygen, dim3(nblocks(p.n_paths, 256)), dim3(256), 0, st, b, p, lhs, M);
}
void launch_nerad_apply(const WaveBuffers &b, const float *out, uint32_t capacity, uint32_t render, hipStream_t st) {
  const unsigned blocks = (unsigned)std::min<uint64_t>((capacity + 255) / 256, 16384);
  hipLaunchKernelGGL(k_nerad_apply, dim3(std::max(1u, blocks)), dim3(256), 0, st, b, out, render);
}
void launch_nerad_mean(const WaveBuffers &b, uint32_t n, uint32_t M, float *L_rhs, float *lanes, hipStream_t st) {
  hipLaunchKernelGGL(k_nerad_mean, dim3(nblocks(n, 256)), dim3(256), 0, st, b, n, M, L_rhs, lanes);
}

}  // namespace mtxd
