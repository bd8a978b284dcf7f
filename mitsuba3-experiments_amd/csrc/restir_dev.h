// restir_dev.h — per-lane ReSTIR GI state loads / stores (the planes of
// wavefront.h RestirBuffers), shared by restir.hip's phase kernels and the
// stage-A path megakernel in kernels.hip.
#pragma once
#include "device_common.h"
#include "mtx_core/restir.h"

namespace mtxd {

__device__ __forceinline__ RSample ld_sample(const float4 *b, uint32_t n, uint32_t i) {
  const float4 p0 = b[i], p1 = b[(size_t)n + i], p2 = b[2 * (size_t)n + i], p3 = b[3 * (size_t)n + i],
               p4 = b[4 * (size_t)n + i];
  RSample s;
  s.x_v = V3{p0.x, p0.y, p0.z};
  s.valid = p0.w != 0.f;
  s.n_v = V3{p1.x, p1.y, p1.z};
  s.p_q = p1.w;
  s.x_s = V3{p2.x, p2.y, p2.z};
  s.n_s = V3{p3.x, p3.y, p3.z};
  s.L_o = V3{p4.x, p4.y, p4.z};
  return s;
}

__device__ __forceinline__ void st_sample(float4 *b, uint32_t n, uint32_t i, const RSample &s) {
  b[i] = make_float4(s.x_v.x, s.x_v.y, s.x_v.z, s.valid ? 1.f : 0.f);
  b[(size_t)n + i] = make_float4(s.n_v.x, s.n_v.y, s.n_v.z, s.p_q);
  b[2 * (size_t)n + i] = make_float4(s.x_s.x, s.x_s.y, s.x_s.z, 0.f);
  b[3 * (size_t)n + i] = make_float4(s.n_s.x, s.n_s.y, s.n_s.z, 0.f);
  b[4 * (size_t)n + i] = make_float4(s.L_o.x, s.L_o.y, s.L_o.z, 0.f);
}

__device__ __forceinline__ RReservoir ld_res(const float4 *b, uint32_t n, uint32_t i) {
  RReservoir r;
  r.z = ld_sample(b, n, i);
  const float4 p5 = b[5 * (size_t)n + i];
  r.w = p5.x;
  r.W = p5.y;
  r.M = __float_as_uint(p5.z);
  return r;
}

__device__ __forceinline__ void st_res(float4 *b, uint32_t n, uint32_t i, const RReservoir &r) {
  st_sample(b, n, i, r.z);
  b[5 * (size_t)n + i] = make_float4(r.w, r.W, __uint_as_float(r.M), 0.f);
}

__device__ __forceinline__ Pcg32 ld_rng(uint4 m) {
  Pcg32 g;
  g.state = ((uint64_t)m.y << 32) | (uint64_t)m.x;
  g.seq = m.z;
  return g;
}

__device__ __forceinline__ uint4 st_rng(const Pcg32 &g, uint32_t w) {
  return make_uint4((uint32_t)g.state, (uint32_t)(g.state >> 32), g.seq, w);
}

__device__ __forceinline__ float4 f4(V3 v, float w) { return make_float4(v.x, v.y, v.z, w); }


}  // namespace mtxd
