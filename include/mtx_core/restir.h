// ReSTIR GI per-lane primitives (restirgi.py), shared by the device kernels
// and the CPU oracle so both evaluate the same IEEE operation sequence.
//
//   RSample / RReservoir      restirgi.py:103-149 (RestirSample, RestirReservoir)
//   res_update / res_merge    restirgi.py:120-149
//   p_hat                     restirgi.py:84-85
//   similar                   restirgi.py:175-180 (thresholds :152-153)
//   jacobian_J                restirgi.py:42-53 (J, the variant the integrator calls)
//   project_prev              PerspectiveCamera::sample_direction (upstream),
//                             called at restirgi.py:370-372
//   pixel_index               restirgi.py:170-173 (to_idx) with the clamp fixed
//                             to [0, size-1] (reference off-by-one)
//
// Sample layout in HBM (5 float4 planes; reservoir = 5 planes + 1):
//   0: x_v.xyz, valid (0/1)   1: n_v.xyz, p_q   2: x_s.xyz, 0
//   3: n_s.xyz, 0             4: L_o.rgb, 0     5: w, W, M (u32 bits), 0
#pragma once
#include "../mtx.h"
#include "common.h"

namespace mtx {

struct RSample {
  V3 x_v, n_v, x_s, n_s, L_o;
  float p_q;
  bool valid;
};

struct RReservoir {
  RSample z;
  float w, W;
  uint32_t M;
};

MTX_HD RSample rsample_zero() {
  RSample s;
  s.x_v = s.n_v = s.x_s = s.n_s = s.L_o = v3s(0.f);
  s.p_q = 0.f;
  s.valid = false;
  return s;
}

MTX_HD RReservoir rres_zero() {
  RReservoir r;
  r.z = rsample_zero();
  r.w = 0.f;
  r.W = 0.f;
  r.M = 0u;
  return r;
}

// cos(25 * pi / 180) evaluated in double (Python float), compared as float32.
constexpr float kRestirCosThreshold = 0.906307787036649963f;
constexpr float kRestirDistThreshold = 0.1f;

MTX_HD float p_hat(V3 f) { return norm(f); }

MTX_HD bool similar(const RSample &a, const RSample &b) {
  const float dist = norm(a.x_v - b.x_v);
  bool s = dist < kRestirDistThreshold;
  s = s && (dot(a.n_v, b.n_v) > kRestirCosThreshold);
  return s;
}

// RestirReservoir.update: the draw `u` is consumed whether or not `active`.
MTX_HD void res_update(RReservoir &r, const RSample &snew, float wnew, bool active, float u) {
  r.w = r.w + (active ? wnew : 0.f);
  r.M = r.M + (active ? 1u : 0u);
  if (active && (u < wnew / r.w)) r.z = snew;
}

// RestirReservoir.merge: weight p * W * M (left to right, M as float).
// res_merge_w does the weight / count update of o = (W, M) and returns
// whether o's sample replaces r.z (so a caller can fetch that sample only
// when it is taken); res_merge is exactly res_update + the count fix-up.
MTX_HD bool res_merge_w(RReservoir &r, float oW, uint32_t oM, float p, bool active, float u) {
  const uint32_t M0 = r.M;
  const float wnew = p * oW * (float)oM;
  r.w = r.w + (active ? wnew : 0.f);
  r.M = active ? M0 + oM : M0;
  return active && (u < wnew / r.w);
}

MTX_HD void res_merge(RReservoir &r, const RReservoir &o, float p, bool active, float u) {
  if (res_merge_w(r, o.W, o.M, p, active, u)) r.z = o.z;
}

MTX_HD float dr_clampf(float x, float lo, float hi) { return fmaxf(fminf(x, hi), lo); }

// restirgi.py:42-53
MTX_HD float jacobian_J(V3 receiver, const RReservoir &nb) {
  const V3 v_new = receiver - nb.z.x_s;
  const float d_new = norm(v_new);
  const float cos_new = dr_clampf(dot(v_new, nb.z.n_s) / d_new, 0.f, 1.f);
  const V3 v_old = nb.z.x_v - nb.z.x_s;
  const float d_old = norm(v_old);
  const float cos_old = dr_clampf(dot(v_old, nb.z.n_s) / d_old, 0.f, 1.f);
  const float div = cos_old * sqr(d_new);
  return div > 0.f ? cos_new * sqr(d_old) / div : 0.f;
}

// PerspectiveCamera::sample_direction: film position (pixels) of world point
// p; returns false (ds.pdf = 0) outside the clip range or the frustum.
MTX_HD bool project_prev(const mtx_camera &c, V3 p, float *ux, float *uy) {
  const V3 rel = p - V3{c.origin[0], c.origin[1], c.origin[2]};
  const V3 r0 = V3{c.inv_rows[0], c.inv_rows[1], c.inv_rows[2]};
  const V3 r1 = V3{c.inv_rows[3], c.inv_rows[4], c.inv_rows[5]};
  const V3 r2 = V3{c.inv_rows[6], c.inv_rows[7], c.inv_rows[8]};
  const float lx = dot(r0, rel), ly = dot(r1, rel), lz = dot(r2, rel);
  if (!(lz >= c.near_clip && lz <= c.far_clip)) return false;
  const float sx = 0.5f * (1.f - lx / (lz * c.tan_x));
  const float sy = 0.5f * (1.f - ly / (lz * c.tan_y));
  if (!(sx >= 0.f && sx <= 1.f && sy >= 0.f && sy <= 1.f)) return false;
  *ux = sx * (float)c.width;
  *uy = sy * (float)c.height;
  return true;
}

MTX_HD uint32_t clamp_pix(int64_t v, uint32_t size) {
  return (uint32_t)(v < 0 ? 0 : (v > (int64_t)size - 1 ? (int64_t)size - 1 : v));
}

// to_idx: pixel -> wavefront index (pixel-major, spp samples per pixel)
MTX_HD uint32_t pixel_index(int64_t x, int64_t y, uint32_t W, uint32_t H, uint32_t spp, uint32_t smp) {
  return (clamp_pix(y, H) * W + clamp_pix(x, W)) * spp + smp;
}

}  // namespace mtx
