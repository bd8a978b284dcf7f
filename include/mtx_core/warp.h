// mtx_core/warp.h — sample warps and shading frames (upstream mitsuba
// include/mitsuba/core/warp.h and frame.h, restated; unverifiable offline).
// Call sites in the reference: BSDF sampling everywhere, mi.warp.square_to_std_normal
// (pssmlt.py:251), square_to_uniform_disk (restirgi.py:305),
// square_to_uniform_hemisphere(_pdf) (restirgi.py:443-444).
#pragma once
#include "common.h"
#include "dmath.h"

namespace mtx {

// Low-distortion concentric disk map (Shirley-Chiu, Dave Cline's branch-free
// form as used upstream).
MTX_HD V2 square_to_uniform_disk_concentric(V2 s) {
  float x = fmaf(2.f, s.x, -1.f), y = fmaf(2.f, s.y, -1.f);
  bool is_zero = (x == 0.f) && (y == 0.f);
  bool q13 = fabsf(x) < fabsf(y);
  float r = q13 ? y : x;
  float rp = q13 ? x : y;
  float phi = 0.25f * kPi * rp / r;
  if (q13) phi = 0.5f * kPi - phi;
  if (is_zero) phi = 0.f;
  float sn, cs;
  dsincos(phi, &sn, &cs);
  return V2{r * cs, r * sn};
}

MTX_HD V3 square_to_cosine_hemisphere(V2 s) {
  V2 p = square_to_uniform_disk_concentric(s);
  float z = safe_sqrt(1.f - fmaf(p.y, p.y, p.x * p.x));
  return V3{p.x, p.y, z};
}
MTX_HD float square_to_cosine_hemisphere_pdf(V3 v) { return kInvPi * v.z; }

MTX_HD V3 square_to_uniform_hemisphere(V2 s) {
  V2 p = square_to_uniform_disk_concentric(s);
  float z = 1.f - fmaf(p.y, p.y, p.x * p.x);
  float sc = sqrtf(z + 1.f);
  return V3{p.x * sc, p.y * sc, z};
}
MTX_HD float square_to_uniform_hemisphere_pdf(V3) { return kInvTwoPi; }

// Uniform sphere (the constant environment's direction sampling):
// z = 1 - 2 s.y, r = safe_sqrt(1 - z^2), phi = 2 pi s.x.
MTX_HD V3 square_to_uniform_sphere(V2 s) {
  const float z = fmaf(-2.f, s.y, 1.f);
  const float r = safe_sqrt(fmaf(-z, z, 1.f));
  float sn, cs;
  dsincos(kTwoPi * s.x, &sn, &cs);
  return V3{r * cs, r * sn, z};
}
MTX_HD float square_to_uniform_sphere_pdf(V3) { return kInvFourPi; }

MTX_HD V2 square_to_uniform_disk(V2 s) {
  float r = sqrtf(s.x);
  float sn, cs;
  dsincos(kTwoPi * s.y, &sn, &cs);
  return V2{cs * r, sn * r};
}

// Box-Muller (pssmlt.py:251 mi.warp.square_to_std_normal).
MTX_HD V2 square_to_std_normal(V2 s) {
  float r = sqrtf(-2.f * dlog(1.f - s.x));
  float sn, cs;
  dsincos(kTwoPi * s.y, &sn, &cs);
  return V2{cs * r, sn * r};
}

// Orthonormal frame around a unit normal (Duff et al. 2017, as upstream
// coordinate_system()).
struct Frame {
  V3 s, t, n;
};
MTX_HD Frame frame_from_normal(V3 n) {
  float sign = (f2u(n.z) & 0x80000000u) ? -1.f : 1.f;
  float a = -1.f / (sign + n.z);
  float b = n.x * n.y * a;
  Frame f;
  f.s = V3{mulsign(sqr(n.x) * a, n.z) + 1.f, mulsign(b, n.z), mulsign_neg(n.x, n.z)};
  f.t = V3{b, fmaf(n.y, n.y * a, sign), -n.y};
  f.n = n;
  return f;
}
MTX_HD V3 to_local(const Frame &f, V3 v) { return V3{dot(v, f.s), dot(v, f.t), dot(v, f.n)}; }
MTX_HD V3 to_world(const Frame &f, V3 v) { return fma3(f.n, v.z, fma3(f.t, v.y, f.s * v.x)); }

MTX_HD V3 reflect_local(V3 wi) { return V3{-wi.x, -wi.y, wi.z}; }
MTX_HD V3 reflect_m(V3 wi, V3 m) {  // fmsub(m, 2*dot(wi,m), wi)
  float d2 = 2.f * dot(wi, m);
  return V3{fmaf(m.x, d2, -wi.x), fmaf(m.y, d2, -wi.y), fmaf(m.z, d2, -wi.z)};
}
MTX_HD V3 refract_local(V3 wi, float cos_theta_t, float eta_ti) {
  return V3{-eta_ti * wi.x, -eta_ti * wi.y, cos_theta_t};
}
MTX_HD V3 refract_m(V3 wi, V3 m, float cos_theta_t, float eta_ti) {
  float k = fmaf(dot(wi, m), eta_ti, cos_theta_t);
  return V3{fmaf(m.x, k, -(wi.x * eta_ti)), fmaf(m.y, k, -(wi.y * eta_ti)), fmaf(m.z, k, -(wi.z * eta_ti))};
}

}  // namespace mtx
