// mtx_core/microfacet.h — Fresnel terms and the GGX / Beckmann microfacet
// distribution with visible-normal sampling (upstream mitsuba
// include/mitsuba/render/fresnel.h and microfacet.h, restated; unverifiable
// offline). Used by the bedroom BSDFs roughconductor (scene.xml:147-155,
// 165-173, 182-190, 208-216), roughdielectric (:174-179) and roughplastic
// (:113-124, :125-136).
#pragma once
#include "common.h"
#include "dmath.h"
#include "warp.h"

namespace mtx {

struct FresnelResult {
  float r, cos_theta_t, eta_it, eta_ti;
};

// Unpolarized dielectric Fresnel reflectance.
MTX_HD FresnelResult fresnel_dielectric(float cos_theta_i, float eta) {
  bool outside = cos_theta_i >= 0.f;
  float rcp_eta = 1.f / eta;
  float eta_it = outside ? eta : rcp_eta;
  float eta_ti = outside ? rcp_eta : eta;
  float cos_theta_t_sqr = fmaf(-fmaf(-cos_theta_i, cos_theta_i, 1.f), sqr(eta_ti), 1.f);
  float cos_i_abs = fabsf(cos_theta_i);
  float cos_t_abs = safe_sqrt(cos_theta_t_sqr);
  bool index_matched = eta == 1.f;
  bool special = index_matched || cos_i_abs == 0.f;
  float r_sc = index_matched ? 0.f : 1.f;
  float a_s = fmaf(-eta_it, cos_t_abs, cos_i_abs) / fmaf(eta_it, cos_t_abs, cos_i_abs);
  float a_p = fmaf(-eta_it, cos_i_abs, cos_t_abs) / fmaf(eta_it, cos_i_abs, cos_t_abs);
  float r = 0.5f * (sqr(a_s) + sqr(a_p));
  if (special) r = r_sc;
  FresnelResult fr;
  fr.r = r;
  fr.cos_theta_t = mulsign_neg(cos_t_abs, cos_theta_i);
  fr.eta_it = eta_it;
  fr.eta_ti = eta_ti;
  return fr;
}

// Conductor Fresnel with complex IOR (eta_r + i eta_i), "Optics" (Moeller 1988)
// form used upstream.
MTX_HD float fresnel_conductor(float cos_theta_i, float eta_r, float eta_i) {
  float c2 = sqr(cos_theta_i);
  float s2 = 1.f - c2;
  float s4 = sqr(s2);
  float temp_1 = sqr(eta_r) - sqr(eta_i) - s2;
  float a_2_pb_2 = safe_sqrt(sqr(temp_1) + 4.f * sqr(eta_i) * sqr(eta_r));
  float a = safe_sqrt(0.5f * (a_2_pb_2 + temp_1));
  float term_1 = a_2_pb_2 + c2;
  float term_2 = 2.f * cos_theta_i * a;
  float r_s = (term_1 - term_2) / (term_1 + term_2);
  float term_3 = a_2_pb_2 * c2 + s4;
  float term_4 = term_2 * s2;
  float r_p = r_s * (term_3 - term_4) / (term_3 + term_4);
  return 0.5f * (r_s + r_p);
}

enum : uint32_t { MICROFACET_GGX = 0, MICROFACET_BECKMANN = 1 };

// Isotropic distribution, visible-normal sampling (sample_visible = true).
struct Microfacet {
  uint32_t type;
  float alpha;

  MTX_HD float eval(V3 m) const {
    float alpha_uv = alpha * alpha;
    float cos_theta = m.z, cos_theta_2 = sqr(cos_theta);
    float result;
    if (type == MICROFACET_BECKMANN) {
      float e = -(sqr(m.x / alpha) + sqr(m.y / alpha)) / cos_theta_2;
      result = dexp(e) / (kPi * alpha_uv * sqr(cos_theta_2));
    } else {
      result = 1.f / (kPi * alpha_uv * sqr(sqr(m.x / alpha) + sqr(m.y / alpha) + sqr(m.z)));
    }
    return (result * cos_theta > 1e-20f) ? result : 0.f;
  }

  MTX_HD float smith_g1(V3 v, V3 m) const {
    float xy_alpha_2 = sqr(alpha * v.x) + sqr(alpha * v.y);
    float tan_theta_alpha_2 = xy_alpha_2 / sqr(v.z);
    float result;
    if (type == MICROFACET_BECKMANN) {
      float a = rsqrt_(tan_theta_alpha_2), a_sqr = sqr(a);
      result = (a >= 1.6f) ? 1.f
                           : (3.535f * a + 2.181f * a_sqr) / (1.f + 2.276f * a + 2.577f * a_sqr);
    } else {
      result = 2.f / (1.f + sqrtf(1.f + tan_theta_alpha_2));
    }
    if (xy_alpha_2 == 0.f) result = 1.f;
    if (dot(v, m) * v.z <= 0.f) result = 0.f;
    return result;
  }

  MTX_HD float G(V3 wi, V3 wo, V3 m) const { return smith_g1(wi, m) * smith_g1(wo, m); }

  MTX_HD V2 sample_visible_11(float cos_theta_i, V2 s) const {
    if (type == MICROFACET_BECKMANN) {
      const float kSqrtPiInv = 0.56418958354775628695f;
      float tan_theta_i = safe_sqrt(fmaf(-cos_theta_i, cos_theta_i, 1.f)) / cos_theta_i;
      float cot_theta_i = 1.f / tan_theta_i;
      float maxval = derf(cot_theta_i);
      s.x = fmaxf(fminf(s.x, 1.f - 1e-6f), 1e-6f);
      s.y = fmaxf(fminf(s.y, 1.f - 1e-6f), 1e-6f);
      float x = maxval - (maxval + 1.f) * derf(sqrtf(-dlog(s.x)));
      s.x *= 1.f + maxval + kSqrtPiInv * tan_theta_i * dexp(-sqr(cot_theta_i));
      for (int i = 0; i < 3; ++i) {
        float slope = derfinv(x);
        float value = 1.f + x + kSqrtPiInv * tan_theta_i * dexp(-sqr(slope)) - s.x;
        float derivative = 1.f - slope * tan_theta_i;
        x -= value / derivative;
      }
      return V2{derfinv(x), derfinv(2.f * s.y - 1.f)};
    }
    V2 p = square_to_uniform_disk_concentric(s);
    float sc = 0.5f * (1.f + cos_theta_i);
    p.y = lerp(safe_sqrt(1.f - sqr(p.x)), p.y, sc);
    float x = p.x, y = p.y, z = safe_sqrt(1.f - fmaf(p.y, p.y, p.x * p.x));
    float sin_theta_i = safe_sqrt(1.f - sqr(cos_theta_i));
    float nrm = 1.f / fmaf(sin_theta_i, y, cos_theta_i * z);
    return V2{fmaf(cos_theta_i, y, -(sin_theta_i * z)) * nrm, x * nrm};
  }

  // Returns the sampled microfacet normal and its density (w.r.t. m).
  MTX_HD V3 sample(V3 wi, V2 s, float *pdf) const {
    V3 wi_p = normalize(V3{alpha * wi.x, alpha * wi.y, wi.z});
    float sin_theta_2 = fmaf(wi_p.x, wi_p.x, sqr(wi_p.y));
    float inv_sin_theta = rsqrt_(sin_theta_2);
    float cphi = clampf(wi_p.x * inv_sin_theta, -1.f, 1.f);
    float sphi = clampf(wi_p.y * inv_sin_theta, -1.f, 1.f);
    if (fabsf(sin_theta_2) <= 4.f * 5.9604644775390625e-8f) {
      cphi = 1.f;
      sphi = 0.f;
    }
    float cos_theta = wi_p.z;
    V2 slope = sample_visible_11(cos_theta, s);
    V2 sl = V2{fmaf(cphi, slope.x, -(sphi * slope.y)) * alpha, fmaf(sphi, slope.x, cphi * slope.y) * alpha};
    V3 m = normalize(V3{-sl.x, -sl.y, 1.f});
    *pdf = eval(m) * smith_g1(wi, m) * absdot(wi, m) / wi.z;
    return m;
  }

  MTX_HD float pdf(V3 wi, V3 m) const { return eval(m) * smith_g1(wi, m) * absdot(wi, m) / wi.z; }
};

}  // namespace mtx
