// mtx_core/bsdf.h — the bedroom BSDF table as a switch-dispatched device
// function (replaces Dr.Jit vcalls on mi.BSDF). Semantics restated from
// upstream Mitsuba 3 plugins (unverifiable offline): diffuse, twosided,
// roughplastic (nonlinear), conductor, roughconductor, dielectric,
// roughdielectric and mask, as used by data/bedroom/scene.xml:26-219.
// Reference call sites: bsdf.eval_pdf_sample (path.py:254, path-mis.py:107,
// restirgi.py:540, nrc.py:58), bsdf.sample (pssmltsimple.py:84,
// restirgi.py:436), bsdf.eval_pdf (pssmltsimple.py:93), bsdf.eval
// (restirgi.py:268), bsdf.flags() (path.py:245).
#pragma once
#include "../mtx.h"
#include "common.h"
#include "microfacet.h"
#include "warp.h"

namespace mtx {

// Mitsuba BSDFFlags
enum : uint32_t {
  BF_NULL = 0x01,
  BF_DIFFUSE_REFLECTION = 0x02,
  BF_DIFFUSE_TRANSMISSION = 0x04,
  BF_GLOSSY_REFLECTION = 0x08,
  BF_GLOSSY_TRANSMISSION = 0x10,
  BF_DELTA_REFLECTION = 0x20,
  BF_DELTA_TRANSMISSION = 0x40,
  BF_SMOOTH = 0x02 | 0x04 | 0x08 | 0x10,
  BF_DELTA = 0x01 | 0x20 | 0x40,
};

struct BSDFSample {
  V3 wo;
  float pdf;
  float eta;
  uint32_t type;
};

// Scene data a BSDF evaluation may read (textures, roughplastic tables).
struct BsdfData {
  const mtx_texture *textures;
  const float *texels;
  const float *tables;
  // the material colour at the shading point when a caller looked it up
  // already (one texture fetch per shading point instead of one per BSDF call)
  V3 col = V3{0.f, 0.f, 0.f};
  bool has_col = false;
};

MTX_HD uint32_t bsdf_flags(const mtx_material &m) {
  uint32_t f = 0;
  switch (m.type) {
    case MTX_MAT_DIFFUSE: f = BF_DIFFUSE_REFLECTION; break;
    case MTX_MAT_ROUGHPLASTIC: f = BF_GLOSSY_REFLECTION | BF_DIFFUSE_REFLECTION; break;
    case MTX_MAT_CONDUCTOR: f = BF_DELTA_REFLECTION; break;
    case MTX_MAT_ROUGHCONDUCTOR: f = BF_GLOSSY_REFLECTION; break;
    case MTX_MAT_DIELECTRIC: f = BF_DELTA_REFLECTION | BF_DELTA_TRANSMISSION; break;
    case MTX_MAT_ROUGHDIELECTRIC: f = BF_GLOSSY_REFLECTION | BF_GLOSSY_TRANSMISSION; break;
    default: f = 0;
  }
  if (m.flags & MTX_MF_MASK) f |= BF_NULL;
  return f;
}

// Repeat wrap ((i % w) + w) % w for w > 0; the integer division (about 25
// instructions on the device) only for i outside [-w, 2w), which a texture
// coordinate in [0, 1] never reaches. Same integers in every case.
MTX_HD int wrap_repeat(int i, int w) {
  if (i >= 0 && i < w) return i;
  if (i < 0 && i >= -w) return i + w;
  if (i >= w && i - w < w) return i - w;
  return ((i % w) + w) % w;
}

// Bilinear bitmap lookup with repeat wrapping (upstream BitmapTexture::eval).
MTX_HD V3 texture_eval(const BsdfData &d, int32_t tex, V2 uv) {
  const mtx_texture t = d.textures[tex];
  const int w = (int)t.width, h = (int)t.height;
  float ux = fmaf(uv.x, (float)w, -0.5f);
  float uy = fmaf(uv.y, (float)h, -0.5f);
  float fx = floorf(ux), fy = floorf(uy);
  int ix = (int)fx, iy = (int)fy;
  float w1x = ux - fx, w1y = uy - fy;
  float w0x = 1.f - w1x, w0y = 1.f - w1y;
  int x0 = wrap_repeat(ix, w), y0 = wrap_repeat(iy, h);
  int x1 = wrap_repeat(ix + 1, w), y1 = wrap_repeat(iy + 1, h);
  const float *base = d.texels + t.offset;
  const float *f00 = base + 3 * ((uint64_t)y0 * w + x0);
  const float *f10 = base + 3 * ((uint64_t)y0 * w + x1);
  const float *f01 = base + 3 * ((uint64_t)y1 * w + x0);
  const float *f11 = base + 3 * ((uint64_t)y1 * w + x1);
  V3 r;
  r.x = fmaf(w0x, fmaf(w0y, f00[0], w1y * f01[0]), w1x * fmaf(w0y, f10[0], w1y * f11[0]));
  r.y = fmaf(w0x, fmaf(w0y, f00[1], w1y * f01[1]), w1x * fmaf(w0y, f10[1], w1y * f11[1]));
  r.z = fmaf(w0x, fmaf(w0y, f00[2], w1y * f01[2]), w1x * fmaf(w0y, f10[2], w1y * f11[2]));
  return r;
}

MTX_HD V3 mat_color(const BsdfData &d, const mtx_material &m, V2 uv) {
  if (d.has_col) return d.col;
  if (m.tex >= 0) return texture_eval(d, m.tex, uv);
  return V3{m.rgb[0], m.rgb[1], m.rgb[2]};
}

// roughplastic lerp_gather over the 64-entry transmittance table
MTX_HD float lerp_table(const float *tab, float x) {
  x *= (float)(MTX_ROUGH_TRANSMITTANCE_RES - 1);
  uint32_t idx = (uint32_t)x;
  if (idx > MTX_ROUGH_TRANSMITTANCE_RES - 2) idx = MTX_ROUGH_TRANSMITTANCE_RES - 2;
  float v0 = tab[idx], v1 = tab[idx + 1];
  return lerp(v0, v1, x - (float)idx);
}

MTX_HD Microfacet mat_distr(const mtx_material &m) {
  Microfacet d;
  d.type = (m.flags & MTX_MF_BECKMANN) ? MICROFACET_BECKMANN : MICROFACET_GGX;
  d.alpha = m.alpha;
  return d;
}

// ---------------------------------------------------------------------------
// One-sided base BSDFs. `wi` and `wo` are in the local shading frame.
// ---------------------------------------------------------------------------

// roughplastic eval + pdf (one copy, shared by eval_pdf and sample)
MTX_HD void roughplastic_eval_pdf(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, V3 wo, V3 *val,
                                  float *pdf) {
  float ci = wi.z, co = wo.z;
  if (!(ci > 0.f && co > 0.f)) return;
  Microfacet distr = mat_distr(m);
  const float *tab = d.tables + m.table;
  // --- eval ---
  V3 H = normalize(wo + wi);
  float D = distr.eval(H);
  float F = fresnel_dielectric(dot(wi, H), m.eta).r;
  float G = distr.G(wi, wo, H);
  float spec = F * D * G / (4.f * ci);
  V3 result = v3s(spec);
  float t_i = lerp_table(tab, ci), t_o = lerp_table(tab, co);
  V3 diff = mat_color(d, m, uv);
  V3 denom = (m.flags & MTX_MF_NONLINEAR) ? (v3s(1.f) - diff * m.internal_refl) : v3s(1.f - m.internal_refl);
  diff = diff / denom;
  float inv_eta_2 = 1.f / sqr(m.eta);
  diff = diff * (kInvPi * inv_eta_2 * co * t_i * t_o);
  *val = result + diff;
  // --- pdf ---
  float prob_specular = (1.f - t_i) * m.spec_weight;
  float prob_diffuse = t_i * (1.f - m.spec_weight);
  prob_specular = prob_specular / (prob_specular + prob_diffuse);
  prob_diffuse = 1.f - prob_specular;
  float p = distr.eval(H) * distr.smith_g1(wi, H) / (4.f * ci);
  p *= prob_specular;
  p = p + prob_diffuse * square_to_cosine_hemisphere_pdf(wo);
  *pdf = p;
}

// eval + pdf together (upstream eval_pdf)
MTX_HD void base_eval_pdf(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, V3 wo, V3 *val, float *pdf) {
  float ci = wi.z, co = wo.z;
  *val = v3s(0.f);
  *pdf = 0.f;
  switch (m.type) {
    case MTX_MAT_DIFFUSE: {
      if (ci > 0.f && co > 0.f) {
        V3 r = mat_color(d, m, uv);
        *val = r * kInvPi * co;
        *pdf = square_to_cosine_hemisphere_pdf(wo);
      }
      break;
    }
    case MTX_MAT_ROUGHPLASTIC:
      roughplastic_eval_pdf(d, m, uv, wi, wo, val, pdf);
      break;
    case MTX_MAT_ROUGHCONDUCTOR: {
      if (!(ci > 0.f && co > 0.f)) break;
      Microfacet distr = mat_distr(m);
      V3 H = normalize(wo + wi);
      float D = distr.eval(H);
      if (D != 0.f) {
        float G = distr.G(wi, wo, H);
        float res = D * G / (4.f * ci);
        float cdh = dot(wi, H);
        V3 F = V3{fresnel_conductor(cdh, m.eta_rgb[0], m.k_rgb[0]), fresnel_conductor(cdh, m.eta_rgb[1], m.k_rgb[1]),
                  fresnel_conductor(cdh, m.eta_rgb[2], m.k_rgb[2])};
        F = F * V3{m.rgb[0], m.rgb[1], m.rgb[2]};
        *val = F * res;
      }
      if (dot(wi, H) > 0.f && dot(wo, H) > 0.f) *pdf = distr.eval(H) * distr.smith_g1(wi, H) / (4.f * ci);
      break;
    }
    case MTX_MAT_ROUGHDIELECTRIC: {
      if (ci == 0.f) break;
      Microfacet distr = mat_distr(m);
      bool refl = ci * co > 0.f;
      float inv_eta = 1.f / m.eta;
      float eta = ci > 0.f ? m.eta : inv_eta;
      float ieta = ci > 0.f ? inv_eta : m.eta;
      V3 H = normalize(wi + wo * (refl ? 1.f : eta));
      H = mulsign3(H, H.z);
      float D = distr.eval(H);
      float F = fresnel_dielectric(dot(wi, H), m.eta).r;
      float G = distr.G(wi, wo, H);
      float dih = dot(wi, H), doh = dot(wo, H);
      if (refl) {
        *val = v3s(F * D * G / (4.f * fabsf(ci)));
      } else {
        float scale = sqr(ieta);
        float v = fabsf((scale * (1.f - F) * D * G * eta * eta * dih * doh) / (ci * sqr(dih + eta * doh)));
        *val = v3s(v);
      }
      bool side_ok = (dih * ci > 0.f) && (doh * co > 0.f);
      if (side_ok) {
        float dwh_dwo = refl ? 1.f / (4.f * doh) : (eta * eta * doh) / sqr(dih + eta * doh);
        float prob = distr.pdf(mulsign3(wi, ci), H);
        prob *= refl ? F : (1.f - F);
        *pdf = prob * fabsf(dwh_dwo);
      }
      break;
    }
    default: break;  // delta BSDFs: eval = pdf = 0
  }
}

MTX_HD V3 base_sample(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, float u1, V2 u2, BSDFSample *bs) {
  float ci = wi.z;
  bs->wo = v3s(0.f);
  bs->pdf = 0.f;
  bs->eta = 1.f;
  bs->type = 0;
  V3 weight = v3s(0.f);
  // The rough materials draw their microfacet normal in one shared call (one
  // inlined copy of the visible-normal sampler instead of three); same inputs,
  // same arithmetic as calling it inside each case.
  bool need_mf = m.type == MTX_MAT_ROUGHCONDUCTOR || m.type == MTX_MAT_ROUGHDIELECTRIC;
  V3 wi_mf = m.type == MTX_MAT_ROUGHDIELECTRIC ? mulsign3(wi, ci) : wi;
  float rp_prob_specular = 0.f;
  bool rp_specular = false;
  if (m.type == MTX_MAT_ROUGHPLASTIC && ci > 0.f) {
    const float *tab = d.tables + m.table;
    float t_i = lerp_table(tab, ci);
    float prob_specular = (1.f - t_i) * m.spec_weight;
    float prob_diffuse = t_i * (1.f - m.spec_weight);
    rp_prob_specular = prob_specular / (prob_specular + prob_diffuse);
    rp_specular = u1 < rp_prob_specular;
    need_mf = rp_specular;
  }
  float mf_pdf = 0.f;
  V3 mf_n = v3s(0.f);
  if (need_mf) mf_n = mat_distr(m).sample(wi_mf, u2, &mf_pdf);
  switch (m.type) {
    case MTX_MAT_DIFFUSE: {
      bs->wo = square_to_cosine_hemisphere(u2);
      bs->pdf = square_to_cosine_hemisphere_pdf(bs->wo);
      bs->eta = 1.f;
      bs->type = BF_DIFFUSE_REFLECTION;
      if (ci > 0.f && bs->pdf > 0.f) weight = mat_color(d, m, uv);
      break;
    }
    case MTX_MAT_CONDUCTOR: {
      bs->wo = reflect_local(wi);
      bs->pdf = 1.f;
      bs->eta = 1.f;
      bs->type = BF_DELTA_REFLECTION;
      if (ci > 0.f) {
        weight = V3{fresnel_conductor(ci, m.eta_rgb[0], m.k_rgb[0]), fresnel_conductor(ci, m.eta_rgb[1], m.k_rgb[1]),
                    fresnel_conductor(ci, m.eta_rgb[2], m.k_rgb[2])} *
                 V3{m.rgb[0], m.rgb[1], m.rgb[2]};
      }
      break;
    }
    case MTX_MAT_DIELECTRIC: {
      FresnelResult fr = fresnel_dielectric(ci, m.eta);
      float r_i = fr.r, t_i = 1.f - r_i;
      bool sel_r = u1 <= r_i;
      bs->pdf = sel_r ? r_i : t_i;
      bs->type = sel_r ? BF_DELTA_REFLECTION : BF_DELTA_TRANSMISSION;
      bs->wo = sel_r ? reflect_local(wi) : refract_local(wi, fr.cos_theta_t, fr.eta_ti);
      bs->eta = sel_r ? 1.f : fr.eta_it;
      float w = 1.f;
      if (!sel_r) w *= sqr(fr.eta_ti);
      weight = v3s(w);
      break;
    }
    case MTX_MAT_ROUGHCONDUCTOR: {
      Microfacet distr = mat_distr(m);
      float pdf = mf_pdf;
      V3 mn = mf_n;
      bs->wo = reflect_m(wi, mn);
      bs->eta = 1.f;
      bs->type = BF_GLOSSY_REFLECTION;
      bool active = ci > 0.f && pdf != 0.f && bs->wo.z > 0.f;
      float w = distr.smith_g1(bs->wo, mn);
      bs->pdf = pdf / (4.f * dot(bs->wo, mn));
      float cdm = dot(wi, mn);
      V3 F = V3{fresnel_conductor(cdm, m.eta_rgb[0], m.k_rgb[0]), fresnel_conductor(cdm, m.eta_rgb[1], m.k_rgb[1]),
                fresnel_conductor(cdm, m.eta_rgb[2], m.k_rgb[2])} *
             V3{m.rgb[0], m.rgb[1], m.rgb[2]};
      if (active) weight = F * w;
      break;
    }
    case MTX_MAT_ROUGHDIELECTRIC: {
      Microfacet distr = mat_distr(m);
      float pdf = mf_pdf;
      V3 mn = mf_n;
      bool active = pdf != 0.f;
      FresnelResult fr = fresnel_dielectric(dot(wi, mn), m.eta);
      float F = fr.r;
      bool sel_r = u1 <= F && active;
      float w = 1.f;
      pdf *= sel_r ? F : (1.f - F);
      bs->eta = sel_r ? 1.f : fr.eta_it;
      bs->type = sel_r ? BF_GLOSSY_REFLECTION : BF_GLOSSY_TRANSMISSION;
      float dwh_dwo;
      if (sel_r) {
        bs->wo = reflect_m(wi, mn);
        active = active && (bs->wo.z * ci > 0.f);
        dwh_dwo = 1.f / (4.f * dot(bs->wo, mn));
      } else {
        bs->wo = refract_m(wi, mn, fr.cos_theta_t, fr.eta_ti);
        active = active && (bs->wo.z * ci < 0.f);
        w *= sqr(fr.eta_ti);
        float doh = dot(bs->wo, mn);
        dwh_dwo = (sqr(bs->eta) * doh) / sqr(dot(wi, mn) + bs->eta * doh);
      }
      w *= distr.smith_g1(bs->wo, mn);
      bs->pdf = pdf * fabsf(dwh_dwo);
      if (active) weight = v3s(w);
      break;
    }
    case MTX_MAT_ROUGHPLASTIC: {
      if (!(ci > 0.f)) break;
      bs->eta = 1.f;
      if (rp_specular) {
        bs->wo = reflect_m(wi, mf_n);
        bs->type = BF_GLOSSY_REFLECTION;
      } else {
        bs->wo = square_to_cosine_hemisphere(u2);
        bs->type = BF_DIFFUSE_REFLECTION;
      }
      V3 val = v3s(0.f);
      float pdf = 0.f;
      roughplastic_eval_pdf(d, m, uv, wi, bs->wo, &val, &pdf);
      bs->pdf = pdf;
      if (pdf > 0.f) weight = val / pdf;
      break;
    }
    default: break;
  }
  return weight;
}

// ---------------------------------------------------------------------------
// Wrapped BSDFs: mask(opacity, twosided(base)) / twosided(base) / base.
// ---------------------------------------------------------------------------

MTX_HD void twosided_eval_pdf(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, V3 wo, V3 *val, float *pdf) {
  // one call of the base BSDF (flipped to the front side when wi.z < 0)
  const bool two = (m.flags & MTX_MF_TWOSIDED) != 0, flip = two && wi.z < 0.f;
  if (two && !(wi.z > 0.f) && !flip) {
    *val = v3s(0.f);
    *pdf = 0.f;
    return;
  }
  base_eval_pdf(d, m, uv, flip ? V3{wi.x, wi.y, -wi.z} : wi, flip ? V3{wo.x, wo.y, -wo.z} : wo, val, pdf);
}

MTX_HD V3 twosided_sample(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, float u1, V2 u2, BSDFSample *bs) {
  const bool two = (m.flags & MTX_MF_TWOSIDED) != 0, flip = two && wi.z < 0.f;
  if (two && !(wi.z > 0.f) && !flip) {
    bs->wo = v3s(0.f);
    bs->pdf = 0.f;
    bs->eta = 0.f;
    bs->type = 0;
    return v3s(0.f);
  }
  const V3 w = base_sample(d, m, uv, flip ? V3{wi.x, wi.y, -wi.z} : wi, u1, u2, bs);
  if (flip) bs->wo.z = -bs->wo.z;
  return w;
}

// BSDF::eval_pdf (value includes the cosine foreshortening, as upstream)
MTX_HD void bsdf_eval_pdf(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, V3 wo, V3 *val, float *pdf) {
  twosided_eval_pdf(d, m, uv, wi, wo, val, pdf);
  if (m.flags & MTX_MF_MASK) {
    *val = *val * m.opacity;
    *pdf = *pdf * m.opacity;
  }
}

// BSDF::sample -> (BSDFSample, weight = value/pdf)
MTX_HD V3 bsdf_sample(const BsdfData &d, const mtx_material &m, V2 uv, V3 wi, float u1, V2 u2, BSDFSample *bs) {
  // mask: nested lobe with probability `opacity`, else a Null pass-through.
  // The factors opacity / (1 - opacity) cancel in the weight and are not
  // included in bs.pdf (upstream mask.cpp).
  const bool mask = (m.flags & MTX_MF_MASK) != 0;
  if (!mask || u1 < m.opacity) return twosided_sample(d, m, uv, wi, mask ? u1 / m.opacity : u1, u2, bs);
  bs->wo = -wi;
  bs->eta = 1.f;
  bs->pdf = 1.f;
  bs->type = BF_NULL;
  return v3s(1.f);
}

}  // namespace mtx
