// mtx_core/interaction.h — surface interactions, ray spawning, the rectangle
// area emitter, the constant environment emitter, the perspective sensor and
// the two MIS weight variants.
// Upstream semantics restated (unverifiable offline):
//   Mesh::compute_surface_interaction, Interaction::spawn_ray(_to),
//   Scene::sample_emitter_direction / pdf_emitter_direction,
//   AreaEmitter + Rectangle, ConstantBackgroundEmitter (`constant`),
//   PerspectiveCamera::sample_ray.
#pragma once
#include "../mtx.h"
#include "bsdf.h"
#include "common.h"
#include "warp.h"

namespace mtx {

// Pointers to the scene arrays (HBM on the device, host memory in the oracle).
struct SceneView {
  const int32_t *nodes;         // closest-hit BVH (mtx.h, 16 words per node)
  const float *tri_geom;        // its leaf-order triangle records (the scene's triangle order)
  const int32_t *occ_nodes;     // occlusion BVH (mtx.h, 20 words per node)
  const float *occ_tri_geom;    // its own leaf-order copy of the records
  const uint32_t *tri_vidx;
  const uint32_t *tri_shape;
  const float *vpos;
  const float *vnormal;
  const float *vuv;
  const mtx_shape *shapes;
  const mtx_material *materials;
  const mtx_emitter *emitters;
  BsdfData bsdf;
  uint32_t n_tris, n_emitters;  // n_emitters: area emitters
  mtx_camera camera;
  // constant environment (scene.environment(), path-mis.py:41): emitter index
  // n_emitters when has_env; the scene's bounding sphere (env_bsphere)
  uint32_t has_env;
  float env_radiance[3], env_center[3], env_radius;
};

// The environment's emitter index (after the area emitters), -1 without one,
// and the number of emitters the uniform pick chooses from.
MTX_HD int32_t env_index(const SceneView &s) { return s.has_env ? (int32_t)s.n_emitters : -1; }
MTX_HD uint32_t emitter_count(const SceneView &s) { return s.n_emitters + (s.has_env ? 1u : 0u); }

// ConstantBackgroundEmitter::set_scene: the bounding sphere of the scene's
// bounding box (centre, |centre - min|), its radius grown by a ray epsilon.
MTX_HD void env_bsphere(const float *vpos, uint32_t n_verts, float center[3], float *radius) {
  V3 lo = v3s(kInf), hi = v3s(-kInf);
  for (uint32_t i = 0; i < n_verts; ++i) {
    lo = V3{fminf(lo.x, vpos[3 * i]), fminf(lo.y, vpos[3 * i + 1]), fminf(lo.z, vpos[3 * i + 2])};
    hi = V3{fmaxf(hi.x, vpos[3 * i]), fmaxf(hi.y, vpos[3 * i + 1]), fmaxf(hi.z, vpos[3 * i + 2])};
  }
  if (n_verts == 0 || !(lo.x <= hi.x && lo.y <= hi.y && lo.z <= hi.z)) {  // invalid box
    center[0] = center[1] = center[2] = 0.f;
    *radius = kRayEpsilon;
    return;
  }
  const V3 c = (lo + hi) * 0.5f;
  center[0] = c.x;
  center[1] = c.y;
  center[2] = c.z;
  *radius = fmaxf(kRayEpsilon, norm(c - lo) * (1.f + kRayEpsilon));
}

struct SurfaceInteraction {
  float t;
  V3 p;
  V3 n;  // geometric normal
  Frame sh;
  V2 uv;
  V3 wi;  // local
  uint32_t prim;
  int32_t material;  // -1 for an invalid interaction
  int32_t emitter;
  bool valid;
};

MTX_HD V3 load3(const float *p, uint32_t i) { return V3{p[3 * i + 0], p[3 * i + 1], p[3 * i + 2]}; }

// Hit record -> SurfaceInteraction (upstream Mesh::compute_surface_interaction:
// p = b0*p0 + b1*p1 + b2*p2, geometric normal from the winding, shading
// normal from barycentric vertex normals unless face_normals; frame from the
// shading normal with coordinate_system()). si_from_vertices is the shared
// arithmetic; the host gathers the vertices through tri_vidx, the device from
// per-triangle shading records holding the same floats.
MTX_HD SurfaceInteraction si_invalid(float t, uint32_t prim, V3 ray_d) {
  SurfaceInteraction si;
  si.t = kInf;
  si.prim = prim;
  si.valid = false;
  si.material = -1;
  si.emitter = -1;
  si.p = v3s(0.f);
  si.n = V3{0.f, 0.f, 1.f};
  si.sh = frame_from_normal(si.n);
  si.uv = V2{0.f, 0.f};
  si.wi = -ray_d;
  (void)t;
  return si;
}

MTX_HD SurfaceInteraction si_from_vertices(float t, uint32_t prim, float u, float v, V3 ray_d, V3 p0, V3 p1, V3 p2,
                                           uint32_t material, int32_t emitter, bool use_n, V3 n0, V3 n1, V3 n2,
                                           bool use_uv, V2 t0, V2 t1, V2 t2) {
  SurfaceInteraction si;
  si.t = t;
  si.prim = prim;
  si.valid = true;
  float b1 = u, b2 = v, b0 = 1.f - b1 - b2;
  si.p = fma3(p0, b0, fma3(p1, b1, p2 * b2));
  V3 dp0 = p1 - p0, dp1 = p2 - p0;
  si.n = normalize(cross(dp0, dp1));
  si.material = (int32_t)material;
  si.emitter = emitter;
  V3 ns = si.n;
  if (use_n) ns = normalize(fma3(n0, b0, fma3(n1, b1, n2 * b2)));
  if (use_uv) {
    si.uv = V2{fmaf(t0.x, b0, fmaf(t1.x, b1, t2.x * b2)), fmaf(t0.y, b0, fmaf(t1.y, b1, t2.y * b2))};
  } else {
    si.uv = V2{b1, b2};
  }
  si.sh = frame_from_normal(ns);
  si.wi = to_local(si.sh, -ray_d);
  return si;
}

MTX_HD SurfaceInteraction compute_si(const SceneView &s, float t, uint32_t prim, float u, float v, V3 ray_d) {
  if (prim == 0xffffffffu) {  // a miss: si.emitter(scene) is the environment, if any
    SurfaceInteraction si = si_invalid(t, prim, ray_d);
    si.emitter = env_index(s);
    return si;
  }
  const uint32_t i0 = s.tri_vidx[3 * prim + 0], i1 = s.tri_vidx[3 * prim + 1], i2 = s.tri_vidx[3 * prim + 2];
  const V3 p0 = load3(s.vpos, i0), p1 = load3(s.vpos, i1), p2 = load3(s.vpos, i2);
  const mtx_shape sh = s.shapes[s.tri_shape[prim]];
  const bool use_n = !(sh.flags & 1u) && s.vnormal;
  const bool use_uv = (sh.flags & 2u) && s.vuv;
  V3 n0 = v3s(0.f), n1 = v3s(0.f), n2 = v3s(0.f);
  V2 t0 = V2{0.f, 0.f}, t1 = t0, t2 = t0;
  if (use_n) {
    n0 = load3(s.vnormal, i0);
    n1 = load3(s.vnormal, i1);
    n2 = load3(s.vnormal, i2);
  }
  if (use_uv) {
    t0 = V2{s.vuv[2 * i0], s.vuv[2 * i0 + 1]};
    t1 = V2{s.vuv[2 * i1], s.vuv[2 * i1 + 1]};
    t2 = V2{s.vuv[2 * i2], s.vuv[2 * i2 + 1]};
  }
  return si_from_vertices(t, prim, u, v, ray_d, p0, p1, p2, sh.material, sh.emitter, use_n, n0, n1, n2, use_uv, t0,
                          t1, t2);
}

// Interaction::offset_p / spawn_ray / spawn_ray_to
MTX_HD V3 offset_p(V3 p, V3 n, V3 d) {
  float mag = (1.f + hmax(vabs(p))) * kRayEpsilon;
  mag = mulsign(mag, dot(n, d));
  return fma3(n, mag, p);
}
struct Ray {
  V3 o, d;
  float maxt;
};
MTX_HD Ray spawn_ray(V3 p, V3 n, V3 d) { return Ray{offset_p(p, n, d), d, kLargest}; }
MTX_HD Ray spawn_ray_to(V3 p, V3 n, V3 t) {
  V3 o = offset_p(p, n, t - p);
  V3 d = t - o;
  float dist = norm(d);
  d = d / dist;
  return Ray{o, d, dist * (1.f - kShadowEpsilon)};
}

// ------------------------- area emitter -----------------------------------

struct DirectionSample {
  V3 p, n, d;
  float dist, pdf;
  int32_t emitter;
};

// Scene::sample_emitter_direction(ref, sample, test_visibility) without the
// visibility test (the caller traces the shadow ray): uniform emitter pick,
// Rectangle::sample_position, Shape::sample_direction (area -> solid angle),
// AreaEmitter::sample_direction (one-sided). Returns the emitter weight
// (radiance / pdf, times the emitter count); `ds.pdf` includes the pick pdf.
MTX_HD V3 sample_emitter_direction(const SceneView &s, V3 ref_p, V2 u, DirectionSample *ds) {
  const uint32_t count = emitter_count(s);
  const float count_f = (float)count;
  float scaled = u.x * count_f;
  uint32_t index = (uint32_t)scaled;
  if (index > count - 1u) index = count - 1u;
  u.x = scaled - (float)index;
  if ((int32_t)index == env_index(s)) {
    // ConstantBackgroundEmitter::sample_direction: a uniform sphere direction
    // and a target point two bounding radii away (the radius grown to reach
    // a reference point outside the sphere); weight radiance / pdf
    const V3 d = square_to_uniform_sphere(u);
    const V3 ctr = V3{s.env_center[0], s.env_center[1], s.env_center[2]};
    const float radius = fmaxf(s.env_radius, norm(ref_p - ctr));
    const float dist = 2.f * radius;
    ds->p = fma3(d, dist, ref_p);
    ds->n = -d;
    ds->d = d;
    ds->dist = dist;
    ds->pdf = square_to_uniform_sphere_pdf(d);
    ds->emitter = (int32_t)index;
    V3 spec = V3{s.env_radiance[0], s.env_radiance[1], s.env_radiance[2]} / ds->pdf;
    ds->pdf *= 1.f / count_f;
    spec = spec * count_f;
    if (!(ds->pdf != 0.f)) spec = v3s(0.f);
    return spec;
  }
  const mtx_emitter e = s.emitters[index];
  // Rectangle::sample_position: to_world.transform_affine((2u-1, 2v-1, 0))
  float lx = fmaf(u.x, 2.f, -1.f), ly = fmaf(u.y, 2.f, -1.f);
  V3 c0 = V3{e.col0[0], e.col0[1], e.col0[2]}, c1 = V3{e.col1[0], e.col1[1], e.col1[2]};
  V3 ctr = V3{e.center[0], e.center[1], e.center[2]};
  V3 p = fma3(c0, lx, fma3(c1, ly, ctr));
  ds->p = p;
  ds->n = V3{e.normal[0], e.normal[1], e.normal[2]};
  ds->emitter = (int32_t)index;
  // Shape::sample_direction
  V3 d = p - ref_p;
  float dist_squared = squared_norm(d);
  ds->dist = sqrtf(dist_squared);
  ds->d = d / ds->dist;
  float dp = absdot(ds->d, ds->n);
  float x = dist_squared / dp;
  ds->pdf = e.inv_area * (isfinite_(x) ? x : 0.f);
  // AreaEmitter::sample_direction: one-sided, non-zero pdf
  bool active = dot(ds->d, ds->n) < 0.f && ds->pdf != 0.f;
  V3 spec = v3s(0.f);
  if (active) spec = V3{e.radiance[0], e.radiance[1], e.radiance[2]} / ds->pdf;
  // Scene: account for the discrete pick probability
  ds->pdf *= 1.f / count_f;
  spec = spec * count_f;
  if (!(ds->pdf != 0.f)) spec = v3s(0.f);
  return spec;
}

// Scene::pdf_emitter_direction(ref, ds) for ds = DirectionSample3f(scene, si, ref):
// shape pdf_position * dist^2 / |cos|, zero unless the emitter faces ref.
MTX_HD float pdf_emitter_direction(const SceneView &s, int32_t emitter, V3 ds_d, float ds_dist, V3 ds_n) {
  if (emitter < 0) return 0.f;
  if (emitter == env_index(s))  // ConstantBackgroundEmitter::pdf_direction
    return square_to_uniform_sphere_pdf(ds_d) * (1.f / (float)emitter_count(s));
  const mtx_emitter e = s.emitters[emitter];
  float dp = absdot(ds_d, ds_n);
  float pdf = e.inv_area * ((dp != 0.f) ? sqr(ds_dist) / dp : 0.f);
  if (!(dot(ds_d, ds_n) < 0.f)) pdf = 0.f;
  return pdf * (1.f / (float)emitter_count(s));
}

// AreaEmitter::eval(si): radiance if the front side is seen.
MTX_HD V3 emitter_eval(const SceneView &s, int32_t emitter, V3 wi_local) {
  if (emitter < 0) return v3s(0.f);
  if (emitter == env_index(s))  // ConstantBackgroundEmitter::eval: the radiance, any direction
    return V3{s.env_radiance[0], s.env_radiance[1], s.env_radiance[2]};
  const mtx_emitter e = s.emitters[emitter];
  if (!(wi_local.z > 0.f)) return v3s(0.f);
  return V3{e.radiance[0], e.radiance[1], e.radiance[2]};
}

// --------------------------- sensor ----------------------------------------

// PerspectiveCamera::sample_ray for a film-normalised position in [0,1]^2
// (fov along x, +x of the camera maps to the left of the image).
MTX_HD Ray camera_ray(const mtx_camera &c, V2 pos) {
  V3 dl = V3{(1.f - 2.f * pos.x) * c.tan_x, (1.f - 2.f * pos.y) * c.tan_y, 1.f};
  dl = normalize(dl);
  V3 ax = V3{c.axis_x[0], c.axis_x[1], c.axis_x[2]};
  V3 ay = V3{c.axis_y[0], c.axis_y[1], c.axis_y[2]};
  V3 az = V3{c.axis_z[0], c.axis_z[1], c.axis_z[2]};
  V3 d = fma3(ax, dl.x, fma3(ay, dl.y, az * dl.z));
  float inv_z = 1.f / dl.z;
  float near_t = c.near_clip * inv_z, far_t = c.far_clip * inv_z;
  V3 o = V3{c.origin[0], c.origin[1], c.origin[2]};
  o = fma3(d, near_t, o);
  return Ray{o, d, far_t - near_t};
}

// ------------------------------ MIS ----------------------------------------

// path.py:10-18 (variant A): a^2/(a^2+b^2), 0 if not finite.
MTX_HD float mis_weight_a(float pdf_a, float pdf_b) {
  float a2 = sqr(pdf_a), b2 = sqr(pdf_b);
  float w = a2 / (a2 + b2);
  return isfinite_(w) ? w : 0.f;
}
// path-mis.py:9-15 (variant B, also pssmlt.py:9-15, restirgi.py:75-81):
// select(pdf_a > 0, a^2 / fma(b, b, a^2), 0).
MTX_HD float mis_weight_b(float pdf_a, float pdf_b) {
  float a2 = sqr(pdf_a);
  return pdf_a > 0.f ? a2 / fmaf(pdf_b, pdf_b, a2) : 0.f;
}

}  // namespace mtx
