// oracle/oracle.cpp — CPU restatement of the reference hot path.
//
// TEST INFRASTRUCTURE ONLY. Nothing in the product (libmtx, the mtx Python
// package's render path) may link, load or call this library; it is used by
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
// checker / timed CPU baseline.
//
// What it restates, one scalar lane at a time, exactly in the order of the
// reference source:
//   * path-mis.py:24-155   PathIntegrator.sample      -> orc_path_mis()
//   * path.py:194-302      Path.sample                -> orc_path()
//   * nrc.py:25-125        NRCIntegrator.sample       -> orc_nrc()
//   * path.py:27-192       transcribed SamplingIntegrator.render/render_sample
//                          (lane -> pixel, film jitter, camera ray, block.put)
//   * pssmlt.py / pssmltsimple.py Pssmlt.render      -> orc_pssmlt_render()
//   * pssmltpath.py:17-190 PssmltPath.sample          -> orc_pssmlt_path_sample()
//   * restirgi.py:182-457 RestirIntegrator.render    -> orc_restir_frame()
//   * prefix_sum.py:9-36, hashgrid.py:8-90, reductions.py:12-54
//   * nerad.py:118-310 IntersectionSampler.sample / Integrator.sample_rhs
//                          (training samples)      -> orc_nerad_lhs/_rhs()
// The upstream per-lane primitives these loops call (Scene.ray_intersect,
// BSDF, emitter, sampler) come from include/mtx_core;
// the BVH traversal below is an independent scalar re-implementation over
// the scene's node arrays, with the same child-visit order as the device
// kernel so that visit counts can be compared exactly.
//
// Parity status: the reference's own implementation (Mitsuba 3 / Dr.Jit /
// Embree) is absent from the reference tree (empty submodule, SURVEY.md
// §8c), so results at the upstream boundary are "parity unpinned"; the
// in-repo KATs (hashgrid.py:93-98, reductions.py:57-63, prefix_sum.py:39-54)
// pin the primitives.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <omp.h>

#include <algorithm>
#include <parallel/algorithm>
#include <vector>

#include "mtx.h"
#include "mtx_core/bsdf.h"
#include "mtx_core/geometry.h"
#include "mtx_core/interaction.h"
#include "mtx_core/restir.h"
#include "mtx_core/field.h"
#include "mtx_core/rng.h"
#include "mtx_core/warp.h"
#include "mtx_core/nerad.h"

using namespace mtx;

namespace {

SceneView make_view(const mtx_scene_desc *d) {
  SceneView s;
  s.nodes = d->nodes;
  s.tri_geom = d->tri_geom;
  if (!d->occ_nodes || !d->occ_tri_geom) {
    std::fprintf(stderr, "oracle: the scene desc needs its occlusion BVH (occ_nodes, occ_tri_geom)\n");
    std::abort();
  }
  s.occ_nodes = d->occ_nodes;
  s.occ_tri_geom = d->occ_tri_geom;
  s.tri_vidx = d->tri_vidx;
  s.tri_shape = d->tri_shape;
  s.vpos = d->vpos;
  s.vnormal = d->vnormal;
  s.vuv = d->vuv;
  s.shapes = d->shapes;
  s.materials = d->materials;
  s.emitters = d->emitters;
  s.bsdf.textures = d->textures;
  s.bsdf.texels = d->texels;
  s.bsdf.tables = d->tables;
  s.n_tris = d->n_tris;
  s.n_emitters = d->n_emitters;
  s.camera = d->camera;
  s.has_env = d->has_env ? 1u : 0u;
  for (int k = 0; k < 3; ++k) s.env_radiance[k] = d->env_radiance[k];
  env_bsphere(d->vpos, d->n_verts, s.env_center, &s.env_radius);
  return s;
}

struct Hit {
  float t, u, v;
  uint32_t prim;
};

// Diagnostic (tools/ only): visits per node index < g_hist_len are counted
// into g_hist while orc_node_visit_hist runs (the top-of-tree share of node
// fetches that an LDS-resident tree top would serve).
static uint64_t *g_hist = nullptr;
static uint32_t g_hist_len = 0;

// Scalar closest-hit traversal of the 4-wide BVH (mtx.h) in the device
// kernels' per-ray order: a node's hit children sorted by entry distance
// (mtx_core/geometry.h wide_node_order), the nearest visited next and the
// others pushed far-to-near; a leaf's triangles in index order. Ties on t
// go to the smaller prim, so the hit does not depend on the order; the
// visit counts do, and match the device (device_common.h trace_loop_closest).
Hit trace_closest(const SceneView &s, V3 o, V3 d, float maxt, uint32_t *nodes_visited, uint32_t *tris_visited) {
  TraceRay r = make_trace_ray(o, d, maxt);
  Hit h{maxt, 0.f, 0.f, 0xffffffffu};
  float tbest = maxt;
  int32_t stack[3 * MTX_BVH_MAX_DEPTH + 2];
  int sp = 0;
  int32_t node = 0;
  uint32_t nv = 0, tv = 0;
  while (true) {
    if (node >= 0) {
      const int32_t *w = s.nodes + MTX_BVH_NODE_WORDS * (size_t)node;
      const float *f = reinterpret_cast<const float *>(w);
      ++nv;
      if (g_hist && (uint32_t)node < g_hist_len) {
#pragma omp atomic
        ++g_hist[node];
      }
      uint32_t key[4];
      const int n = wide_node_order(r, f[0], f[1], f[2], (uint32_t)w[3], (uint32_t)w[8], (uint32_t)w[9],
                                    (uint32_t)w[10], (uint32_t)w[11], (uint32_t)w[12], (uint32_t)w[13], tbest, key);
      if (n > 0) {
        for (int rr = n - 1; rr >= 1; --rr) stack[sp++] = wide_ref(key[rr], w[4], w[5], w[6], w[7]);
        node = wide_ref(key[0], w[4], w[5], w[6], w[7]);
        continue;
      }
    } else {
      uint32_t first, count;
      leaf_decode(node, &first, &count);
      for (uint32_t k = 0; k < count; ++k) {
        uint32_t prim = first + k;
        const float *g = s.tri_geom + 12 * (size_t)prim;
        float t, u, v;
        ++tv;
        if (tri_intersect(r, V3{g[0], g[1], g[2]}, V3{g[4], g[5], g[6]}, V3{g[8], g[9], g[10]}, tbest, &t, &u, &v)) {
          if (t < tbest || (t == tbest && prim < h.prim)) {
            tbest = t;
            h.t = t;
            h.u = u;
            h.v = v;
            h.prim = prim;
          }
        }
      }
    }
    if (sp == 0) break;
    node = stack[--sp];
  }
  if (nodes_visited) *nodes_visited = nv;
  if (tris_visited) *tris_visited = tv;
  if (h.prim == 0xffffffffu) h.t = kInf;
  return h;
}

// Scalar any-hit traversal of the 8-wide occlusion BVH (mtx.h) in the device
// kernels' per-ray order (mtx_core/geometry.h cw_node_hits): a visited node
// yields a node group (child_base, the hit inner children as mask bits in
// octant order, imask) and a triangle group (tri_base, the hit leaves'
// triangles as mask bits); the triangle group is tested first, one triangle
// per step in ascending offset, then the next child of the node group (the
// lowest bit) is visited with the rest of the group pushed; an empty group
// pops the next one. The answer (any triangle hit in (0, maxt]) does not
// depend on the tree; the visit counts do, and match the device
// (device_common.h trace_loop_occ).
bool trace_any(const SceneView &s, V3 o, V3 d, float maxt, uint32_t *nodes_visited, uint32_t *tris_visited) {
  TraceRay r = make_trace_ray(o, d, maxt);
  const uint32_t oct = ray_octant(r);
  uint32_t stack[2 * (MTX_BVH_MAX_DEPTH + 2)];
  int sp = 0;
  uint32_t gbase = 0, ghits = (1u << (24 + oct)) | 1u;  // the root: node 0 in slot 0
  uint32_t tbase = 0, thits = 0;
  uint32_t nv = 0, tv = 0;
  bool hit = false;
  while (true) {
    if (thits) {
      const uint32_t prim = tbase + (uint32_t)ctz32(thits);
      thits &= thits - 1u;
      const float *g = s.occ_tri_geom + 12 * (size_t)prim;
      float t, u, v;
      ++tv;
      if (tri_intersect(r, V3{g[0], g[1], g[2]}, V3{g[4], g[5], g[6]}, V3{g[8], g[9], g[10]}, maxt, &t, &u, &v)) {
        hit = true;
        break;
      }
    } else if (ghits >> 24) {
      const uint32_t p = (uint32_t)ctz32(ghits >> 24);
      ghits &= ~(1u << (24 + p));
      const uint32_t node = cw_inner_child(gbase, ghits & 0xffu, oct, p);
      if (ghits >> 24) {
        stack[sp++] = gbase;
        stack[sp++] = ghits;
      }
      const uint32_t *w = reinterpret_cast<const uint32_t *>(s.occ_nodes) + MTX_OCC_NODE_WORDS * (size_t)node;
      const float *f = reinterpret_cast<const float *>(w);
      ++nv;
      if (g_hist && node < g_hist_len) {
#pragma omp atomic
        ++g_hist[node];
      }
      const uint32_t hm = cw_node_hits(r, oct, f[0], f[1], f[2], w[3], w[6], w[7], w + 8, maxt);
      gbase = w[4];
      ghits = (hm & 0xff000000u) | (w[3] >> 24);
      tbase = w[5];
      thits = hm & 0x00ffffffu;
    } else if (sp > 0) {
      ghits = stack[--sp];
      gbase = stack[--sp];
    } else {
      break;
    }
  }
  if (nodes_visited) *nodes_visited = nv;
  if (tris_visited) *tris_visited = tv;
  return hit;
}

Hit brute_closest(const SceneView &s, V3 o, V3 d, float maxt) {
  TraceRay r = make_trace_ray(o, d, maxt);
  Hit h{maxt, 0.f, 0.f, 0xffffffffu};
  float tbest = maxt;
  for (uint32_t prim = 0; prim < s.n_tris; ++prim) {
    const float *g = s.tri_geom + 12 * (size_t)prim;
    float t, u, v;
    if (tri_intersect(r, V3{g[0], g[1], g[2]}, V3{g[4], g[5], g[6]}, V3{g[8], g[9], g[10]}, tbest, &t, &u, &v)) {
      if (t < tbest || (t == tbest && prim < h.prim)) {
        tbest = t;
        h = Hit{t, u, v, prim};
      }
    }
  }
  if (h.prim == 0xffffffffu) h.t = kInf;
  return h;
}

SurfaceInteraction intersect(const SceneView &s, const Ray &ray) {
  Hit h = trace_closest(s, ray.o, ray.d, ray.maxt, nullptr, nullptr);
  return compute_si(s, h.t, h.prim, h.u, h.v, ray.d);
}

// scene.sample_emitter_direction(si, u, test_visibility=True) (upstream)
V3 sample_emitter_visible(const SceneView &s, const SurfaceInteraction &si, V2 u, DirectionSample *ds) {
  V3 spec = sample_emitter_direction(s, si.p, u, ds);
  Ray sr = spawn_ray_to(si.p, si.n, ds->p);
  if (trace_any(s, sr.o, sr.d, sr.maxt, nullptr, nullptr)) spec = v3s(0.f);
  return spec;
}

bool smooth(const SceneView &s, const SurfaceInteraction &si) {
  if (!si.valid) return false;
  return (bsdf_flags(s.materials[si.material]) & BF_SMOOTH) != 0;
}

// bsdf.eval_pdf_sample on si (null BSDF for an invalid interaction)
V3 eval_pdf_sample(const SceneView &s, const SurfaceInteraction &si, V3 wo, float u1, V2 u2, V3 *val, float *pdf,
                   BSDFSample *bs) {
  if (!si.valid) {
    *val = v3s(0.f);
    *pdf = 0.f;
    bs->wo = v3s(0.f);
    bs->pdf = 0.f;
    bs->eta = 0.f;
    bs->type = 0;
    return v3s(0.f);
  }
  const mtx_material &m = s.materials[si.material];
  bsdf_eval_pdf(s.bsdf, m, si.uv, si.wi, wo, val, pdf);
  return bsdf_sample(s.bsdf, m, si.uv, si.wi, u1, u2, bs);
}

// ------------------------- path-mis.py:24-155 ------------------------------
V3 orc_path_mis(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, uint32_t rr_depth, bool *valid_out) {
  V3 throughput = v3s(1.f), result = v3s(0.f);
  float eta = 1.f;
  uint32_t depth = 0;
  bool valid_ray = s.has_env != 0;  // scene.environment() is not None (:41; None for the bedroom)
  V3 prev_p = v3s(0.f);
  float prev_bsdf_pdf = 1.f;
  bool prev_bsdf_delta = true;
  bool active = true;
  while (active) {
    SurfaceInteraction si = intersect(s, ray);  // :69-71
    // Direct emission (:75-86)
    V3 rel = si.p - prev_p;
    float dist = norm(rel);
    V3 ds_d = si.valid ? rel / dist : to_world(si.sh, si.wi) * -1.f;
    float em_pdf = prev_bsdf_delta ? 0.f : pdf_emitter_direction(s, si.emitter, ds_d, dist, si.sh.n);
    float mis_bsdf = mis_weight_b(prev_bsdf_pdf, em_pdf);
    V3 le = (prev_bsdf_pdf > 0.f) ? emitter_eval(s, si.emitter, si.wi) : v3s(0.f);
    result = fma3v(throughput, le * mis_bsdf, result);
    bool active_next = (depth + 1 < max_depth) && si.valid;  // :88
    // Emitter sampling (:94-98)
    bool active_em = active_next && smooth(s, si);
    V2 u_em = rng.next_2d();
    DirectionSample ds{};
    V3 em_weight = v3s(0.f);
    if (active_em) em_weight = sample_emitter_visible(s, si, u_em, &ds);
    V3 wo = to_local(si.sh, ds.d);
    // BSDF eval + sample (:104-109)
    float s1 = rng.next_1d();
    V2 s2 = rng.next_2d();
    V3 bsdf_val;
    float bsdf_pdf;
    BSDFSample bs;
    V3 bsdf_weight = eval_pdf_sample(s, si, wo, s1, s2, &bsdf_val, &bsdf_pdf, &bs);
    // Emitter sampling contribution (:115-117)
    float mi_em = mis_weight_b(ds.pdf, bsdf_pdf);
    if (active_em) result = fma3v(throughput, bsdf_val * em_weight * mi_em, result);
    // BSDF sampling (:121-137)
    ray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));
    throughput = throughput * bsdf_weight;
    eta *= bs.eta;
    valid_ray = valid_ray || (active && si.valid && !(bs.type & BF_NULL));
    prev_p = si.p;
    prev_bsdf_pdf = bs.pdf;
    prev_bsdf_delta = (bs.type & BF_DELTA) != 0;
    // Stopping criterion (:141-153)
    if (si.valid) depth += 1;
    float throughput_max = hmax(throughput);
    float rr_prop = fminf(throughput_max * sqr(eta), 0.95f);
    bool rr_active = depth >= rr_depth;
    bool rr_continue = rng.next_1d() < rr_prop;
    if (rr_active) throughput = throughput * rcp(rr_prop);
    active = active_next && (!rr_active || rr_continue) && (throughput_max != 0.f);
  }
  *valid_out = valid_ray;
  return valid_ray ? result : v3s(0.f);  // :155
}

// ---------------------------- simple.py:14-116 -----------------------------
// BSDF-sampling-only path tracer ("integrator"); the test estimator without
// NEE that the NEE + MIS integrators must agree with in expectation.
V3 orc_simple(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, uint32_t rr_depth, bool *valid_out) {
  V3 f = v3s(1.f), L = v3s(0.f);
  float eta = 1.f;
  uint32_t depth = 0;
  float prev_bsdf_pdf = 1.f;
  bool active = true;
  while (active) {  // :55
    SurfaceInteraction si = intersect(s, ray);  // :57-59
    V3 le = (prev_bsdf_pdf > 0.f) ? emitter_eval(s, si.emitter, si.wi) : v3s(0.f);
    L = fma3v(f, le, L);  // :69-70
    bool active_next = (depth + 1 < max_depth) && si.valid;  // :72
    float s1 = rng.next_1d();  // :77-78
    V2 s2 = rng.next_2d();
    BSDFSample bs{};
    bs.wo = v3s(0.f);
    V3 bsdf_weight = v3s(0.f);
    if (active_next)  // bsdf.sample(..., active_next) (:80)
      bsdf_weight = bsdf_sample(s.bsdf, s.materials[si.material], si.uv, si.wi, s1, s2, &bs);
    ray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));  // :86
    f = f * bsdf_weight;  // :98
    eta *= bs.eta;
    prev_bsdf_pdf = bs.pdf;
    if (si.valid) depth += 1;  // :106
    float fmax_ = hmax(f);
    float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);  // :110
    bool rr_active = depth >= rr_depth;
    bool rr_continue = rng.next_1d() < rr_prob;
    if (rr_active) f = f * rcp(rr_prob);  // :114
    active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);  // :116
  }
  *valid_out = depth != 0;  // :118
  return L;
}

// ---------------------------- path.py:194-302 ------------------------------
V3 orc_path(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, uint32_t rr_depth, bool *valid_out) {
  V3 L = v3s(0.f), f = v3s(1.f);
  float eta = 1.f;
  uint32_t depth = 1;
  bool active = depth < max_depth;  // :235 (self.max_depth)
  SurfaceInteraction si;
  if (active) {
    si = intersect(s, ray);  // :238
    L = L + emitter_eval(s, si.emitter, si.wi);  // :239
  } else {
    si = compute_si(s, kInf, 0xffffffffu, 0.f, 0.f, ray.d);
  }
  while (active) {  // :241
    bool active_em = active && smooth(s, si);  // :245
    DirectionSample ds{};
    V3 em_weight = v3s(0.f);
    V2 u_em = rng.next_2d();
    if (active_em) em_weight = sample_emitter_visible(s, si, u_em, &ds);  // :247-249
    active_em = active_em && ds.pdf != 0.f;  // :250
    V3 wo = to_local(si.sh, ds.d);
    float s1 = rng.next_1d();
    V2 s2 = rng.next_2d();
    V3 bsdf_val;
    float bsdf_pdf;
    BSDFSample bs;
    V3 bsdf_weight = eval_pdf_sample(s, si, wo, s1, s2, &bsdf_val, &bsdf_pdf, &bs);  // :254-256
    float mis_em = mis_weight_a(ds.pdf, bsdf_pdf);  // :258
    if (active_em) L = L + f * bsdf_val * em_weight * mis_em;  // :259
    f = f * bsdf_weight;  // :263
    eta *= bs.eta;
    float fmax_ = hmax(f);  // :268
    float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
    bool rr_active = depth >= rr_depth;
    bool rr_continue = rng.next_1d() < rr_prob;
    if (rr_active) f = f * rcp(rr_prob);  // :274
    active = active && (fmax_ != 0.f);
    active = active && (!rr_active || rr_continue);
    Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));  // :280
    SurfaceInteraction si2 = active ? intersect(s, nray) : compute_si(s, kInf, 0xffffffffu, 0.f, 0.f, nray.d);
    bool bsdf_delta = (bs.type & BF_DELTA) != 0;
    V3 rel = si2.p - si.p;
    float dist = norm(rel);
    V3 ds_d = si2.valid ? rel / dist : to_world(si2.sh, si2.wi) * -1.f;
    float em_pdf = bsdf_delta ? 0.f : pdf_emitter_direction(s, si2.emitter, ds_d, dist, si2.sh.n);  // :287-288
    float mis_bsdf = mis_weight_a(bs.pdf, em_pdf);  // :290
    V3 le = (bs.pdf > 0.f) ? emitter_eval(s, si2.emitter, si2.wi) : v3s(0.f);
    if (active) L = L + f * le * mis_bsdf;  // :292
    si = si2;
    if (active) depth += 1;  // :297
    active = active && depth < max_depth;
    active = active && si.valid;
  }
  *valid_out = depth != 0;
  return L;
}

// ----------------------------- nrc.py:25-125 -------------------------------
// With `query` (the radiance-cache option, MTX_RENDER_NRC_CACHE, SURVEY §8f
// item 3) the segment stopped by the spread criterion traces its BSDF ray one
// more time; a valid hit becomes the cache query (p, -d, f) written as
// query[0..9] = {1, p.xyz, wi.xyz, f.xyz}. L itself is unchanged.
V3 orc_nrc(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, float c, bool *valid_out,
           float *query = nullptr) {
  if (query)
    for (int k = 0; k < 10; ++k) query[k] = 0.f;
  SurfaceInteraction si = intersect(s, ray);  // :117
  const bool primary_valid = si.valid;
  bool active = si.valid;  // :119
  float a0 = squared_norm(ray.o - si.p) / (kFourPi * fabsf(si.wi.z));  // :121
  // next_segment (:25-102)
  V3 L = v3s(0.f), f = v3s(1.f);
  float eta = 1.f;
  uint32_t depth = 1;
  float spread = 0.f;
  while (active) {
    bool active_em = active && smooth(s, si);
    V2 u_em = rng.next_2d();
    DirectionSample ds{};
    V3 em_weight = v3s(0.f);
    if (active) em_weight = sample_emitter_visible(s, si, u_em, &ds);  // :51-53 (uses `active`)
    active_em = active_em && ds.pdf != 0.f;
    V3 wo = to_local(si.sh, ds.d);
    float s1 = rng.next_1d();
    V2 s2 = rng.next_2d();
    V3 bsdf_val;
    float bsdf_pdf;
    BSDFSample bs;
    V3 bsdf_weight = eval_pdf_sample(s, si, wo, s1, s2, &bsdf_val, &bsdf_pdf, &bs);
    float mis_em = mis_weight_b(ds.pdf, bsdf_pdf);
    if (active_em) L = L + f * bsdf_val * em_weight * mis_em;  // :62
    f = f * bsdf_weight;
    eta *= bs.eta;
    float a = sqr(spread);  // :70-71
    const bool stopped = active && !(a < c * a0);
    active = active && (a < c * a0);
    Ray nray = spawn_ray(si.p, si.n, to_world(si.sh, bs.wo));
    if (stopped && query) {
      SurfaceInteraction sq = intersect(s, nray);
      if (sq.valid) {
        const float qv[10] = {1.f, sq.p.x, sq.p.y, sq.p.z, -nray.d.x, -nray.d.y, -nray.d.z, f.x, f.y, f.z};
        for (int k = 0; k < 10; ++k) query[k] = qv[k];
      }
    }
    SurfaceInteraction si2 = active ? intersect(s, nray) : compute_si(s, kInf, 0xffffffffu, 0.f, 0.f, nray.d);
    bool bsdf_delta = (bs.type & BF_DELTA) != 0;
    V3 rel = si2.p - si.p;
    float dist = norm(rel);
    V3 ds_d = si2.valid ? rel / dist : to_world(si2.sh, si2.wi) * -1.f;
    float em_pdf = bsdf_delta ? 0.f : pdf_emitter_direction(s, si2.emitter, ds_d, dist, si2.sh.n);
    float mis_bsdf = mis_weight_b(bs.pdf, em_pdf);
    V3 le = (bs.pdf > 0.f) ? emitter_eval(s, si2.emitter, si2.wi) : v3s(0.f);
    if (active) L = L + f * le * mis_bsdf;  // :85
    spread += sqrtf(squared_norm(si2.p - si.p) / (bs.pdf * fabsf(si2.wi.z)));  // :91-93
    si = si2;
    if (active) depth += 1;
    active = active && depth < max_depth;
    active = active && si.valid;
  }
  *valid_out = primary_valid;  // :125
  return L;
}

// Dr.Jit clamp(x, lo, hi) = maximum(minimum(x, hi), lo) with NaN-ignoring
// minimum/maximum: clamp(NaN, 0, 1) = 1.
inline float dr_clamp(float x, float lo, float hi) { return fmaxf(fminf(x, hi), lo); }

// ----------------------- pssmltsimple.py:16-133 ----------------------------
// One proposal of a chain: BSDF-only tracer (no NEE, no MIS); the local BSDF
// direction of every bounce is mutated against the current path's vertex
// (mutate, :135-142) and written to the proposed vertex buffer.
V3 orc_pssmlt_sample(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, uint32_t rr_depth, bool large_step,
                     const V3 *path_v, V3 *prop_v) {
  V3 f = v3s(1.f), L = v3s(0.f);
  float eta = 1.f;
  uint32_t depth = 0;
  float prev_bsdf_pdf = 1.f;
  bool active = true;
  while (active) {
    SurfaceInteraction si = intersect(s, ray);  // :62-64
    V3 le = (prev_bsdf_pdf > 0.f) ? emitter_eval(s, si.emitter, si.wi) : v3s(0.f);
    L = fma3v(f, le, L);  // :74
    bool active_next = (depth + 1 < max_depth) && si.valid;  // :76
    float s1 = rng.next_1d();  // :81-82
    V2 s2 = rng.next_2d();
    BSDFSample bs{};
    V3 w = v3s(0.f);
    const mtx_material *mat = si.valid ? &s.materials[si.material] : nullptr;
    if (mat) w = bsdf_sample(s.bsdf, *mat, si.uv, si.wi, s1, s2, &bs);  // :84
    if (!active_next) w = v3s(0.f);  // sample(..., active_next): weight masked
    // mutate (:135-142): a = 0.1
    V3 old = path_v[depth];
    V3 vwo = large_step ? bs.wo : normalize(old * 0.9f + bs.wo * 0.1f);
    V3 val = v3s(0.f);
    float pdf = 0.f;
    if (mat) bsdf_eval_pdf(s.bsdf, *mat, si.uv, si.wi, vwo, &val, &pdf);  // :93
    if (pdf <= 0.f) vwo = bs.wo;  // :95
    if (pdf > 0.f) w = val / pdf;  // :96
    prop_v[depth] = vwo;  // :99
    ray = spawn_ray(si.p, si.n, to_world(si.sh, vwo));  // :101
    f = f * w;
    eta *= bs.eta;
    prev_bsdf_pdf = bs.pdf;
    if (si.valid) depth += 1;  // :121
    float fmax_ = hmax(f);
    float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
    bool rr_active = depth >= rr_depth;
    bool rr_continue = rng.next_1d() < rr_prob;
    if (rr_active) f = f * rcp(rr_prob);
    active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);
  }
  return L;
}

// --------------------------- pssmltpath.py:17-190 ---------------------------
// One proposal with NEE + MIS. Vertex = (local wo, emitter sample); both are
// mutated against the current path's vertex and written to the proposal.
V3 orc_pssmlt_path_sample(const SceneView &s, Pcg32 &rng, Ray ray, uint32_t max_depth, uint32_t rr_depth,
                          bool large_step, const V3 *path_v, const V2 *path_es, V3 *prop_v, V2 *prop_es) {
  V3 f = v3s(1.f), L = v3s(0.f);
  float eta = 1.f;
  uint32_t depth = 0;
  V3 prev_p = v3s(0.f);  // prev_si = zeros (:42)
  float prev_bsdf_pdf = 1.f;
  bool prev_bsdf_delta = true;
  bool active = true;
  while (active) {
    SurfaceInteraction si = intersect(s, ray);  // :67
    V3 rel = si.p - prev_p;                      // :71-82
    float dist = norm(rel);
    V3 ds_d = si.valid ? rel / dist : to_world(si.sh, si.wi) * -1.f;
    float em_pdf = prev_bsdf_delta ? 0.f : pdf_emitter_direction(s, si.emitter, ds_d, dist, si.sh.n);
    float mis_bsdf = mis_weight_b(prev_bsdf_pdf, em_pdf);
    V3 le = (prev_bsdf_pdf > 0.f) ? emitter_eval(s, si.emitter, si.wi) : v3s(0.f);
    L = fma3v(f, le * mis_bsdf, L);
    bool active_next = (depth + 1 < max_depth) && si.valid;  // :84
    float s1 = rng.next_1d();                                 // :99-101
    V2 s2 = rng.next_2d();
    BSDFSample bs{};
    V3 w = v3s(0.f);
    const mtx_material *mat = si.valid ? &s.materials[si.material] : nullptr;
    if (mat) w = bsdf_sample(s.bsdf, *mat, si.uv, si.wi, s1, s2, &bs);
    V2 um = rng.next_2d();  // :104 mutate(path[depth], wo, next_2d, large_step)
    V3 vwo;
    V2 es;
    if (large_step) {
      vwo = bs.wo;
      es = um;
    } else {  // :176-188
      vwo = normalize(path_v[depth] * 0.99f + bs.wo * 0.01f);
      V2 g = square_to_std_normal(um);
      es = V2{dr_clamp(g.x * 0.1f + path_es[depth].x, 0.f, 1.f), dr_clamp(g.y * 0.1f + path_es[depth].y, 0.f, 1.f)};
    }
    V3 val = v3s(0.f);
    float pdf = 0.f;
    if (mat) bsdf_eval_pdf(s.bsdf, *mat, si.uv, si.wi, vwo, &val, &pdf);  // :107
    if (pdf <= 0.f) vwo = bs.wo;                                          // :109
    if (pdf > 0.f) w = val / pdf;                                         // :110
    ray = spawn_ray(si.p, si.n, to_world(si.sh, vwo));                    // :114
    bool active_em = active_next && smooth(s, si);                        // :118
    if (active_em) {                                                      // :120-134
      DirectionSample ds{};
      V3 em_weight = sample_emitter_visible(s, si, es, &ds);
      V3 wo = to_local(si.sh, ds.d);
      V3 ev;
      float epdf;
      bsdf_eval_pdf(s.bsdf, *mat, si.uv, si.wi, wo, &ev, &epdf);
      float mi_em = mis_weight_b(ds.pdf, epdf);
      L = fma3v(f, ev * em_weight * mi_em, L);
    }
    prop_v[depth] = vwo;  // :138
    prop_es[depth] = es;
    f = f * w;
    eta *= bs.eta;
    prev_p = si.p;
    prev_bsdf_pdf = bs.pdf;
    prev_bsdf_delta = (bs.type & BF_DELTA) != 0;
    if (si.valid) depth += 1;  // :154
    float fmax_ = hmax(f);
    float rr_prob = fminf(fmax_ * sqr(eta), 0.95f);
    bool rr_active = depth >= rr_depth;
    bool rr_continue = rng.next_1d() < rr_prob;
    if (rr_active) f = f * rcp(rr_prob);
    active = active_next && (!rr_active || rr_continue) && (fmax_ != 0.f);
  }
  return L;
}

V3 run_integrator(const SceneView &s, const mtx_render_args &a, Pcg32 &rng, const Ray &ray, bool *valid,
                  float *query = nullptr) {
  switch (a.integrator) {
    case MTX_INT_PATH: return orc_path(s, rng, ray, a.max_depth, a.rr_depth, valid);
    case MTX_INT_NRC: return orc_nrc(s, rng, ray, a.max_depth, a.nrc_c, valid, (a.flags & 4u) ? query : nullptr);
    case MTX_INT_SIMPLE: return orc_simple(s, rng, ray, a.max_depth, a.rr_depth, valid);
    default: return orc_path_mis(s, rng, ray, a.max_depth, a.rr_depth, valid);
  }
}

}  // namespace

// ===========================================================================
// C entry points (ctypes)
// ===========================================================================
extern "C" {

int orc_trace(const mtx_scene_desc *d, uint64_t n, const float *rays, int any_hit, int brute, uint32_t *hits,
              uint32_t *visits) {
  SceneView s = make_view(d);
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const float *r = rays + 8 * i;
    V3 o{r[0], r[1], r[2]}, dd{r[4], r[5], r[6]};
    float maxt = r[3];
    uint32_t nv = 0, tv = 0;
    if (any_hit == 1) {
      hits[i] = trace_any(s, o, dd, maxt, &nv, &tv) ? 1u : 0u;
    } else {
      Hit h = brute ? brute_closest(s, o, dd, maxt) : trace_closest(s, o, dd, maxt, &nv, &tv);
      hits[4 * i + 0] = f2u(h.t);
      hits[4 * i + 1] = h.prim;
      hits[4 * i + 2] = f2u(h.u);
      hits[4 * i + 3] = f2u(h.v);
    }
    if (visits) {
      visits[2 * i] = nv;
      visits[2 * i + 1] = tv;
    }
  }
  return 0;
}

// orc_trace with the per-node visit histogram of nodes [0, hist_len) (tools/ diagnostic)
int orc_node_visit_hist(const mtx_scene_desc *d, uint64_t n, const float *rays, int any_hit, uint64_t *hist,
                        uint32_t hist_len) {
  std::vector<uint32_t> hits(any_hit ? n : 4 * n);
  g_hist = hist;
  g_hist_len = hist_len;
  const int rc = orc_trace(d, n, rays, any_hit, 0, hits.data(), nullptr);
  g_hist = nullptr;
  g_hist_len = 0;
  return rc;
}

// SamplingIntegrator.sample() for given rays (see mtx_sample_rays).
int orc_sample_rays(const mtx_scene_desc *d, const mtx_render_args *a, uint64_t n, const float *rays,
                    const uint32_t *lanes, uint32_t rng_skip, float *L, uint8_t *valid) {
  SceneView s = make_view(d);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    Pcg32 rng = sampler_lane(a->seed, lanes[i]);
    for (uint32_t k = 0; k < rng_skip; ++k) rng.next_u32();
    const float *r = rays + 6 * i;
    Ray ray{V3{r[0], r[1], r[2]}, V3{r[3], r[4], r[5]}, kLargest};
    bool v = false;
    V3 res = run_integrator(s, *a, rng, ray, &v);
    L[3 * i] = res.x;
    L[3 * i + 1] = res.y;
    L[3 * i + 2] = res.z;
    valid[i] = v ? 1 : 0;
  }
  return 0;
}

// Per-sample radiance for film rows [y0,y1): lane = (y*W + x)*spp_total +
// sample_offset + s; writes L (3 per sample) and the film position (2 per
// sample) in (pixel, s) order. Used by the per-lane parity tests.
// `query` (NULL, or 10 floats per sample): NRC radiance-cache queries, see
// orc_nrc; all zero for samples without one.
int orc_render_samples_q(const mtx_scene_desc *d, const mtx_render_args *a, float *L, float *pos, float *query) {
  SceneView s = make_view(d);
  const uint32_t W = s.camera.width, H = s.camera.height;
  const uint64_t npx = (uint64_t)(a->y1 - a->y0) * W;
  const uint32_t spp = a->spp;
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t p = 0; p < (int64_t)npx; ++p) {
    uint32_t y = a->y0 + (uint32_t)(p / W), x = (uint32_t)(p % W);
    for (uint32_t k = 0; k < spp; ++k) {
      uint32_t lane = (uint32_t)(((uint64_t)y * W + x) * a->spp_total + a->sample_offset + k);
      Pcg32 rng = sampler_lane(a->seed, lane);
      V2 u = rng.next_2d();  // path.py:45
      float sx = (float)x + u.x, sy = (float)y + u.y;
      V2 adj = V2{sx / (float)W, sy / (float)H};
      Ray ray = camera_ray(s.camera, adj);  // path.py:60-62
      bool v = false;
      uint64_t o = (uint64_t)p * spp + k;
      float qbuf[10];
      V3 res = run_integrator(s, *a, rng, ray, &v, qbuf);
      if (query)
        for (int j = 0; j < 10; ++j) query[10 * o + j] = (a->integrator == MTX_INT_NRC && (a->flags & 4u)) ? qbuf[j] : 0.f;
      L[3 * o] = res.x;
      L[3 * o + 1] = res.y;
      L[3 * o + 2] = res.z;
      pos[2 * o] = sx;
      pos[2 * o + 1] = sy;
    }
  }
  return 0;
}

int orc_render_samples(const mtx_scene_desc *d, const mtx_render_args *a, float *L, float *pos) {
  return orc_render_samples_q(d, a, L, pos, nullptr);
}

// Film accumulation in the fixed order documented in DESIGN.md ("Film"):
// the samples of a pixel fall into `nslots` partial slots by their global
// sample index g (film_slot: slot k holds g in [floor(k T / 8), floor((k+1)
// T / 8)) of spp_total = T samples when nslots = 8; one slot otherwise);
// per slot, stage 1 sums each source pixel's samples (g ascending) into its
// 3x3 tent footprint and stage 2 gathers the 9 neighbours (dy, dx
// ascending); the film is the fixed binary tree of the slot films
// (mtx_core/common.h film_tree8). A sample-range shard of the same render
// holds whole slots, so ranks combined by the same tree reproduce the
// one-device film bit for bit (N = 1, 2, 4, 8).
int orc_film_slots(uint32_t W, uint32_t y0, uint32_t y1, uint32_t spp, uint32_t spp_total, uint32_t sample_offset,
                   uint32_t nslots, const float *L, const float *pos, float *film) {
  const uint32_t rows = y1 - y0;
  const uint32_t NS = nslots == 8 ? 8u : 1u;
  std::vector<float> acc((size_t)NS * rows * W * 36, 0.f);
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < (int64_t)rows * W; ++p) {
    int x = (int)(p % W), y = (int)(y0 + p / W);
    for (uint32_t k = 0; k < spp; ++k) {
      const uint32_t slot = NS == 8 ? film_slot(sample_offset + k, spp_total) : 0u;
      float *a = &acc[36 * ((size_t)slot * rows * W + (size_t)p)];
      uint64_t o = (uint64_t)p * spp + k;
      float sx = pos[2 * o], sy = pos[2 * o + 1];
      float lr = L[3 * o], lg = L[3 * o + 1], lb = L[3 * o + 2];
      for (int dy = 0; dy < 3; ++dy) {
        float wy = fmaxf(0.f, 1.f - fabsf(sy - ((float)(y + dy - 1) + 0.5f)));
        for (int dx = 0; dx < 3; ++dx) {
          float wx = fmaxf(0.f, 1.f - fabsf(sx - ((float)(x + dx - 1) + 0.5f)));
          float w = wx * wy;
          float *c = a + 4 * (dy * 3 + dx);
          c[0] = c[0] + lr * w;
          c[1] = c[1] + lg * w;
          c[2] = c[2] + lb * w;
          c[3] = c[3] + w;
        }
      }
    }
  }
  const uint32_t FW = W + 2, FH = rows + 2;
#pragma omp parallel for schedule(static)
  for (int64_t q = 0; q < (int64_t)FW * FH; ++q) {
    int px = (int)(q % FW) - 1, py = (int)(y0 + q / FW) - 1;
    V4 sl[8];
    for (uint32_t k = 0; k < NS; ++k) {
      float r = 0.f, g = 0.f, b = 0.f, w = 0.f;
      for (int dy = 0; dy < 3; ++dy)
        for (int dx = 0; dx < 3; ++dx) {
          int sxp = px - dx + 1, syp = py - dy + 1;
          if (sxp < 0 || sxp >= (int)W || syp < (int)y0 || syp >= (int)y1) continue;
          const float *c = &acc[36 * ((size_t)k * rows * W + (size_t)(syp - y0) * W + sxp) + 4 * (dy * 3 + dx)];
          r = r + c[0];
          g = g + c[1];
          b = b + c[2];
          w = w + c[3];
        }
      sl[k] = V4{r, g, b, w};
    }
    const V4 f = NS == 8 ? film_tree8(sl) : sl[0];
    film[4 * q] = f.x;
    film[4 * q + 1] = f.y;
    film[4 * q + 2] = f.z;
    film[4 * q + 3] = f.w;
  }
  return 0;
}

int orc_film(uint32_t W, uint32_t y0, uint32_t y1, uint32_t spp, const float *L, const float *pos, float *film) {
  return orc_film_slots(W, y0, y1, spp, spp, 0, 1, L, pos, film);
}

int orc_render(const mtx_scene_desc *d, const mtx_render_args *a, float *film) {
  const uint32_t W = d->camera.width;
  const uint64_t ns = (uint64_t)(a->y1 - a->y0) * W * a->spp;
  std::vector<float> L(3 * ns), pos(2 * ns);
  orc_render_samples(d, a, L.data(), pos.data());
  return orc_film_slots(W, a->y0, a->y1, a->spp, a->spp_total, a->sample_offset, 8, L.data(), pos.data(), film);
}


// --------------------------- pssmlt.py:112-228 -----------------------------
// Pssmlt.render for film rows [y0,y1): chains lane = pixel*spp + s (pssmlt.py
// :188-193), `iterations` Metropolis steps (200 in the reference, :208) with a
// large step every 50 (:206-209) and aggregation when i % 50 > 40 (:210).
// Writes the tent film (fixed order: iteration, then pixel, then chain) and,
// if chain_out != NULL, the final chain state (Lc.xyz, cw, offset.xy).
int orc_pssmlt_render(const mtx_scene_desc *d, const mtx_render_args *a, uint32_t iterations, float *film,
                      float *chain_out) {
  SceneView s = make_view(d);
  const uint32_t W = s.camera.width, H = s.camera.height, spp = a->spp, D = a->max_depth;
  const uint32_t rows = a->y1 - a->y0;
  const uint64_t npx = (uint64_t)rows * W;
  std::vector<float> acc(npx * 36, 0.f);
  const float kSqrt01 = 0.31622776601683794f;
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t p = 0; p < (int64_t)npx; ++p) {
    const uint32_t y = a->y0 + (uint32_t)(p / W), x = (uint32_t)(p % W);
    std::vector<V3> path_v((size_t)spp * D, v3s(0.f)), prop_v((size_t)spp * D, v3s(0.f));
    const bool with_nee = a->integrator == MTX_INT_PSSMLT_PATH;  // pssmltpath.py
    std::vector<V2> path_es(with_nee ? (size_t)spp * D : 0, V2{0.f, 0.f}), prop_es(path_es);
    std::vector<Pcg32> rng(spp);
    std::vector<V2> off(spp, V2{0.5f, 0.5f});
    std::vector<V3> Lc(spp, v3s(0.f));
    std::vector<float> cw(spp, 0.f);
    // chains [sample_offset, sample_offset + spp) of the pixel's spp_total (a chain shard)
    const uint32_t spp_total = a->spp_total ? a->spp_total : spp;
    for (uint32_t k = 0; k < spp; ++k)
      rng[k] = sampler_lane(a->seed, (uint32_t)(((uint64_t)y * W + x) * spp_total + a->sample_offset + k));
    float *ac = &acc[36 * (size_t)p];
    for (uint32_t it = 0; it < iterations; ++it) {
      const bool large = it % 50 == 0, agg = it % 50 > 40;
      for (uint32_t k = 0; k < spp; ++k) {
        Pcg32 &r = rng[k];
        V2 u = r.next_2d();  // :126
        V2 po;
        if (large) {
          po = u;
        } else {  // mutate_offset (:245-255)
          V2 g = square_to_std_normal(u);
          po = V2{dr_clamp(g.x * kSqrt01 + off[k].x, 0.f, 1.f), dr_clamp(g.y * kSqrt01 + off[k].y, 0.f, 1.f)};
        }
        V2 sp = V2{((float)x + po.x) / (float)W, ((float)y + po.y) / (float)H};  // :128
        Ray ray = camera_ray(s.camera, sp);
        V3 Lp = with_nee ? orc_pssmlt_path_sample(s, r, ray, D, a->rr_depth, large, &path_v[(size_t)k * D],
                                                   &path_es[(size_t)k * D], &prop_v[(size_t)k * D],
                                                   &prop_es[(size_t)k * D])
                         : orc_pssmlt_sample(s, r, ray, D, a->rr_depth, large, &path_v[(size_t)k * D],
                                             &prop_v[(size_t)k * D]);
        float acc_a = dr_clamp(luminance(Lp) / luminance(Lc[k]), 0.f, 1.f);  // :137
        bool accept = r.next_1d() < acc_a;                                  // :138-140
        if (accept) cw[k] = acc_a; else cw[k] += 1.f - acc_a;               // :143-144
        if (accept) {
          off[k] = po;
          Lc[k] = Lp;
          for (uint32_t dd = 0; dd < D; ++dd) path_v[(size_t)k * D + dd] = prop_v[(size_t)k * D + dd];  // :155-158
          if (with_nee)
            for (uint32_t dd = 0; dd < D; ++dd) path_es[(size_t)k * D + dd] = prop_es[(size_t)k * D + dd];
        }
      }
      if (agg) {  // block.put(pos, L / cw) at the integer pixel position (:161-165)
        for (uint32_t k = 0; k < spp; ++k) {
          V3 res = Lc[k] / cw[k];
          for (int dy = 0; dy < 3; ++dy) {
            float wy = fmaxf(0.f, 1.f - fabsf((float)y - ((float)((int)y + dy - 1) + 0.5f)));
            for (int dx = 0; dx < 3; ++dx) {
              float wx = fmaxf(0.f, 1.f - fabsf((float)x - ((float)((int)x + dx - 1) + 0.5f)));
              float w = wx * wy;
              float *c = ac + 4 * (dy * 3 + dx);
              c[0] = c[0] + res.x * w;
              c[1] = c[1] + res.y * w;
              c[2] = c[2] + res.z * w;
              c[3] = c[3] + w;
            }
          }
        }
      }
    }
    if (chain_out)
      for (uint32_t k = 0; k < spp; ++k) {
        float *o = chain_out + 6 * ((size_t)p * spp + k);
        o[0] = Lc[k].x; o[1] = Lc[k].y; o[2] = Lc[k].z; o[3] = cw[k]; o[4] = off[k].x; o[5] = off[k].y;
      }
  }
  const uint32_t FW = W + 2, FH = rows + 2;
  for (int64_t q = 0; q < (int64_t)FW * FH; ++q) {
    int px = (int)(q % FW) - 1, py = (int)(a->y0 + q / FW) - 1;
    float r = 0.f, g = 0.f, b = 0.f, w = 0.f;
    for (int dy = 0; dy < 3; ++dy)
      for (int dx = 0; dx < 3; ++dx) {
        int sxp = px - dx + 1, syp = py - dy + 1;
        if (sxp < 0 || sxp >= (int)W || syp < (int)a->y0 || syp >= (int)a->y1) continue;
        const float *c = &acc[36 * ((size_t)(syp - a->y0) * W + sxp) + 4 * (dy * 3 + dx)];
        r = r + c[0]; g = g + c[1]; b = b + c[2]; w = w + c[3];
      }
    film[4 * q] = r; film[4 * q + 1] = g; film[4 * q + 2] = b; film[4 * q + 3] = w;
  }
  return 0;
}

}  // extern "C"

// ------------------------- restirgi.py:182-457 -----------------------------
// One RestirIntegrator.render() call (one frame) over the whole film, phase by
// phase exactly as the reference evaluates them: sample_initial (:412-457),
// temporal_resampling (:365-410), spatial_resampling (:274-363),
// render_final (:261-272) and block.put at the integer pixel (:236-242).
// Persistent state (float planes, layout in mtx_core/restir.h) is owned by
// the caller: cur (5 planes, written), prev (5 planes, read; ignored at frame
// 0 where prev_sample = sample), tres / sres (6 planes), radius (1 float).
namespace {

RSample rs_load(const float *b, size_t n, size_t i) {
  const float *p0 = b + 4 * i, *p1 = b + 4 * (n + i), *p2 = b + 4 * (2 * n + i), *p3 = b + 4 * (3 * n + i),
              *p4 = b + 4 * (4 * n + i);
  RSample s;
  s.x_v = V3{p0[0], p0[1], p0[2]};
  s.valid = p0[3] != 0.f;
  s.n_v = V3{p1[0], p1[1], p1[2]};
  s.p_q = p1[3];
  s.x_s = V3{p2[0], p2[1], p2[2]};
  s.n_s = V3{p3[0], p3[1], p3[2]};
  s.L_o = V3{p4[0], p4[1], p4[2]};
  return s;
}

void rs_store(float *b, size_t n, size_t i, const RSample &s) {
  float *p0 = b + 4 * i, *p1 = b + 4 * (n + i), *p2 = b + 4 * (2 * n + i), *p3 = b + 4 * (3 * n + i),
        *p4 = b + 4 * (4 * n + i);
  p0[0] = s.x_v.x; p0[1] = s.x_v.y; p0[2] = s.x_v.z; p0[3] = s.valid ? 1.f : 0.f;
  p1[0] = s.n_v.x; p1[1] = s.n_v.y; p1[2] = s.n_v.z; p1[3] = s.p_q;
  p2[0] = s.x_s.x; p2[1] = s.x_s.y; p2[2] = s.x_s.z; p2[3] = 0.f;
  p3[0] = s.n_s.x; p3[1] = s.n_s.y; p3[2] = s.n_s.z; p3[3] = 0.f;
  p4[0] = s.L_o.x; p4[1] = s.L_o.y; p4[2] = s.L_o.z; p4[3] = 0.f;
}

RReservoir rr_load(const float *b, size_t n, size_t i) {
  RReservoir r;
  r.z = rs_load(b, n, i);
  const float *p5 = b + 4 * (5 * n + i);
  r.w = p5[0];
  r.W = p5[1];
  memcpy(&r.M, &p5[2], 4);
  return r;
}

void rr_store(float *b, size_t n, size_t i, const RReservoir &r) {
  rs_store(b, n, i, r.z);
  float *p5 = b + 4 * (5 * n + i);
  p5[0] = r.w;
  p5[1] = r.W;
  memcpy(&p5[2], &r.M, 4);
  p5[3] = 0.f;
}

}  // namespace

extern "C" int orc_restir_frame(const mtx_scene_desc *d, const mtx_render_args *a, const mtx_camera *prev_cam,
                                float *cur, const float *prev, float *tres, float *sres, float *radius,
                                float *film) {
  SceneView s = make_view(d);
  const uint32_t W = s.camera.width, H = s.camera.height, spp = a->spp;
  const size_t n = (size_t)W * H * spp;
  const bool bias = a->restir_flags & MTX_RESTIR_BIAS_CORRECTION;
  const bool jac = a->restir_flags & MTX_RESTIR_JACOBIAN;
  const bool bsdf_sampling = a->restir_flags & MTX_RESTIR_BSDF_SAMPLING;
  const bool ss_reuse = a->restir_flags & MTX_RESTIR_SPATIAL_SPATIAL;
  if (a->frame == 0) {  // :217-226
    memset(tres, 0, sizeof(float) * 24 * n);
    memset(sres, 0, sizeof(float) * 24 * n);
    for (size_t i = 0; i < n; ++i) radius[i] = a->initial_search_radius;
    prev = cur;  // :230-231 prev_sample = sample (read after sample_initial)
  }
  std::vector<Pcg32> rng(n);
  std::vector<float> hitrec(4 * n), pdir(3 * n), emit(3 * n);

  // ---- sample_initial (:412-457)
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const uint32_t x = (uint32_t)(i / spp % W), y = (uint32_t)(i / W / spp);  // :206-208
    Pcg32 r = sampler_lane(a->seed, (uint32_t)i);
    const V2 u = r.next_2d();  // :211-213
    const V2 sp = V2{((float)x + u.x) / (float)W, ((float)y + u.y) / (float)H};
    const Ray ray = camera_ray(s.camera, sp);
    const Hit h = trace_closest(s, ray.o, ray.d, ray.maxt, nullptr, nullptr);
    const SurfaceInteraction si = compute_si(s, h.t, h.prim, h.u, h.v, ray.d);
    hitrec[4 * i] = h.t;
    memcpy(&hitrec[4 * i + 1], &h.prim, 4);
    hitrec[4 * i + 2] = h.u;
    hitrec[4 * i + 3] = h.v;
    pdir[3 * i] = ray.d.x; pdir[3 * i + 1] = ray.d.y; pdir[3 * i + 2] = ray.d.z;
    const V3 em = emitter_eval(s, si.emitter, si.wi);  // :421-423
    emit[3 * i] = em.x; emit[3 * i + 1] = em.y; emit[3 * i + 2] = em.z;
    RSample S = rsample_zero();
    S.valid = si.valid;
    if (si.valid) {
      S.x_v = si.p;
      S.n_v = si.n;
    }
    V3 wo;
    float pdf;
    if (bsdf_sampling) {  // :431-438
      const float s1 = r.next_1d();
      const V2 s2 = r.next_2d();
      BSDFSample bs;
      bs.wo = v3s(0.f);
      bs.pdf = 0.f;
      if (si.valid) bsdf_sample(s.bsdf, s.materials[si.material], si.uv, si.wi, s1, s2, &bs);
      wo = bs.wo;
      pdf = bs.pdf;
    } else {  // :440-444
      wo = square_to_uniform_hemisphere(r.next_2d());
      pdf = square_to_uniform_hemisphere_pdf(wo);
    }
    S.p_q = pdf;
    if (si.valid) {
      const Ray ray2 = spawn_ray(si.p, si.n, to_world(si.sh, wo));  // :448
      bool v = false;
      S.L_o = orc_path_mis(s, r, ray2, a->max_depth, a->rr_depth, &v);  // :450 (sample_ray :459-588)
      const SurfaceInteraction si2 = intersect(s, ray2);                // :452
      if (si2.valid) {
        S.x_s = si2.p;
        S.n_s = si2.n;
      }
    } else {
      // zero-direction ray from an invalid interaction: one missed iteration
      // of sample_ray (6 draws), radiance 0 (ReSTIR GI)
      for (int k = 0; k < 6; ++k) r.next_u32();
    }
    rs_store(cur, n, i, S);
    rng[i] = r;
  }

  // ---- temporal_resampling (:365-410)
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const uint32_t smp = (uint32_t)(i % spp);
    Pcg32 &r = rng[i];
    const RSample S = rs_load(cur, n, i);
    float ux = 0.f, uy = 0.f;
    bool valid = project_prev(*prev_cam, S.x_v, &ux, &uy);
    RSample Sprev = rsample_zero();
    if (valid) Sprev = rs_load(prev, n, pixel_index((int64_t)ux, (int64_t)uy, W, H, spp, smp));
    valid = valid && similar(S, Sprev);
    const RReservoir R = valid ? rr_load(tres, n, i) : rres_zero();
    RReservoir Rn = rres_zero();
    float phat = p_hat(S.L_o);
    const float w = S.p_q > 0.f ? phat / S.p_q : 0.f;
    res_update(Rn, S, w, true, r.next_1d());
    res_merge(Rn, R, p_hat(R.z.L_o), true, r.next_1d());
    phat = p_hat(Rn.z.L_o);
    Rn.W = (phat * (float)Rn.M > 0.f) ? Rn.w / ((float)Rn.M * phat) : 0.f;
    if (a->max_M_temporal) Rn.M = std::min(Rn.M, a->max_M_temporal);
    rr_store(tres, n, i, Rn);
  }

  // ---- spatial_resampling (:274-363)
  std::vector<float> result(3 * n), pos(2 * n);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const uint32_t smp = (uint32_t)(i % spp);
    const int64_t x = (int64_t)(i / spp % W), y = (int64_t)(i / W / spp);
    Pcg32 &r = rng[i];
    const RReservoir Rs = rr_load(sres, n, i);
    RReservoir Rn = rres_zero();
    const RSample q = rs_load(cur, n, i);
    uint32_t Z = 0;
    if (ss_reuse) {
      res_merge(Rn, Rs, p_hat(Rs.z.L_o), true, r.next_1d());
      Z += Rs.M;
    }
    const int max_iter = (a->max_M_spatial == 0 || (double)Rs.M < a->max_M_spatial / 2.0) ? 9 : 3;
    bool any_reused = false;
    uint32_t qM[9];
    V3 qp[9];
    bool qa[9];
    const float rad = radius[i];
    for (int k = 0; k < 9; ++k) {
      bool active = k < max_iter;
      const V2 d2 = square_to_uniform_disk(r.next_2d());
      const V2 off = V2{d2.x * rad, d2.y * rad};
      const uint32_t idx = pixel_index(x + (int32_t)off.x, y + (int32_t)off.y, W, H, spp, smp);
      const RSample qn = rs_load(cur, n, idx);
      active = active && similar(qn, q);
      const RReservoir Rk = active ? rr_load(tres, n, idx) : rres_zero();
      bool shadowed = false;
      if (active) {
        const Ray sr = spawn_ray_to(q.x_v, q.n_v, Rk.z.x_s);
        shadowed = trace_any(s, sr.o, sr.d, sr.maxt, nullptr, nullptr);
      }
      const float jf = jac ? dr_clampf(jacobian_J(q.x_v, Rk), 0.f, 1000.f) : 1.0f;
      const float phat = (!active || shadowed) ? 0.f : p_hat(Rk.z.L_o) * jf;
      res_merge(Rn, Rk, phat, active, r.next_1d());
      qM[k] = Rk.M;
      qp[k] = Rk.z.x_v;
      qa[k] = active;
      any_reused = any_reused || active;
    }
    const float phat = p_hat(Rn.z.L_o);
    if (bias) {
      for (int k = 0; k < 9; ++k) {
        bool active = qa[k];
        if (active) {
          const Ray br = spawn_ray_to(Rn.z.x_s, Rn.z.n_s, qp[k]);
          active = !trace_any(s, br.o, br.d, br.maxt, nullptr, nullptr);
        }
        Z += active ? qM[k] : 0u;
      }
      Rn.W = ((float)Z * phat > 0.f) ? Rn.w / ((float)Z * phat) : 0.f;
    } else {
      Rn.W = (phat * (float)Rn.M > 0.f) ? Rn.w / ((float)Rn.M * phat) : 0.f;
    }
    radius[i] = fmaxf(any_reused ? rad : rad / 2.f, a->minimal_search_radius);
    if (a->max_M_spatial) Rn.M = std::min(Rn.M, a->max_M_spatial);
    rr_store(sres, n, i, Rn);

    // ---- render_final (:261-272)
    uint32_t prim;
    memcpy(&prim, &hitrec[4 * i + 1], 4);
    const SurfaceInteraction si =
        compute_si(s, hitrec[4 * i], prim, hitrec[4 * i + 2], hitrec[4 * i + 3],
                   V3{pdir[3 * i], pdir[3 * i + 1], pdir[3 * i + 2]});
    V3 beta = v3s(0.f);
    if (si.valid) {
      float pdf_unused;
      const V3 wo = to_local(si.sh, normalize(Rn.z.x_s - si.p));
      bsdf_eval_pdf(s.bsdf, s.materials[si.material], si.uv, si.wi, wo, &beta, &pdf_unused);
    }
    const V3 res = beta * Rn.z.L_o * Rn.W + V3{emit[3 * i], emit[3 * i + 1], emit[3 * i + 2]};
    result[3 * i] = res.x; result[3 * i + 1] = res.y; result[3 * i + 2] = res.z;
    pos[2 * i] = (float)x;
    pos[2 * i + 1] = (float)y;
  }
  return orc_film(W, 0, H, spp, result.data(), pos.data(), film);
}

extern "C" {

// ------------------------- nerad.py:86-106 features -------------------------
// The radiance-field encoder restated in mtx_core/field.h (shared with the
// device), driven from a mtx_field_desc as mtx_field_upload does.
int orc_field_features(const mtx_field_desc *f, uint64_t n, const float *p, const float *wi, uint16_t *out) {
  FieldEncoding e{};
  e.table = f->table;
  e.n_levels = f->n_levels;
  e.n_features = f->n_features;
  e.log2_table = f->log2_table;
  for (uint32_t l = 0; l < f->n_levels; ++l) {
    const double scale = exp2((double)l * log2((double)f->per_level_scale)) * f->base_res - 1.0;
    e.level_scale[l] = (float)scale;
    e.level_res[l] = (uint32_t)ceil((double)(float)scale) + 1u;
  }
  for (int k = 0; k < 3; ++k) {
    e.bbox_min[k] = f->bbox_min[k];
    e.bbox_max[k] = f->bbox_max[k];
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i)
    field_features(e, V3{p[3 * i], p[3 * i + 1], p[3 * i + 2]}, V3{wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]},
                   out + 64 * i, 64);
  return 0;
}

// ------------------------------- RNG KATs ----------------------------------
int orc_rng_stream(uint32_t seed, uint32_t lane0, uint32_t n_lanes, uint32_t n_draws, float *out) {
  for (uint32_t l = 0; l < n_lanes; ++l) {
    Pcg32 r = sampler_lane(seed, lane0 + l);
    for (uint32_t k = 0; k < n_draws; ++k) out[(size_t)l * n_draws + k] = r.next_1d();
  }
  return 0;
}

// --------------------------- prefix_sum.py:9-36 ----------------------------
// Hillis-Steele: for i in 0..floor(log2 n): x[j] = x[j] + x[j - 2^i], j >= 2^i,
// with copy-on-write (gather all, then scatter).
int orc_prefix_sum_f32_hs(const float *in, float *out, uint64_t n) {
  std::vector<float> x(in, in + n), y(n);
  if (n == 0) return 0;
  int passes = 0;
  while ((1ull << (passes + 1)) <= n) ++passes;  // floor(log2 n)
  for (int i = 0; i <= passes; ++i) {
    uint64_t st = 1ull << i;
    if (st >= n) break;
    y = x;
    for (uint64_t j = st; j < n; ++j) y[j] = x[j] + x[j - st];
    x.swap(y);
  }
  memcpy(out, x.data(), n * sizeof(float));
  return 0;
}

int orc_prefix_sum_u32(const uint32_t *in, uint32_t *out, uint64_t n, int inclusive) {
  uint32_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t v = in[i];
    if (inclusive) {
      acc += v;
      out[i] = acc;
    } else {
      out[i] = acc;
      acc += v;
    }
  }
  return 0;
}

// ------------------------------ hashgrid.py --------------------------------
// hash (:8-12) on u32 with wraparound; bbmin/bbmax are scalars over all three
// axes (:33-41); cell_offset is the exclusive scan of cell_size (:65-76);
// within a cell, sample indices are listed in ascending order (the reference
// order is race-defined, :53).
int orc_hashgrid(const float *p, uint64_t n, uint32_t res, uint32_t n_cells, uint32_t *cell, uint32_t *cell_size,
                 uint32_t *cell_offset, uint32_t *sample_idx) {
  const float *px = p, *py = p + n, *pz = p + 2 * n;
  float bbmin = INFINITY, bbmax = -INFINITY;
  for (uint64_t i = 0; i < n; ++i) {
    bbmin = fminf(bbmin, fminf(px[i], fminf(py[i], pz[i])));
    bbmax = fmaxf(bbmax, fmaxf(px[i], fmaxf(py[i], pz[i])));
  }
  float ext = bbmax - bbmin, fres = (float)res;
  for (uint32_t c = 0; c < n_cells; ++c) cell_size[c] = 0;
  std::vector<uint32_t> rank(n);
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t x = (uint32_t)((px[i] - bbmin) / ext * fres);
    uint32_t y = (uint32_t)((py[i] - bbmin) / ext * fres);
    uint32_t z = (uint32_t)((pz[i] - bbmin) / ext * fres);
    uint32_t h = ((x * 73856093u) ^ (y * 19349663u) ^ (z * 83492791u)) % n_cells;
    cell[i] = h;
    rank[i] = cell_size[h]++;
  }
  uint32_t acc = 0;
  for (uint32_t c = 0; c < n_cells; ++c) {
    cell_offset[c] = acc;
    acc += cell_size[c];
  }
  for (uint64_t i = 0; i < n; ++i) sample_idx[cell_offset[cell[i]] + rank[i]] = (uint32_t)i;
  return 0;
}

// ------------------- multi-core CPU baselines (OpenMP) ----------------------
// The same results as the sequential restatements above (tested equal),
// computed with every host thread: bench.py's cpu_baseline leg times these
// for the primitive lines (all host cores). Not used as checkers.

// u32 scan: per-thread chunk sums, exclusive scan of the chunk sums, local pass.
int orc_prefix_sum_u32_mt(const uint32_t *in, uint32_t *out, uint64_t n, int inclusive) {
  const int T = omp_get_max_threads();
  std::vector<uint32_t> part(T + 1, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
    uint32_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += in[i];
    part[t + 1] = s;
#pragma omp barrier
#pragma omp single
    for (int k = 0; k < T; ++k) part[k + 1] += part[k];
    uint32_t acc = part[t];
    for (uint64_t i = lo; i < hi; ++i) {
      const uint32_t v = in[i];
      if (inclusive) {
        acc += v;
        out[i] = acc;
      } else {
        out[i] = acc;
        acc += v;
      }
    }
  }
  return 0;
}

// Hillis-Steele passes in the reference's order, each pass over all threads.
int orc_prefix_sum_f32_hs_mt(const float *in, float *out, uint64_t n) {
  std::vector<float> x(in, in + n), y(n);
  for (uint64_t st = 1; st < n; st <<= 1) {
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < (int64_t)n; ++j) y[j] = (uint64_t)j >= st ? x[j] + x[j - st] : x[j];
    x.swap(y);
  }
  if (n) memcpy(out, x.data(), n * sizeof(float));
  return 0;
}

// Hash grid: bbox (parallel reduction), cells in parallel, then a parallel
// sort of (cell, index) pairs (libstdc++ parallel mode) = ascending index
// within a cell, and the run bounds in parallel.
int orc_hashgrid_mt(const float *p, uint64_t n, uint32_t res, uint32_t n_cells, uint32_t *cell, uint32_t *cell_size,
                    uint32_t *cell_offset, uint32_t *sample_idx) {
  const float *px = p, *py = p + n, *pz = p + 2 * n;
  float bbmin = INFINITY, bbmax = -INFINITY;
#pragma omp parallel for reduction(min : bbmin) reduction(max : bbmax)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    bbmin = fminf(bbmin, fminf(px[i], fminf(py[i], pz[i])));
    bbmax = fmaxf(bbmax, fmaxf(px[i], fmaxf(py[i], pz[i])));
  }
  const float ext = bbmax - bbmin, fres = (float)res;
  std::vector<uint64_t> key(n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const uint32_t x = (uint32_t)((px[i] - bbmin) / ext * fres);
    const uint32_t y = (uint32_t)((py[i] - bbmin) / ext * fres);
    const uint32_t z = (uint32_t)((pz[i] - bbmin) / ext * fres);
    const uint32_t h = ((x * 73856093u) ^ (y * 19349663u) ^ (z * 83492791u)) % n_cells;
    cell[i] = h;
    key[i] = ((uint64_t)h << 32) | (uint64_t)i;
  }
  __gnu_parallel::sort(key.begin(), key.end());
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < (int64_t)n_cells; ++c) cell_size[c] = 0;
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < (int64_t)n; ++k) {
    const uint32_t c = (uint32_t)(key[k] >> 32);
    sample_idx[k] = (uint32_t)key[k];
    if (k == 0 || (uint32_t)(key[k - 1] >> 32) != c) cell_offset[c] = (uint32_t)k;  // run start
  }
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < (int64_t)n; ++k) {
    const uint32_t c = (uint32_t)(key[k] >> 32);
    if (k + 1 == (int64_t)n || (uint32_t)(key[k + 1] >> 32) != c) cell_size[c] = (uint32_t)(k + 1) - cell_offset[c];
  }
  // empty cells: offset = start of the next non-empty run (exclusive scan)
  uint32_t next = (uint32_t)n;
  for (int64_t c = (int64_t)n_cells - 1; c >= 0; --c) {
    if (cell_size[c]) next = cell_offset[c];
    else cell_offset[c] = next;
  }
  return 0;
}

// Scatter-reduce: parallel sort of (target, index) pairs, then every target
// folds its values in ascending index order (targets in parallel).
int orc_scatter_reduce_f32_mt(int op, float *target, uint64_t n_target, const float *value, const uint32_t *index,
                              uint64_t n_value) {
  std::vector<uint64_t> key(n_value);
  for (uint64_t i = 0; i < n_value; ++i)
    if (index[i] >= n_target) return -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n_value; ++i) key[i] = ((uint64_t)index[i] << 32) | (uint64_t)i;
  __gnu_parallel::sort(key.begin(), key.end());
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < (int64_t)n_value; ++k) {
    const uint32_t t = (uint32_t)(key[k] >> 32);
    if (k > 0 && (uint32_t)(key[k - 1] >> 32) == t) continue;  // not the run start
    float a = target[t];
    for (int64_t j = k; j < (int64_t)n_value && (uint32_t)(key[j] >> 32) == t; ++j) {
      const float b = value[(uint32_t)key[j]];
      a = op == 0 ? a + b : (op == 1 ? fminf(a, b) : (op == 2 ? fmaxf(a, b) : a * b));
    }
    target[t] = a;
  }
  return 0;
}

// ----------------------------- reductions.py -------------------------------
// Every target index receives func(target, value) for each of its values,
// applied in ascending value-index order. func: 0 add, 1 min, 2 max, 3 mul.
int orc_scatter_reduce_f32(int op, float *target, uint64_t n_target, const float *value, const uint32_t *index,
                           uint64_t n_value) {
  for (uint64_t i = 0; i < n_value; ++i) {
    uint32_t t = index[i];
    if (t >= n_target) return -1;
    float a = target[t], b = value[i];
    target[t] = op == 0 ? a + b : (op == 1 ? fminf(a, b) : (op == 2 ? fmaxf(a, b) : a * b));
  }
  return 0;
}

}  // extern "C"

// --------------------- per-lane primitive probes (tests) -------------------
extern "C" {

// op: 0 sin, 1 cos, 2 log, 3 exp, 4 erf, 5 erfinv
int orc_dmath(int op, const float *x, float *out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    float s, c;
    switch (op) {
      case 0: dsincos(x[i], &s, &c); out[i] = s; break;
      case 1: dsincos(x[i], &s, &c); out[i] = c; break;
      case 2: out[i] = dlog(x[i]); break;
      case 3: out[i] = dexp(x[i]); break;
      case 4: out[i] = derf(x[i]); break;
      case 5: out[i] = derfinv(x[i]); break;
      default: return -1;
    }
  }
  return 0;
}

// BSDF probe for material `mat` of a scene: for each i, with local wi[i],
// wo[i], uv[i] and samples u[i] = (u1, u2x, u2y):
//   out[16 i + 0..2]  eval value at wo, [3] eval pdf at wo
//   out[16 i + 4..6]  sampled wo, [7] sample pdf, [8] eta, [9] type (bits)
//   out[16 i + 10..12] sample weight, [13..15] eval value at the sampled wo
//   out2[i]           eval pdf at the sampled wo
int orc_bsdf_probe(const mtx_scene_desc *d, uint32_t mat, uint64_t n, const float *wi, const float *wo,
                   const float *uv, const float *u, float *out, float *out2) {
  SceneView s = make_view(d);
  if (mat >= d->n_materials) return -1;
  const mtx_material &m = s.materials[mat];
  for (uint64_t i = 0; i < n; ++i) {
    V3 a{wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]}, b{wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]};
    V2 t{uv[2 * i], uv[2 * i + 1]};
    V3 val;
    float pdf;
    bsdf_eval_pdf(s.bsdf, m, t, a, b, &val, &pdf);
    BSDFSample bs;
    V3 w = bsdf_sample(s.bsdf, m, t, a, u[3 * i], V2{u[3 * i + 1], u[3 * i + 2]}, &bs);
    V3 val2;
    float pdf2;
    bsdf_eval_pdf(s.bsdf, m, t, a, bs.wo, &val2, &pdf2);
    float *o = out + 16 * i;
    o[0] = val.x; o[1] = val.y; o[2] = val.z; o[3] = pdf;
    o[4] = bs.wo.x; o[5] = bs.wo.y; o[6] = bs.wo.z; o[7] = bs.pdf; o[8] = bs.eta; o[9] = u2f(bs.type);
    o[10] = w.x; o[11] = w.y; o[12] = w.z;
    o[13] = val2.x; o[14] = val2.y; o[15] = val2.z;
    out2[i] = pdf2;
  }
  return 0;
}

// Probes of the shared sensor / ray-spawn / emitter primitives (mtx_core/
// interaction.h) for the independent numpy pins of tests/test_core_pins.py.
// 16 floats in, 16 floats out per item:
//   op 0 camera_ray(in[0..1])                    -> o[0..2], d[3..5], maxt[6]
//   op 1 spawn_ray(p=in[0..2], n=in[3..5], d=in[6..8])    -> o, d, maxt
//   op 2 spawn_ray_to(p=in[0..2], n=in[3..5], t=in[6..8]) -> o, d, maxt
//   op 3 sample_emitter_direction(ref=in[0..2], u=in[3..4])
//        -> weight[0..2], p[3..5], n[6..8], d[9..11], dist[12], pdf[13], emitter[14]
//   op 4 pdf_emitter_direction(emitter=in[0], d=in[1..3], dist=in[4], n=in[5..7]) -> pdf[0];
//        emitter_eval(emitter, wi_local=in[8..10]) -> [1..3]
int orc_probe(const mtx_scene_desc *d, int op, uint64_t n, const float *in, float *out) {
  SceneView s = make_view(d);
  for (uint64_t i = 0; i < n; ++i) {
    const float *a = in + 16 * i;
    float *o = out + 16 * i;
    for (int k = 0; k < 16; ++k) o[k] = 0.f;
    V3 x{a[0], a[1], a[2]}, y{a[3], a[4], a[5]}, z{a[6], a[7], a[8]};
    Ray r{};
    switch (op) {
      case 0: r = camera_ray(s.camera, V2{a[0], a[1]}); break;
      case 1: r = spawn_ray(x, y, z); break;
      case 2: r = spawn_ray_to(x, y, z); break;
      case 3: {
        DirectionSample ds{};
        V3 w = sample_emitter_direction(s, x, V2{a[3], a[4]}, &ds);
        o[0] = w.x; o[1] = w.y; o[2] = w.z;
        o[3] = ds.p.x; o[4] = ds.p.y; o[5] = ds.p.z;
        o[6] = ds.n.x; o[7] = ds.n.y; o[8] = ds.n.z;
        o[9] = ds.d.x; o[10] = ds.d.y; o[11] = ds.d.z;
        o[12] = ds.dist; o[13] = ds.pdf; o[14] = (float)ds.emitter;
        continue;
      }
      case 4: {
        const int32_t e = (int32_t)a[0];
        o[0] = pdf_emitter_direction(s, e, V3{a[1], a[2], a[3]}, a[4], V3{a[5], a[6], a[7]});
        V3 le = emitter_eval(s, e, V3{a[8], a[9], a[10]});
        o[1] = le.x; o[2] = le.y; o[3] = le.z;
        continue;
      }
      default: return -1;
    }
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z;
    o[6] = r.maxt;
  }
  return 0;
}

// ReSTIR GI reservoir primitives of mtx_core/restir.h item by item, for the
// float64 transcription of restirgi.py in tests/test_restir_pins.py. 16
// floats in / out per item (u32 counts and pixel coordinates as exact
// floats):
//   op 0 p_hat(f = in[0..2]) -> out[0]                       (:84-85)
//   op 1 similar(x_v, n_v of a = in[0..5], of b = in[6..11]) -> out[0] 0 / 1  (:175-180)
//   op 2 res_update(w = in[0], M = in[1], wnew = in[2], active = in[3], u = in[4])
//        -> out w, M, taken                                   (:120-134)
//   op 3 res_merge_w(w = in[0], M = in[1], o.W = in[2], o.M = in[3], p = in[4],
//        active = in[5], u = in[6]) -> out w, M, taken         (:136-141)
//   op 4 jacobian_J(receiver = in[0..2], z.x_s = in[3..5], z.n_s = in[6..8],
//        z.x_v = in[9..11]) -> out[0]                          (:42-53)
//   op 5 pixel_index(x = in[0], y = in[1], W, H, spp, smp = in[2..5]) -> out[0]  (:170-173)
int orc_restir_probe(int op, uint64_t n, const float *in, float *out) {
  for (uint64_t i = 0; i < n; ++i) {
    const float *a = in + 16 * i;
    float *o = out + 16 * i;
    for (int k = 0; k < 16; ++k) o[k] = 0.f;
    auto v3 = [&](int k) { return V3{a[k], a[k + 1], a[k + 2]}; };
    switch (op) {
      case 0: o[0] = p_hat(v3(0)); break;
      case 1: {
        RSample x = rsample_zero(), y = rsample_zero();
        x.x_v = v3(0);
        x.n_v = v3(3);
        y.x_v = v3(6);
        y.n_v = v3(9);
        o[0] = similar(x, y) ? 1.f : 0.f;
        break;
      }
      case 2: {
        RReservoir r = rres_zero();
        r.w = a[0];
        r.M = (uint32_t)a[1];
        RSample s = rsample_zero();
        s.valid = true;
        res_update(r, s, a[2], a[3] != 0.f, a[4]);
        o[0] = r.w;
        o[1] = (float)r.M;
        o[2] = r.z.valid ? 1.f : 0.f;
        break;
      }
      case 3: {
        RReservoir r = rres_zero();
        r.w = a[0];
        r.M = (uint32_t)a[1];
        const bool taken = res_merge_w(r, a[2], (uint32_t)a[3], a[4], a[5] != 0.f, a[6]);
        o[0] = r.w;
        o[1] = (float)r.M;
        o[2] = taken ? 1.f : 0.f;
        break;
      }
      case 4: {
        RReservoir nb = rres_zero();
        nb.z.x_s = v3(3);
        nb.z.n_s = v3(6);
        nb.z.x_v = v3(9);
        o[0] = jacobian_J(v3(0), nb);
        break;
      }
      case 5:
        o[0] = (float)pixel_index((int64_t)a[0], (int64_t)a[1], (uint32_t)a[2], (uint32_t)a[3], (uint32_t)a[4],
                                  (uint32_t)a[5]);
        break;
      default: return -1;
    }
  }
  return 0;
}

// Surface interaction from explicit vertex data (mtx_core/interaction.h
// si_from_vertices, the arithmetic compute_si and the device's shading
// records share) for the float64 pins of tests/test_shared_pins.py.
// 40 floats in per item: t u v | ray_d[3] | p0 p1 p2 [9] | use_n | n0 n1 n2 [9] |
// use_uv | uv0 uv1 uv2 [6] | pad. 24 floats out: p[3] n[3] s[3] t[3] ns[3] uv[2] wi[3] pad.
int orc_si_probe(uint64_t n, const float *in, float *out) {
  for (uint64_t i = 0; i < n; ++i) {
    const float *a = in + 40 * i;
    float *o = out + 24 * i;
    auto v3 = [&](int k) { return V3{a[k], a[k + 1], a[k + 2]}; };
    const SurfaceInteraction si =
        si_from_vertices(a[0], 0u, a[1], a[2], v3(3), v3(6), v3(9), v3(12), 0u, -1, a[15] != 0.f, v3(16), v3(19),
                         v3(22), a[25] != 0.f, V2{a[26], a[27]}, V2{a[28], a[29]}, V2{a[30], a[31]});
    const V3 q[6] = {si.p, si.n, si.sh.s, si.sh.t, si.sh.n, V3{si.uv.x, si.uv.y, 0.f}};
    for (int k = 0; k < 6; ++k) {
      o[3 * k] = q[k].x;
      o[3 * k + 1] = q[k].y;
      o[3 * k + 2] = q[k].z;
    }
    o[17] = si.wi.x;
    o[18] = si.wi.y;
    o[19] = si.wi.z;
  }
  return 0;
}

// Bitmap lookups (mtx_core/bsdf.h texture_eval) of texture `tex` of a scene
// at n uv pairs; 3 floats out per item.
int orc_tex_probe(const mtx_scene_desc *d, uint32_t tex, uint64_t n, const float *uv, float *out) {
  SceneView s = make_view(d);
  if (tex >= d->n_textures) return -1;
  for (uint64_t i = 0; i < n; ++i) {
    const V3 c = texture_eval(s.bsdf, (int32_t)tex, V2{uv[2 * i], uv[2 * i + 1]});
    out[3 * i] = c.x;
    out[3 * i + 1] = c.y;
    out[3 * i + 2] = c.z;
  }
  return 0;
}

// Warps used by the integrators (upstream mitsuba/core/warp.h).
// op: 0 cosine hemisphere (3), 1 uniform disk concentric (2), 2 uniform
// disk (2), 3 std normal (2), 4 uniform hemisphere (3)
int orc_warp(int op, const float *u, float *out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    V2 s{u[2 * i], u[2 * i + 1]};
    float *o = out + 3 * i;
    V3 v{0, 0, 0};
    V2 p{0, 0};
    switch (op) {
      case 0: v = square_to_cosine_hemisphere(s); break;
      case 1: p = square_to_uniform_disk_concentric(s); v = V3{p.x, p.y, 0}; break;
      case 2: p = square_to_uniform_disk(s); v = V3{p.x, p.y, 0}; break;
      case 3: p = square_to_std_normal(s); v = V3{p.x, p.y, 0}; break;
      case 4: v = square_to_uniform_hemisphere(s); break;
      default: return -1;
    }
    o[0] = v.x; o[1] = v.y; o[2] = v.z;
  }
  return 0;
}

}  // extern "C"

namespace {

// ------------------------ nerad.py:118-310 (training samples) ----------------
struct NeradHost {
  std::vector<DiscreteDist> dists;
  NeradTables t;
};

NeradHost nerad_tables(const mtx_nerad_tables *h) {
  NeradHost r;
  r.dists.resize(h->n_shapes);
  for (uint32_t k = 0; k < h->n_shapes; ++k) {
    const uint32_t off = h->tri_off[k];
    r.dists[k] = DiscreteDist{h->tri_pmf + off, h->tri_cdf + off, h->tri_off[k + 1] - off, h->tri_valid[2 * k],
                              h->tri_valid[2 * k + 1], h->tri_sum[k], h->tri_norm[k]};
  }
  r.t.shape = DiscreteDist{h->shape_pmf, h->shape_cdf, h->n_shapes, h->shape_valid[0], h->shape_valid[1],
                           h->shape_sum, h->shape_norm};
  r.t.tri_dist = r.dists.data();
  r.t.tri_off = h->tri_off;
  r.t.tri_prim = h->tri_prim;
  return r;
}

// IntersectionSampler.sample (:291-310) of point i: the surface interaction
// of the sampled (triangle, barycentrics), seen along -wi_world.
SurfaceInteraction nerad_point(const SceneView &s, const NeradTables &t, uint32_t seed, uint32_t i, V3 *wi_world,
                               SurfaceSample *ss) {
  Pcg32 rng = sampler_lane(seed, i);
  *ss = nerad_surface_sample(t, s.shapes, s.materials, rng);
  const SurfaceInteraction f = compute_si(s, 1.f, ss->prim, ss->b1, ss->b2, V3{0.f, 0.f, 1.f});
  *wi_world = to_world(f.sh, ss->wi_local);
  return compute_si(s, 1.f, ss->prim, ss->b1, ss->b2, *wi_world * -1.f);
}

// bsdf.sample on si (null BSDF for an invalid interaction)
V3 sample_or_null(const SceneView &s, const SurfaceInteraction &si, float u1, V2 u2, BSDFSample *bs) {
  if (!si.valid) {
    bs->wo = v3s(0.f);
    bs->pdf = 0.f;
    bs->eta = 0.f;
    bs->type = 0;
    return v3s(0.f);
  }
  return bsdf_sample(s.bsdf, s.materials[si.material], si.uv, si.wi, u1, u2, bs);
}

// Integrator.sample_rhs (:174-233) for one lane, without the field term:
// L_nee (:197-200), the path weight f of the stop vertex (zero if invalid,
// :214-219), its emission Le and its field query (p, si.to_world(si.wi)).
// The caller forms L = L_nee + f * (Le + Field(query)) (:226-229).
void orc_nerad_lane(const SceneView &s, const SurfaceInteraction &si, Pcg32 &rng, float *o) {
  V3 L = v3s(0.f);
  DirectionSample ds{};
  const V3 em = sample_emitter_visible(s, si, rng.next_2d(), &ds);  // :197
  const mtx_material &m = s.materials[si.material];
  V3 val;
  float pdf;
  bsdf_eval_pdf(s.bsdf, m, si.uv, si.wi, to_local(si.sh, ds.d), &val, &pdf);  // :198
  L = L + val * mis_weight_b(ds.pdf, pdf) * em;                              // :200
  const float u1 = rng.next_1d();
  const V2 u2 = rng.next_2d();
  BSDFSample bs;
  const V3 w = bsdf_sample(s.bsdf, m, si.uv, si.wi, u1, u2, &bs);  // :204-206
  SurfaceInteraction si2 = intersect(s, spawn_ray(si.p, si.n, to_world(si.sh, bs.wo)));  // :208-209
  bool active = si2.valid;
  const V3 rel = si2.p - si.p;
  const float dist = norm(rel);
  const float em_pdf = pdf_emitter_direction(s, si2.emitter, rel / dist, dist, si2.sh.n);  // :213-216
  V3 f = w * mis_weight_b(bs.pdf, em_pdf);                                                // :217
  // next_smooth_si (:124-164)
  V3 f2 = v3s(1.f);
  float t1 = rng.next_1d();
  V2 t2 = rng.next_2d();
  BSDFSample b2;
  V3 w2 = sample_or_null(s, si2, t1, t2, &b2);
  bool chain = (b2.type & BF_DELTA) != 0;
  uint32_t depth = 0;
  while (chain) {
    f2 = f2 * w2;
    si2 = intersect(s, spawn_ray(si2.p, si2.n, to_world(si2.sh, b2.wo)));
    t1 = rng.next_1d();
    t2 = rng.next_2d();
    w2 = sample_or_null(s, si2, t1, t2, &b2);
    depth += 1;
    chain = (b2.type & BF_DELTA) != 0 && depth < 10;
  }
  active = active && si2.valid;  // :217
  f = f * f2;                    // :218
  if (!active) f = f * 0.f;      // :219
  const V3 le = emitter_eval(s, si2.emitter, si2.wi);
  const V3 wi = to_world(si2.sh, si2.wi);
  const float vals[16] = {L.x, L.y, L.z, f.x, f.y, f.z, le.x, le.y, le.z, si2.valid ? 1.f : 0.f,
                          si2.p.x, si2.p.y, si2.p.z, wi.x, wi.y, wi.z};
  for (int k = 0; k < 16; ++k) o[k] = vals[k];
}

// Integrator.sample (nerad.py:235-254) for one camera lane, without the
// field term: next_smooth_si from the first hit, f (zero if invalid, :250),
// Le and the field query; the caller forms L = Field * f + Le (:251-252).
void orc_nerad_render_lane(const SceneView &s, Pcg32 &rng, const Ray &ray, float *o) {
  SurfaceInteraction si = intersect(s, ray);  // :247
  V3 f = v3s(1.f);
  float t1 = rng.next_1d();
  V2 t2 = rng.next_2d();
  BSDFSample bs;
  V3 w = sample_or_null(s, si, t1, t2, &bs);
  bool chain = (bs.type & BF_DELTA) != 0;
  uint32_t depth = 0;
  while (chain) {
    f = f * w;
    si = intersect(s, spawn_ray(si.p, si.n, to_world(si.sh, bs.wo)));
    t1 = rng.next_1d();
    t2 = rng.next_2d();
    w = sample_or_null(s, si, t1, t2, &bs);
    depth += 1;
    chain = (bs.type & BF_DELTA) != 0 && depth < 10;
  }
  f = f * (si.valid ? 1.f : 0.f);
  const V3 le = emitter_eval(s, si.emitter, si.wi);
  const V3 wi = to_world(si.sh, si.wi);
  const float vals[16] = {0.f, 0.f, 0.f, f.x, f.y, f.z, le.x, le.y, le.z, si.valid ? 1.f : 0.f,
                          si.p.x, si.p.y, si.p.z, wi.x, wi.y, wi.z};
  for (int k = 0; k < 16; ++k) o[k] = vals[k];
}

}  // namespace

extern "C" {

// IntersectionSampler.sample for n points: 9 floats each (prim bits, b1, b2,
// p, wi_world), as mtx_nerad_lhs.
int orc_nerad_lhs(const mtx_scene_desc *d, const mtx_nerad_tables *h, uint32_t seed, uint32_t n, float *out) {
  SceneView s = make_view(d);
  NeradHost nt = nerad_tables(h);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    V3 wi;
    SurfaceSample ss;
    const SurfaceInteraction si = nerad_point(s, nt.t, seed, (uint32_t)i, &wi, &ss);
    float *o = out + 9 * i;
    uint32_t pb = ss.prim;
    memcpy(o, &pb, 4);
    o[1] = ss.b1;
    o[2] = ss.b2;
    o[3] = si.p.x;
    o[4] = si.p.y;
    o[5] = si.p.z;
    o[6] = wi.x;
    o[7] = wi.y;
    o[8] = wi.z;
  }
  return 0;
}

// sample_rhs lanes (batch * M, lane = point * M + j): 16 floats per lane, see
// orc_nerad_lane.
int orc_nerad_rhs(const mtx_scene_desc *d, const mtx_nerad_tables *h, uint32_t lhs_seed, uint32_t rhs_seed,
                  uint32_t batch, uint32_t M, float *lanes) {
  SceneView s = make_view(d);
  NeradHost nt = nerad_tables(h);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t i = 0; i < (int64_t)batch * M; ++i) {
    V3 wi;
    SurfaceSample ss;
    const SurfaceInteraction si = nerad_point(s, nt.t, lhs_seed, (uint32_t)(i / M), &wi, &ss);
    Pcg32 rng = sampler_lane(rhs_seed, (uint32_t)i);
    orc_nerad_lane(s, si, rng, lanes + 16 * i);
  }
  return 0;
}

// Integrator.sample lanes of a render (camera lanes as orc_render_samples):
// 16 floats per sample (see orc_nerad_render_lane) and the film position.
int orc_nerad_render_samples(const mtx_scene_desc *d, const mtx_render_args *a, float *lanes, float *pos) {
  SceneView s = make_view(d);
  const uint32_t W = s.camera.width, H = s.camera.height;
  const uint64_t npx = (uint64_t)(a->y1 - a->y0) * W;
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t p = 0; p < (int64_t)npx; ++p) {
    const uint32_t y = a->y0 + (uint32_t)(p / W), x = (uint32_t)(p % W);
    for (uint32_t k = 0; k < a->spp; ++k) {
      const uint32_t lane = (uint32_t)(((uint64_t)y * W + x) * a->spp_total + a->sample_offset + k);
      Pcg32 rng = sampler_lane(a->seed, lane);
      const V2 u = rng.next_2d();
      const float sx = (float)x + u.x, sy = (float)y + u.y;
      const Ray ray = camera_ray(s.camera, V2{sx / (float)W, sy / (float)H});
      const uint64_t o = (uint64_t)p * a->spp + k;
      orc_nerad_render_lane(s, rng, ray, lanes + 16 * o);
      pos[2 * o] = sx;
      pos[2 * o + 1] = sy;
    }
  }
  return 0;
}

}  // extern "C"
