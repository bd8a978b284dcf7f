// api.cpp — libmtx C ABI (include/mtx.h): device context, scene upload,
// wavefront scheduling and the primitive entry points.
//
// The host side of the replaced path: upstream SamplingIntegrator::render
// (transcribed at path.py:103-192) seeds the sampler over W*H*spp lanes,
// traces one Dr.Jit wavefront and splats into an ImageBlock. Here the same
// lanes are processed in chunks of whole pixels; each chunk runs
// raygen -> [trace, shade, shadow] x max_depth -> film stage 1 on one HIP
// stream with no host synchronisation (the persistent kernels read their
// queue lengths from device counters), then one film gather per call.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <initializer_list>
#include <string>
#include <vector>

#include "mtx.h"
#include "mtx_core/interaction.h"
#include "prims.h"
#include "wavefront.h"

static thread_local char g_err[1024] = "";

void mtx_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) {                                                                       \
      mtx_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return MTX_E_HIP;                                                                           \
    }                                                                                             \
  } while (0)

namespace {

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
};

int dalloc(DevBuf &b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return MTX_OK;
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  if (bytes == 0) return MTX_OK;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    mtx_set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    b.p = nullptr;
    return MTX_E_OOM;
  }
  b.bytes = bytes;
  return MTX_OK;
}

void dfree(DevBuf &b) {
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

template <class T>
int upload(DevBuf &b, const T *src, size_t count, hipStream_t st) {
  if (!src || count == 0) {
    dfree(b);
    return MTX_OK;
  }
  int rc = dalloc(b, count * sizeof(T));
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, st));
  return MTX_OK;
}

}  // namespace

// Second wavefront of the two-stream render (mtx_render's path / path-mis /
// nrc / simple integrators): its own path state, queues, counters, claim
// cursors and traversal spill area, on its own stream. The film's chunks
// alternate between the two wavefronts, so one chunk's kernels fill the
// GPU while the other's persistent trace launches drain their tails.
struct Wave2 {
  hipStream_t stream = nullptr;
  hipEvent_t start = nullptr, done = nullptr;
  DevBuf ray_o, ray_d, thr, L, prev, misc, pos, hit, q0, q1, shadow, counters, xheads, stack_ovf, cq_perm, cq_cursor;
  DevBuf cq_p, cq_d, cq_t, cq_count, f_feat, f_out;  // NRC radiance-cache queries of its chunks
  uint32_t capacity = 0;
};

struct mtx_ctx {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  Wave2 w2;
  uint32_t *q_pinned = nullptr;  // per-chunk cache-query counts of a stats render (pinned, kQSlots)
  uint32_t streams = MTX_STREAMS;  // 1: every chunk on `stream` (MTX_STREAMS env: A/B)
  uint32_t streams_max_log2 = 27;  // two streams for renders of <= 2^this paths (MTX_STREAMS_MAX_LOG2: A/B)
  bool has_scene = false;
  // scene
  DevBuf stack_ovf;  // traversal stack entries beyond the LDS part
  DevBuf shade_rec;  // per-triangle shading records
  // radiance field (mtx_field_upload)
  DevBuf field_table, field_frag, fq_p, fq_d, f_feat, f_out;
  DevBuf cq_p, cq_d, cq_t, cq_count;  // NRC cache queries of a chunk
  mtx::FieldEncoding field{};
  uint32_t field_hidden = 0;
  bool has_field = false;
  DevBuf field_w16;  // plain fp16 weights (training forward / backward)
  uint32_t field_n_in = 0, field_n_w = 0;
  uint64_t field_n_table = 0;  // fp16 table entries
  // field training (mtx_field_train_init): fp32 master parameters [table |
  // weights], Adam moments, gradients, per-batch scratch
  DevBuf tr_p, tr_m, tr_v, tr_g, tr_wpart, tr_loss, tr_out, tr_dfeat, tr_feat, tr_flag, tr_target;
  mtx_field_opt opt{};
  bool training = false;
  uint32_t adam_t = 0, good_steps = 0;
  float scale = 1.f;
  // neural radiosity surface tables (mtx_nerad_upload) and batch buffers
  DevBuf nr_shape_pmf, nr_shape_cdf, nr_tri_off, nr_tri_pmf, nr_tri_cdf, nr_tri_prim, nr_dists;
  mtx::NeradTables nr{};
  bool has_nerad = false;
  uint32_t scene_n_shapes = 0;
  DevBuf nr_lhs, nr_qp, nr_qd, nr_Lrhs, nr_lanes;
  DevBuf nodes, tri, occ_nodes, occ_tri, tri_vidx, tri_shape, vpos, vnormal, vuv, shapes, materials, emitters, textures, texels, tables;
  mtxd::DevScene scene{};
  // wavefront
  DevBuf ray_o, ray_d, thr, L, prev, misc, pos, hit, q0, q1, shadow, counters, stats;
  DevBuf xheads, rs_heads;  // per-XCD claim cursors of the persistent trace kernels
  uint32_t capacity = 0;
  DevBuf mlt_cur, mlt_L, mlt_prop, vpath, vprop;  // PSSMLT chain state
  DevBuf vpath_es, vprop_es;                       // pssmltpath emitter samples
  uint32_t mlt_capacity = 0, mlt_depth = 0, mlt_es_capacity = 0, mlt_es_depth = 0;
  // ReSTIR GI frame state (restirgi.py:217-226): kept across mtx_render calls
  DevBuf rs_samp[2], rs_tres, rs_sres, rs_radius, rs_hit, rs_dir, rs_emit, rs_rng, rs_rays, rs_count, rs_occ, rs_qM, rs_nbr, rs_xs, rs_ns;
  uint32_t rs_n = 0, rs_cur = 0, rs_pending_frame = 0;
  bool rs_valid = false, rs_pending_b = false;
  mtx_camera rs_prev_cam{};
  // film
  DevBuf contrib, film;
  // scratch for sample_rays / trace / primitives
  DevBuf s0, s1, s2, s3, s4, s5, s6;
  int trace_grid = 0, closest_grid = 0, shade_grid = 0;  // persistent grids: any hit, closest hit, shade
  size_t max_lds = 160 * 1024;  // LDS one workgroup may hold (gfx950: the CU's 160 KiB)
  // tuning knobs (environment, read at context creation): LDS stack entries
  // of the persistent traversal, chunk path order
  uint32_t lds_stack = mtxd::kLdsStack;
  uint32_t lds_top = MTX_LDS_TOP;          // closest-hit tree nodes kept in LDS per block (MTX_LDS_TOP env: A/B)
  uint32_t occ_lds_top = MTX_OCC_LDS_TOP;  // occlusion tree nodes kept in LDS per block (MTX_OCC_LDS_TOP)
  uint32_t occ_lds_stack = mtxd::kOccLdsStack;
  uint32_t trace_batch = 128;  // queue entries per claim (256: +0.6 % closest, +1 % at spp 32; 64: +5 %)
  uint32_t urefill = 24;  // refill a wave once 24 lanes are idle (16: closest +1.3 %, 32: +2 %; 4-wide BVH)
  uint32_t occ_urefill = 12;  // any hit on the 8-wide tree (MTX_OCC_UREFILL; 8-16 alike, 24: shadow +1 ms, 32/40: +2/+3 ms)
  uint32_t xcd_claim = 1;
  // ReSTIR GI: a band of at most this many paths runs its stage A in the
  // per-lane megakernel on one wavefront (MTX_MEGA_PATHS, 0 = off; default
  // 0xffffffff = twice the resident lanes of the megakernel's grid,
  // 2 x mega_grid x kShadeBlock)
  uint32_t mega_paths = 0xffffffffu;
  int mega_grid = 0;
  // such a band's whole stage A (raygen .. collect) in one per-lane launch
  // (kernels.hip k_rs_stage_a; MTX_RS_FUSED=0: raygen, trace, k_rs_begin, the
  // megakernel and k_rs_collect as separate launches)
  uint32_t rs_fused = 1;
  // NRC cache query order: MTX_CACHE_SORT=1 Morton-sorted (host sync; measured slower), 2 grouped
  // by region on the device with one eighth of the rows per XCD (field.hip)
  uint32_t cache_sort = MTX_CACHE_SORT;
  // NRC cache encoder: level-major lanes (field.hip k_field_encode_lm; MTX_ENCODE_LM=0: query-major)
  uint32_t encode_lm = MTX_ENCODE_LM;
  // NRC cache: encode + MLP + apply in one launch (field.hip k_field_cache_fused; MTX_CACHE_FUSED=0: three)
  uint32_t cache_fused = 1;
  DevBuf cq_keys, cq_perm, cq_ws;
  std::vector<hipEvent_t> events;
  hipEvent_t prim_ev[2] = {nullptr, nullptr};
  double last_device_ms = 0.0;
};

extern "C" {

int mtx_abi_version(void) { return MTX_ABI_VERSION; }

// Diagnostic export (not in mtx.h): the shade kernel's per-phase stamp sums of
// an MTX_DIAG_STAMPS build (tools/shade_stamps.py); returns the segment
// count, or -1 in production builds.
int mtx_diag_shade_stamps(unsigned long long *out) { return mtxd::shade_stamps(out); }

const char *mtx_last_error(void) { return g_err; }

int mtx_ctx_create(int hip_device, mtx_ctx **out) {
  if (!out) {
    mtx_set_error("mtx_ctx_create: out is NULL");
    return MTX_E_ARG;
  }
  *out = nullptr;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (hip_device < 0 || hip_device >= n) {
    mtx_set_error("mtx_ctx_create: device %d out of range (%d devices)", hip_device, n);
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(hip_device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, hip_device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    mtx_set_error("mtx_ctx_create: device %d is %s, libmtx is built for gfx950", hip_device, prop.gcnArchName);
    return MTX_E_UNSUPPORTED;
  }
  mtx_ctx *c = new mtx_ctx();
  c->device = hip_device;
  c->n_cu = prop.multiProcessorCount;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    mtx_set_error("hipStreamCreate failed: %s", hipGetErrorString(e));
    return MTX_E_HIP;
  }
  // Persistent grids: every CU filled to the kernels' occupancy (the trace
  // grid is recomputed per scene: its LDS stack depends on the BVH depth).
  c->trace_grid = c->closest_grid = c->n_cu * 8;
  c->shade_grid = c->n_cu * mtxd::shade_blocks_per_cu();
  {
    // a gfx950 workgroup may hold the CU's whole 160 KiB of LDS (the attribute
    // may report the 64 KiB that needs no opt-in; the kernels launch above it)
    int v = 0;
    c->max_lds = 160 * 1024;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, hip_device) == hipSuccess &&
        (size_t)v > c->max_lds)
      c->max_lds = (size_t)v;
  }
  if (const char *e = getenv("MTX_LDS_STACK")) c->lds_stack = std::max(1, std::min(MTX_BVH_MAX_DEPTH + 1, atoi(e)));
  if (const char *e = getenv("MTX_LDS_TOP")) c->lds_top = (uint32_t)std::max(0, std::min(256, atoi(e)));
  if (const char *e = getenv("MTX_OCC_LDS_TOP")) c->occ_lds_top = (uint32_t)std::max(0, std::min(192, atoi(e)));
  if (const char *e = getenv("MTX_OCC_LDS_STACK"))
    c->occ_lds_stack = std::max(1, std::min(MTX_BVH_MAX_DEPTH + 1, atoi(e)));
  if (const char *e = getenv("MTX_STREAMS_MAX_LOG2")) c->streams_max_log2 = (uint32_t)std::max(16, std::min(31, atoi(e)));
  if (const char *e = getenv("MTX_STREAMS")) c->streams = (uint32_t)std::max(1, std::min(2, atoi(e)));
  if (const char *e = getenv("MTX_TRACE_BATCH")) c->trace_batch = (uint32_t)std::max(1, std::min(1 << 16, atoi(e)));
  if (const char *e = getenv("MTX_UREFILL")) c->urefill = (uint32_t)std::max(1, std::min(64, atoi(e)));
  if (const char *e = getenv("MTX_OCC_UREFILL")) c->occ_urefill = (uint32_t)std::max(1, std::min(64, atoi(e)));
  if (const char *e = getenv("MTX_XCD_CLAIM")) c->xcd_claim = atoi(e) != 0;
  if (const char *e = getenv("MTX_RS_FUSED")) c->rs_fused = atoi(e) ? 1u : 0u;
  if (const char *e = getenv("MTX_MEGA_PATHS")) c->mega_paths = (uint32_t)strtoul(e, nullptr, 0);
  if (const char *e = getenv("MTX_CACHE_FUSED")) c->cache_fused = atoi(e) ? 1u : 0u;
  if (const char *e = getenv("MTX_ENCODE_LM")) c->encode_lm = atoi(e) ? 1u : 0u;
  if (const char *e = getenv("MTX_CACHE_SORT")) c->cache_sort = (uint32_t)std::max(0, std::min(2, atoi(e)));
  *out = c;
  return MTX_OK;
}

void mtx_ctx_destroy(mtx_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->w2.stream) hipStreamSynchronize(c->w2.stream);
  DevBuf *bufs[] = {&c->nodes,  &c->tri, &c->occ_nodes, &c->occ_tri, &c->tri_vidx, &c->tri_shape, &c->vpos,     &c->vnormal, &c->vuv,
                    &c->shapes, &c->materials, &c->emitters, &c->textures, &c->texels, &c->tables, &c->ray_o,
                    &c->ray_d,  &c->thr,     &c->L,        &c->prev,      &c->misc,     &c->pos,     &c->hit,
                    &c->q0,     &c->q1,      &c->shadow,   &c->counters, &c->xheads, &c->rs_heads,  &c->stats,    &c->contrib, &c->film,
                    &c->mlt_cur, &c->mlt_L, &c->mlt_prop, &c->vpath, &c->vprop, &c->vpath_es, &c->vprop_es,
                    &c->stack_ovf, &c->shade_rec, &c->field_table, &c->field_frag, &c->fq_p, &c->fq_d,
                    &c->f_feat, &c->f_out, &c->cq_p, &c->cq_d, &c->cq_t, &c->cq_count, &c->rs_samp[0], &c->rs_samp[1], &c->rs_tres, &c->rs_sres, &c->rs_radius, &c->rs_hit,
                    &c->rs_dir, &c->rs_emit, &c->rs_rng, &c->rs_rays, &c->rs_count, &c->rs_occ, &c->rs_qM, &c->rs_nbr, &c->rs_xs, &c->rs_ns,
                    &c->s0,     &c->s1,      &c->s2,       &c->s3,        &c->s4,       &c->s5, &c->s6,
                    &c->cq_keys, &c->cq_perm, &c->cq_ws,
                    &c->field_w16, &c->tr_p, &c->tr_m, &c->tr_v, &c->tr_g, &c->tr_wpart, &c->tr_loss, &c->tr_out,
                    &c->tr_dfeat, &c->tr_feat, &c->tr_flag, &c->tr_target, &c->nr_shape_pmf, &c->nr_shape_cdf,
                    &c->nr_tri_off, &c->nr_tri_pmf, &c->nr_tri_cdf, &c->nr_tri_prim, &c->nr_dists, &c->nr_lhs,
                    &c->nr_qp, &c->nr_qd, &c->nr_Lrhs, &c->nr_lanes};
  for (DevBuf *b : bufs) dfree(*b);
  Wave2 &w = c->w2;
  for (DevBuf *b : {&w.ray_o, &w.ray_d, &w.thr, &w.L, &w.prev, &w.misc, &w.pos, &w.hit, &w.q0, &w.q1, &w.shadow,
                    &w.counters, &w.xheads, &w.stack_ovf, &w.cq_p, &w.cq_d, &w.cq_t, &w.cq_count, &w.f_feat,
                    &w.f_out, &w.cq_perm, &w.cq_cursor})
    dfree(*b);
  if (w.start) hipEventDestroy(w.start);
  if (w.done) hipEventDestroy(w.done);
  if (w.stream) hipStreamDestroy(w.stream);
  for (hipEvent_t ev : c->events) hipEventDestroy(ev);
  if (c->q_pinned) hipHostFree(c->q_pinned);
  for (hipEvent_t ev : c->prim_ev)
    if (ev) hipEventDestroy(ev);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

// Caller-supplied occlusion trees: their triangle records must be the
// scene's (a stale pair would answer shadow rays against other geometry).
// With d->occ_perm the claimed correspondence is checked record by record
// and as a permutation; without it the records of both arrays are sorted
// and matched. perm[i] = scene triangle of occlusion triangle i.
static int occ_match(const mtx_scene_desc *d, std::vector<uint32_t> &perm) {
  const uint32_t n = d->n_tris;
  auto rec = [](const float *g, uint32_t i, int w) {
    uint32_t x;
    memcpy(&x, g + 12 * (size_t)i + 4 * (w / 3) + (w % 3), 4);
    return x;
  };
  auto same = [&](uint32_t i, uint32_t j) {
    for (int w = 0; w < 9; ++w)
      if (rec(d->occ_tri_geom, i, w) != rec(d->tri_geom, j, w)) return false;
    return true;
  };
  perm.assign(n, 0u);
  if (d->occ_perm) {
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t j = d->occ_perm[i];
      if (j >= n || seen[j] || !same(i, j)) {
        mtx_set_error("mtx_scene_upload: occ_perm[%u] = %u does not map occlusion triangle %u to an unused scene "
                      "triangle with the same record",
                      i, j, i);
        return MTX_E_ARG;
      }
      seen[j] = 1;
      perm[i] = j;
    }
    return MTX_OK;
  }
  std::vector<uint32_t> a(n), b(n);
  for (uint32_t i = 0; i < n; ++i) a[i] = b[i] = i;
  auto less = [&](const float *g) {
    return [&, g](uint32_t x, uint32_t y) {
      for (int w = 0; w < 9; ++w) {
        const uint32_t u = rec(g, x, w), v = rec(g, y, w);
        if (u != v) return u < v;
      }
      return x < y;
    };
  };
  std::sort(a.begin(), a.end(), less(d->occ_tri_geom));
  std::sort(b.begin(), b.end(), less(d->tri_geom));
  for (uint32_t k = 0; k < n; ++k) {
    if (!same(a[k], b[k])) {
      mtx_set_error("mtx_scene_upload: occ_tri_geom is not a permutation of tri_geom (occ_nodes / occ_tri_geom "
                    "must come from mtx_bvh_build_occlusion over this tri_geom)");
      return MTX_E_ARG;
    }
    perm[a[k]] = b[k];
  }
  return MTX_OK;
}

int mtx_scene_upload(mtx_ctx *c, const mtx_scene_desc *d) {
  if (!c || !d) {
    mtx_set_error("mtx_scene_upload: null argument");
    return MTX_E_ARG;
  }
  if (!d->nodes || !d->tri_geom || !d->tri_vidx || !d->tri_shape || !d->vpos || !d->shapes || !d->materials ||
      d->n_tris == 0 || d->n_nodes == 0 || (d->n_emitters == 0 && !d->has_env) || (d->n_emitters && !d->emitters)) {
    mtx_set_error("mtx_scene_upload: incomplete scene (need geometry, BVH, shapes, materials, >=1 emitter)");
    return MTX_E_ARG;
  }
  // The occlusion BVH: given, or built here over the triangle records.
  const bool occ_given = d->occ_nodes && d->occ_tri_geom && d->n_occ_nodes > 0;
  if (!occ_given && (d->occ_nodes || d->occ_tri_geom)) {
    mtx_set_error("mtx_scene_upload: occ_nodes and occ_tri_geom go together (both NULL: built here)");
    return MTX_E_ARG;
  }
  std::vector<int32_t> occ_nodes_v;
  std::vector<float> occ_geom_v;
  std::vector<uint32_t> occ_perm_v;
  const int32_t *occ_nodes = d->occ_nodes;
  const float *occ_geom = d->occ_tri_geom;
  uint32_t n_occ = d->n_occ_nodes;
  int rc = 0;
  if (!occ_given) {
    occ_nodes_v.resize(((size_t)d->n_tris + 1) * MTX_OCC_NODE_WORDS);
    occ_geom_v.resize(12 * (size_t)d->n_tris);
    if ((rc = mtx_bvh_build_occlusion(d->tri_geom, d->n_tris, occ_nodes_v.data(), &n_occ, occ_geom_v.data(),
                                      nullptr, nullptr)))
      return rc;
    occ_nodes = occ_nodes_v.data();
    occ_geom = occ_geom_v.data();
  } else if ((rc = occ_match(d, occ_perm_v))) {  // given trees: their records must be this scene's
    return rc;
  }
  // Validate both trees (mtx.h) on the host so that no kernel can read out
  // of bounds, and find their depths (stack entries: a 4-wide level pushes
  // at most 3 node references, an 8-wide level one node group); also
  // rejects cycles.
  uint32_t bvh_depth = 0, occ_depth = 0;
  {
    std::vector<std::pair<int32_t, uint32_t>> todo{{0, 0u}};
    uint64_t visited = 0;
    while (!todo.empty()) {
      auto [nd, dep] = todo.back();
      todo.pop_back();
      bvh_depth = std::max(bvh_depth, dep + 1);
      if (++visited > d->n_nodes || dep >= MTX_BVH_MAX_DEPTH) {
        mtx_set_error("mtx_scene_upload: BVH is not a tree of depth <= %d", MTX_BVH_MAX_DEPTH);
        return MTX_E_ARG;
      }
      const int32_t *w = d->nodes + MTX_BVH_NODE_WORDS * (size_t)nd;
      const uint32_t nch = (uint32_t)w[3] >> 24;
      if (nch < 1 || nch > MTX_BVH_WIDTH) {
        mtx_set_error("mtx_scene_upload: node %d has %u children", nd, nch);
        return MTX_E_ARG;
      }
      for (uint32_t k = 0; k < nch; ++k) {
        const int32_t ch = w[4 + k];
        if (ch >= 0) {
          if ((uint32_t)ch >= d->n_nodes) {
            mtx_set_error("mtx_scene_upload: node %d child %d out of range", nd, ch);
            return MTX_E_ARG;
          }
          todo.push_back({ch, dep + 1});
        } else {
          uint32_t x = (uint32_t)(~ch), first = x >> 3, cnt = (x & 7u) + 1;
          if ((uint64_t)first + cnt > d->n_tris) {
            mtx_set_error("mtx_scene_upload: leaf [%u,+%u) exceeds %u triangles", first, cnt, d->n_tris);
            return MTX_E_ARG;
          }
        }
      }
    }
  }
  {
    std::vector<std::pair<uint32_t, uint32_t>> todo{{0u, 0u}};
    uint64_t visited = 0;
    while (!todo.empty()) {
      auto [nd, dep] = todo.back();
      todo.pop_back();
      occ_depth = std::max(occ_depth, dep + 1);
      if (++visited > n_occ || dep >= MTX_BVH_MAX_DEPTH) {
        mtx_set_error("mtx_scene_upload: occlusion BVH is not a tree of depth <= %d", MTX_BVH_MAX_DEPTH);
        return MTX_E_ARG;
      }
      const uint32_t *w = reinterpret_cast<const uint32_t *>(occ_nodes) + MTX_OCC_NODE_WORDS * (size_t)nd;
      const uint32_t imask = w[3] >> 24, child_base = w[4], tri_base = w[5];
      uint32_t inner = 0;
      for (uint32_t sl = 0; sl < MTX_OCC_WIDTH; ++sl) {
        const uint32_t m = (w[6 + (sl >> 2)] >> (8 * (sl & 3))) & 0xffu;
        const bool is_inner = (imask >> sl) & 1u;
        if (is_inner) {
          const uint32_t ch = child_base + inner++;
          if (m != (0x20u | (24u + sl)) || ch >= n_occ) {
            mtx_set_error("mtx_scene_upload: occlusion node %u slot %u: bad inner child", nd, sl);
            return MTX_E_ARG;
          }
          todo.push_back({ch, dep + 1});
        } else if (m != 0) {
          const uint32_t cb = m >> 5, off = m & 31u, cnt = cb == 1 ? 1u : cb == 3 ? 2u : cb == 7 ? 3u : 0u;
          if (cnt == 0 || off + cnt > 24 || (uint64_t)tri_base + off + cnt > d->n_tris) {
            mtx_set_error("mtx_scene_upload: occlusion node %u slot %u: bad leaf", nd, sl);
            return MTX_E_ARG;
          }
        }
      }
    }
  }
  for (uint64_t i = 0; i < 3ull * d->n_tris; ++i)
    if (d->tri_vidx[i] >= d->n_verts) {
      mtx_set_error("mtx_scene_upload: vertex index out of range");
      return MTX_E_ARG;
    }
  for (uint32_t i = 0; i < d->n_tris; ++i)
    if (d->tri_shape[i] >= d->n_shapes) {
      mtx_set_error("mtx_scene_upload: shape index out of range");
      return MTX_E_ARG;
    }
  for (uint32_t i = 0; i < d->n_shapes; ++i) {
    if (d->shapes[i].material >= d->n_materials ||
        (d->shapes[i].emitter >= 0 && (uint32_t)d->shapes[i].emitter >= d->n_emitters)) {
      mtx_set_error("mtx_scene_upload: shape %u references a missing material/emitter", i);
      return MTX_E_ARG;
    }
  }
  for (uint32_t i = 0; i < d->n_materials; ++i) {
    const mtx_material &m = d->materials[i];
    if (m.tex >= 0) {
      if ((uint32_t)m.tex >= d->n_textures || !d->textures) {
        mtx_set_error("mtx_scene_upload: material %u texture out of range", i);
        return MTX_E_ARG;
      }
      const mtx_texture &t = d->textures[m.tex];
      if (t.offset + 3ull * t.width * t.height > d->n_texels || t.width == 0 || t.height == 0) {
        mtx_set_error("mtx_scene_upload: texture %d exceeds texel buffer", m.tex);
        return MTX_E_ARG;
      }
    }
    if (m.type == MTX_MAT_ROUGHPLASTIC && (m.table < 0 || (uint32_t)m.table + MTX_ROUGH_TRANSMITTANCE_RES > d->n_tables)) {
      mtx_set_error("mtx_scene_upload: roughplastic material %u has no transmittance table", i);
      return MTX_E_ARG;
    }
  }
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = c->stream;
  if ((rc = upload(c->nodes, d->nodes, (size_t)MTX_BVH_NODE_WORDS * d->n_nodes, st))) return rc;
  if ((rc = upload(c->occ_nodes, occ_nodes, (size_t)MTX_OCC_NODE_WORDS * n_occ, st))) return rc;
  for (int tree = 0; tree < 2; ++tree) {
    // device triangles packed to 36 B (the ABI's 48-B records carry 3 pad
    // words): 3.6 instead of 2.7 triangles per 128-B line, same load count
    const float *src = tree ? occ_geom : d->tri_geom;
    std::vector<float> g9(9ull * d->n_tris);
    for (size_t i = 0; i < d->n_tris; ++i)
      for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 3; ++j) g9[9 * i + 3 * k + j] = src[12 * i + 4 * k + j];
    if ((rc = upload(tree ? c->occ_tri : c->tri, g9.data(), g9.size(), st))) return rc;
    HIP_TRY(hipStreamSynchronize(st));  // g9 is freed at scope exit
  }
  if ((rc = upload(c->tri_vidx, d->tri_vidx, 3ull * d->n_tris, st))) return rc;
  if ((rc = upload(c->tri_shape, d->tri_shape, (size_t)d->n_tris, st))) return rc;
  if ((rc = upload(c->vpos, d->vpos, 3ull * d->n_verts, st))) return rc;
  if ((rc = upload(c->vnormal, d->vnormal, d->vnormal ? 3ull * d->n_verts : 0, st))) return rc;
  if ((rc = upload(c->vuv, d->vuv, d->vuv ? 2ull * d->n_verts : 0, st))) return rc;
  if ((rc = upload(c->shapes, d->shapes, d->n_shapes, st))) return rc;
  c->scene_n_shapes = d->n_shapes;
  c->has_nerad = false;  // surface tables belong to the previous scene
  if ((rc = upload(c->materials, d->materials, d->n_materials, st))) return rc;
  if ((rc = upload(c->emitters, d->emitters, d->n_emitters, st))) return rc;
  if ((rc = upload(c->textures, d->textures, d->n_textures, st))) return rc;
  if ((rc = upload(c->texels, d->texels, d->n_texels, st))) return rc;
  if ((rc = upload(c->tables, d->tables, d->n_tables, st))) return rc;
  {
    // per-triangle shading records (compute_si_dev)
    std::vector<float> rec(32 * (size_t)d->n_tris, 0.f);
    for (uint32_t t = 0; t < d->n_tris; ++t) {
      float *r = &rec[32 * (size_t)t];
      const mtx_shape &sh = d->shapes[d->tri_shape[t]];
      const uint32_t use_n = (!(sh.flags & 1u) && d->vnormal) ? 1u : 0u;
      const uint32_t use_uv = ((sh.flags & 2u) && d->vuv) ? 2u : 0u;
      for (int k = 0; k < 3; ++k) {
        const uint32_t vi = d->tri_vidx[3 * (size_t)t + k];
        for (int a = 0; a < 3; ++a) r[4 * k + a] = d->vpos[3 * (size_t)vi + a];
        if (use_n)
          for (int a = 0; a < 3; ++a) r[12 + 4 * k + a] = d->vnormal[3 * (size_t)vi + a];
        if (use_uv) {
          r[24 + 2 * k] = d->vuv[2 * (size_t)vi];
          r[24 + 2 * k + 1] = d->vuv[2 * (size_t)vi + 1];
        }
      }
      // bits 8..12: shading class of the material (read by no kernel since
      // the block-level material sort was measured slower and removed)
      const mtx_material &m = d->materials[sh.material];
      const uint32_t cls = 1u + ((m.type & 7u) << 2 | (m.tex >= 0 ? 2u : 0u) | ((m.flags & MTX_MF_MASK) ? 1u : 0u));
      const uint32_t mat = sh.material, fl = use_n | use_uv | (cls << 8);
      const int32_t em = sh.emitter;
      memcpy(&r[3], &mat, 4);
      memcpy(&r[7], &em, 4);
      memcpy(&r[11], &fl, 4);
    }
    if ((rc = upload(c->shade_rec, rec.data(), rec.size(), st))) return rc;
    HIP_TRY(hipStreamSynchronize(st));  // rec is freed at scope exit
  }
  HIP_TRY(hipStreamSynchronize(st));
  mtxd::DevScene &s = c->scene;
  s.nodes = (const int4 *)c->nodes.p;
  s.tri = (const float *)c->tri.p;
  s.occ_nodes = (const int4 *)c->occ_nodes.p;
  s.occ_tri = (const float *)c->occ_tri.p;
  s.tri_vidx = (const uint32_t *)c->tri_vidx.p;
  s.tri_shape = (const uint32_t *)c->tri_shape.p;
  s.vpos = (const float *)c->vpos.p;
  s.vnormal = (const float *)c->vnormal.p;
  s.vuv = (const float *)c->vuv.p;
  s.shapes = (const mtx_shape *)c->shapes.p;
  s.shade_rec = (const float4 *)c->shade_rec.p;
  s.materials = (const mtx_material *)c->materials.p;
  s.emitters = (const mtx_emitter *)c->emitters.p;
  s.textures = (const mtx_texture *)c->textures.p;
  s.texels = (const float *)c->texels.p;
  s.tables = (const float *)c->tables.p;
  s.n_tris = d->n_tris;
  s.n_emitters = d->n_emitters;
  s.camera = d->camera;
  s.has_env = d->has_env ? 1u : 0u;
  for (int k = 0; k < 3; ++k) s.env_radiance[k] = d->env_radiance[k];
  mtx::env_bsphere(d->vpos, d->n_verts, s.env_center, &s.env_radius);
  // LDS per trace block (8 blocks of 256 threads per CU fill the 160 KB):
  // closest hit 16 x 4-B stack entries per lane + 64 nodes of 64 B,
  // occlusion 8 x 8-B entries + 48 nodes of 80 B
  s.stack_entries = 3 * bvh_depth + 1;
  s.lds_entries = std::min<uint32_t>(s.stack_entries, c->lds_stack);
  s.lds_top = std::min<uint32_t>(d->n_nodes, c->lds_top);
  s.occ_stack_entries = occ_depth + 1;
  s.occ_lds_entries = std::min<uint32_t>(s.occ_stack_entries, c->occ_lds_stack);
  s.occ_lds_top = std::min<uint32_t>(n_occ, c->occ_lds_top);
  s.trace_batch = c->trace_batch;
  s.urefill = c->urefill;
  s.occ_urefill = c->occ_urefill;
  s.xcd_claim = c->xcd_claim;
  c->trace_grid = c->n_cu * mtxd::trace_blocks_per_cu(s);
  c->closest_grid = c->n_cu * mtxd::closest_blocks_per_cu(s);
  c->mega_grid = c->n_cu * mtxd::mega_blocks_per_cu(s);
  s.ovf_threads = (uint32_t)std::max(c->trace_grid, c->closest_grid) * mtxd::kTraceBlock;
  if ((rc = dalloc(c->stack_ovf, mtxd::stack_ovf_bytes(s)))) return rc;
  s.stack_ovf = c->stack_ovf.p;
  c->has_scene = true;
  return MTX_OK;
}

}  // extern "C"

namespace {

// Default wavefront: up to 256 Mi paths (~328 B of state each, ~82 GB) so a
// 1280x720 spp=256 frame runs as one chunk (fewer queue tails), bounded by
// 40 % of the free HBM.
constexpr uint32_t kDefaultChunk = 1u << 28;
constexpr size_t kPathStateBytes = 328;
constexpr size_t kCacheQueryBytes = 16 * 3 + 128 + 12;  // ensure_cache: query planes, features, outputs
// `ways` wavefronts of the returned size are allocated (2 for a two-stream
// render), each with the NRC cache-query buffers when `cache`: the budget is
// 40 % of the free HBM for all of them together. Buffers this context already
// holds (every wavefront's) count as available.
uint32_t default_chunk(mtx_ctx *c, const mtx_render_args *a, uint32_t ways, bool cache) {
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 1u << 22;
  // PSSMLT chains also keep the current and proposed path vertices
  const size_t per_path =
      kPathStateBytes + (cache ? kCacheQueryBytes : 0) +
      (a->integrator == MTX_INT_PSSMLT_SIMPLE ? 32ull * std::max<uint32_t>(a->max_depth, 1) + 48
       : a->integrator == MTX_INT_PSSMLT_PATH ? 48ull * std::max<uint32_t>(a->max_depth, 1) + 48
                                              : 0);
  const size_t held = ways > 1 ? std::min<size_t>(c->capacity, c->w2.capacity) : c->capacity;
  const size_t fit = std::max<size_t>((size_t)((double)free_b * 0.4) / (per_path * std::max<uint32_t>(ways, 1)), held);
  return (uint32_t)std::max<size_t>(1u << 20, std::min<size_t>(kDefaultChunk, fit));
}

int ensure_wavefront(mtx_ctx *c, uint32_t cap, uint32_t max_depth) {
  int rc;
  if (cap > c->capacity) {
    if ((rc = dalloc(c->ray_o, 32ull * cap))) return rc;  // two planes (bounce parity), wavefront.h
    if ((rc = dalloc(c->ray_d, 32ull * cap))) return rc;
    if ((rc = dalloc(c->thr, 32ull * cap))) return rc;
    if ((rc = dalloc(c->L, 48ull * cap))) return rc;  // queue planes 0 / 1 + the per-path plane

    if ((rc = dalloc(c->prev, 32ull * cap))) return rc;
    if ((rc = dalloc(c->misc, 48ull * cap))) return rc;
    if ((rc = dalloc(c->pos, 8ull * cap))) return rc;
    if ((rc = dalloc(c->hit, 16ull * cap))) return rc;
    if ((rc = dalloc(c->q0, 4ull * cap))) return rc;
    if ((rc = dalloc(c->q1, 4ull * cap))) return rc;
    if ((rc = dalloc(c->shadow, sizeof(mtxd::ShadowRec) * (size_t)cap))) return rc;
    c->capacity = cap;
  }
  if ((rc = dalloc(c->counters, 16ull * (max_depth + 2)))) return rc;
  if ((rc = dalloc(c->xheads, 8ull * mtxd::kXSlotWords * (max_depth + 2)))) return rc;
  if ((rc = dalloc(c->stats, 8 * 8))) return rc;
  return MTX_OK;
}

mtxd::WaveBuffers buffers(mtx_ctx *c) {
  mtxd::WaveBuffers b;
  b.ray_o[0] = (float4 *)c->ray_o.p;
  b.ray_o[1] = b.ray_o[0] + c->capacity;
  b.ray_d[0] = (float4 *)c->ray_d.p;
  b.ray_d[1] = b.ray_d[0] + c->capacity;
  b.ray_par = 0;
  b.thr[0] = (float4 *)c->thr.p;
  b.thr[1] = b.thr[0] + c->capacity;
  for (int k = 0; k < 3; ++k) b.L[k] = (float4 *)c->L.p + (size_t)k * c->capacity;
  b.prev[0] = (float4 *)c->prev.p;
  b.prev[1] = b.prev[0] + c->capacity;
  for (int k = 0; k < 3; ++k) b.misc[k] = (uint4 *)c->misc.p + (size_t)k * c->capacity;
  b.pos = (float2 *)c->pos.p;
  b.hit = (float4 *)c->hit.p;
  b.queue[0] = (uint32_t *)c->q0.p;
  b.queue[1] = (uint32_t *)c->q1.p;
  b.shadow = (mtxd::ShadowRec *)c->shadow.p;
  b.counters = (uint32_t *)c->counters.p;
  b.xheads = (uint32_t *)c->xheads.p;
  b.stats = (unsigned long long *)c->stats.p;
  b.capacity = c->capacity;
  b.mlt_cur = (float4 *)c->mlt_cur.p;
  b.mlt_L = (float4 *)c->mlt_L.p;
  b.mlt_prop = (float2 *)c->mlt_prop.p;
  b.vpath = (float4 *)c->vpath.p;
  b.vprop = (float4 *)c->vprop.p;
  b.vpath_es = (float2 *)c->vpath_es.p;
  b.vprop_es = (float2 *)c->vprop_es.p;
  b.cq_p = (float4 *)c->cq_p.p;
  b.cq_d = (float4 *)c->cq_d.p;
  b.cq_t = (float4 *)c->cq_t.p;
  b.cq_count = (uint32_t *)c->cq_count.p;
  return b;
}

// The second wavefront (Wave2): buffers for `cap` paths, its stream and
// events, and a traversal spill area of its own (two trace launches may run
// at once).
int ensure_wavefront2(mtx_ctx *c, uint32_t cap, uint32_t max_depth) {
  int rc;
  Wave2 &w = c->w2;
  if (!w.stream) {
    HIP_TRY(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&w.start, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
  }
  if (cap > w.capacity) {
    for (DevBuf *b : {&w.ray_o, &w.ray_d, &w.thr, &w.prev})
      if ((rc = dalloc(*b, 32ull * cap))) return rc;
    for (DevBuf *b : {&w.L, &w.misc})
      if ((rc = dalloc(*b, 48ull * cap))) return rc;
    if ((rc = dalloc(w.hit, 16ull * cap))) return rc;
    if ((rc = dalloc(w.pos, 8ull * cap))) return rc;
    if ((rc = dalloc(w.q0, 4ull * cap))) return rc;
    if ((rc = dalloc(w.q1, 4ull * cap))) return rc;
    if ((rc = dalloc(w.shadow, sizeof(mtxd::ShadowRec) * (size_t)cap))) return rc;
    w.capacity = cap;
  }
  if ((rc = dalloc(w.counters, 16ull * (max_depth + 2)))) return rc;
  if ((rc = dalloc(w.xheads, 8ull * mtxd::kXSlotWords * (max_depth + 2)))) return rc;
  const mtxd::DevScene &s = c->scene;
  if ((rc = dalloc(w.stack_ovf, mtxd::stack_ovf_bytes(s)))) return rc;
  return MTX_OK;
}

mtxd::WaveBuffers buffers2(mtx_ctx *c) {
  mtxd::WaveBuffers b = buffers(c);  // shared: stats, the PSSMLT / cache planes (unused by this path)
  Wave2 &w = c->w2;
  b.ray_o[0] = (float4 *)w.ray_o.p;
  b.ray_o[1] = b.ray_o[0] + w.capacity;
  b.ray_d[0] = (float4 *)w.ray_d.p;
  b.ray_d[1] = b.ray_d[0] + w.capacity;
  b.thr[0] = (float4 *)w.thr.p;
  b.thr[1] = b.thr[0] + w.capacity;
  for (int k = 0; k < 3; ++k) b.L[k] = (float4 *)w.L.p + (size_t)k * w.capacity;
  b.prev[0] = (float4 *)w.prev.p;
  b.prev[1] = b.prev[0] + w.capacity;
  for (int k = 0; k < 3; ++k) b.misc[k] = (uint4 *)w.misc.p + (size_t)k * w.capacity;
  b.pos = (float2 *)w.pos.p;
  b.hit = (float4 *)w.hit.p;
  b.queue[0] = (uint32_t *)w.q0.p;
  b.queue[1] = (uint32_t *)w.q1.p;
  b.shadow = (mtxd::ShadowRec *)w.shadow.p;
  b.counters = (uint32_t *)w.counters.p;
  b.xheads = (uint32_t *)w.xheads.p;
  b.capacity = w.capacity;
  b.cq_p = (float4 *)w.cq_p.p;  // null unless ensure_cache2
  b.cq_d = (float4 *)w.cq_d.p;
  b.cq_t = (float4 *)w.cq_t.p;
  b.cq_count = (uint32_t *)w.cq_count.p;
  return b;
}

// Zeroes a chunk's queue counters and the per-XCD claim cursors.
hipError_t reset_counters(const mtxd::WaveBuffers &b, uint32_t depth, hipStream_t st) {
  hipError_t e = hipMemsetAsync(b.counters, 0, 16ull * (depth + 2), st);
  if (e != hipSuccess) return e;
  return hipMemsetAsync(b.xheads, 0, 8ull * mtxd::kXSlotWords * (depth + 2), st);
}

int ensure_mlt(mtx_ctx *c, uint32_t cap, uint32_t max_depth, bool emitter_samples) {
  int rc;
  if (emitter_samples && (!c->vpath_es.p || c->mlt_es_capacity != c->capacity || max_depth > c->mlt_es_depth)) {
    const size_t wc = c->capacity;
    if ((rc = dalloc(c->vpath_es, 8 * wc * max_depth))) return rc;
    if ((rc = dalloc(c->vprop_es, 8 * wc * max_depth))) return rc;
    c->mlt_es_capacity = c->capacity;
    c->mlt_es_depth = max_depth;
  }
  if (cap > c->mlt_capacity || max_depth > c->mlt_depth || c->mlt_capacity != c->capacity) {
    // vertex buffers are indexed [depth * wavefront capacity + chain]
    const size_t wc = c->capacity;
    if ((rc = dalloc(c->mlt_cur, 16 * wc))) return rc;
    if ((rc = dalloc(c->mlt_L, 16 * wc))) return rc;
    if ((rc = dalloc(c->mlt_prop, 8 * wc))) return rc;
    if ((rc = dalloc(c->vpath, 16 * wc * max_depth))) return rc;
    if ((rc = dalloc(c->vprop, 16 * wc * max_depth))) return rc;
    c->mlt_capacity = c->capacity;
    c->mlt_depth = max_depth;
  }
  return MTX_OK;
}

// NRC radiance-cache buffers for `cap` paths (queries <= paths).
int ensure_cache(mtx_ctx *c, uint32_t cap) {
  int rc;
  if (!c->has_field) {
    mtx_set_error("mtx_render: NRC cache requested but no radiance field uploaded (mtx_field_upload)");
    return MTX_E_ARG;
  }
  if ((rc = dalloc(c->cq_p, 16ull * cap))) return rc;
  if ((rc = dalloc(c->cq_d, 16ull * cap))) return rc;
  if ((rc = dalloc(c->cq_t, 16ull * cap))) return rc;
  if ((rc = dalloc(c->cq_count, 16))) return rc;
  if ((rc = dalloc(c->f_feat, 128ull * cap))) return rc;
  if ((rc = dalloc(c->f_out, 12ull * cap))) return rc;
  return MTX_OK;
}

// The second wavefront's cache-query buffers (two-stream NRC + cache render).
int ensure_cache2(mtx_ctx *c, uint32_t cap) {
  int rc;
  Wave2 &w = c->w2;
  if ((rc = dalloc(w.cq_p, 16ull * cap))) return rc;
  if ((rc = dalloc(w.cq_d, 16ull * cap))) return rc;
  if ((rc = dalloc(w.cq_t, 16ull * cap))) return rc;
  if ((rc = dalloc(w.cq_count, 16))) return rc;
  if ((rc = dalloc(w.f_feat, 128ull * cap))) return rc;
  if ((rc = dalloc(w.f_out, 12ull * cap))) return rc;
  return MTX_OK;
}

int check_args(mtx_ctx *c, const mtx_render_args *a) {
  if (!c || !a) {
    mtx_set_error("null context or args");
    return MTX_E_ARG;
  }
  if (!c->has_scene) {
    mtx_set_error("no scene uploaded");
    return MTX_E_NOSCENE;
  }
  if (a->integrator != MTX_INT_PATH && a->integrator != MTX_INT_PATH_MIS && a->integrator != MTX_INT_NRC &&
      a->integrator != MTX_INT_PSSMLT_SIMPLE && a->integrator != MTX_INT_RESTIR_GI &&
      a->integrator != MTX_INT_PSSMLT_PATH && a->integrator != MTX_INT_NERAD && a->integrator != MTX_INT_SIMPLE) {
    mtx_set_error("integrator %u is not supported by this entry point", a->integrator);
    return MTX_E_UNSUPPORTED;
  }
  if (a->max_depth > 0xfffe) {
    mtx_set_error("max_depth %u too large", a->max_depth);
    return MTX_E_ARG;
  }
  return MTX_OK;
}

constexpr uint32_t kQSlots = 4096;  // chunks whose cache-query counts one stats render records

// Event-pair timer per kernel class.
struct Timer {
  mtx_ctx *c;
  bool on;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pairs[6];  // trace, shadow, shade, all, encode, mlp
  uint64_t cache_queries = 0;
  uint32_t q_used = 0;  // chunk query counts copied (asynchronously) into c->q_pinned
  uint32_t streams = 1;  // wavefronts / streams of the render (mtx_stats.streams)
  size_t next = 0;
  hipEvent_t get() {
    if (next >= c->events.size()) {
      hipEvent_t e;
      hipEventCreate(&e);
      c->events.push_back(e);
    }
    return c->events[next++];
  }
  hipEvent_t begin(int k, hipStream_t st = nullptr) {
    if (!on) return nullptr;
    hipEvent_t e0 = get();
    hipEventRecord(e0, st ? st : c->stream);
    return e0;
  }
  void end(int k, hipEvent_t e0, hipStream_t st = nullptr) {
    if (!on) return;
    hipEvent_t e1 = get();
    hipEventRecord(e1, st ? st : c->stream);
    pairs[k].push_back({e0, e1});
  }
  double total(int k) {
    double ms = 0;
    for (auto &p : pairs[k]) {
      float t = 0;
      hipEventElapsedTime(&t, p.first, p.second);
      ms += t;
    }
    return ms;
  }
};

// Encode + MLP + L += T * out for the chunk's compacted cache queries (on
// `stream` with the feature / output buffers of the chunk's wavefront: the
// context's by default, the second wavefront's in a two-stream render).
int run_cache(mtx_ctx *c, const mtxd::WaveBuffers &b, uint32_t cap, Timer &tm, bool nerad_render = false,
               hipStream_t stream = nullptr, DevBuf *feat = nullptr, DevBuf *out = nullptr, DevBuf *perm_buf = nullptr,
               DevBuf *cursor_buf = nullptr) {
  hipStream_t st = stream ? stream : c->stream;
  DevBuf &f_feat = feat ? *feat : c->f_feat, &f_out = out ? *out : c->f_out;
  const uint32_t *perm = nullptr;
  int xcd_split = 0;
  hipEvent_t e = tm.begin(4, st);
  if (c->cache_sort == 2 && !nerad_render) {
    // region-grouped rows, the blocks of each XCD on one eighth of them
    // (field.hip k_field_encode xcd_split): device-only, no host round trip
    DevBuf &pb = perm_buf ? *perm_buf : c->cq_perm, &cb = cursor_buf ? *cursor_buf : c->cq_keys;
    if (!dalloc(pb, 4ull * cap) && !dalloc(cb, 4ull * 32768)) {
      mtxd::field_bucket_queries(c->field, b.cq_p, b.cq_count, cap, (uint32_t *)cb.p, (uint32_t *)pb.p, c->n_cu, st);
      perm = (const uint32_t *)pb.p;
      xcd_split = 1;
    }
  } else if (c->cache_sort && !nerad_render && st == c->stream) {
    // encode the queries in Morton order (a stable sort of 24-bit cell codes
    // with the hash-grid group-by): the hash-grid corner gathers of
    // neighbouring rows then share table lines. The MLP row order follows;
    // k_cache_apply maps row q back to query perm[q]. Results are unchanged
    // (every query's features and MLP column are its own).
    uint32_t nq = 0;
    if (hipMemcpyAsync(&nq, b.cq_count, 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
        hipStreamSynchronize(c->stream) == hipSuccess && nq > 0 && !dalloc(c->cq_keys, 4ull * nq) &&
        !dalloc(c->cq_perm, 4ull * nq) && !dalloc(c->cq_ws, mtxd::sort24_workspace_bytes(nq))) {
      mtxd::field_morton_keys(c->field, b.cq_p, nq, (uint32_t *)c->cq_keys.p, c->stream);
      if (mtxd::sort24((const uint32_t *)c->cq_keys.p, nq, (uint32_t *)c->cq_perm.p, c->cq_ws.p, c->stream) ==
          MTX_OK)
        perm = (const uint32_t *)c->cq_perm.p;
    }
  }
  // the fused pass only when its LDS fits a workgroup (n_hidden <= 14)
  const bool fused = c->cache_fused && !nerad_render && mtxd::field_cache_fused_lds(c->field_hidden) <= c->max_lds;
  int rc = MTX_OK;
  if (fused) {
    // encode + MLP + L += T * out in one launch (field.hip k_field_cache_fused),
    // timed as the encode
    rc = mtxd::field_cache_fused(c->field, b.cq_p, b.cq_d, b.cq_t, b.cq_count, cap, perm, xcd_split,
                                 c->field_frag.p, c->field_hidden, b.L[mtxd::kFinal], c->n_cu, st);
    tm.end(4, e, st);
    if (rc) return rc;
  } else {
    rc = mtxd::field_encode(c->field, b.cq_p, b.cq_d, b.cq_count, cap, (uint16_t *)f_feat.p, st, perm, xcd_split,
                            (int)c->encode_lm);
    tm.end(4, e, st);
    if (rc) return rc;
    e = tm.begin(5, st);
    rc = mtxd::field_mlp((const uint16_t *)f_feat.p, b.cq_count, cap, c->field_frag.p, c->field_hidden,
                         (float *)f_out.p, c->n_cu, st);
    tm.end(5, e, st);
    if (rc) return rc;
    if (nerad_render)
      mtxd::launch_nerad_apply(b, (const float *)f_out.p, cap, 1, st);
    else
      mtxd::launch_cache_apply(b, (const float *)f_out.p, cap, st, perm);
    HIP_TRY(hipGetLastError());
  }
  if (tm.on) {  // counted after the render's final synchronisation (fill_stats): no per-chunk sync
    if (!c->q_pinned && hipHostMalloc((void **)&c->q_pinned, 4 * kQSlots) != hipSuccess) c->q_pinned = nullptr;
    if (c->q_pinned && tm.q_used < kQSlots) {
      hipMemcpyAsync(c->q_pinned + tm.q_used++, b.cq_count, 4, hipMemcpyDeviceToHost, st);
    } else {  // more chunks than pinned slots: count this one synchronously (never dropped)
      uint32_t nq = 0;
      if (hipMemcpyAsync(&nq, b.cq_count, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
          hipStreamSynchronize(st) == hipSuccess)
        tm.cache_queries += nq;
    }
  }
  return MTX_OK;
}

// One bounce of a chunk: closest hit, shade, NEE shadow rays.
void launch_bounce(mtx_ctx *c, const mtxd::WaveBuffers &b, const mtxd::ChunkParams &p, Timer &tm,
                   uint64_t *n_trace, uint64_t *n_shadow, const mtxd::DevScene &s, hipStream_t st, uint32_t bounce) {
  // nerad RHS lanes start at their surface point (no bounce-0 trace) and
  // trace NEE rays at that point only
  const bool nerad = p.integrator == MTX_INT_NERAD_RHS, nerad_render = p.integrator == MTX_INT_NERAD;
  hipEvent_t e;
  // past its second vertex the nerad RHS chain only continues through
  // delta surfaces (next_smooth_si): a small queue, traced and shaded by
  // an eighth of the persistent grid (dispatching the full grid of
  // immediately-exiting blocks costs more than the work)
  const int div = (nerad && bounce >= 2) ? 8 : 1;
  if (!(nerad && bounce == 0)) {
    e = tm.begin(0, st);
    mtxd::launch_trace_closest(s, b, bounce, p.stats, std::max(1, c->closest_grid / div), st);
    tm.end(0, e, st);
    ++*n_trace;
  }
  e = tm.begin(2, st);
  mtxd::launch_shade(s, b, p, bounce, std::max(1, c->shade_grid / div), st);
  tm.end(2, e, st);
  if (p.integrator != MTX_INT_PSSMLT_SIMPLE && p.integrator != MTX_INT_SIMPLE && !nerad_render &&
      !(nerad && bounce > 0)) {  // PSSMLT, simple and the nerad render trace no NEE rays
    e = tm.begin(1, st);
    mtxd::launch_trace_shadow(s, b, bounce, p.stats, c->trace_grid, st);
    tm.end(1, e, st);
    ++*n_shadow;
  }
}

// Bounces of a chunk's loop (an NRC cache query needs one more trace + shade
// after the last segment).
uint32_t bounce_iters(const mtxd::ChunkParams &p) {
  return std::max<uint32_t>(p.max_depth, 1) + (p.nrc_cache ? 1u : 0u);
}

// Paths a depth limit left queued keep their result in a queue plane.
void finish_bounces(const mtxd::WaveBuffers &b, const mtxd::ChunkParams &p, hipStream_t st) {
  if (p.integrator != MTX_INT_NERAD_RHS && p.integrator != MTX_INT_NERAD)
    mtxd::launch_flush_tail(b, bounce_iters(p), b.capacity, p.integrator, st);
}

// Runs one chunk's bounce loop (rays already generated, counters[0] set).
void run_bounces(mtx_ctx *c, const mtxd::WaveBuffers &b, const mtxd::ChunkParams &p, Timer &tm,
                 uint64_t *n_trace, uint64_t *n_shadow, const mtxd::DevScene *scene = nullptr,
                 hipStream_t stream = nullptr) {
  const mtxd::DevScene &s = scene ? *scene : c->scene;
  hipStream_t st = stream ? stream : c->stream;
  const uint32_t depth_iters = bounce_iters(p);
  for (uint32_t bounce = 0; bounce < depth_iters; ++bounce) {
    launch_bounce(c, b, p, tm, n_trace, n_shadow, s, st, bounce);
    // Deep paths (max_depth 65, scene.xml:6): stop launching once the queue
    // has drained (checked every 8 bounces).
    if (depth_iters > 16 && (bounce & 7) == 7 && bounce + 1 < depth_iters) {
      uint32_t cnt = 0;
      hipMemcpyAsync(&cnt, b.counters + 4 * (bounce + 1), 4, hipMemcpyDeviceToHost, st);
      hipStreamSynchronize(st);
      if (cnt == 0) return;
    }
  }
  finish_bounces(b, p, st);
}

int fill_stats(mtx_ctx *c, mtx_stats *stats, bool want_stats, Timer &tm, uint64_t n_trace, uint64_t n_shadow,
               uint64_t paths) {
  if (!stats) return MTX_OK;
  memset(stats, 0, sizeof(*stats));
  if (want_stats) {
    unsigned long long h[8];
    HIP_TRY(hipMemcpy(h, c->stats.p, 64, hipMemcpyDeviceToHost));
    stats->nodes_closest = h[0];
    stats->tris_closest = h[1];
    stats->nodes_shadow = h[2];
    stats->tris_shadow = h[3];
    stats->rays_closest = h[4];
    stats->rays_shadow = h[5];
    stats->wave_node_iters = h[6];
    stats->wave_leaf_iters = h[7];
  }
  stats->trace_launches = n_trace;
  stats->shadow_launches = n_shadow;
  stats->streams = tm.streams;
  stats->paths = paths;
  if (tm.on) {
    stats->trace_ms = tm.total(0);
    stats->shadow_ms = tm.total(1);
    stats->shade_ms = tm.total(2);
    stats->cache_encode_ms = tm.total(4);
    stats->cache_mlp_ms = tm.total(5);
    for (uint32_t i = 0; i < tm.q_used; ++i) tm.cache_queries += c->q_pinned[i];
    stats->cache_queries = tm.cache_queries;
    stats->other_ms = tm.total(3) - stats->trace_ms - stats->shadow_ms - stats->shade_ms - stats->cache_encode_ms -
                      stats->cache_mlp_ms;
  }
  return MTX_OK;
}

int ensure_restir(mtx_ctx *c, uint32_t n) {
  int rc;
  if (c->rs_n != n) {
    c->rs_valid = false;
    const size_t N = n;
    for (int k = 0; k < 2; ++k)
      if ((rc = dalloc(c->rs_samp[k], 5 * 16 * N))) return rc;
    if ((rc = dalloc(c->rs_tres, 6 * 16 * N))) return rc;
    if ((rc = dalloc(c->rs_sres, 6 * 16 * N))) return rc;
    if ((rc = dalloc(c->rs_radius, 4 * N))) return rc;
    if ((rc = dalloc(c->rs_hit, 16 * N))) return rc;
    if ((rc = dalloc(c->rs_dir, 16 * N))) return rc;
    if ((rc = dalloc(c->rs_emit, 16 * N))) return rc;
    if ((rc = dalloc(c->rs_rng, 16 * N))) return rc;
    if ((rc = dalloc(c->rs_rays, 9 * 32 * N))) return rc;
    if ((rc = dalloc(c->rs_count, 16))) return rc;
    if ((rc = dalloc(c->rs_heads, 4ull * mtxd::kXSlotWords))) return rc;
    if ((rc = dalloc(c->rs_occ, 18 * N))) return rc;
    if ((rc = dalloc(c->rs_qM, 10 * 4 * N))) return rc;
    if ((rc = dalloc(c->rs_nbr, 10 * 4 * N))) return rc;
    if ((rc = dalloc(c->rs_xs, 16 * N))) return rc;
    if ((rc = dalloc(c->rs_ns, 16 * N))) return rc;
    c->rs_n = n;
  }
  return MTX_OK;
}

// One RestirIntegrator.render() frame (restirgi.py:182-258) over the whole
// film; the kernel sequence is documented in restir.hip.
int render_restir(mtx_ctx *c, const mtx_render_args *a, float4 *film_dev, Timer &tm, uint64_t *n_trace,
                  uint64_t *n_shadow, bool want_stats) {
  const mtx_camera &cam = c->scene.camera;
  const uint32_t W = cam.width, H = cam.height, spp = a->spp;
  if (a->sample_offset != 0 || a->spp_total != spp) {
    mtx_set_error("mtx_render: ReSTIR GI needs spp_total = spp and sample_offset = 0");
    return MTX_E_ARG;
  }
  if (c->scene.has_env) {
    // restirgi.py's reservoirs keep the first secondary hit (x_s, n_s) and
    // its visibility; a secondary ray escaping to an environment has no such
    // point, and the reference's handling of it is not restated here
    mtx_set_error("mtx_render: ReSTIR GI with an environment emitter is not supported");
    return MTX_E_UNSUPPORTED;
  }
  const uint64_t n64 = (uint64_t)W * H * spp;
  if (n64 * 18 >= (1ull << 32)) {
    mtx_set_error("mtx_render: ReSTIR GI frame too large (%llu lanes)", (unsigned long long)n64);
    return MTX_E_ARG;
  }
  const bool only_a = (a->restir_flags & MTX_RESTIR_STAGE_A) != 0;
  const bool only_b = (a->restir_flags & MTX_RESTIR_STAGE_B) != 0;
  if (only_a && only_b) {
    mtx_set_error("mtx_render: ReSTIR stage A and stage B flags are exclusive");
    return MTX_E_ARG;
  }
  const bool run_a = !only_b, run_b = !only_a;
  const uint32_t n = (uint32_t)n64;
  const uint32_t lane0 = a->y0 * W * spp, nb = (a->y1 - a->y0) * W * spp;
  const uint32_t depth = std::max<uint32_t>(a->max_depth, 1);
  int rc;
  if ((rc = ensure_wavefront(c, nb, depth))) return rc;
  if ((rc = ensure_restir(c, n))) return rc;
  if (run_a && a->frame != 0 && !c->rs_valid) {
    mtx_set_error("mtx_render: ReSTIR GI frame %u without the state of frame 0 (film size or scene changed?)",
                  a->frame);
    return MTX_E_ARG;
  }
  if (only_b && (!c->rs_pending_b || c->rs_pending_frame != a->frame)) {
    mtx_set_error("mtx_render: ReSTIR stage B of frame %u without its stage A", a->frame);
    return MTX_E_ARG;
  }
  hipStream_t st = c->stream;
  if (run_a && a->frame == 0) {  // restirgi.py:217-229
    HIP_TRY(hipMemsetAsync(c->rs_tres.p, 0, 6 * 16 * (size_t)n, st));
    HIP_TRY(hipMemsetAsync(c->rs_sres.p, 0, 6 * 16 * (size_t)n, st));
    HIP_TRY(hipMemsetAsync(c->rs_samp[0].p, 0, 5 * 16 * (size_t)n, st));
    HIP_TRY(hipMemsetAsync(c->rs_samp[1].p, 0, 5 * 16 * (size_t)n, st));
    uint32_t bits;
    memcpy(&bits, &a->initial_search_radius, 4);
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)c->rs_radius.p, (int)bits, n, st));
    c->rs_prev_cam = cam;
    c->rs_cur = 0;
  }
  mtxd::WaveBuffers b = buffers(c);
  mtxd::RestirBuffers r{};
  r.cur = (float4 *)c->rs_samp[c->rs_cur].p;
  r.prev = a->frame == 0 ? r.cur : (const float4 *)c->rs_samp[c->rs_cur ^ 1].p;
  r.tres = (float4 *)c->rs_tres.p;
  r.sres = (float4 *)c->rs_sres.p;
  r.radius = (float *)c->rs_radius.p;
  r.prim_hit = (float4 *)c->rs_hit.p;
  r.prim_dir = (float4 *)c->rs_dir.p;
  r.emit = (float4 *)c->rs_emit.p;
  r.rng = (uint4 *)c->rs_rng.p;
  r.test_rays = (float4 *)c->rs_rays.p;
  r.test_count = (uint32_t *)c->rs_count.p;
  r.test_heads = (uint32_t *)c->rs_heads.p;
  r.occ = (uint8_t *)c->rs_occ.p;
  r.qM = (uint32_t *)c->rs_qM.p;
  r.nbr = (uint32_t *)c->rs_nbr.p;
  r.n = n;
  r.lane0 = lane0;
  r.nb = nb;
  r.prev_cam = c->rs_prev_cam;
  r.flags = a->restir_flags;
  r.xcd_remap = c->xcd_claim;
  r.max_M_temporal = a->max_M_temporal;
  r.max_M_spatial = a->max_M_spatial;
  r.initial_radius = a->initial_search_radius;
  r.minimal_radius = a->minimal_search_radius;
  r.frame = a->frame;
  b.rs_xs = (float4 *)c->rs_xs.p;
  b.rs_ns = (float4 *)c->rs_ns.p;

  mtxd::ChunkParams p{};
  p.integrator = MTX_INT_RESTIR_GI;
  p.max_depth = a->max_depth;
  p.rr_depth = a->rr_depth;
  p.seed = a->seed;
  p.spp = spp;
  p.spp_total = spp;
  p.width = W;
  p.height = H;
  p.px0 = a->y0 * W;
  p.n_px = (a->y1 - a->y0) * W;
  p.band_y0 = a->y0;
  p.band_px = (a->y1 - a->y0) * W;
  p.n_paths = nb;
  p.restir = 1;
  p.stats = want_stats ? 1 : 0;
  if (want_stats) HIP_TRY(hipMemsetAsync(c->stats.p, 0, 64, c->stream));
  hipEvent_t e;
  if (run_a) {
    // Stage A is per lane up to and including the temporal resampling (which
    // reads this frame's lane and the complete previous frame), so the band's
    // rows split into two halves traced on two wavefronts / streams: one
    // half's kernels fill the tails of the other's short (~2 M-ray)
    // persistent launches. Same lanes, same draws: bit-identical.
    // A band of at most mega_max paths (default: twice the megakernel's
    // resident lanes, 2 x mega_grid x kShadeBlock) runs all of its secondary
    // paths in the path megakernel on ONE wavefront instead (the band is not
    // split into halves then): one launch of at most the resident blocks,
    // whose waves claim the queued paths 64 at a time.
    const uint32_t rows = a->y1 - a->y0;
    const uint32_t mega_max =
        c->mega_paths == 0xffffffffu ? 2u * (uint32_t)c->mega_grid * mtxd::kShadeBlock : c->mega_paths;
    const bool mega_all = !p.stats && nb <= mega_max;
    const bool two = !mega_all && c->streams > 1 && rows >= 2 && nb >= (1u << 16);
    if (two) tm.streams = 2;
    const uint32_t ym = two ? a->y0 + rows / 2 : a->y1;
    mtxd::DevScene s2 = c->scene;
    mtxd::WaveBuffers bw2{};
    if (two) {
      if ((rc = ensure_wavefront2(c, (a->y1 - ym) * W * spp, depth))) return rc;
      bw2 = buffers2(c);
      s2.stack_ovf = c->w2.stack_ovf.p;
      HIP_TRY(hipEventRecord(c->w2.start, st));  // after the frame-0 clears
      HIP_TRY(hipStreamWaitEvent(c->w2.stream, c->w2.start, 0));
    }
    // The halves' launches are enqueued interleaved, step by step (prologue,
    // each bounce, epilogue), so the second stream starts at once instead of
    // after the host has queued all of the first half's launches.
    const int halves = two ? 2 : 1;
    hipStream_t sh[2] = {st, c->w2.stream};
    if (mega_all && c->rs_fused) {
      // the whole stage A up to k_rs_collect in one per-lane launch
      // (kernels.hip k_rs_stage_a), then the temporal pass
      HIP_TRY(reset_counters(b, depth, st));
      e = tm.begin(0, st);
      mtxd::launch_rs_stage_a(c->scene, b, p, r,
                              std::max(1, std::min<int>(c->mega_grid, (nb + mtxd::kShadeBlock - 1) / mtxd::kShadeBlock)),
                              st);
      tm.end(0, e, st);
      ++*n_trace;
      mtxd::launch_restir_temporal(r, p, st);
    }
    const bool fused = mega_all && c->rs_fused;
    const mtxd::DevScene *sc[2] = {&c->scene, &s2};
    mtxd::WaveBuffers bh[2], b1[2];
    mtxd::ChunkParams ph[2];
    mtxd::RestirBuffers rh[2];
    for (int h = 0; h < (fused ? 0 : halves); ++h) {
      const uint32_t ya = h ? ym : a->y0, yb = h ? a->y1 : ym;
      bh[h] = h ? bw2 : b;
      bh[h].rs_xs = b.rs_xs + (size_t)(ya - a->y0) * W * spp;  // path-indexed within the half
      bh[h].rs_ns = b.rs_ns + (size_t)(ya - a->y0) * W * spp;
      ph[h] = p;
      ph[h].px0 = ya * W;
      ph[h].n_px = (yb - ya) * W;
      ph[h].n_paths = ph[h].n_px * spp;
      rh[h] = r;
      rh[h].lane0 = ya * W * spp;
      rh[h].nb = ph[h].n_paths;
      // sample_initial: primary rays and their closest hits
      HIP_TRY(reset_counters(bh[h], depth, sh[h]));
      mtxd::launch_raygen_camera(*sc[h], bh[h], ph[h], sh[h]);
      e = tm.begin(0, sh[h]);
      mtxd::launch_trace_closest(*sc[h], bh[h], 0, ph[h].stats, c->closest_grid, sh[h]);
      tm.end(0, e, sh[h]);
      ++*n_trace;
      HIP_TRY(reset_counters(bh[h], depth, sh[h]));
      mtxd::launch_restir_begin(*sc[h], bh[h], ph[h], rh[h], sh[h]);
      b1[h] = bh[h];  // k_rs_begin left the secondary rays in the parity-1 planes
      b1[h].ray_par = 1;
    }
    // sample_ray (the path-mis loop): with mega_all (halves == 1) the whole
    // band runs all its bounces in the path megakernel (no counters: STATS
    // renders keep the wavefront kernels)
    bool mega[2] = {false, false};
    for (int h = 0; h < (fused ? 0 : halves); ++h) {
      mega[h] = mega_all;
      if (!mega[h]) continue;
      e = tm.begin(0, sh[h]);
      mtxd::launch_path_mega(*sc[h], b1[h], ph[h],
                             std::max(1, std::min<int>(c->mega_grid, (ph[h].n_paths + mtxd::kShadeBlock - 1) /
                                                                         mtxd::kShadeBlock)),
                             sh[h]);
      tm.end(0, e, sh[h]);
      ++*n_trace;
    }
    const uint32_t iters = fused ? 0u : bounce_iters(p);
    for (uint32_t bounce = 0; bounce < iters; ++bounce)
      for (int h = 0; h < halves; ++h)
        if (!mega[h]) launch_bounce(c, b1[h], ph[h], tm, n_trace, n_shadow, *sc[h], sh[h], bounce);
    for (int h = 0; h < (fused ? 0 : halves); ++h) {
      if (!mega[h]) finish_bounces(b1[h], ph[h], sh[h]);
      mtxd::launch_restir_collect(bh[h], ph[h], rh[h], sh[h]);
      mtxd::launch_restir_temporal(rh[h], ph[h], sh[h]);
    }
    if (two) {  // stage B reads every lane of the band
      HIP_TRY(hipEventRecord(c->w2.done, c->w2.stream));
      HIP_TRY(hipStreamWaitEvent(st, c->w2.done, 0));
    }
  }
  if (run_b) {
    // spatial_resampling (reads samples / temporal reservoirs of rows outside
    // the band: a row-banded caller imports them between stage A and B)
    HIP_TRY(hipMemsetAsync(r.test_count, 0, 16, st));
    HIP_TRY(hipMemsetAsync(r.test_heads, 0, 4ull * mtxd::kXSlotWords, st));
    mtxd::launch_restir_spatial_rays(r, p, st);
    e = tm.begin(1);
    mtxd::launch_trace_test(c->scene, r, 0, c->trace_grid, st);
    tm.end(1, e);
    ++*n_shadow;
    HIP_TRY(hipMemsetAsync(r.test_count, 0, 16, st));
    HIP_TRY(hipMemsetAsync(r.test_heads, 0, 4ull * mtxd::kXSlotWords, st));
    mtxd::launch_restir_spatial_merge(r, p, st);
    if (a->restir_flags & MTX_RESTIR_BIAS_CORRECTION) {
      e = tm.begin(1);
      mtxd::launch_trace_test(c->scene, r, 9 * n, c->trace_grid, st);
      tm.end(1, e);
      ++*n_shadow;
      mtxd::launch_restir_bias_finish(r, p, st);
    }
    mtxd::launch_restir_final(c->scene, b, p, r, st);
    mtxd::launch_film_src(b, p, (float4 *)c->contrib.p, st);
    mtxd::launch_film_gather((const float4 *)c->contrib.p, film_dev, W, a->y0, a->y1, 1, 1u, st);
  }
  HIP_TRY(hipGetLastError());
  if (only_a) {
    c->rs_pending_b = true;
    c->rs_pending_frame = a->frame;
    c->rs_valid = a->frame != 0 ? c->rs_valid : false;
    return MTX_OK;
  }
  // restirgi.py:245-247: prev_sensor <- sensor, prev_sample <- sample
  c->rs_pending_b = false;
  c->rs_prev_cam = cam;
  c->rs_cur ^= 1;
  c->rs_valid = true;
  return MTX_OK;
}

}  // namespace

extern "C" {

int mtx_render(mtx_ctx *c, const mtx_render_args *a, float *film_rgbw, int film_on_device, mtx_stats *stats) {
  int rc = check_args(c, a);
  if (rc) return rc;
  const mtx_camera &cam = c->scene.camera;
  const uint32_t W = cam.width, H = cam.height;
  if (!film_rgbw || a->spp == 0 || a->y1 <= a->y0 || a->y1 > H || a->spp_total < a->sample_offset + a->spp) {
    mtx_set_error("mtx_render: bad film/rows/spp arguments");
    return MTX_E_ARG;
  }
  if ((uint64_t)W * H * a->spp_total >= (1ull << 32)) {
    mtx_set_error("mtx_render: W*H*spp_total exceeds the 32-bit sampler lane space");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  const uint32_t band_px = (a->y1 - a->y0) * W;
  const bool nrc_cache = a->integrator == MTX_INT_NRC && (a->flags & 4u);
  const bool nerad_render = a->integrator == MTX_INT_NERAD;
  const bool mlt = a->integrator == MTX_INT_PSSMLT_SIMPLE || a->integrator == MTX_INT_PSSMLT_PATH;
  // two wavefronts on two streams (Wave2): the band splits into at least two
  // chunks that alternate between them (the caller's chunk size still caps a
  // chunk), so one chunk's kernels fill the tails of the other's persistent
  // trace launches (~0.2 ms per launch that does not shrink with the rays).
  // Renders of 2^16 .. 2^27 paths: the bench's per-rank share at N >= 2
  // (spp 32: 26.8 -> 25.9 ms per step; spp 128: 91.6 -> 90.2 ms); at spp 256
  // (2^27.8 paths) it gains 0.5 % and would blur the per-kernel event times
  // the N = 1 roofline is measured with. Path-state integrators without a
  // per-chunk cache pass only.
  const uint64_t n_paths_all = (uint64_t)band_px * a->spp;
  // (NRC + cache: each wavefront has its own query / feature buffers, so one
  // chunk's cache pass overlaps the other's bounces; not with the Morton sort)
  const bool two = c->streams > 1 && !mlt && !(nrc_cache && c->cache_sort == 1) && !nerad_render &&
                   a->integrator != MTX_INT_RESTIR_GI && n_paths_all >= (1u << 16) &&
                   n_paths_all <= (1ull << c->streams_max_log2);
  // the default chunk is sized for every wavefront the render allocates
  const uint32_t chunk_paths =
      a->chunk_paths ? a->chunk_paths : default_chunk(c, a, two ? 2u : 1u, nrc_cache || nerad_render);
  uint32_t px_per_chunk = std::min(std::max<uint32_t>(1, chunk_paths / a->spp), band_px);
  if (two) px_per_chunk = std::min(px_per_chunk, (band_px + 1) / 2);
  const uint32_t cap = px_per_chunk * a->spp;
  if ((rc = ensure_wavefront(c, cap, std::max<uint32_t>(a->max_depth, 1)))) return rc;
  if (two && (rc = ensure_wavefront2(c, cap, std::max<uint32_t>(a->max_depth, 1)))) return rc;
  if ((nrc_cache || nerad_render) && (rc = ensure_cache(c, cap))) return rc;
  if (two && nrc_cache && (rc = ensure_cache2(c, cap))) return rc;
  // sample-sharded film renders: 8 partial slots (GPU-count-invariant films,
  // DESIGN.md "Film"); PSSMLT splats and ReSTIR frames: one
  const uint32_t film_slots = (mlt || a->integrator == MTX_INT_RESTIR_GI) ? 1u : 8u;
  // the slots [sample_offset, sample_offset + spp) falls in (FilmSlots: slot k
  // takes global samples [end(k - 1), end(k)), slot 7 everything past end(6))
  uint32_t slot_mask = 1u;
  if (film_slots == 8) {
    slot_mask = 0;
    for (uint32_t k = 0; k < 8; ++k) {
      const uint64_t lo = k ? mtx::film_slot_end(k - 1, a->spp_total) : 0u;
      const uint64_t hi = k < 7 ? mtx::film_slot_end(k, a->spp_total) : ~0ull;
      if (std::max<uint64_t>(lo, a->sample_offset) < std::min<uint64_t>(hi, (uint64_t)a->sample_offset + a->spp))
        slot_mask |= 1u << k;
    }
  }
  if ((rc = dalloc(c->contrib, 9ull * 16 * band_px * film_slots))) return rc;
  const size_t film_floats = 4ull * (W + 2) * (a->y1 - a->y0 + 2);
  float4 *film_dev = (float4 *)film_rgbw;
  if (!film_on_device) {
    if ((rc = dalloc(c->film, film_floats * 4))) return rc;
    film_dev = (float4 *)c->film.p;
  }
  const bool want_stats = stats && (a->flags & 1u);
  Timer tm{c, stats && (a->flags & 2u)};
  if (two) tm.streams = 2;
  if (a->integrator == MTX_INT_RESTIR_GI) {
    hipEvent_t e_all = tm.begin(3);
    uint64_t n_trace = 0, n_shadow = 0;
    if ((rc = render_restir(c, a, film_dev, tm, &n_trace, &n_shadow, want_stats))) return rc;
    tm.end(3, e_all);
    // stage A writes no film: no copy, and no wait unless stats were asked
    // for (the caller's stage B follows on the same stream)
    const bool stage_a = (a->restir_flags & MTX_RESTIR_STAGE_A) != 0;
    if (!film_on_device && !stage_a)
      HIP_TRY(hipMemcpyAsync(film_rgbw, film_dev, film_floats * 4, hipMemcpyDeviceToHost, c->stream));
    if (!stage_a || stats) HIP_TRY(hipStreamSynchronize(c->stream));
    return fill_stats(c, stats, want_stats, tm, n_trace, n_shadow, (uint64_t)W * H * a->spp);
  }
  if (mlt) {
    if ((rc = ensure_mlt(c, cap, std::max<uint32_t>(a->max_depth, 1), a->integrator == MTX_INT_PSSMLT_PATH)))
      return rc;
    HIP_TRY(hipMemsetAsync(c->contrib.p, 0, 9ull * 16 * band_px, c->stream));
  }
  mtxd::WaveBuffers b = buffers(c);
  if (want_stats) HIP_TRY(hipMemsetAsync(b.stats, 0, 64, c->stream));
  uint64_t n_trace = 0, n_shadow = 0;
  hipEvent_t e_all = tm.begin(3);
  mtxd::WaveBuffers b2{};
  mtxd::DevScene s2{};
  if (two) {
    // the second stream starts after everything queued on the first
    b2 = buffers2(c);
    s2 = c->scene;
    s2.stack_ovf = c->w2.stack_ovf.p;
    HIP_TRY(hipEventRecord(c->w2.start, c->stream));
    HIP_TRY(hipStreamWaitEvent(c->w2.stream, c->w2.start, 0));
  }
  uint32_t chunk_index = 0;
  for (uint32_t px0 = a->y0 * W; px0 < a->y1 * W; px0 += px_per_chunk, ++chunk_index) {
    const bool second = two && (chunk_index & 1u);
    hipStream_t st = second ? c->w2.stream : c->stream;
    const mtxd::WaveBuffers &bc = second ? b2 : b;
    const mtxd::DevScene &sc = second ? s2 : c->scene;
    mtxd::ChunkParams p{};
    p.integrator = a->integrator;
    p.max_depth = a->max_depth;
    p.rr_depth = a->rr_depth;
    p.seed = a->seed;
    p.spp = a->spp;
    p.spp_total = a->spp_total;
    p.sample_offset = a->sample_offset;
    p.width = W;
    p.height = H;
    p.px0 = px0;
    p.n_px = std::min(px_per_chunk, a->y1 * W - px0);
    p.band_y0 = a->y0;
    p.band_px = (a->y1 - a->y0) * W;
    p.film_slots = film_slots;
    p.slot_mask = slot_mask;
    p.n_paths = p.n_px * a->spp;
    p.nrc_c = a->nrc_c;
    p.stats = want_stats ? 1 : 0;
      p.nrc_cache = nrc_cache ? 1u : 0u;
    // the film (and the cache apply) read an ending path's L only; PSSMLT's
    // chain kernels read its sampler state (mtx_sample_rays' k_collect and
    // ReSTIR's k_rs_collect build their own ChunkParams, which keep it)
    p.drop_end_misc = mlt ? 0u : 1u;
    p.ident0 = 1;  // raygen_camera / mlt_begin queue every path at its own position
    if (mlt) {
      // Pssmlt.render (pssmlt.py:167-228): all iterations of this chunk's chains
      const uint32_t iters = a->iterations ? a->iterations : 200;
      mtxd::launch_mlt_init(b, p, c->stream);
      for (uint32_t it = 0; it < iters; ++it) {
        p.large_step = (it % 50 == 0) ? 1u : 0u;  // reset_interval = 50 (:209)
        HIP_TRY(reset_counters(b, std::max<uint32_t>(a->max_depth, 1), c->stream));
        mtxd::launch_mlt_begin(c->scene, b, p, c->stream);
        run_bounces(c, b, p, tm, &n_trace, &n_shadow);
        mtxd::launch_mlt_end(b, p, c->stream);
        if (it % 50 > 40) mtxd::launch_mlt_film(b, p, (float4 *)c->contrib.p, c->stream);  // bootstrapping = 40
      }
      continue;
    }
    HIP_TRY(reset_counters(bc, std::max<uint32_t>(a->max_depth, 1), st));
    if (nrc_cache || nerad_render) HIP_TRY(hipMemsetAsync(bc.cq_count, 0, 4, st));
    mtxd::launch_raygen_camera(sc, bc, p, st);
    run_bounces(c, bc, p, tm, &n_trace, &n_shadow, &sc, st);
    if (nrc_cache) {
      if (second)
        rc = run_cache(c, bc, p.n_paths, tm, false, st, &c->w2.f_feat, &c->w2.f_out, &c->w2.cq_perm,
                       &c->w2.cq_cursor);
      else
        rc = run_cache(c, b, p.n_paths, tm);
      if (rc) return rc;
    }
    if (nerad_render && (rc = run_cache(c, b, p.n_paths, tm, true))) return rc;
    mtxd::launch_film_src(bc, p, (float4 *)c->contrib.p, st);
  }
  if (two) {  // the film gather reads both wavefronts' contributions
    HIP_TRY(hipEventRecord(c->w2.done, c->w2.stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->w2.done, 0));
  }
  mtxd::launch_film_gather((const float4 *)c->contrib.p, film_dev, W, a->y0, a->y1, film_slots, slot_mask, c->stream);
  tm.end(3, e_all);
  HIP_TRY(hipGetLastError());
  if (!film_on_device)
    HIP_TRY(hipMemcpyAsync(film_rgbw, film_dev, film_floats * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return fill_stats(c, stats, want_stats, tm, n_trace, n_shadow, (uint64_t)band_px * a->spp);
}

int mtx_set_camera(mtx_ctx *c, const mtx_camera *cam) {
  if (!c || !cam) {
    mtx_set_error("mtx_set_camera: null argument");
    return MTX_E_ARG;
  }
  if (!c->has_scene) {
    mtx_set_error("no scene uploaded");
    return MTX_E_NOSCENE;
  }
  if (cam->width != c->scene.camera.width || cam->height != c->scene.camera.height) {
    mtx_set_error("mtx_set_camera: film size changed (%ux%u -> %ux%u)", c->scene.camera.width,
                  c->scene.camera.height, cam->width, cam->height);
    return MTX_E_ARG;
  }
  c->scene.camera = *cam;
  return MTX_OK;
}

int mtx_restir_rows(mtx_ctx *c, int which, uint32_t row0, uint32_t nrows, void *buf, int to_state) {
  if (!c || !buf || which < 0 || which > 2) {
    mtx_set_error("mtx_restir_rows: bad argument");
    return MTX_E_ARG;
  }
  if (!c->rs_n || !c->has_scene) {
    mtx_set_error("mtx_restir_rows: no ReSTIR GI state");
    return MTX_E_ARG;
  }
  const uint32_t W = c->scene.camera.width, H = c->scene.camera.height;
  if (row0 + nrows > H || nrows == 0) {
    mtx_set_error("mtx_restir_rows: rows [%u, %u) outside the film", row0, row0 + nrows);
    return MTX_E_ARG;
  }
  const size_t n = c->rs_n, per_row = n / H;  // lanes per row (W * spp)
  (void)W;
  if (which == 2 && (!c->rs_valid || c->rs_pending_b)) {
    mtx_set_error("mtx_restir_rows: the previous frame's samples exist between complete frames only");
    return MTX_E_ARG;
  }
  const int planes = which == 1 ? 6 : 5;
  // which = 0: the current frame's samples (before stage B swaps them);
  // 2: the previous frame's (what k_rs_temporal reads through prev_cam)
  char *state = (char *)(which == 0 ? c->rs_samp[c->rs_cur].p
                                    : which == 2 ? c->rs_samp[c->rs_cur ^ 1].p : c->rs_tres.p);
  char *dev = (char *)buf;
  HIP_TRY(hipSetDevice(c->device));
  for (int k = 0; k < planes; ++k) {
    char *s = state + 16 * ((size_t)k * n + (size_t)row0 * per_row);
    char *d = dev + 16 * (size_t)k * nrows * per_row;
    const size_t bytes = 16 * (size_t)nrows * per_row;
    HIP_TRY(hipMemcpyAsync(to_state ? s : d, to_state ? d : s, bytes, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

int mtx_restir_state(mtx_ctx *c, int which, float *out, uint64_t n_floats) {
  if (!c || !out) {
    mtx_set_error("mtx_restir_state: null argument");
    return MTX_E_ARG;
  }
  if (!c->rs_valid) {
    mtx_set_error("mtx_restir_state: no ReSTIR GI frame rendered");
    return MTX_E_ARG;
  }
  const uint64_t n = c->rs_n;
  const void *src = nullptr;
  uint64_t need = 0;
  switch (which) {
    case 0: src = c->rs_samp[c->rs_cur ^ 1].p; need = 20 * n; break;  // the frame just rendered
    case 1: src = c->rs_tres.p; need = 24 * n; break;
    case 2: src = c->rs_sres.p; need = 24 * n; break;
    case 3: src = c->rs_radius.p; need = n; break;
    default:
      mtx_set_error("mtx_restir_state: which=%d not in 0..3", which);
      return MTX_E_ARG;
  }
  if (n_floats != need) {
    mtx_set_error("mtx_restir_state: need %llu floats, got %llu", (unsigned long long)need,
                  (unsigned long long)n_floats);
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpy(out, src, 4 * need, hipMemcpyDeviceToHost));
  return MTX_OK;
}

// Device-pointer entry points (the *_dev functions of mtx.h): every buffer
// must be memory of the context's device (hipMalloc'd, e.g. a torch CUDA
// tensor's data_ptr); host memory is refused with MTX_E_ARG.
static bool on_device(const mtx_ctx *c, const void *p) {
  if (!p) return false;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky "invalid value" of an unregistered host pointer
    return false;
  }
  return (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged) && at.device == c->device;
}
static int need_device(const mtx_ctx *c, const char *fn, std::initializer_list<const void *> ptrs) {
  int k = 0;
  for (const void *p : ptrs) {
    if (p && !on_device(c, p)) {
      mtx_set_error("%s: argument %d is not device memory of device %d", fn, k, c->device);
      return MTX_E_ARG;
    }
    ++k;
  }
  return MTX_OK;
}

static int sample_rays_impl(mtx_ctx *c, const mtx_render_args *a, uint64_t n, const float *rays,
                            const uint32_t *lanes, uint32_t rng_skip, float *L, uint8_t *valid, bool dev);

int mtx_sample_rays(mtx_ctx *c, const mtx_render_args *a, uint64_t n, const float *rays, const uint32_t *lanes,
                    uint32_t rng_skip, float *L, uint8_t *valid) {
  return sample_rays_impl(c, a, n, rays, lanes, rng_skip, L, valid, false);
}

int mtx_sample_rays_dev(mtx_ctx *c, const mtx_render_args *a, uint64_t n, const float *rays, const uint32_t *lanes,
                        uint32_t rng_skip, float *L, uint8_t *valid) {
  if (c && n && (!rays || !lanes || !L || !valid)) {
    mtx_set_error("mtx_sample_rays_dev: null buffer");
    return MTX_E_ARG;
  }
  if (c && n) {
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = need_device(c, "mtx_sample_rays_dev", {rays, lanes, L, valid})) return rc;
  }
  return sample_rays_impl(c, a, n, rays, lanes, rng_skip, L, valid, true);
}

static int sample_rays_impl(mtx_ctx *c, const mtx_render_args *a, uint64_t n, const float *rays,
                            const uint32_t *lanes, uint32_t rng_skip, float *L, uint8_t *valid, bool dev) {
  int rc = check_args(c, a);
  if (rc) return rc;
  if (a->integrator == MTX_INT_PSSMLT_SIMPLE || a->integrator == MTX_INT_PSSMLT_PATH ||
      a->integrator == MTX_INT_RESTIR_GI) {
    mtx_set_error("mtx_sample_rays: PSSMLT / ReSTIR GI are render-level algorithms (use mtx_render)");
    return MTX_E_UNSUPPORTED;
  }
  if (n == 0) return MTX_OK;
  if (!rays || !lanes || !L || !valid) {
    mtx_set_error("mtx_sample_rays: null buffer");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  const uint32_t chunk = a->chunk_paths ? a->chunk_paths : default_chunk(c, a, 1u, false);
  const uint32_t cap = (uint32_t)std::min<uint64_t>(n, chunk);
  if ((rc = ensure_wavefront(c, cap, std::max<uint32_t>(a->max_depth, 1)))) return rc;
  const bool nrc_cache = a->integrator == MTX_INT_NRC && (a->flags & 4u);
  const bool nerad_render = a->integrator == MTX_INT_NERAD;
  if ((nrc_cache || nerad_render) && (rc = ensure_cache(c, cap))) return rc;
  if (!dev) {
    if ((rc = dalloc(c->s0, 24ull * cap))) return rc;
    if ((rc = dalloc(c->s1, 4ull * cap))) return rc;
    if ((rc = dalloc(c->s2, 12ull * cap))) return rc;
    if ((rc = dalloc(c->s3, 1ull * cap))) return rc;
  }
  mtxd::WaveBuffers b = buffers(c);
  Timer tm{c, false};
  uint64_t nt = 0, ns = 0;
  for (uint64_t off = 0; off < n; off += cap) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(cap, n - off);
    // the chunk's rays / lanes / outputs: the caller's device buffers, or the
    // context's staging copies of the host ones
    const float *d_rays = dev ? rays + 6 * off : (const float *)c->s0.p;
    const uint32_t *d_lanes = dev ? lanes + off : (const uint32_t *)c->s1.p;
    float *d_L = dev ? L + 3 * off : (float *)c->s2.p;
    uint8_t *d_valid = dev ? valid + off : (uint8_t *)c->s3.p;
    if (!dev) {
      HIP_TRY(hipMemcpyAsync(c->s0.p, rays + 6 * off, 24ull * m, hipMemcpyHostToDevice, c->stream));
      HIP_TRY(hipMemcpyAsync(c->s1.p, lanes + off, 4ull * m, hipMemcpyHostToDevice, c->stream));
    }
    mtxd::ChunkParams p{};
    p.integrator = a->integrator;
    p.max_depth = a->max_depth;
    p.rr_depth = a->rr_depth;
    p.seed = a->seed;
    p.spp = 1;
    p.spp_total = 1;
    p.width = c->scene.camera.width;
    p.height = c->scene.camera.height;
    p.n_paths = m;
    p.nrc_c = a->nrc_c;
    p.nrc_cache = nrc_cache ? 1u : 0u;
    HIP_TRY(reset_counters(b, std::max<uint32_t>(a->max_depth, 1), c->stream));
    if (nrc_cache || nerad_render) HIP_TRY(hipMemsetAsync(b.cq_count, 0, 4, c->stream));
    mtxd::launch_raygen_rays(c->scene, b, p, d_rays, d_lanes, rng_skip, c->stream);
    run_bounces(c, b, p, tm, &nt, &ns);
    if (nrc_cache && (rc = run_cache(c, b, m, tm))) return rc;
    if (nerad_render && (rc = run_cache(c, b, m, tm, true))) return rc;
    mtxd::launch_collect(b, p, d_L, d_valid, c->stream);
    HIP_TRY(hipGetLastError());
    if (!dev) {
      HIP_TRY(hipMemcpyAsync(L + 3 * off, c->s2.p, 12ull * m, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(valid + off, c->s3.p, m, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));  // the staging buffers are reused by the next chunk
    }
  }
  if (dev) HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

static int trace_impl(mtx_ctx *c, uint64_t n, const float *rays, int any_hit, uint32_t *hits, uint32_t *visits,
                      bool dev);

int mtx_trace(mtx_ctx *c, uint64_t n, const float *rays, int any_hit, uint32_t *hits, uint32_t *visits) {
  return trace_impl(c, n, rays, any_hit, hits, visits, false);
}

int mtx_trace_dev(mtx_ctx *c, uint64_t n, const float *rays, int any_hit, uint32_t *hits, uint32_t *visits) {
  if (c && rays && hits && n) {
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = need_device(c, "mtx_trace_dev", {rays, hits, visits})) return rc;
  }
  return trace_impl(c, n, rays, any_hit, hits, visits, true);
}

static int trace_impl(mtx_ctx *c, uint64_t n, const float *rays, int any_hit, uint32_t *hits, uint32_t *visits,
                      bool dev) {
  if (!c || !rays || !hits) {
    mtx_set_error("mtx_trace: null argument");
    return MTX_E_ARG;
  }
  if (!c->has_scene) {
    mtx_set_error("no scene uploaded");
    return MTX_E_NOSCENE;
  }
  if (any_hit < 0 || any_hit > 1) {
    mtx_set_error("mtx_trace: mode %d (0 closest hit, 1 any hit)", any_hit);
    return MTX_E_ARG;
  }
  if (n == 0) return MTX_OK;
  if (n >= (1ull << 31)) {
    mtx_set_error("mtx_trace: too many rays");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  const size_t hit_words = any_hit == 1 ? n : 4 * n;
  if (dev) {
    mtxd::launch_trace_raw(c->scene, (const float4 *)rays, (uint32_t)n, any_hit, hits, visits, c->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MTX_OK;
  }
  if ((rc = dalloc(c->s0, 32ull * n))) return rc;
  if ((rc = dalloc(c->s1, 4ull * hit_words))) return rc;
  if (visits && (rc = dalloc(c->s2, 8ull * n))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s0.p, rays, 32ull * n, hipMemcpyHostToDevice, c->stream));
  mtxd::launch_trace_raw(c->scene, (const float4 *)c->s0.p, (uint32_t)n, any_hit, (uint32_t *)c->s1.p,
                         visits ? (uint32_t *)c->s2.p : nullptr, c->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(hits, c->s1.p, 4ull * hit_words, hipMemcpyDeviceToHost, c->stream));
  if (visits) HIP_TRY(hipMemcpyAsync(visits, c->s2.p, 8ull * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

// ------------------------------- primitives -------------------------------

// HIP-event bracket around the device work of one primitive call.
static int prim_timer_begin(mtx_ctx *c) {
  for (int k = 0; k < 2; ++k)
    if (!c->prim_ev[k]) HIP_TRY(hipEventCreate(&c->prim_ev[k]));
  HIP_TRY(hipEventRecord(c->prim_ev[0], c->stream));
  return MTX_OK;
}
static int prim_timer_end(mtx_ctx *c) {
  HIP_TRY(hipEventRecord(c->prim_ev[1], c->stream));
  return MTX_OK;
}
static void prim_timer_read(mtx_ctx *c) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, c->prim_ev[0], c->prim_ev[1]) == hipSuccess) c->last_device_ms = ms;
}

double mtx_last_device_ms(mtx_ctx *c) { return c ? c->last_device_ms : 0.0; }

int mtx_field_upload(mtx_ctx *c, const mtx_field_desc *f) {
  if (!c || !f || !f->table || !f->weights) {
    mtx_set_error("mtx_field_upload: null argument");
    return MTX_E_ARG;
  }
  if (f->n_levels == 0 || f->n_levels > mtx::kFieldMaxLevels || f->n_features < 1 || f->n_features > 2 ||
      f->log2_table < 4 || f->log2_table > 26 || f->n_hidden > 16 ||
      f->n_in != 3 + f->n_levels * f->n_features + 3 + 16 || f->n_in > 64 || f->base_res < 1 ||
      !(f->per_level_scale >= 1.f)) {
    mtx_set_error("mtx_field_upload: unsupported field shape (n_in must be 3 + L*F + 19 <= 64)");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  const size_t table_halfs = (size_t)f->n_levels * ((size_t)1 << f->log2_table) * f->n_features;
  if ((rc = upload(c->field_table, f->table, table_halfs, c->stream))) return rc;
  const uint32_t n_frag = mtxd::field_frag_count(f->n_hidden);
  std::vector<uint16_t> frag((size_t)n_frag * 64 * 8);
  mtxd::field_prepack(f->weights, f->n_in, f->n_hidden, frag.data());
  if ((rc = upload(c->field_frag, frag.data(), frag.size(), c->stream))) return rc;
  const uint32_t n_w = 64u * f->n_in + f->n_hidden * 4096u + 3u * 64u;
  if ((rc = upload(c->field_w16, f->weights, n_w, c->stream))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->field_n_in = f->n_in;
  c->field_n_w = n_w;
  c->field_n_table = table_halfs;
  c->training = false;  // a new field: mtx_field_train_init starts over
  mtx::FieldEncoding &e = c->field;
  e.table = (const uint16_t *)c->field_table.p;
  e.n_levels = f->n_levels;
  e.n_features = f->n_features;
  e.log2_table = f->log2_table;
  for (uint32_t l = 0; l < f->n_levels; ++l) {
    const double scale = std::exp2((double)l * std::log2((double)f->per_level_scale)) * f->base_res - 1.0;
    e.level_scale[l] = (float)scale;
    e.level_res[l] = (uint32_t)std::ceil((double)(float)scale) + 1u;
  }
  for (int k = 0; k < 3; ++k) {
    e.bbox_min[k] = f->bbox_min[k];
    e.bbox_max[k] = f->bbox_max[k];
  }
  c->field_hidden = f->n_hidden;
  c->has_field = true;
  return MTX_OK;
}

static int field_stage_queries(mtx_ctx *c, uint64_t n, const float *p, const float *wi) {
  int rc;
  if ((rc = dalloc(c->fq_p, 16 * n))) return rc;
  if ((rc = dalloc(c->fq_d, 16 * n))) return rc;
  std::vector<float> tp(4 * n), td(4 * n);
  for (uint64_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      tp[4 * i + k] = p[3 * i + k];
      td[4 * i + k] = wi[3 * i + k];
    }
  HIP_TRY(hipMemcpy(c->fq_p.p, tp.data(), 16 * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->fq_d.p, td.data(), 16 * n, hipMemcpyHostToDevice));
  return MTX_OK;
}

static int field_check(mtx_ctx *c, uint64_t n) {
  if (!c || !c->has_field) {
    mtx_set_error("no radiance field uploaded (mtx_field_upload)");
    return MTX_E_ARG;
  }
  if (n >= (1ull << 31)) {
    mtx_set_error("too many field queries");
    return MTX_E_ARG;
  }
  return MTX_OK;
}

int mtx_field_features(mtx_ctx *c, uint64_t n, const float *p, const float *wi, uint16_t *feat) {
  int rc = field_check(c, n);
  if (rc) return rc;
  if (n == 0) return MTX_OK;
  if (!p || !wi || !feat) {
    mtx_set_error("mtx_field_features: null buffer");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = field_stage_queries(c, n, p, wi))) return rc;
  if ((rc = dalloc(c->f_feat, 128 * n))) return rc;
  if ((rc = prim_timer_begin(c))) return rc;
  mtxd::field_encode(c->field, (const float4 *)c->fq_p.p, (const float4 *)c->fq_d.p, nullptr, (uint32_t)n,
                     (uint16_t *)c->f_feat.p, c->stream);
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(feat, c->f_feat.p, 128 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_field_mlp(mtx_ctx *c, uint64_t n, const uint16_t *feat, float *out) {
  int rc = field_check(c, n);
  if (rc) return rc;
  if (n == 0) return MTX_OK;
  if (!feat || !out) {
    mtx_set_error("mtx_field_mlp: null buffer");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = dalloc(c->f_feat, 128 * n))) return rc;
  if ((rc = dalloc(c->f_out, 12 * n))) return rc;
  HIP_TRY(hipMemcpyAsync(c->f_feat.p, feat, 128 * n, hipMemcpyHostToDevice, c->stream));
  if ((rc = prim_timer_begin(c))) return rc;
  mtxd::field_mlp((const uint16_t *)c->f_feat.p, nullptr, (uint32_t)n, c->field_frag.p, c->field_hidden,
                  (float *)c->f_out.p, c->n_cu, c->stream);
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->f_out.p, 12 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_field_eval(mtx_ctx *c, uint64_t n, const float *p, const float *wi, float *out) {
  int rc = field_check(c, n);
  if (rc) return rc;
  if (n == 0) return MTX_OK;
  if (!p || !wi || !out) {
    mtx_set_error("mtx_field_eval: null buffer");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = field_stage_queries(c, n, p, wi))) return rc;
  if ((rc = dalloc(c->f_feat, 128 * n))) return rc;
  if ((rc = dalloc(c->f_out, 12 * n))) return rc;
  if ((rc = prim_timer_begin(c))) return rc;
  mtxd::field_encode(c->field, (const float4 *)c->fq_p.p, (const float4 *)c->fq_d.p, nullptr, (uint32_t)n,
                     (uint16_t *)c->f_feat.p, c->stream);
  mtxd::field_mlp((const uint16_t *)c->f_feat.p, nullptr, (uint32_t)n, c->field_frag.p, c->field_hidden,
                  (float *)c->f_out.p, c->n_cu, c->stream);
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->f_out.p, 12 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_prefix_sum_u32(mtx_ctx *c, const uint32_t *in, uint32_t *out, uint64_t n, int inclusive) {
  if (!c || (n && (!in || !out))) {
    mtx_set_error("mtx_prefix_sum_u32: null argument");
    return MTX_E_ARG;
  }
  if (n == 0) return MTX_OK;
  if (n >= (1ull << 32)) {
    mtx_set_error("mtx_prefix_sum_u32: n >= 2^32");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s0, 4 * n))) return rc;
  if ((rc = dalloc(c->s1, 4 * n))) return rc;
  if ((rc = dalloc(c->s2, mtxd::scan_workspace_bytes(n)))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s0.p, in, 4 * n, hipMemcpyHostToDevice, c->stream));
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::scan_u32((const uint32_t *)c->s0.p, (uint32_t *)c->s1.p, n, inclusive, c->s2.p, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->s1.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_prefix_sum_f32_hs(mtx_ctx *c, const float *in, float *out, uint64_t n) {
  if (!c || (n && (!in || !out))) {
    mtx_set_error("mtx_prefix_sum_f32_hs: null argument");
    return MTX_E_ARG;
  }
  if (n == 0) return MTX_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s0, 4 * n))) return rc;
  if ((rc = dalloc(c->s1, 4 * n))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s0.p, in, 4 * n, hipMemcpyHostToDevice, c->stream));
  float *res = nullptr;
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::scan_f32_hs((float *)c->s0.p, (float *)c->s1.p, n, &res, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, res, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_prefix_sum_u32_dev(mtx_ctx *c, const uint32_t *in, uint32_t *out, uint64_t n, int inclusive) {
  if (!c || (n && (!in || !out))) {
    mtx_set_error("mtx_prefix_sum_u32_dev: null argument");
    return MTX_E_ARG;
  }
  if (n == 0) return MTX_OK;
  if (n >= (1ull << 32)) {
    mtx_set_error("mtx_prefix_sum_u32_dev: n >= 2^32");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = need_device(c, "mtx_prefix_sum_u32_dev", {in, out}))) return rc;
  if ((rc = dalloc(c->s2, mtxd::scan_workspace_bytes(n)))) return rc;
  if ((rc = prim_timer_begin(c))) return rc;
  if ((rc = mtxd::scan_u32(in, out, n, inclusive, c->s2.p, c->stream))) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_prefix_sum_f32_hs_dev(mtx_ctx *c, const float *in, float *out, uint64_t n) {
  if (!c || (n && (!in || !out))) {
    mtx_set_error("mtx_prefix_sum_f32_hs_dev: null argument");
    return MTX_E_ARG;
  }
  if (n == 0) return MTX_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = need_device(c, "mtx_prefix_sum_f32_hs_dev", {in, out}))) return rc;
  if ((rc = dalloc(c->s1, 4 * n))) return rc;  // ping-pong partner of out
  if ((rc = prim_timer_begin(c))) return rc;
  if ((rc = mtxd::scan_f32_hs_to(in, out, (float *)c->s1.p, n, c->stream))) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_hashgrid_build_dev(mtx_ctx *c, const float *p, uint64_t n, uint32_t resolution, uint32_t n_cells,
                           uint32_t *cell, uint32_t *cell_size, uint32_t *cell_offset, uint32_t *sample_idx) {
  if (!c || !p || !cell || !cell_size || !cell_offset || !sample_idx || n == 0 || n_cells == 0) {
    mtx_set_error("mtx_hashgrid_build_dev: bad argument");
    return MTX_E_ARG;
  }
  if (n >= (1ull << 31)) {
    mtx_set_error("mtx_hashgrid_build_dev: n too large");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = need_device(c, "mtx_hashgrid_build_dev", {p, cell, cell_size, cell_offset, sample_idx}))) return rc;
  if ((rc = dalloc(c->s5, mtxd::hashgrid_workspace_bytes(n, n_cells)))) return rc;
  if ((rc = prim_timer_begin(c))) return rc;
  if ((rc = mtxd::hashgrid_build(p, n, resolution, n_cells, cell, cell_size, cell_offset, sample_idx, c->s5.p,
                                 c->stream)))
    return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_hashgrid_build(mtx_ctx *c, const float *p, uint64_t n, uint32_t resolution, uint32_t n_cells, uint32_t *cell,
                       uint32_t *cell_size, uint32_t *cell_offset, uint32_t *sample_idx) {
  if (!c || !p || !cell || !cell_size || !cell_offset || !sample_idx || n == 0 || n_cells == 0) {
    mtx_set_error("mtx_hashgrid_build: bad argument");
    return MTX_E_ARG;
  }
  if (n >= (1ull << 31)) {
    mtx_set_error("mtx_hashgrid_build: n too large");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s0, 12 * n))) return rc;
  if ((rc = dalloc(c->s1, 4 * n))) return rc;           // cell
  if ((rc = dalloc(c->s2, 4 * (size_t)n_cells))) return rc;   // size
  if ((rc = dalloc(c->s3, 4 * (size_t)n_cells))) return rc;   // offset
  if ((rc = dalloc(c->s4, 4 * n))) return rc;           // sample_idx
  if ((rc = dalloc(c->s5, mtxd::hashgrid_workspace_bytes(n, n_cells)))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s0.p, p, 12 * n, hipMemcpyHostToDevice, c->stream));
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::hashgrid_build((const float *)c->s0.p, n, resolution, n_cells, (uint32_t *)c->s1.p, (uint32_t *)c->s2.p,
                            (uint32_t *)c->s3.p, (uint32_t *)c->s4.p, c->s5.p, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(cell, c->s1.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(cell_size, c->s2.p, 4ull * n_cells, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(cell_offset, c->s3.p, 4ull * n_cells, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(sample_idx, c->s4.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_group_by_u32(mtx_ctx *c, const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size,
                     uint32_t *key_offset, uint32_t *order) {
  if (!c || !keys || !key_size || !key_offset || !order || n == 0 || n_keys == 0) {
    mtx_set_error("mtx_group_by_u32: bad argument");
    return MTX_E_ARG;
  }
  if (n >= (1ull << 31)) {
    mtx_set_error("mtx_group_by_u32: n too large");
    return MTX_E_ARG;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (keys[i] >= n_keys) {
      mtx_set_error("mtx_group_by_u32: keys[%llu] = %u out of range", (unsigned long long)i, keys[i]);
      return MTX_E_ARG;
    }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s1, 4 * n))) return rc;                // keys
  if ((rc = dalloc(c->s2, 4 * (size_t)n_keys))) return rc;   // size
  if ((rc = dalloc(c->s3, 4 * (size_t)n_keys))) return rc;   // offset
  if ((rc = dalloc(c->s4, 4 * n))) return rc;                // order
  if ((rc = dalloc(c->s5, mtxd::hashgrid_workspace_bytes(n, n_keys)))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s1.p, keys, 4 * n, hipMemcpyHostToDevice, c->stream));
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::group_by_u32((const uint32_t *)c->s1.p, n, n_keys, (uint32_t *)c->s2.p, (uint32_t *)c->s3.p,
                          (uint32_t *)c->s4.p, c->s5.p, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(key_size, c->s2.p, 4ull * n_keys, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(key_offset, c->s3.p, 4ull * n_keys, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(order, c->s4.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_group_by_u32_dev(mtx_ctx *c, const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size,
                         uint32_t *key_offset, uint32_t *order) {
  if (!c || !keys || !key_size || !key_offset || !order || n == 0 || n_keys == 0) {
    mtx_set_error("mtx_group_by_u32_dev: bad argument");
    return MTX_E_ARG;
  }
  if (n >= (1ull << 31)) {
    mtx_set_error("mtx_group_by_u32_dev: n too large");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s5, mtxd::hashgrid_workspace_bytes(n, n_keys)))) return rc;
  if ((rc = dalloc(c->s6, 64))) return rc;
  // the keys are device data: range-checked on the device before any
  // kernel indexes with them
  HIP_TRY(hipMemsetAsync(c->s6.p, 0, 4, c->stream));
  mtxd::keys_in_range(keys, n, n_keys, (uint32_t *)c->s6.p, c->stream);
  uint32_t bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->s6.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (bad) {
    mtx_set_error("mtx_group_by_u32_dev: a key is >= n_keys (%u)", n_keys);
    return MTX_E_ARG;
  }
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::group_by_u32(keys, n, n_keys, key_size, key_offset, order, c->s5.p, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_scatter_reduce_f32_dev(mtx_ctx *c, int op, float *target, uint64_t n_target, const float *value,
                               const uint32_t *index, uint64_t n_value) {
  if (!c || !target || (n_value && (!value || !index)) || op < 0 || op > 3) {
    mtx_set_error("mtx_scatter_reduce_f32_dev: bad argument");
    return MTX_E_ARG;
  }
  if (n_value == 0 || n_target == 0) return MTX_OK;
  if (n_value >= (1ull << 31) || n_target >= (1ull << 31)) {
    mtx_set_error("mtx_scatter_reduce_f32_dev: size too large");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = need_device(c, "mtx_scatter_reduce_f32_dev", {target, value, index}))) return rc;
  if ((rc = dalloc(c->s3, mtxd::scatter_workspace_bytes(n_target, n_value)))) return rc;
  if ((rc = dalloc(c->s6, 64))) return rc;
  // the indices are device data: range-checked on the device first
  HIP_TRY(hipMemsetAsync(c->s6.p, 0, 4, c->stream));
  mtxd::keys_in_range(index, n_value, (uint32_t)n_target, (uint32_t *)c->s6.p, c->stream);
  uint32_t bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, c->s6.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (bad) {
    mtx_set_error("mtx_scatter_reduce_f32_dev: an index is >= n_target (%llu)", (unsigned long long)n_target);
    return MTX_E_ARG;
  }
  if ((rc = prim_timer_begin(c))) return rc;
  if ((rc = mtxd::scatter_reduce_f32(op, target, n_target, value, index, n_value, c->s3.p, c->stream))) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

int mtx_scatter_reduce_f32(mtx_ctx *c, int op, float *target, uint64_t n_target, const float *value,
                           const uint32_t *index, uint64_t n_value) {
  if (!c || !target || (n_value && (!value || !index)) || op < 0 || op > 3) {
    mtx_set_error("mtx_scatter_reduce_f32: bad argument");
    return MTX_E_ARG;
  }
  if (n_value == 0 || n_target == 0) return MTX_OK;
  if (n_value >= (1ull << 31) || n_target >= (1ull << 31)) {
    mtx_set_error("mtx_scatter_reduce_f32: size too large");
    return MTX_E_ARG;
  }
  for (uint64_t i = 0; i < n_value; ++i)
    if (index[i] >= n_target) {
      mtx_set_error("mtx_scatter_reduce_f32: index[%llu] = %u out of range", (unsigned long long)i, index[i]);
      return MTX_E_ARG;
    }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = dalloc(c->s0, 4 * n_target))) return rc;
  if ((rc = dalloc(c->s1, 4 * n_value))) return rc;
  if ((rc = dalloc(c->s2, 4 * n_value))) return rc;
  if ((rc = dalloc(c->s3, mtxd::scatter_workspace_bytes(n_target, n_value)))) return rc;
  HIP_TRY(hipMemcpyAsync(c->s0.p, target, 4 * n_target, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->s1.p, value, 4 * n_value, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->s2.p, index, 4 * n_value, hipMemcpyHostToDevice, c->stream));
  if ((rc = prim_timer_begin(c))) return rc;
  rc = mtxd::scatter_reduce_f32(op, (float *)c->s0.p, n_target, (const float *)c->s1.p, (const uint32_t *)c->s2.p,
                                n_value, c->s3.p, c->stream);
  if (rc) return rc;
  if ((rc = prim_timer_end(c))) return rc;
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(target, c->s0.p, 4 * n_target, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  prim_timer_read(c);
  return MTX_OK;
}

}  // extern "C"

// ============================================================================
// Radiance-field training and neural radiosity samples (nerad.py:121-375)
// ============================================================================
static int train_check(mtx_ctx *c) {
  if (!c || !c->has_field) {
    mtx_set_error("no radiance field uploaded (mtx_field_upload)");
    return MTX_E_ARG;
  }
  if (!c->training) {
    mtx_set_error("field training not initialised (mtx_field_train_init)");
    return MTX_E_ARG;
  }
  return MTX_OK;
}

// Forward + backward of the field for n points (queries qp / qd on the
// device, targets 3n floats on the device): gradients of scale * loss in
// tr_g = [table | weights], network outputs in tr_out, loss (unscaled) on
// the host.
static int field_backward(mtx_ctx *c, const float4 *qp, const float4 *qd, const float *target, uint32_t n,
                          float scale, double *loss) {
  int rc;
  const uint32_t LF = c->field.n_levels * c->field.n_features;
  const uint32_t blocks = (n + 63) / 64;
  const uint64_t n_params = c->field_n_table + c->field_n_w;
  if ((rc = dalloc(c->tr_feat, 128ull * n))) return rc;
  if ((rc = dalloc(c->tr_out, 12ull * n))) return rc;
  if ((rc = dalloc(c->tr_loss, 4ull * blocks))) return rc;
  if ((rc = dalloc(c->tr_wpart, 4ull * blocks * c->field_n_w))) return rc;
  if ((rc = dalloc(c->tr_dfeat, 4ull * n * LF))) return rc;
  if ((rc = dalloc(c->tr_g, 4 * n_params))) return rc;
  mtxd::field_encode(c->field, qp, qd, nullptr, n, (uint16_t *)c->tr_feat.p, c->stream);
  HIP_TRY(hipMemsetAsync(c->tr_g.p, 0, 4 * c->field_n_table, c->stream));
  float *g = (float *)c->tr_g.p;
  mtxd::field_train_launch((const uint16_t *)c->tr_feat.p, n, (const uint16_t *)c->field_w16.p, c->field_n_in,
                           c->field_hidden, target, (float)(2.0 * scale / (3.0 * n)), (float *)c->tr_out.p,
                           (float *)c->tr_loss.p, (float *)c->tr_wpart.p, g + c->field_n_table,
                           (float *)c->tr_dfeat.p, LF, c->stream);
  mtxd::field_encode_bwd_launch(c->field, qp, n, (const float *)c->tr_dfeat.p, g, c->stream);
  HIP_TRY(hipGetLastError());
  if (loss) {
    std::vector<float> part(blocks);
    HIP_TRY(hipMemcpyAsync(part.data(), c->tr_loss.p, 4ull * blocks, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double sq = 0.0;
    for (float x : part) sq += x;
    *loss = sq / (3.0 * n);
  }
  return MTX_OK;
}

// GradScaler.step(opt): finite check of the scaled gradients, Adam on the
// unscaled ones (skipped on inf / NaN), scale update; the fp16 table and
// weights are rewritten by the Adam kernel and re-packed for the MFMA MLP.
static int field_opt_step(mtx_ctx *c, mtx_train_stats *st) {
  const uint64_t n_params = c->field_n_table + c->field_n_w;
  int rc;
  if ((rc = dalloc(c->tr_flag, 16))) return rc;
  HIP_TRY(hipMemsetAsync(c->tr_flag.p, 0, 4, c->stream));
  mtxd::grad_check_launch((const float *)c->tr_g.p, n_params, (uint32_t *)c->tr_flag.p, c->stream);
  uint32_t found = 0;
  HIP_TRY(hipMemcpyAsync(&found, c->tr_flag.p, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const mtx_field_opt &o = c->opt;
  if (!found) {
    ++c->adam_t;
    const double t = c->adam_t;
    const float lr_t = (float)(o.lr * std::sqrt(1.0 - std::pow((double)o.beta_2, t)) /
                               (1.0 - std::pow((double)o.beta_1, t)));
    mtxd::adam_launch((float *)c->tr_p.p, (float *)c->tr_m.p, (float *)c->tr_v.p, (const float *)c->tr_g.p, n_params,
                      lr_t, o.beta_1, o.beta_2, o.epsilon, 1.f / c->scale, (const uint32_t *)c->tr_flag.p,
                      (uint16_t *)c->field_table.p, c->field_n_table, (uint16_t *)c->field_w16.p, c->stream);
    mtxd::field_prepack_launch((const uint16_t *)c->field_w16.p, c->field_n_in, c->field_hidden,
                               (uint16_t *)c->field_frag.p, c->stream);
    HIP_TRY(hipGetLastError());
    if (++c->good_steps >= o.growth_interval) {
      c->scale *= o.growth_factor;
      c->good_steps = 0;
    }
  } else {
    c->scale *= o.backoff_factor;
    c->good_steps = 0;
  }
  if (st) {
    st->found_inf = found;
    st->scale = c->scale;
    st->step = c->adam_t;
  }
  return MTX_OK;
}

struct PhaseTimer {
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  hipStream_t st;
  explicit PhaseTimer(hipStream_t s) : st(s) {
    for (auto &e : ev) hipEventCreate(&e);
  }
  ~PhaseTimer() {
    for (auto &e : ev) hipEventDestroy(e);
  }
  void mark(int i) { hipEventRecord(ev[i], st); }
  double ms(int a, int b) {
    float t = 0.f;
    hipEventElapsedTime(&t, ev[a], ev[b]);
    return t;
  }
};

static int nerad_check(mtx_ctx *c, const mtx_nerad_args *a, bool need_field = true) {
  if (!c || !a) {
    mtx_set_error("null context or args");
    return MTX_E_ARG;
  }
  if (!c->has_scene || !c->has_nerad) {
    mtx_set_error("nerad: upload a scene and its surface tables (mtx_nerad_upload) first");
    return MTX_E_NOSCENE;
  }
  if (need_field && !c->has_field) {
    mtx_set_error("nerad: no radiance field uploaded (mtx_field_upload)");
    return MTX_E_ARG;
  }
  if (a->batch == 0 || a->M == 0 || (uint64_t)a->batch * a->M >= (1ull << 31)) {
    mtx_set_error("nerad: bad batch %u / M %u", a->batch, a->M);
    return MTX_E_ARG;
  }
  return MTX_OK;
}

static int nerad_lhs_dev(mtx_ctx *c, const mtx_nerad_args *a) {
  int rc;
  if ((rc = dalloc(c->nr_lhs, 48ull * a->batch))) return rc;
  if ((rc = dalloc(c->nr_qp, 16ull * a->batch))) return rc;
  if ((rc = dalloc(c->nr_qd, 16ull * a->batch))) return rc;
  mtxd::launch_nerad_lhs(c->scene, c->nr, a->lhs_seed, a->batch, (float4 *)c->nr_lhs.p, (float4 *)c->nr_qp.p,
                         (float4 *)c->nr_qd.p, c->stream);
  HIP_TRY(hipGetLastError());
  return MTX_OK;
}

// sample_rhs (nerad.py:174-233) for the points in nr_lhs: L_rhs in nr_Lrhs.
static int nerad_rhs_dev(mtx_ctx *c, const mtx_nerad_args *a, float *lanes_dev, uint32_t *queries,
                         mtx_train_stats *st = nullptr) {
  int rc;
  const uint32_t n = a->batch * a->M;
  const uint32_t bounces = 12;  // first vertex, its BSDF hit, <= 10 next_smooth_si traces (:146)
  if ((rc = ensure_wavefront(c, n, bounces))) return rc;
  if ((rc = ensure_cache(c, n))) return rc;
  if ((rc = dalloc(c->nr_Lrhs, 12ull * a->batch))) return rc;
  mtxd::WaveBuffers b = buffers(c);
  mtxd::ChunkParams p{};
  p.integrator = MTX_INT_NERAD_RHS;
  p.max_depth = bounces;
  p.seed = a->rhs_seed;
  p.spp = p.spp_total = 1;
  p.n_paths = n;
  p.n_px = n;
  const bool counters = st && (a->flags & 1u);
  p.stats = counters ? 1u : 0u;
  HIP_TRY(reset_counters(b, bounces, c->stream));
  HIP_TRY(hipMemsetAsync(b.cq_count, 0, 4, c->stream));
  if (counters) HIP_TRY(hipMemsetAsync(b.stats, 0, 64, c->stream));
  mtxd::launch_nerad_raygen(b, p, (const float4 *)c->nr_lhs.p, a->M, c->stream);
  Timer tm{c, st != nullptr};
  uint64_t nt = 0, ns = 0;
  run_bounces(c, b, p, tm, &nt, &ns);
  mtxd::field_encode(c->field, b.cq_p, b.cq_d, b.cq_count, n, (uint16_t *)c->f_feat.p, c->stream);
  mtxd::field_mlp((const uint16_t *)c->f_feat.p, b.cq_count, n, c->field_frag.p, c->field_hidden,
                  (float *)c->f_out.p, c->n_cu, c->stream);
  mtxd::launch_nerad_apply(b, (const float *)c->f_out.p, n, 0, c->stream);
  mtxd::launch_nerad_mean(b, a->batch, a->M, (float *)c->nr_Lrhs.p, lanes_dev, c->stream);
  HIP_TRY(hipGetLastError());
  if (queries) HIP_TRY(hipMemcpyAsync(queries, b.cq_count, 4, hipMemcpyDeviceToHost, c->stream));
  if (st) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    st->ms_trace = tm.total(0);
    if (counters) {
      unsigned long long h[8];
      HIP_TRY(hipMemcpy(h, b.stats, 64, hipMemcpyDeviceToHost));
      st->nodes_closest = h[0];
      st->tris_closest = h[1];
      st->rays_closest = h[4];
    }
  }
  return MTX_OK;
}

extern "C" {

int mtx_field_train_init(mtx_ctx *c, const mtx_field_opt *opt) {
  if (!c || !opt || !c->has_field) {
    mtx_set_error("mtx_field_train_init: null argument or no field uploaded");
    return MTX_E_ARG;
  }
  if (!(opt->lr > 0.f) || !(opt->init_scale > 0.f) || opt->growth_interval == 0) {
    mtx_set_error("mtx_field_train_init: bad optimiser settings");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t n_params = c->field_n_table + c->field_n_w;
  int rc;
  if ((rc = dalloc(c->tr_p, 4 * n_params))) return rc;
  if ((rc = dalloc(c->tr_m, 4 * n_params))) return rc;
  if ((rc = dalloc(c->tr_v, 4 * n_params))) return rc;
  mtxd::half_to_float_launch((const uint16_t *)c->field_table.p, c->field_n_table, (float *)c->tr_p.p, c->stream);
  mtxd::half_to_float_launch((const uint16_t *)c->field_w16.p, c->field_n_w, (float *)c->tr_p.p + c->field_n_table,
                             c->stream);
  HIP_TRY(hipMemsetAsync(c->tr_m.p, 0, 4 * n_params, c->stream));
  HIP_TRY(hipMemsetAsync(c->tr_v.p, 0, 4 * n_params, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->opt = *opt;
  c->adam_t = 0;
  c->good_steps = 0;
  c->scale = opt->init_scale;
  c->training = true;
  return MTX_OK;
}

int mtx_field_grad(mtx_ctx *c, uint64_t n, const float *p, const float *wi, const float *target, float scale,
                   float *out, double *loss, float *grad_table, float *grad_weights) {
  int rc = field_check(c, n);
  if (rc) return rc;
  if (n == 0 || !p || !wi || !target) {
    mtx_set_error("mtx_field_grad: empty batch or null input");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = field_stage_queries(c, n, p, wi))) return rc;
  if ((rc = upload(c->tr_target, target, 3 * n, c->stream))) return rc;
  if ((rc = field_backward(c, (const float4 *)c->fq_p.p, (const float4 *)c->fq_d.p, (const float *)c->tr_target.p,
                           (uint32_t)n, scale, loss)))
    return rc;
  const float *g = (const float *)c->tr_g.p;
  if (out) HIP_TRY(hipMemcpyAsync(out, c->tr_out.p, 12 * n, hipMemcpyDeviceToHost, c->stream));
  if (grad_table) HIP_TRY(hipMemcpyAsync(grad_table, g, 4 * c->field_n_table, hipMemcpyDeviceToHost, c->stream));
  if (grad_weights)
    HIP_TRY(hipMemcpyAsync(grad_weights, g + c->field_n_table, 4ull * c->field_n_w, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

int mtx_field_train_step(mtx_ctx *c, uint64_t n, const float *p, const float *wi, const float *target,
                         mtx_train_stats *stats) {
  int rc = field_check(c, n);
  if (rc || (rc = train_check(c))) return rc;
  if (n == 0 || !p || !wi || !target) {
    mtx_set_error("mtx_field_train_step: empty batch or null input");
    return MTX_E_ARG;
  }
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = field_stage_queries(c, n, p, wi))) return rc;
  if ((rc = upload(c->tr_target, target, 3 * n, c->stream))) return rc;
  double loss = 0.0;
  if ((rc = field_backward(c, (const float4 *)c->fq_p.p, (const float4 *)c->fq_d.p, (const float *)c->tr_target.p,
                           (uint32_t)n, c->scale, &loss)))
    return rc;
  mtx_train_stats st{};
  st.loss = loss;
  if ((rc = field_opt_step(c, &st))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (stats) *stats = st;
  return MTX_OK;
}

int mtx_field_params(mtx_ctx *c, float *table, float *weights, float *m, float *v) {
  int rc = train_check(c);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t nt = c->field_n_table, nw = c->field_n_w;
  if (table) HIP_TRY(hipMemcpy(table, c->tr_p.p, 4 * nt, hipMemcpyDeviceToHost));
  if (weights) HIP_TRY(hipMemcpy(weights, (const float *)c->tr_p.p + nt, 4 * nw, hipMemcpyDeviceToHost));
  if (m) HIP_TRY(hipMemcpy(m, c->tr_m.p, 4 * (nt + nw), hipMemcpyDeviceToHost));
  if (v) HIP_TRY(hipMemcpy(v, c->tr_v.p, 4 * (nt + nw), hipMemcpyDeviceToHost));
  return MTX_OK;
}

int mtx_nerad_upload(mtx_ctx *c, const mtx_nerad_tables *t) {
  if (!c || !t || !c->has_scene) {
    mtx_set_error("mtx_nerad_upload: null argument or no scene");
    return MTX_E_ARG;
  }
  const uint32_t S = t->n_shapes, E = t->n_entries;
  if (S != c->scene_n_shapes || !t->shape_pmf || !t->shape_cdf || !t->tri_off || !t->tri_pmf || !t->tri_cdf ||
      !t->tri_prim || !t->tri_sum || !t->tri_norm || !t->tri_valid || t->tri_off[S] != E ||
      t->shape_valid[0] > t->shape_valid[1] || t->shape_valid[1] >= S) {
    mtx_set_error("mtx_nerad_upload: tables do not match the scene (%u shapes)", c->scene_n_shapes);
    return MTX_E_ARG;
  }
  for (uint32_t k = 0; k < S; ++k) {
    const uint32_t cnt = t->tri_off[k + 1] - t->tri_off[k];
    if (t->tri_off[k + 1] < t->tri_off[k] || cnt == 0 || t->tri_valid[2 * k] > t->tri_valid[2 * k + 1] ||
        t->tri_valid[2 * k + 1] >= cnt) {
      mtx_set_error("mtx_nerad_upload: bad triangle range of shape %u", k);
      return MTX_E_ARG;
    }
  }
  for (uint32_t i = 0; i < E; ++i)
    if (t->tri_prim[i] >= c->scene.n_tris) {
      mtx_set_error("mtx_nerad_upload: tri_prim[%u] out of range", i);
      return MTX_E_ARG;
    }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = upload(c->nr_shape_pmf, t->shape_pmf, S, c->stream))) return rc;
  if ((rc = upload(c->nr_shape_cdf, t->shape_cdf, S, c->stream))) return rc;
  if ((rc = upload(c->nr_tri_off, t->tri_off, S + 1, c->stream))) return rc;
  if ((rc = upload(c->nr_tri_pmf, t->tri_pmf, E, c->stream))) return rc;
  if ((rc = upload(c->nr_tri_cdf, t->tri_cdf, E, c->stream))) return rc;
  if ((rc = upload(c->nr_tri_prim, t->tri_prim, E, c->stream))) return rc;
  std::vector<mtx::DiscreteDist> d(S);
  for (uint32_t k = 0; k < S; ++k) {
    const uint32_t off = t->tri_off[k];
    d[k].pmf = (const float *)c->nr_tri_pmf.p + off;
    d[k].cdf = (const float *)c->nr_tri_cdf.p + off;
    d[k].n = t->tri_off[k + 1] - off;
    d[k].valid_lo = t->tri_valid[2 * k];
    d[k].valid_hi = t->tri_valid[2 * k + 1];
    d[k].sum = t->tri_sum[k];
    d[k].normalization = t->tri_norm[k];
  }
  if ((rc = upload(c->nr_dists, d.data(), S, c->stream))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  mtx::NeradTables &n = c->nr;
  n.shape.pmf = (const float *)c->nr_shape_pmf.p;
  n.shape.cdf = (const float *)c->nr_shape_cdf.p;
  n.shape.n = S;
  n.shape.valid_lo = t->shape_valid[0];
  n.shape.valid_hi = t->shape_valid[1];
  n.shape.sum = t->shape_sum;
  n.shape.normalization = t->shape_norm;
  n.tri_dist = (const mtx::DiscreteDist *)c->nr_dists.p;
  n.tri_off = (const uint32_t *)c->nr_tri_off.p;
  n.tri_prim = (const uint32_t *)c->nr_tri_prim.p;
  c->has_nerad = true;
  return MTX_OK;
}

int mtx_nerad_lhs(mtx_ctx *c, const mtx_nerad_args *a, float *out) {
  int rc = nerad_check(c, a, false);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = nerad_lhs_dev(c, a))) return rc;
  if (out) {
    std::vector<float> raw(12ull * a->batch);
    HIP_TRY(hipMemcpyAsync(raw.data(), c->nr_lhs.p, 48ull * a->batch, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (uint64_t i = 0; i < a->batch; ++i) {
      const float *r = raw.data() + 12 * i;
      float *o = out + 9 * i;
      o[0] = r[3];  // prim bits
      o[1] = r[7];
      o[2] = r[8];
      o[3] = r[0];
      o[4] = r[1];
      o[5] = r[2];
      o[6] = r[4];
      o[7] = r[5];
      o[8] = r[6];
    }
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

int mtx_nerad_rhs(mtx_ctx *c, const mtx_nerad_args *a, float *L_rhs, float *lanes) {
  int rc = nerad_check(c, a);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = nerad_lhs_dev(c, a))) return rc;
  float *lanes_dev = nullptr;
  if (lanes) {
    if ((rc = dalloc(c->nr_lanes, 12ull * a->batch * a->M))) return rc;
    lanes_dev = (float *)c->nr_lanes.p;
  }
  if ((rc = nerad_rhs_dev(c, a, lanes_dev, nullptr))) return rc;
  if (L_rhs) HIP_TRY(hipMemcpyAsync(L_rhs, c->nr_Lrhs.p, 12ull * a->batch, hipMemcpyDeviceToHost, c->stream));
  if (lanes) HIP_TRY(hipMemcpyAsync(lanes, lanes_dev, 12ull * a->batch * a->M, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MTX_OK;
}

int mtx_nerad_step(mtx_ctx *c, const mtx_nerad_args *a, mtx_train_stats *stats) {
  int rc = nerad_check(c, a);
  if (rc || (rc = train_check(c))) return rc;
  HIP_TRY(hipSetDevice(c->device));
  PhaseTimer pt(c->stream);
  pt.mark(0);
  if ((rc = nerad_lhs_dev(c, a))) return rc;  // si_lhs = isampler.sample(sampler_lhs) (:365)
  pt.mark(1);
  uint32_t nq = 0;
  mtx_train_stats st{};
  if ((rc = nerad_rhs_dev(c, a, nullptr, &nq, &st))) return rc;  // L_rhs = sample_rhs(si_lhs) (:368)
  pt.mark(2);
  double loss = 0.0;  // L_lhs = Field(si_lhs), loss, backward (:367-372)
  if ((rc = field_backward(c, (const float4 *)c->nr_qp.p, (const float4 *)c->nr_qd.p, (const float *)c->nr_Lrhs.p,
                           a->batch, c->scale, &loss)))
    return rc;
  st.loss = loss;
  if ((rc = field_opt_step(c, &st))) return rc;  // scaler.step(opt) (:373)
  pt.mark(3);
  HIP_TRY(hipStreamSynchronize(c->stream));
  st.rhs_queries = nq;
  st.ms_lhs = pt.ms(0, 1);
  st.ms_rhs = pt.ms(1, 2);
  st.ms_train = pt.ms(2, 3);
  st.ms_total = pt.ms(0, 3);
  if (stats) *stats = st;
  return MTX_OK;
}

}  // extern "C"
