// wavefront.h — device-side data layout of the MI355X wavefront integrator
// and the host-visible launch wrappers implemented in the .hip files.
//
// A chunk of C paths lives in HBM as SoA arrays of 16-byte records (one
// dwordx4 load/store per field group per lane):
//   ray_o  float4  o.xyz, maxt
//   ray_d  float4  d.xyz, a0 (NRC footprint, nrc.py:121)
//   thr    float4  throughput.xyz, eta
//   prev   float4  prev_si.p.xyz, spread (NRC, nrc.py:91-93)
//   L      float4  result.xyz, prev_bsdf_pdf
//   misc   uint4   rng.state lo/hi, rng.seq, depth | flags << 16
//   pos    float2  film sample position (block.put position, path.py:101)
//   hit    float4  t, prim, u, v (written by the closest-hit traversal)
// ray_o / ray_d / thr / prev / L / misc travel with the path's queue entry:
// two planes each, by bounce parity, indexed by queue position (the trace
// and shade kernels read them coalesced; the shade stores a continuing
// path's next state at its append slot). L and misc have a third, per-path
// plane that an ending path's state lands in (film, chain and ReSTIR
// kernels). pos is per path, hit per queue position. Paths of a chunk are
// pixel-major: path = q * spp + s for sample s of the chunk's pixel q.
// Queues are u32 path indices compacted per 256-thread block (ballot + mbcnt
// + LDS, one atomic per block step); shadow rays are 64-byte records.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtx.h"
#include "mtx_core/nerad.h"

namespace mtxd {

enum : uint32_t {
  PF_VALID_RAY = 1u,   // path-mis.py:129-133 valid_ray
  PF_PREV_DELTA = 2u,  // path-mis.py:137 prev_bsdf_delta
  PF_PRIMARY_VALID = 4u,
  PF_CACHE_QUERY = 8u,  // NRC: the next hit is the radiance-cache query
};

#ifndef MTX_TRACE_BLOCK
#define MTX_TRACE_BLOCK 256  // 8 blocks of 4 waves per CU: 20 KB of LDS each (stack + tree top)
#endif
constexpr int kTraceBlock = MTX_TRACE_BLOCK;  // threads per traversal block
constexpr int kShadeBlock = 256;             // threads per shade / path-megakernel block
// LDS part of the persistent traversal stacks (per lane) and the tree tops
// copied into LDS per trace block; both kernels' blocks take ~20 KB (8 per CU):
// closest hit 16 x 4-B node refs + 64 x 64-B nodes, occlusion 8 x 8-B node
// groups + 48 x 80-B nodes
constexpr uint32_t kLdsStack = 16;
constexpr uint32_t kOccLdsStack = 8;
#ifndef MTX_LDS_TOP
#define MTX_LDS_TOP 64  // closest-hit tree nodes copied into LDS per trace block (0 = none)
#endif
#ifndef MTX_OCC_LDS_TOP
#define MTX_OCC_LDS_TOP 48  // occlusion tree nodes copied into LDS per trace block (0 = none)
#endif
#ifndef MTX_SHADE_WARM
#define MTX_SHADE_WARM 1  // k_shade: warm L2 with the next entry's shading record
#endif
#ifndef MTX_CACHE_SORT
#define MTX_CACHE_SORT 2  // NRC cache query order (api.cpp run_cache): 0 as appended, 1 Morton sort, 2 region x XCD
#endif
#ifndef MTX_ENCODE_LM
#define MTX_ENCODE_LM 1  // NRC cache encoder with level-major lanes (field.hip k_field_encode_lm)
#endif
#ifndef MTX_STREAMS
#define MTX_STREAMS 2  // mtx_render: chunks alternate between two wavefronts on two streams (1 = one)
#endif

// Per-XCD claim cursors of the persistent trace kernels: kXcds words,
// kXHeadStride words (128 B) apart; one slot per trace launch of a chunk.
constexpr uint32_t kXcds = 8;
constexpr uint32_t kXHeadStride = 32;
constexpr uint32_t kXSlotWords = kXcds * kXHeadStride;

struct DevScene {
  const int4 *nodes;      // closest-hit BVH: 4 x int4 per node (the 64-B ABI node, mtx.h)
  const float *tri;       // its leaf-order triangles, 9 floats each (v0, e1, e2; device_common.h load_tri)
  const int4 *occ_nodes;  // occlusion BVH: 5 x int4 per node (the 80-B ABI node, mtx.h)
  const float *occ_tri;   // its own leaf-order copy of the triangles (9 floats each)
  const uint32_t *tri_vidx;
  const uint32_t *tri_shape;
  const float *vpos;
  const float *vnormal;
  const float *vuv;
  const mtx_shape *shapes;
  const float4 *shade_rec;  // 8 float4 per triangle (device_common.h compute_si_dev)
  const mtx_material *materials;
  const mtx_emitter *emitters;
  const mtx_texture *textures;
  const float *texels;
  const float *tables;
  uint32_t n_tris, n_emitters;
  uint32_t stack_entries;  // closest hit: 3 x depth + 1 stack entries per lane (4-B node refs)
  uint32_t lds_entries;    // persistent kernels: stack entries kept in LDS
  uint32_t lds_top;        // persistent kernels: nodes [0, lds_top) read from a per-block LDS copy
  uint32_t occ_stack_entries, occ_lds_entries, occ_lds_top;  // the same for the occlusion tree
                                                             // (depth + 1 entries: 8-B node groups)
  uint32_t trace_batch;    // persistent kernels: queue entries claimed per atomic
  void *stack_ovf;         // persistent kernels: entries beyond the LDS part, [entry][thread]
                           // (int32 node refs for closest hit, uint2 node groups for occlusion)
  uint32_t ovf_threads;    // threads of the persistent trace grid
  uint32_t urefill;        // persistent kernels: refill a wave once this many lanes are idle
  uint32_t occ_urefill;    // the same for the any-hit kernels
  uint32_t xcd_claim;      // persistent kernels: claim rays from the own XCD's queue segment first
  mtx_camera camera;
  // constant environment (mtx_core/interaction.h SceneView: emitter index n_emitters)
  uint32_t has_env;
  float env_radiance[3], env_center[3], env_radius;
};

// Global spill area of a wavefront's traversals (the deeper of the two
// trees' needs; closest-hit and any-hit launches of one wavefront never
// overlap).
inline size_t stack_ovf_bytes(const DevScene &s) {
  const size_t a = (size_t)(s.stack_entries - s.lds_entries) * sizeof(int32_t);
  const size_t b = (size_t)(s.occ_stack_entries - s.occ_lds_entries) * sizeof(uint2);
  const size_t n = (a > b ? a : b) * s.ovf_threads;
  return n > 8 ? n : 8;
}

// Shadow-ray record (64 B): o.xyz maxt | d.xyz L index | t | x (L index =
// plane * capacity + position of the path's L, WaveBuffers). As make_shadow
// builds it: t = T.xyz flags, x = X.xyz 0; flags bit0: fma form
// L = fma(T, X, L) (path-mis.py:117) else L = L + X (path.py:259, nrc.py:62);
// bits 1..3: the occluded-case contribution of that channel is NaN
// (non-finite BSDF value / MIS weight), see DESIGN.md. As k_shade stores it
// for the integrators whose L it stores (kernels.hip make_shadow, flag bit
// 4): t = the L after an unoccluded ray | flags, x = the L before it.
constexpr int kFinal = 2;  // the per-path plane of L / misc

struct ShadowRec {
  float4 o;
  float4 d;
  float4 t;
  float4 x;
};

struct WaveBuffers {
  // rays of bounce b at ray_o / ray_d[(b + ray_par) & 1][k] for queue position
  // k: the trace loads them coalesced, the shade writes the next ray at its
  // append slot (no path-indexed scatter on either side)
  float4 *ray_o[2], *ray_d[2];
  uint32_t ray_par;
  // throughput and previous vertex move with the ray the same way (the nerad
  // integrators keep them path-indexed in plane 0: k_nerad_apply reads them)
  float4 *thr[2], *prev[2];
  // result and sampler state: planes 0 / 1 by queue position (bounce parity,
  // as the rays), plane kFinal by path -- a path's state lands there when it
  // ends (k_shade; k_flush_tail for paths still queued after the last
  // bounce), where the film, k_collect and the PSSMLT / ReSTIR / nerad
  // kernels read it. The three L planes are contiguous (capacity apart):
  // a shadow record addresses its target as plane * capacity + index.
  float4 *L[3];
  uint4 *misc[3];
  float2 *pos;
  float4 *hit;
  uint32_t *queue[2];
  ShadowRec *shadow;
  uint32_t *counters;   // per bounce b: [4b+0] rays of bounce b, [4b+1] shadow rays of bounce b-1 (one 8-B pair with the queue shade b-1 fills), [4b+2], [4b+3] unused
  uint32_t *xheads;     // per bounce b: slot 2b closest-hit, 2b+1 shadow claim cursors (kXSlotWords each)
  unsigned long long *stats;  // nodes_c, tris_c, nodes_s, tris_s, rays_c, rays_s
  uint32_t capacity;
  // PSSMLT chain state (pssmlt.py:196-200): offset.xy, cumulative weight | L | proposed offset,
  // and the current / proposed path vertices (PathVert.wo, depth-major: [depth * capacity + chain]).
  float4 *mlt_cur;
  float4 *mlt_L;
  float2 *mlt_prop;
  float4 *vpath;
  float4 *vprop;
  float2 *vpath_es;  // pssmltpath.py PathVert.emitter_sample (current / proposed)
  float2 *vprop_es;
  // ReSTIR GI: first hit of the secondary path (restirgi.py:452-455), written
  // by the bounce-0 shade (path order).
  float4 *rs_xs;
  float4 *rs_ns;
  // NRC radiance-cache queries (compacted): p, -d, (T, path), count
  float4 *cq_p, *cq_d, *cq_t;
  uint32_t *cq_count;
};

// ReSTIR GI frame state (restirgi.py:217-226, 230-231). Sample / reservoir
// planes as in mtx_core/restir.h; `n` = W*H*spp lanes of one frame.
struct RestirBuffers {
  float4 *cur;        // 5 planes: this frame's samples
  const float4 *prev; // 5 planes: previous frame's samples (== cur at frame 0)
  float4 *tres;       // 6 planes: temporal reservoirs
  float4 *sres;       // 6 planes: spatial reservoirs
  float *radius;      // search radius per lane
  float4 *prim_hit;   // primary closest hit (t, prim, u, v)
  float4 *prim_dir;   // primary ray direction
  float4 *emit;       // emittance at the primary hit (:421-423)
  uint4 *rng;         // sampler state between the phases
  float4 *test_rays;  // compacted visibility tests: (o, maxt), (d, slot)
  uint32_t *test_count;  // [0] count
  uint32_t *test_heads;  // per-XCD claim cursors of k_trace_test (kXSlotWords)
  uint8_t *occ;       // 18 per lane: spatial tests [0,9), bias-correction tests [9,18)
  uint32_t *qM;       // 10 per lane: Q.M with bit 31 = active, [9] = Z before the loop
  uint32_t *nbr;      // 10 per lane: the 9 spatial candidates' lanes, [9] = active mask (rays -> merge)
  uint32_t n;      // lanes of the whole frame (state arrays)
  uint32_t lane0;  // first lane of the rows this call computes
  uint32_t nb;     // lanes this call computes (row band)
  mtx_camera prev_cam;
  uint32_t flags, max_M_temporal, max_M_spatial;
  uint32_t xcd_remap;  // k_rs_* neighbour passes: XCD-banded block order
  float initial_radius, minimal_radius;
  uint32_t frame;
};

struct ChunkParams {
  uint32_t integrator, max_depth, rr_depth, seed;
  uint32_t spp, spp_total, sample_offset;
  uint32_t width, height;
  uint32_t px0, n_px;   // first film pixel (y*W+x) of the chunk and pixel count
  uint32_t band_y0;     // first row of the rendered band (film/contrib origin)
  uint32_t band_px;     // pixels of the band (contrib: film_slots x 9 planes of band_px float4)
  uint32_t film_slots;  // 8: partial-slot film (mtx_core/common.h film_slot); 0 / 1: one slot
  uint32_t slot_mask;   // film_slots == 8: the slots this render's samples fall in (the others are
                        // neither written nor read: they are zero, and x + 0 is x in the slot tree)
  uint32_t n_paths;
  float nrc_c;
  uint32_t stats;
  uint32_t large_step;  // PSSMLT: i % 50 == 0 (pssmlt.py:209)
  uint32_t restir;      // ReSTIR GI secondary paths (path-mis loop, restirgi.py:459-588)
  uint32_t nrc_cache;     // NRC: query the radiance field where the spread criterion stops
  uint32_t drop_end_misc; // film render: an ending path's sampler state is never read (its L is)
  uint32_t ident0;        // the bounce-0 queue is the identity (raygen): not stored, k_shade uses position = path
};

// -------- launch wrappers (kernels.hip) --------
int trace_blocks_per_cu(const DevScene &s);    // any-hit kernels
int closest_blocks_per_cu(const DevScene &s);  // k_trace_closest
int shade_blocks_per_cu();
int mega_blocks_per_cu(const DevScene &s);
// all bounces of a short path-mis / path wavefront in one kernel (k_path_mega)
void launch_path_mega(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, int grid, hipStream_t st);
// ReSTIR GI stage A of a short band (raygen .. collect) in one per-lane launch (kernels.hip)
void launch_rs_stage_a(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                       int grid, hipStream_t st);
int shade_stamps(unsigned long long *out);  // diagnostic builds (MTX_DIAG_STAMPS)
void launch_raygen_camera(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, hipStream_t st);
void launch_raygen_rays(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const float *rays,
                        const uint32_t *lanes, uint32_t rng_skip, hipStream_t st);
void launch_trace_closest(const DevScene &s, const WaveBuffers &b, uint32_t bounce, uint32_t stats, int grid,
                          hipStream_t st);
void launch_trace_shadow(const DevScene &s, const WaveBuffers &b, uint32_t bounce, uint32_t stats, int grid,
                         hipStream_t st);
void launch_shade(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, uint32_t bounce, int grid,
                  hipStream_t st);
void launch_film_src(const WaveBuffers &b, const ChunkParams &p, float4 *contrib, hipStream_t st);
void launch_film_gather(const float4 *contrib, float4 *film, uint32_t width, uint32_t y0, uint32_t y1,
                        uint32_t nslots, uint32_t slot_mask, hipStream_t st);
void launch_mlt_init(const WaveBuffers &b, const ChunkParams &p, hipStream_t st);
void launch_mlt_begin(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, hipStream_t st);
void launch_mlt_end(const WaveBuffers &b, const ChunkParams &p, hipStream_t st);
void launch_mlt_film(const WaveBuffers &b, const ChunkParams &p, float4 *contrib, hipStream_t st);
void launch_flush_tail(const WaveBuffers &b, uint32_t bounce, uint32_t capacity, uint32_t integrator,
                       hipStream_t st);
void launch_collect(const WaveBuffers &b, const ChunkParams &p, float *L_out, uint8_t *valid_out, hipStream_t st);
// perm (optional): MLP row q belongs to cache query perm[q]
void launch_cache_apply(const WaveBuffers &b, const float *out, uint32_t capacity, hipStream_t st,
                        const uint32_t *perm = nullptr);
// ReSTIR GI (restir.hip)
void launch_restir_begin(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                         hipStream_t st);
void launch_restir_collect(const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r, hipStream_t st);
void launch_restir_temporal(const RestirBuffers &r, const ChunkParams &p, hipStream_t st);
void launch_restir_spatial_rays(const RestirBuffers &r, const ChunkParams &p, hipStream_t st);
void launch_restir_spatial_merge(const RestirBuffers &r, const ChunkParams &p, hipStream_t st);
void launch_restir_bias_finish(const RestirBuffers &r, const ChunkParams &p, hipStream_t st);
void launch_restir_final(const DevScene &s, const WaveBuffers &b, const ChunkParams &p, const RestirBuffers &r,
                         hipStream_t st);
void launch_trace_test(const DevScene &s, const RestirBuffers &r, uint32_t occ_base, int grid, hipStream_t st);
void launch_trace_raw(const DevScene &s, const float4 *rays, uint32_t n, int any_hit, uint32_t *hits,
                      uint32_t *visits, hipStream_t st);
// neural radiosity training samples (nerad.hip)
void launch_nerad_lhs(const DevScene &s, const mtx::NeradTables &t, uint32_t seed, uint32_t n, float4 *lhs,
                      float4 *qp, float4 *qd, hipStream_t st);
void launch_nerad_raygen(const WaveBuffers &b, const ChunkParams &p, const float4 *lhs, uint32_t M, hipStream_t st);
void launch_nerad_apply(const WaveBuffers &b, const float *out, uint32_t capacity, uint32_t render,
                        hipStream_t st);
void launch_nerad_mean(const WaveBuffers &b, uint32_t n, uint32_t M, float *L_rhs, float *lanes, hipStream_t st);

}  // namespace mtxd
