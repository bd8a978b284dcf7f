/* mtx.h — C ABI of libmtx, the MI355X (gfx950) wavefront path-tracing
 * integrator that replaces the per-bounce `sample()` loop of
 * DoeringChristian/mitsuba3-experiments.
 *
 * Plain C: fixed-width integers, floats, pointers and sizes only. Every entry
 * point returns 0 on success and a negative MTX_E* code on failure; the
 * message is available from mtx_last_error() (thread-local). No exceptions
 * cross the ABI. Host buffers are caller-owned and only read/written during
 * the call; calls are synchronous with respect to their outputs. A context
 * is bound to one HIP device and is not thread-safe: one host thread per
 * context (ctypes releases the GIL during the call, so N Python threads or N
 * processes can drive N GPUs).
 *
 * What each entry point replaces in the reference (file:line under the
 * reference root) is stated above its declaration. The ctypes binding a
 * maintainer adds on the reference side is in INTEGRATION.md.
 */
#ifndef MTX_H_
#define MTX_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTX_ABI_VERSION 8

enum {
  MTX_OK = 0,
  MTX_E_ARG = -1,     /* bad argument / shape mismatch */
  MTX_E_HIP = -2,     /* HIP runtime error */
  MTX_E_NOSCENE = -3, /* no scene uploaded */
  MTX_E_OOM = -4,     /* device allocation failed */
  MTX_E_UNSUPPORTED = -5
};

/* ------------------------------------------------------------------ */
/* Scene layout (SoA records copied to HBM as-is by mtx_scene_upload). */
/* ------------------------------------------------------------------ */

/* Material types: the 8 BSDF plugins of data/bedroom/scene.xml:26-219. */
enum {
  MTX_MAT_DIFFUSE = 1,         /* diffuse (rgb or bitmap reflectance) */
  MTX_MAT_ROUGHPLASTIC = 2,    /* roughplastic (ggx/beckmann, nonlinear) */
  MTX_MAT_CONDUCTOR = 3,       /* conductor (smooth) */
  MTX_MAT_ROUGHCONDUCTOR = 4,  /* roughconductor (ggx/beckmann) */
  MTX_MAT_DIELECTRIC = 5,      /* dielectric (smooth) */
  MTX_MAT_ROUGHDIELECTRIC = 6  /* roughdielectric */
};
/* Material flags. A `mask` BSDF is its nested BSDF + MTX_MF_MASK + opacity;
 * a `twosided` wrapper is MTX_MF_TWOSIDED on the nested BSDF. */
enum {
  MTX_MF_TWOSIDED = 1,
  MTX_MF_MASK = 2,
  MTX_MF_BECKMANN = 4, /* microfacet distribution: 0 = ggx */
  MTX_MF_NONLINEAR = 8
};

#define MTX_ROUGH_TRANSMITTANCE_RES 64

typedef struct mtx_material {
  uint32_t type;
  uint32_t flags;
  int32_t tex;           /* bitmap texture index for (diffuse_)reflectance, -1 = use rgb */
  float opacity;         /* mask opacity */
  float rgb[3];          /* reflectance | diffuse_reflectance | specular_reflectance */
  float alpha;           /* microfacet roughness */
  float eta;             /* int_ior / ext_ior (dielectric, roughdielectric, roughplastic) */
  float eta_rgb[3];      /* conductor eta (real part) */
  float k_rgb[3];        /* conductor k (imaginary part) */
  float spec_weight;     /* roughplastic specular sampling weight */
  float internal_refl;   /* roughplastic internal reflectance */
  int32_t table;         /* roughplastic: offset (floats) of its 64-entry external transmittance table */
} mtx_material;

typedef struct mtx_texture {
  uint32_t width, height;
  uint64_t offset; /* offset (in floats) into texels[], RGB interleaved, linear */
} mtx_texture;

/* Area emitter on a `rectangle` shape (scene.xml:706-731). */
typedef struct mtx_emitter {
  float center[3];  /* to_world translation */
  float col0[3];    /* to_world * (1,0,0) */
  float col1[3];    /* to_world * (0,1,0) */
  float normal[3];  /* normalize(inverse-transpose(to_world) * (0,0,1)) */
  float inv_area;   /* 1 / |cross(2 col0, 2 col1)| */
  float radiance[3];
} mtx_emitter;

typedef struct mtx_shape {
  uint32_t material;
  int32_t emitter; /* -1 if not an emitter */
  uint32_t flags;  /* bit0: face_normals / no vertex normals, bit1: has uv */
  uint32_t pad;
} mtx_shape;

/* Perspective sensor (scene.xml:10-25). */
typedef struct mtx_camera {
  float origin[3];  /* to_world translation */
  float axis_x[3];  /* to_world columns */
  float axis_y[3];
  float axis_z[3];
  float tan_x, tan_y; /* tan(fov_x/2), tan(fov_x/2) / aspect */
  float near_clip, far_clip;
  uint32_t width, height;
  float inv_rows[9];  /* rows of inverse([axis_x axis_y axis_z]) (world -> camera) */
  uint32_t pad;
} mtx_camera;

/* A scene carries two BVHs over the same triangles (round 4: each is the
 * faster form for its query):
 *
 * Closest-hit BVH node (64 B, Scene.ray_intersect): up to 4 children with
 * 8-bit quantised boxes, collapsed from a binned-SAH BVH2 by dynamic
 * programming over the 4-wide tree's SAH (bvh_build.cpp); visited near child
 * first (the traversal sorts the four entry distances). Breadth-first, the
 * inner children of a node consecutive and first in slot order, then its
 * leaves, whose triangle ranges are consecutive. Words:
 *   f[0..2] = origin.xyz (fp32);  w[3] = bytes [ex, ey, ez, n_children],
 *             e* int8 in [-32, 31]: axis scale 2^e
 *   i[4..7] = child refs: >= 0 inner node index,
 *             < 0 leaf: ~c = (first_tri << 3) | (count - 1)
 *   w[8..13] = q_lo.x, q_hi.x, q_lo.y, q_hi.y, q_lo.z, q_hi.z: one byte per
 *             child (child k in bits 8k..8k+7); bound = origin + q * 2^e in
 *             fp32, conservative (contains the child's padded box)
 *   w[14], w[15] = 0
 * Its leaf order is THE triangle order of the scene (tri_geom, tri_vidx,
 * tri_shape, hit records' prim). Triangles are 12 floats (48 B):
 *   v0.xyz, 0, e1 = v1-v0 .xyz, 0, e2 = v2-v0 .xyz, 0 */
#define MTX_BVH_WIDTH 4
#define MTX_BVH_MAX_LEAF 8
#define MTX_BVH_NODE_WORDS 16
#define MTX_BVH_MAX_DEPTH 40

/* Occlusion BVH node (80 B, Scene.ray_test: any hit; a compressed 8-wide
 * node after Ylitie, Karras & Laine 2017), built over the closest-hit
 * tree's triangle records (mtx_bvh_build_occlusion) with its own leaf order
 * and its own copy of the records (occ_tri_geom): up to 8 children with
 * 8-bit quantised boxes, collapsed from a binned-SAH BVH2 by dynamic
 * programming over the 8-wide tree's SAH. The children sit in slots chosen
 * so that visiting slot s at position s ^ octant(ray) (octant bit a set when
 * the direction's component a is negative) is approximately front to back:
 * no per-visit sort. Breadth-first; a node's inner children are consecutive
 * from child_base in slot order, its leaves' triangles consecutive from
 * tri_base in slot order. Words:
 *   f[0..2]  origin.xyz (fp32)
 *   w[3]     bytes [ex, ey, ez, imask]: int8 axis exponents in [-32, 31]
 *            (axis scale 2^e); imask bit s set: slot s holds an inner node
 *   w[4]     child_base: node index of the first inner child; the inner
 *            child in slot s is child_base + popcount(imask & ((1 << s) - 1))
 *   w[5]     tri_base: first triangle (occlusion leaf order) of the leaves
 *   w[6..7]  meta, one byte per slot (slot s in byte s of the 8):
 *              0 = empty; inner: 0x20 | (24 + s);
 *              leaf of n = 1..3 triangles: ((1 << n) - 1) << 5 | offset,
 *              its triangles tri_base + offset .. + n - 1 (offset + n <= 24)
 *   w[8..19] q_lo.x, q_hi.x, q_lo.y, q_hi.y, q_lo.z, q_hi.z: 8 bytes each
 *            (two words, slot s in byte s); bound = origin + q * 2^e in
 *            fp32, conservative (contains the child's padded box); empty
 *            slots hold q_lo 255, q_hi 0 */
#define MTX_OCC_WIDTH 8
#define MTX_OCC_MAX_LEAF 3
#define MTX_OCC_NODE_WORDS 20

typedef struct mtx_scene_desc {
  uint32_t n_tris, n_nodes, n_verts, n_shapes;
  uint32_t n_materials, n_emitters, n_textures, flags;
  const int32_t *nodes;      /* closest-hit BVH: MTX_BVH_NODE_WORDS (16) words per node */
  const float *tri_geom;     /* 12 floats per triangle (leaf order) */
  const uint32_t *tri_vidx;  /* 3 vertex indices per triangle (leaf order) */
  const uint32_t *tri_shape; /* shape index per triangle (leaf order) */
  const float *vpos;         /* 3 per vertex */
  const float *vnormal;      /* 3 per vertex, may be NULL */
  const float *vuv;          /* 2 per vertex, may be NULL */
  const mtx_shape *shapes;
  const mtx_material *materials;
  const mtx_emitter *emitters;
  const mtx_texture *textures;
  const float *texels;
  uint64_t n_texels;         /* floats */
  const float *tables;       /* roughplastic transmittance tables */
  uint32_t n_tables;         /* floats */
  uint32_t pad0;
  mtx_camera camera;
  /* occlusion BVH (MTX_OCC_NODE_WORDS words per node) and its triangle
   * records (12 floats each, its leaf order): both NULL = mtx_scene_upload
   * builds them (mtx_bvh_build_occlusion over tri_geom) */
  const int32_t *occ_nodes;
  const float *occ_tri_geom;
  uint32_t n_occ_nodes, pad1;
  /* scene triangle (closest-hit leaf order) of each occlusion leaf-order
   * triangle (mtx_bvh_build_occlusion's perm). Given with occ_nodes /
   * occ_tri_geom: mtx_scene_upload checks occ_tri_geom[i] ==
   * tri_geom[occ_perm[i]] for every i and that it is a permutation; NULL
   * with given trees: derived at upload by matching the records, and the
   * trees rejected (MTX_E_ARG) unless occ_tri_geom is a permutation of
   * tri_geom. */
  const uint32_t *occ_perm;
  /* constant environment emitter (Mitsuba `constant`, the scene.environment()
   * of path-mis.py:41 / pssmltpath.py:39 / restirgi.py:475; mtx_core/interaction.h):
   * has_env != 0 adds it as emitter index n_emitters, picked uniformly with the
   * area emitters; its bounding sphere is that of the vertices' box. With
   * has_env, n_emitters may be 0. (ABI 8) */
  float env_radiance[3];
  uint32_t has_env;
} mtx_scene_desc;

/* Integrators (the reference scripts whose sample() loop is replaced). */
enum {
  MTX_INT_PATH = 1,          /* path.py:194-302 ("mypath") */
  MTX_INT_PATH_MIS = 2,      /* path-mis.py:24-155 ("path_test") */
  MTX_INT_NRC = 3,           /* nrc.py:25-125 */
  MTX_INT_PSSMLT_SIMPLE = 4, /* pssmlt.py:167-228 + pssmltsimple.py:16-142 */
  MTX_INT_RESTIR_GI = 5,     /* restirgi.py:182-588 */
  MTX_INT_PSSMLT_PATH = 6,   /* pssmlt.py:167-228 + pssmltpath.py:17-190 ("pssmlt") */
  MTX_INT_NERAD_RHS = 7,     /* nerad.py:174-233 Integrator.sample_rhs (internal: mtx_nerad_*) */
  MTX_INT_NERAD = 8,         /* nerad.py:235-254 Integrator.sample: next_smooth_si + the uploaded field
                                (max_depth = 11: first hit + up to 10 delta bounces) */
  MTX_INT_SIMPLE = 9         /* simple.py:14-116 ("integrator"): BSDF sampling only, no NEE */
};

typedef struct mtx_render_args {
  uint32_t integrator;
  uint32_t max_depth;
  uint32_t rr_depth;
  uint32_t seed;
  uint32_t spp;          /* samples traced per pixel by this call */
  uint32_t spp_total;    /* samples per pixel of the whole job (lane stride) */
  uint32_t sample_offset;/* first global sample index of this call (rank shard) */
  uint32_t y0, y1;       /* film rows [y0, y1) traced by this call */
  uint32_t chunk_paths;  /* wavefront size (0 = default) */
  float nrc_c;           /* NRC spread threshold (nrc.py:123) */
  uint32_t flags;        /* bit0: collect traversal stats, bit1: per-kernel HIP event timing,
                            bit2 (NRC): query the uploaded radiance field where the spread
                            criterion ends a segment (NRC radiance cache) */
  uint32_t iterations;   /* PSSMLT Metropolis iterations (pssmlt.py:208: 200; 0 = 200) */
  uint32_t frame;        /* ReSTIR GI frame index (restirgi.py self.n); 0 resets the reservoirs */
  /* ReSTIR GI properties (restirgi.py:157-166) */
  uint32_t restir_flags; /* bit0 bias_correction, bit1 jacobian, bit2 bsdf_sampling, bit3 spatial_spatial_reuse */
  uint32_t max_M_temporal; /* 0 = None */
  uint32_t max_M_spatial;  /* 0 = None */
  float initial_search_radius;
  float minimal_search_radius;
  uint32_t reserved;
} mtx_render_args;

enum {
  MTX_RESTIR_BIAS_CORRECTION = 1,
  MTX_RESTIR_JACOBIAN = 2,
  MTX_RESTIR_BSDF_SAMPLING = 4,
  MTX_RESTIR_SPATIAL_SPATIAL = 8,
  /* row-banded frames (multi-GPU): stage A = sample_initial + temporal
   * resampling of rows [y0,y1); stage B = spatial resampling + render_final +
   * film of the same rows. Between them the caller imports the neighbours'
   * halo rows (mtx_restir_rows). Neither flag: the whole frame in one call. */
  MTX_RESTIR_STAGE_A = 16,
  MTX_RESTIR_STAGE_B = 32
};

/* Device-side counters, filled when mtx_render_args.flags has bit0/bit1. */
typedef struct mtx_stats {
  uint64_t rays_closest, rays_shadow;
  uint64_t nodes_closest, tris_closest; /* node / triangle visits */
  uint64_t nodes_shadow, tris_shadow;
  uint64_t trace_launches;              /* closest-hit traversal launches */
  uint64_t shadow_launches;
  double trace_ms, shadow_ms, shade_ms, other_ms; /* HIP-event time, summed */
  uint64_t paths;
  /* closest-hit traversal wave iterations (node phase, leaf phase): SIMD
   * utilisation = visits / (64 * iterations) */
  uint64_t wave_node_iters, wave_leaf_iters;
  /* NRC radiance cache (MTX_RENDER_NRC_CACHE): queries answered, HIP-event
   * time of the feature encoder and of the fused MLP (part of other_ms's
   * complement: other_ms excludes them) */
  uint64_t cache_queries;
  double cache_encode_ms, cache_mlp_ms;
  /* wavefronts / HIP streams the render ran on: > 1 means the per-kernel
   * times above are summed over overlapping launches (wall time is other_ms
   * + the kernels only for a one-stream render) */
  uint32_t streams, reserved;
} mtx_stats;

/* --------------------------- context ------------------------------ */
int mtx_abi_version(void);
const char *mtx_last_error(void);
typedef struct mtx_ctx mtx_ctx;
/* One context per HIP device; owns every device allocation. */
int mtx_ctx_create(int hip_device, mtx_ctx **out);
void mtx_ctx_destroy(mtx_ctx *ctx);

/* --------------------------- scene -------------------------------- */
/* Host-only BVH build over an indexed triangle mesh (replaces the Embree /
 * OptiX acceleration-structure build behind mi.load_file, upstream): binned-
 * SAH BVH2, collapsed to the 4-wide closest-hit node above.
 * nodes_out: capacity (n_tris + 1) * MTX_BVH_NODE_WORDS words; tri_geom_out:
 * 12*n_tris floats; perm_out: n_tris (leaf order -> input triangle index);
 * depth_out: levels of the 4-wide tree (the traversal stack's bound). */
int mtx_bvh_build(const float *vpos, uint32_t n_verts, const uint32_t *tri_vidx, uint32_t n_tris,
                  int32_t *nodes_out, uint32_t *n_nodes_out, float *tri_geom_out, uint32_t *perm_out,
                  uint32_t *depth_out);
/* Host-only occlusion BVH (8-wide node above) over n_tris triangle records
 * (12 floats each, e.g. mtx_bvh_build's tri_geom_out). nodes_out: capacity
 * (n_tris + 1) * MTX_OCC_NODE_WORDS words; tri_geom_out: the same records
 * (bit-identical) in the occlusion tree's leaf order; perm_out (may be NULL):
 * occlusion leaf order -> input record; depth_out: levels of the tree. */
int mtx_bvh_build_occlusion(const float *tri_geom, uint32_t n_tris, int32_t *nodes_out, uint32_t *n_nodes_out,
                            float *tri_geom_out, uint32_t *perm_out, uint32_t *depth_out);
/* Host-only roughplastic precompute (upstream roughplastic constructor):
 * external transmittance table (64 floats) and internal reflectance. */
int mtx_roughplastic_tables(uint32_t distribution, float alpha, float eta, float *table_out,
                            float *internal_refl_out);
/* Copy a scene to HBM (replaces mi.load_file / mi.load_dict scene
 * construction, path.py:308-309, restirgi.py:599). */
int mtx_scene_upload(mtx_ctx *ctx, const mtx_scene_desc *scene);

/* --------------------------- integrators -------------------------- */
/* Render film rows [y0,y1) (+1-pixel tent border) into film_rgbw, an
 * (y1-y0+2) x (width+2) x 4 float buffer (host pointer, or a device pointer
 * when film_on_device != 0): un-normalised RGB*weight and weight sums in a
 * fixed summation order. Replaces mi.render(scene, integrator, spp, seed)
 * driving SamplingIntegrator::render (transcribed path.py:103-192) with the
 * sample() of path.py:194-302 / path-mis.py:24-155 / nrc.py:104-125,
 * Pssmlt.render (pssmlt.py:167-228), and one RestirIntegrator.render frame
 * (restirgi.py:182-258; whole film only, y0 = 0, y1 = height, spp_total =
 * spp; args.frame = 0 resets the reservoirs kept in ctx, later frames reuse
 * them and the camera of the previous frame as prev_sensor). */
int mtx_render(mtx_ctx *ctx, const mtx_render_args *args, float *film_rgbw, int film_on_device,
               mtx_stats *stats);

/* Replace the sensor of the uploaded scene (mi.traverse(sensor).update,
 * test-restir-dynamic.py; restirgi.py:247 keeps the old one as prev_sensor
 * for the next ReSTIR frame). The film size must not change. */
int mtx_set_camera(mtx_ctx *ctx, const mtx_camera *camera);

/* Copy rows [row0, row0+nrows) of the ReSTIR GI state to (to_state = 0) or
 * from (to_state = 1) a device buffer, plane-major (planes x rows x W*spp
 * float4): which = 0 the current frame's samples (5 planes), 1 the temporal
 * reservoirs (6 planes), 2 the previous frame's samples (5 planes; between
 * frames only: the buffer temporal resampling reprojects into,
 * restirgi.py:374-383). The halo exchange of a row-banded frame
 * (restirgi.py:301-313 reads up to search_radius rows away; a
 * moving camera reprojects arbitrarily far, so a banded caller gathers the
 * whole previous-sample buffer with which = 2 before stage A). */
int mtx_restir_rows(mtx_ctx *ctx, int which, uint32_t row0, uint32_t nrows, void *buf, int to_state);

/* Read back ReSTIR GI frame state (test / debugging hook for restirgi.py's
 * self.sample, temporal_reservoir, spatial_reservoir, search_radius):
 * which = 0 samples (5 float4 planes), 1 temporal reservoirs (6 planes),
 * 2 spatial reservoirs (6 planes), 3 search radius (1 float per lane);
 * layout in include/mtx_core/restir.h. n_floats must match exactly. */
int mtx_restir_state(mtx_ctx *ctx, int which, float *out, uint64_t n_floats);

/* Evaluate the integrator's sample() for n given rays (replaces
 * SamplingIntegrator.sample(scene, sampler, ray), path-mis.py:24-31).
 * rays: 6n floats (o.xyz, d.xyz); lanes: n sampler lane ids; each lane's
 * PCG32 stream is seeded with (seed, lane) and advanced by rng_skip draws
 * before the first bounce (the render loop consumes 2 for the film jitter).
 * Outputs: L (3n floats), valid (n bytes). Host pointers. */
int mtx_sample_rays(mtx_ctx *ctx, const mtx_render_args *args, uint64_t n, const float *rays,
                    const uint32_t *lanes, uint32_t rng_skip, float *L, uint8_t *valid);

/* Device-pointer forms (SURVEY §8b mtx_device_ptrs): the reference calls
 * sample(), ray_intersect and its primitives on wavefront-wide Dr.Jit arrays
 * that live on the GPU (path.py:194-202, prefix_sum.py:9-36,
 * hashgrid.py:16-84, reductions.py:12-54). The *_dev functions take buffers
 * in the context's device memory (hipMalloc'd; e.g. a torch CUDA tensor's
 * data_ptr), with the layouts of their host twins, and copy nothing through
 * the host: no staging copy, results written in place. Work runs on the
 * context's stream and is complete on return (the caller orders its own
 * producer of the inputs before the call). A host pointer is refused
 * (MTX_E_ARG); device indices are range-checked on the device. */
int mtx_sample_rays_dev(mtx_ctx *ctx, const mtx_render_args *args, uint64_t n, const float *rays,
                        const uint32_t *lanes, uint32_t rng_skip, float *L, uint8_t *valid);

/* Raw closest-hit / any-hit traversal (Scene.ray_intersect / ray_test,
 * path-mis.py:69-71, restirgi.py:320). rays: 8n floats (o.xyz, tmax, d.xyz,
 * 0); any_hit: 0 closest hit (4-wide tree), 1 any hit (8-wide occlusion
 * tree); hits: 4n words
 * (t, prim, u, v) for closest hit, or n words (1 = occluded) for any hit.
 * visits (optional, 2n u32): node and triangle visits. */
int mtx_trace(mtx_ctx *ctx, uint64_t n, const float *rays, int any_hit, uint32_t *hits,
              uint32_t *visits);
/* mtx_trace on device buffers (Scene.ray_intersect on a device wavefront). */
int mtx_trace_dev(mtx_ctx *ctx, uint64_t n, const float *rays, int any_hit, uint32_t *hits,
                  uint32_t *visits);

/* --------------------------- primitives --------------------------- */
/* prefix_sum.py:9-36: inclusive (or exclusive) scan of u32, device-wide
 * decoupled look-back. Host pointers. */
int mtx_prefix_sum_u32(mtx_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n, int inclusive);
/* prefix_sum.py:9-36 with f32 data in Hillis-Steele summation order
 * (floor(log2 n)+1 passes x[j] += x[j-2^i]), bit-identical to the reference. */
int mtx_prefix_sum_f32_hs(mtx_ctx *ctx, const float *in, float *out, uint64_t n);
/* The two scans on device buffers (prefix_sum.py:9-36 on Dr.Jit arrays); the
 * input is not modified. */
int mtx_prefix_sum_u32_dev(mtx_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n, int inclusive);
int mtx_prefix_sum_f32_hs_dev(mtx_ctx *ctx, const float *in, float *out, uint64_t n);
/* hashgrid.py:16-90: cell = hash(trunc((p-bbmin)/(bbmax-bbmin)*res)) % n_cells,
 * cell_size, exclusive cell_offset, and sample_idx (per-cell order ascending
 * by sample index). p: 3n floats (x[n], y[n], z[n] planes). */
int mtx_hashgrid_build(mtx_ctx *ctx, const float *p, uint64_t n, uint32_t resolution, uint32_t n_cells,
                       uint32_t *cell, uint32_t *cell_size, uint32_t *cell_offset, uint32_t *sample_idx);
/* HashGrid(sample, ...) on device buffers (hashgrid.py:16-84 on Dr.Jit arrays). */
int mtx_hashgrid_build_dev(mtx_ctx *ctx, const float *p, uint64_t n, uint32_t resolution, uint32_t n_cells,
                           uint32_t *cell, uint32_t *cell_size, uint32_t *cell_offset, uint32_t *sample_idx);
/* reductions.py:12-54 scatter_reduce_with for func in {ADD=0, MIN=1, MAX=2,
 * MUL=3}: target[index[i]] = func(target[index[i]], value[i]), each target's
 * values applied in ascending i order (deterministic; the reference's order
 * is race-defined). The reference takes any Python callable (:12, :53): the
 * Python layer folds such a callable over mtx_group_by_u32 /
 * mtx_group_by_u32_dev's groups, round by round (on the device with torch
 * tensors). target is read-modify-write. */
int mtx_scatter_reduce_f32(mtx_ctx *ctx, int op, float *target, uint64_t n_target, const float *value,
                           const uint32_t *index, uint64_t n_value);
/* scatter_reduce_with on device buffers (reductions.py:12-54 on Dr.Jit
 * arrays); target is updated in place; an index >= n_target: MTX_E_ARG. */
int mtx_scatter_reduce_f32_dev(mtx_ctx *ctx, int op, float *target, uint64_t n_target, const float *value,
                               const uint32_t *index, uint64_t n_value);
/* The stable group-by behind mtx_hashgrid_build / mtx_scatter_reduce_f32
 * for caller keys (< n_keys): key_size, exclusive key_offset and order
 * (element indices grouped by key, ascending inside a key). The Python
 * scatter_reduce_with folds an arbitrary callable over it round by round,
 * as reductions.py:21-54 does with one election per round. Host pointers. */
int mtx_group_by_u32(mtx_ctx *ctx, const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size,
                     uint32_t *key_offset, uint32_t *order);
/* mtx_group_by_u32 on DEVICE pointers of the context's device (keys: n u32,
 * key_size / key_offset: n_keys u32, order: n u32), for callers whose data
 * stays in HBM (mtx.primitives.scatter_reduce_with with torch tensors). The
 * keys are range-checked on the device first (MTX_E_ARG if one is >= n_keys);
 * returns after the results are complete. */
int mtx_group_by_u32_dev(mtx_ctx *ctx, const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size,
                         uint32_t *key_offset, uint32_t *order);

/* --------------------------- radiance field ----------------------- */
/* nerad.py:54-106 Field (hash-grid + SH encoding, fp16 MLP with LeakyReLU,
 * no bias), the radiance cache queried by NRC. */
typedef struct mtx_field_desc {
  uint32_t n_levels, n_features, log2_table, base_res; /* grid encoding */
  float per_level_scale;
  float bbox_min[3], bbox_max[3];                     /* scene.bbox() */
  uint32_t n_in;      /* features per query: 3 + n_levels*n_features + 3 + 16, <= 64 */
  uint32_t n_hidden;  /* hidden 64x64 layers (nerad.py:61: 4) */
  const uint16_t *table;   /* fp16 bits [n_levels][2^log2_table][n_features] */
  const uint16_t *weights; /* fp16 bits, row-major W0[64][n_in], W1..Wn[64][64], Wout[3][64] */
} mtx_field_desc;
/* Copy a field to HBM (weights prepacked as MFMA fragments). */
int mtx_field_upload(mtx_ctx *ctx, const mtx_field_desc *field);
/* Features (n x 64 fp16 bits) of n queries (p, wi: 3n floats). Host pointers. */
int mtx_field_features(mtx_ctx *ctx, uint64_t n, const float *p, const float *wi, uint16_t *feat);
/* MLP on n feature rows (n x 64 fp16 bits) -> out (3n floats). Host pointers. */
int mtx_field_mlp(mtx_ctx *ctx, uint64_t n, const uint16_t *feat, float *out);
/* Field(si) for n queries: encode + MLP -> out (3n floats). Host pointers. */
int mtx_field_eval(mtx_ctx *ctx, uint64_t n, const float *p, const float *wi, float *out);

/* ------------------ radiance-field training (nerad.py) ------------------ */
/* nerad.py:336-400: the field above trained by neural radiosity. The fp16
 * table / weights uploaded with mtx_field_upload are the network; training
 * keeps fp32 master copies + Adam moments in the context and re-casts the
 * fp16 field after every step (:389-390). */
typedef struct mtx_field_opt {
  float lr, beta_1, beta_2, epsilon;     /* drjit.opt.Adam(lr=1e-3) defaults (:336-342) */
  float init_scale, growth_factor, backoff_factor;
  uint32_t growth_interval;              /* drjit.opt.GradScaler (:347) */
} mtx_field_opt;
typedef struct mtx_train_stats {
  double loss;        /* mean((L_lhs - L_rhs)^2) of the step, unscaled (:370) */
  float scale;        /* GradScaler scale after the step */
  uint32_t found_inf; /* 1: non-finite gradient, step skipped */
  uint32_t step;      /* Adam steps taken */
  uint32_t rhs_queries;
  double ms_lhs, ms_rhs, ms_train, ms_total; /* HIP-event times of the phases */
  double ms_trace;    /* closest-hit traversal launches of the RHS */
  uint64_t rays_closest, nodes_closest, tris_closest; /* RHS visit counters (args.flags bit 0) */
} mtx_train_stats;
/* Start training the uploaded field (fp32 master copies, zero moments). */
int mtx_field_train_init(mtx_ctx *ctx, const mtx_field_opt *opt);
/* Loss and gradients of scale * loss w.r.t. the table (fp32, n_levels*2^log2_table*n_features)
 * and the weights (fp32, mtx_field_desc order) for n points (p, wi: 3n) and targets (3n);
 * out: the network output (3n). Host pointers; any output may be NULL. No update. */
int mtx_field_grad(mtx_ctx *ctx, uint64_t n, const float *p, const float *wi, const float *target, float scale,
                   float *out, double *loss, float *grad_table, float *grad_weights);
/* One optimiser step on host-supplied points / targets (forward, backward, GradScaler + Adam). */
int mtx_field_train_step(mtx_ctx *ctx, uint64_t n, const float *p, const float *wi, const float *target,
                         mtx_train_stats *stats);
/* fp32 master parameters (table, weights) and Adam moments; any pointer may be NULL. */
int mtx_field_params(mtx_ctx *ctx, float *table, float *weights, float *m, float *v);

/* Surface-area tables of the uploaded scene (IntersectionSampler, nerad.py:281-289): the
 * shape distribution and per shape the distribution over its triangles (entries
 * [tri_off[s], tri_off[s+1]) of tri_pmf / tri_cdf / tri_prim; leaf-order triangles).
 * cdf = double-accumulated inclusive prefix stored as float; *_valid = first / last
 * index with non-zero pmf. */
typedef struct mtx_nerad_tables {
  uint32_t n_shapes, n_entries;
  const float *shape_pmf, *shape_cdf;
  float shape_sum, shape_norm;
  uint32_t shape_valid[2];
  const uint32_t *tri_off;    /* n_shapes + 1 */
  const float *tri_pmf, *tri_cdf;
  const uint32_t *tri_prim;
  const float *tri_sum, *tri_norm; /* n_shapes */
  const uint32_t *tri_valid;       /* 2 per shape */
} mtx_nerad_tables;
int mtx_nerad_upload(mtx_ctx *ctx, const mtx_nerad_tables *t);
typedef struct mtx_nerad_args {
  uint32_t lhs_seed;  /* sampler_lhs.seed(seed(), batch_size) (:387) */
  uint32_t rhs_seed;  /* sampler.seed(seed(), batch_size * M) in sample_rhs (:189) */
  uint32_t batch;     /* batch_size (:258: 2^14) */
  uint32_t M;         /* RHS samples per point (:259: 32) */
  uint32_t flags;     /* bit 0: count traversal visits (slower STATS kernels) */
} mtx_nerad_args;
/* IntersectionSampler.sample for `batch` points (:291-310): 9 floats per point
 * (prim as uint32 bits, b1, b2, p.xyz, wi_world.xyz). */
int mtx_nerad_lhs(mtx_ctx *ctx, const mtx_nerad_args *a, float *out);
/* Integrator.sample_rhs (:174-233) at the mtx_nerad_lhs(a) points with the current field:
 * L_rhs (3 per point); lanes (NULL or 3 * batch * M): every sample's L before the mean. */
int mtx_nerad_rhs(mtx_ctx *ctx, const mtx_nerad_args *a, float *L_rhs, float *lanes);
/* training_step (:363-375) on the device: LHS points, L_lhs = Field(si), L_rhs, loss,
 * backward, GradScaler + Adam, fp16 refresh of the field. */
int mtx_nerad_step(mtx_ctx *ctx, const mtx_nerad_args *a, mtx_train_stats *stats);

/* HIP-event time (ms) of the device work of the last primitive call on ctx
 * (the scan / hash / scatter kernels, without the host<->device copies);
 * used by bench.py to report the primitives against their rooflines. */
double mtx_last_device_ms(mtx_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* MTX_H_ */
