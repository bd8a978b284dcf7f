// device_common.h — device helpers shared by the gfx950 kernel files:
// scene view, wave64 stream compaction, and the two BVH traversals (4-wide
// sorted closest hit, 8-wide compressed any hit) whose visit orders and
// tie-breaking match oracle/oracle.cpp trace_closest / trace_any exactly.
#pragma once
#include <hip/hip_runtime.h>

#include "mtx_core/bsdf.h"
#include "mtx_core/geometry.h"
#include "mtx_core/interaction.h"
#include "mtx_core/rng.h"
#include "wavefront.h"

namespace mtxd {

using namespace mtx;

// Traversal stacks live in LDS, one column of 4-B words per lane
// ([word][lane]): node references (closest hit, 3 x depth + 1 words) or node
// groups (occlusion, depth + 1 entries of two words). mtx_trace's kernel and
// the path megakernel keep the whole stack of either tree in LDS; a thread
// may run both traversals on its one column (the path megakernel does), and
// no thread's words overlap another's.
// (stride kTraceBlock: every kernel that calls traverse_closest / traverse_occ
// runs blocks of kTraceBlock threads; k_path_mega asserts it.)
inline size_t stack_bytes(const DevScene &s) {
  const size_t a = s.stack_entries, b = 2 * (size_t)s.occ_stack_entries;
  return (a > b ? a : b) * sizeof(uint32_t) * kTraceBlock;
}
// The persistent kernels keep only the top lds_entries entries in LDS (so
// LDS does not cap occupancy) and spill deeper entries to a per-thread global
// area ([entry - lds_entries][thread], coalesced per depth), rarely touched.
// Behind the stack columns each block holds an LDS copy of the first lds_top
// nodes of its tree (the top of the breadth-first tree).
inline size_t persistent_stack_bytes(const DevScene &s, bool occ) {
  return occ ? (size_t)s.occ_lds_entries * kTraceBlock * sizeof(uint2) + (size_t)s.occ_lds_top * 80
             : (size_t)s.lds_entries * kTraceBlock * sizeof(int32_t) + (size_t)s.lds_top * 64;
}

__device__ __forceinline__ SceneView make_view(const DevScene &s) {
  SceneView v;
  v.nodes = reinterpret_cast<const int32_t *>(s.nodes);
  v.tri_geom = nullptr;  // device: DevScene::tri (packed, load_tri)
  v.tri_vidx = s.tri_vidx;
  v.tri_shape = s.tri_shape;
  v.vpos = s.vpos;
  v.vnormal = s.vnormal;
  v.vuv = s.vuv;
  v.shapes = s.shapes;
  v.materials = s.materials;
  v.emitters = s.emitters;
  v.bsdf.textures = s.textures;
  v.bsdf.texels = s.texels;
  v.bsdf.tables = s.tables;
  v.n_tris = s.n_tris;
  v.n_emitters = s.n_emitters;
  v.camera = s.camera;
  v.has_env = s.has_env;
  for (int k = 0; k < 3; ++k) {
    v.env_radiance[k] = s.env_radiance[k];
    v.env_center[k] = s.env_center[k];
  }
  v.env_radius = s.env_radius;
  return v;
}

// Device compute_si: the triangle's vertices, normals, uvs and shape fields
// come from one 128-B shading record (DevScene::shade_rec, built at upload in
// leaf order) instead of the tri_vidx -> vertex gathers; same floats, same
// arithmetic (si_from_vertices), so identical to the host compute_si.
//   r0 p0.xyz material | r1 p1.xyz emitter | r2 p2.xyz use flags (bit0 vertex
//   normals, bit1 uvs) | r3..r5 n0..n2 | r6 uv0, uv1 | r7 uv2
__device__ __forceinline__ SurfaceInteraction compute_si_dev(const DevScene &s, float t, uint32_t prim, float u,
                                                             float v, V3 ray_d) {
  if (prim == 0xffffffffu) {  // a miss: the environment, if any (compute_si)
    SurfaceInteraction si = si_invalid(t, prim, ray_d);
    si.emitter = s.has_env ? (int32_t)s.n_emitters : -1;
    return si;
  }
  const float4 *r = s.shade_rec + 8 * (size_t)prim;
  const float4 a = r[0], b = r[1], c = r[2];
  const uint32_t fl = __float_as_uint(c.w);
  const bool use_n = (fl & 1u) != 0, use_uv = (fl & 2u) != 0;
  V3 n0 = v3s(0.f), n1 = v3s(0.f), n2 = v3s(0.f);
  V2 t0 = V2{0.f, 0.f}, t1 = t0, t2 = t0;
  if (use_n) {
    const float4 x = r[3], y = r[4], z = r[5];
    n0 = V3{x.x, x.y, x.z};
    n1 = V3{y.x, y.y, y.z};
    n2 = V3{z.x, z.y, z.z};
  }
  if (use_uv) {
    const float4 x = r[6], y = r[7];
    t0 = V2{x.x, x.y};
    t1 = V2{x.z, x.w};
    t2 = V2{y.x, y.y};
  }
  return si_from_vertices(t, prim, u, v, ray_d, V3{a.x, a.y, a.z}, V3{b.x, b.y, b.z}, V3{c.x, c.y, c.z},
                          __float_as_uint(a.w), (int32_t)__float_as_uint(b.w), use_n, n0, n1, n2, use_uv, t0, t1, t2);
}

// Triangle geometry of leaf-order triangle `prim` of a tree (DevScene::tri
// or ::occ_tri): 9 packed floats (36 B: v0, e1 = v1 - v0, e2 = v2 - v0;
// mtx_scene_upload drops the ABI's pads), three dwordx3 loads.
struct TriGeom {
  V3 p0, e1, e2;
};
__device__ __forceinline__ TriGeom load_tri(const float *tri, uint32_t prim) {
  const float *g = tri + 9 * (size_t)prim;
  TriGeom t;
  t.p0 = V3{g[0], g[1], g[2]};
  t.e1 = V3{g[3], g[4], g[5]};
  t.e2 = V3{g[6], g[7], g[8]};
  return t;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Once-touched per-ray streams (ray planes, hit and shadow records, path
// state) with the non-temporal policy (`nt`). MTX_NT_STREAM bits: 0 the
// trace kernels' loads, 1 the shade kernel's loads, 2 its stores, 3 the trace
// kernels' stores, 4 the camera raygen's stores, 5 the shade kernel's queue
// entries and the film's reads. Default: the shade kernel's stores only
// (shade 62.7 -> 60.6 ms per step); nt loads were slower (shade loads 61.2
// -> 64.0 ms) or neutral, the other stores neutral, and the stores with
// sc1 / sc0 sc1 / nt sc1 slower (66-72 ms): profiles/r6h_ab_nt_stream_bits.jsonl,
// r6i_ab_nt_store_policy.jsonl.
#ifndef MTX_NT_STREAM
#define MTX_NT_STREAM 4
#endif
template <class T>
struct NtVec {  // the vector type of a 4-, 8- or 16-B record for the nt builtins
  static_assert(sizeof(T) == 4 || sizeof(T) == 8 || sizeof(T) == 16, "4-, 8- or 16-B stream records");
  typedef uint32_t type __attribute__((ext_vector_type(sizeof(T) / 4)));
};
template <int BIT, class T>
__device__ __forceinline__ T ld_stream(const T *p) {
  if constexpr ((MTX_NT_STREAM >> BIT) & 1) {
    using V = typename NtVec<T>::type;
    const V v = __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
    T r;
    __builtin_memcpy(&r, &v, sizeof(T));
    return r;
  } else {
    return *p;
  }
}
template <int BIT, class T>
__device__ __forceinline__ void st_stream(T *p, const T &x) {
  if constexpr ((MTX_NT_STREAM >> BIT) & 1) {
    using V = typename NtVec<T>::type;
    V v;
    __builtin_memcpy(&v, &x, sizeof(T));
    __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
  } else {
    *p = x;
  }
}
constexpr int kNtTrace = 0, kNtShade = 1, kNtShadeSt = 2, kNtTraceSt = 3, kNtRaygen = 4, kNtQueue = 5;

// Wave-level stream compaction: every lane of the wave must call this.
// Returns the output slot of a lane with pred = true.
__device__ __forceinline__ uint32_t wave_append(uint32_t *counter, bool pred) {
  const uint64_t mask = __ballot(pred);
  const uint32_t prefix =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
  const uint32_t total = (uint32_t)__popcll(mask);
  uint32_t base = 0;
  if (total) {
    const uint32_t leader = (uint32_t)(__ffsll((unsigned long long)mask) - 1);
    if (lane_id() == leader) base = atomicAdd(counter, total);
    base = __builtin_amdgcn_readlane(base, leader);
  }
  return base + prefix;
}

// Block-level reservation of `cnt` consecutive slots per thread: one
// device-scope atomic per block (same-address atomics from every wave of
// the chip serialise at ~90 per microsecond). Returns this thread's first
// slot; every thread of the block must call it.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_reserve(uint32_t cnt, uint32_t *counter) {
  constexpr int W = BLOCK / 64;
  __shared__ uint32_t wsum[W];
  __shared__ uint32_t bbase;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t x = cnt;  // inclusive prefix inside the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= (uint32_t)off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint32_t v = wsum[w];
      wsum[w] = t;
      t += v;
    }
    bbase = t ? atomicAdd(counter, t) : 0u;
  }
  __syncthreads();
  const uint32_t r = bbase + wsum[wave] + x - cnt;
  __syncthreads();
  return r;
}

// Block-level stream compaction into two queues: one device-scope atomic
// per queue per block step (instead of one per wave) -- same-address atomics
// from every wave of the chip serialise. All threads of the block must call
// it once per step; `parity` alternates between consecutive steps so that the
// LDS slots of one step are not overwritten while a slow wave still reads them.
// The two counters are one 8-byte-aligned pair (c[0], c[1]): a single 64-bit
// atomic reserves both (the low count never carries: it stays below 2^32).
// Inside a block step's range of the second queue the entries with p1_hi
// follow the others (NEE shadow rays: the rays of one emitter together, so
// the any-hit waves that claim them walk one light's shadow frusta).
template <int BLOCK>
__device__ __forceinline__ void block_append2(bool p0, bool p1, bool p1_hi, uint32_t *c, uint32_t parity,
                                              uint32_t &s0, uint32_t &s1) {
  constexpr int W = BLOCK / 64;
  __shared__ uint32_t wcnt[2][3][W];
  __shared__ uint32_t bbase[2][3];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t m0 = __ballot(p0), ml = __ballot(p1 && !p1_hi), mh = __ballot(p1 && p1_hi);
  if (lane == 0) {
    wcnt[parity][0][wave] = (uint32_t)__popcll(m0);
    wcnt[parity][1][wave] = (uint32_t)__popcll(ml);
    wcnt[parity][2][wave] = (uint32_t)__popcll(mh);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t0 = 0, tl = 0, th = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      t0 += wcnt[parity][0][w];
      tl += wcnt[parity][1][w];
      th += wcnt[parity][2][w];
    }
    uint64_t base = 0;
    if (t0 | tl | th)
      base = atomicAdd(reinterpret_cast<unsigned long long *>(c), ((unsigned long long)(tl + th) << 32) | t0);
    bbase[parity][0] = (uint32_t)base;
    bbase[parity][1] = (uint32_t)(base >> 32);
    bbase[parity][2] = (uint32_t)(base >> 32) + tl;
  }
  __syncthreads();
  uint32_t o0 = bbase[parity][0], ol = bbase[parity][1], oh = bbase[parity][2];
  for (uint32_t w = 0; w < wave; ++w) {
    o0 += wcnt[parity][0][w];
    ol += wcnt[parity][1][w];
    oh += wcnt[parity][2][w];
  }
  s0 = o0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
  s1 = p1_hi ? oh + __builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mh, 0u))
             : ol + __builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ml, 0u));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}


// ===========================================================================
// Closest hit: 4-wide BVH (mtx.h). One node visit = four 16-B loads (from
// the block's LDS copy of the tree top, or global memory) and
// mtx_core/geometry.h wide_node_keys_e; the child references ride along the
// 5-exchange sorting network, so the visit order is by entry distance.
// ===========================================================================
// The 64-B node of the block's LDS tree-top copy (inline asm: as plain loads
// the compiler merges an LDS branch and a global branch into flat loads
// through a selected generic pointer, which take the vector-memory path for
// every lane).
__device__ __forceinline__ void lds_node64(const int4 *top, int32_t node, int4 &a, int4 &rf, int4 &qa, int2 &qb) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef int v2i __attribute__((ext_vector_type(2)));
  v4i x0, x1, x2;
  v2i x3;
  const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)top + 64u * (uint32_t)node;
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:16\n\t"
      "ds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b64 %3, %4 offset:48\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)
      : "v"(la));
  a = make_int4(x0.x, x0.y, x0.z, x0.w);
  rf = make_int4(x1.x, x1.y, x1.z, x1.w);
  qa = make_int4(x2.x, x2.y, x2.z, x2.w);
  qb = make_int2(x3.x, x3.y);
}

// Slab tests of a 4-wide node's children (words a, rf, qa, qb of mtx.h) and
// the near-first order: returns the number of hit children, c[] the child
// references sorted by entry distance.
__device__ __forceinline__ int wide_visit_regs(const TraceRay &r, int4 a, int4 rf, int4 qa, int2 qb, float tbest,
                                               int32_t c[4], uint32_t *key_out = nullptr) {
  uint32_t key[4];
  const uint32_t eb = (uint32_t)a.w;
  // the references ride along the compare-exchange network (one compare +
  // four selects per exchange) instead of being picked by the sorted keys'
  // slot bits afterwards: the keys are distinct (slot in the low bits), so
  // the order and the references are those of wide_node_order + wide_ref
  const int n = wide_node_keys_e(r, __int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z),
                                 (int)(int8_t)(uint8_t)(eb & 0xffu), (int)(int8_t)(uint8_t)((eb >> 8) & 0xffu),
                                 (int)(int8_t)(uint8_t)((eb >> 16) & 0xffu), (int)(eb >> 24), (uint32_t)qa.x,
                                 (uint32_t)qa.y, (uint32_t)qa.z, (uint32_t)qa.w, (uint32_t)qb.x, (uint32_t)qb.y,
                                 tbest, key);
  c[0] = rf.x;
  c[1] = rf.y;
  c[2] = rf.z;
  c[3] = rf.w;
#define MTX_CAS2(i, j)                         \
  {                                            \
    const bool sw_ = key[j] < key[i];          \
    const uint32_t ki_ = key[i], kj_ = key[j]; \
    const int32_t ci_ = c[i], cj_ = c[j];      \
    key[i] = sw_ ? kj_ : ki_;                  \
    key[j] = sw_ ? ki_ : kj_;                  \
    c[i] = sw_ ? cj_ : ci_;                    \
    c[j] = sw_ ? ci_ : cj_;                    \
  }
  MTX_CAS2(0, 1) MTX_CAS2(2, 3) MTX_CAS2(0, 2) MTX_CAS2(1, 3) MTX_CAS2(1, 2)
#undef MTX_CAS2
  if (key_out) {
#pragma unroll
    for (int k = 0; k < 4; ++k) key_out[k] = key[k];
  }
  return n;
}

__device__ __forceinline__ int wide_visit(const DevScene &s, const TraceRay &r, int32_t node, float tbest,
                                          int32_t c[4], const int4 *top = nullptr, int top_n = 0,
                                          uint32_t *key_out = nullptr) {
  int4 a, rf, qa;
  int2 qb;
  if (node < top_n) {
    lds_node64(top, node, a, rf, qa, qb);
  } else {
    const int4 *np = s.nodes + 4 * node;
    a = np[0];
    rf = np[1];
    qa = np[2];
    qb = *reinterpret_cast<const int2 *>(np + 3);
  }
  return wide_visit_regs(r, a, rf, qa, qb, tbest, c, key_out);
}

// Per-thread closest-hit traversal in the oracle's order (oracle/oracle.cpp
// trace_closest) for mtx_trace: stk is this thread's LDS column.
__device__ __forceinline__ void traverse_closest(const DevScene &s, int32_t *stk, const TraceRay &r, float &tbest,
                                                 uint32_t &prim_best, float &bu, float &bv, uint32_t &nv,
                                                 uint32_t &tv) {
  int sp = 0;
  int32_t node = 0;
  while (true) {
    if (node >= 0) {
      int32_t cr[4];
      ++nv;
      const int n = wide_visit(s, r, node, tbest, cr);
      if (n > 0) {
#pragma unroll
        for (int rr = 3; rr >= 1; --rr)
          if (rr < n) {
            stk[sp * kTraceBlock] = cr[rr];
            ++sp;
          }
        node = cr[0];
        continue;
      }
    } else {
      uint32_t first, count;
      leaf_decode(node, &first, &count);
      for (uint32_t k = 0; k < count; ++k) {
        const uint32_t prim = first + k;
        const TriGeom g = load_tri(s.tri, prim);
        float t, u, v;
        ++tv;
        if (tri_intersect(r, g.p0, g.e1, g.e2, tbest, &t, &u, &v) &&
            (t < tbest || (t == tbest && prim < prim_best))) {
          tbest = t;
          prim_best = prim;
          bu = u;
          bv = v;
        }
      }
    }
    if (sp == 0) break;
    --sp;
    node = stk[sp * kTraceBlock];
  }
}

// ===========================================================================
// Any hit: 8-wide compressed occlusion BVH (mtx.h). One node visit = five
// 16-B loads and mtx_core/geometry.h cw_node_hits. A lane's traversal state
// is a node group (child_base, hit inner children as bits 24..31 in octant
// order | imask) and a triangle group (tri_base, hit leaves' triangles as
// bits 0..23); the stack holds node groups, one 8-B entry per visited node
// at most.
// ===========================================================================
struct CwVisit {
  uint32_t hits, child_base, tri_base, imask;
};

__device__ __forceinline__ void lds_node80(const int4 *top, uint32_t node, int4 &a, int4 &b, int4 &q0, int4 &q1,
                                           int4 &q2) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i x0, x1, x2, x3, x4;
  const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)top + 80u * node;
  asm volatile(
      "ds_read_b128 %0, %5\n\t"
      "ds_read_b128 %1, %5 offset:16\n\t"
      "ds_read_b128 %2, %5 offset:32\n\t"
      "ds_read_b128 %3, %5 offset:48\n\t"
      "ds_read_b128 %4, %5 offset:64\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3), "=&v"(x4)
      : "v"(la));
  a = make_int4(x0.x, x0.y, x0.z, x0.w);
  b = make_int4(x1.x, x1.y, x1.z, x1.w);
  q0 = make_int4(x2.x, x2.y, x2.z, x2.w);
  q1 = make_int4(x3.x, x3.y, x3.z, x3.w);
  q2 = make_int4(x4.x, x4.y, x4.z, x4.w);
}

__device__ __forceinline__ CwVisit cw_visit_regs(const TraceRay &r, uint32_t oct, int4 a, int4 b, int4 q0, int4 q1,
                                                 int4 q2, float tbest) {
  const uint32_t q[12] = {(uint32_t)q0.x, (uint32_t)q0.y, (uint32_t)q0.z, (uint32_t)q0.w,
                          (uint32_t)q1.x, (uint32_t)q1.y, (uint32_t)q1.z, (uint32_t)q1.w,
                          (uint32_t)q2.x, (uint32_t)q2.y, (uint32_t)q2.z, (uint32_t)q2.w};
  CwVisit v;
  v.hits = cw_node_hits(r, oct, __int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z), (uint32_t)a.w,
                        (uint32_t)b.z, (uint32_t)b.w, q, tbest);
  v.child_base = (uint32_t)b.x;
  v.tri_base = (uint32_t)b.y;
  v.imask = (uint32_t)a.w >> 24;
  return v;
}

__device__ __forceinline__ CwVisit cw_visit(const DevScene &s, const TraceRay &r, uint32_t oct, uint32_t node,
                                            float tbest, const int4 *top, int top_n) {
  int4 a, b, q0, q1, q2;
  if ((int)node < top_n) {
    lds_node80(top, node, a, b, q0, q1, q2);
  } else {
    const int4 *np = s.occ_nodes + 5 * (size_t)node;
    a = np[0];
    b = np[1];
    q0 = np[2];
    q1 = np[3];
    q2 = np[4];
  }
  return cw_visit_regs(r, oct, a, b, q0, q1, q2, tbest);
}

// Per-thread any-hit traversal in the oracle's order (oracle/oracle.cpp
// trace_any) for mtx_trace and the path megakernel: stk is this thread's LDS
// column of words; node group e takes words 2e (base) and 2e + 1 (bits).
__device__ __forceinline__ bool traverse_occ(const DevScene &s, uint32_t *stk, const TraceRay &r, float tmax,
                                             uint32_t &nv, uint32_t &tv) {
  const uint32_t oct = ray_octant(r);
  int sp = 0;
  uint32_t gbase = 0, ghits = (1u << (24 + oct)) | 1u, tbase = 0, thits = 0;
  while (true) {
    if (thits) {
      const uint32_t prim = tbase + (uint32_t)ctz32(thits);
      thits &= thits - 1u;
      const TriGeom g = load_tri(s.occ_tri, prim);
      float t, u, v;
      ++tv;
      if (tri_intersect(r, g.p0, g.e1, g.e2, tmax, &t, &u, &v)) return true;
    } else if (ghits >> 24) {
      const uint32_t p = (uint32_t)ctz32(ghits >> 24);
      ghits &= ~(1u << (24 + p));
      const uint32_t node = cw_inner_child(gbase, ghits & 0xffu, oct, p);
      if (ghits >> 24) {
        stk[(2 * sp) * kTraceBlock] = gbase;
        stk[(2 * sp + 1) * kTraceBlock] = ghits;
        ++sp;
      }
      ++nv;
      const CwVisit v = cw_visit(s, r, oct, node, tmax, nullptr, 0);
      gbase = v.child_base;
      ghits = (v.hits & 0xff000000u) | v.imask;
      tbase = v.tri_base;
      thits = v.hits & 0x00ffffffu;
    } else if (sp > 0) {
      --sp;
      gbase = stk[(2 * sp) * kTraceBlock];
      ghits = stk[(2 * sp + 1) * kTraceBlock];
    } else {
      return false;
    }
  }
}

// ===========================================================================
// Persistent single-step traversal loops (both trees).
//
// Every lane owns one ray at a time. Each iteration a lane with a ray does
// one unit of work: one node visit, then (same iteration) one triangle test
// if it holds triangles to test; nothing waits for the slowest lane of the
// wave to reach a leaf. Finished lanes are refilled from a per-wave
// reservoir of claimed queue indices once s.urefill lanes of the wave are
// idle -- one device-scope atomic per claimed batch. Waves claim rays from
// their own XCD's eighth of the queue first (that XCD's L2 then holds the
// band's nodes). Each ray's visit sequence is the oracle's, with or without
// STATS. Src provides: a Payload type (what a lane carries for its ray),
// load(k, TraceRay&, float &tmax, Payload &) and finish(const Payload &, bool
// any_hit, float t, uint32_t prim, float u, float v).
// ===========================================================================

// Stack entry e of a lane: LDS for e < lds_n, the global spill area above.
// The LDS entry is read unconditionally (clamped) and the global one only on
// the rare deep entries, so the common pop is a ds_read; a select between the
// two pointers would compile to a flat load (vector-memory + LDS counters,
// a texture-path slot per pop).
__device__ __forceinline__ int32_t stack_read(const int32_t *stk, const int32_t *ovf, int e, int lds_n,
                                              uint32_t ovf_threads) {
  int32_t v = stk[min(e, lds_n - 1) * kTraceBlock];
  asm volatile("" : "+v"(v));  // keeps the LDS read (no pointer select + flat load)
  if (e >= lds_n) v = ovf[(size_t)(e - lds_n) * ovf_threads];
  return v;
}
__device__ __forceinline__ uint2 stack_read(const uint2 *stk, const uint2 *ovf, int e, int lds_n,
                                            uint32_t ovf_threads) {
  uint2 v = stk[min(e, lds_n - 1) * kTraceBlock];
  asm volatile("" : "+v"(v.x), "+v"(v.y));
  if (e >= lds_n) v = ovf[(size_t)(e - lds_n) * ovf_threads];
  return v;
}

// XCD of the executing wave (0-7): speed only (which L2 the wave fills).
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kXcds - 1u);
}

// Queue segment k of 8: [count*k/8, count*(k+1)/8).
__device__ __forceinline__ uint32_t xseg_bound(uint32_t count, uint32_t k) {
  return (uint32_t)(((uint64_t)count * k) >> 3);
}

// A wave's reservoir of claimed queue indices. Claims take s.trace_batch
// entries, cut down (to >= 64) when the queue is too short to give every
// wave of the grid a batch: a small queue then still spreads over the chip
// instead of running a few long per-lane chains; waves beyond the batches
// exit at once (start() returns false). Claims come from the own XCD's
// queue segment first, then the next segments. (Guided sizes -- each claim
// its fair share of what the segment has left -- measured much slower:
// closest 61.3 -> 74.0 ms/step at spp 256)
struct RayReservoir {
  uint32_t *heads;
  uint32_t count, batch, seg, tries, res_lo, res_hi;
  bool drained, exhausted;

  __device__ __forceinline__ bool start(const DevScene &s, uint32_t *heads_, uint32_t count_) {
    heads = heads_;
    count = count_;
    const uint32_t n_grid_waves = gridDim.x * (kTraceBlock / 64u);
    batch = max(64u, min(s.trace_batch, (count / n_grid_waves) & ~63u));
    seg = s.xcd_claim ? xcc_id() : 0u;
    tries = s.xcd_claim ? 0u : kXcds - 1u;
    res_lo = res_hi = 0;
    drained = exhausted = false;
    return (blockIdx.x * kTraceBlock + threadIdx.x) / 64u < (count + batch - 1) / batch;
  }

  // [base2, base2 + got2) from the next non-empty segment (wave-uniform; the
  // leader lane does the atomic); true once every segment is drained
  __device__ __forceinline__ bool claim(const DevScene &s, uint32_t leader, uint32_t lane, uint32_t &base2,
                                        uint32_t &got2) {
    while (true) {
      const uint32_t lo = s.xcd_claim ? xseg_bound(count, seg) : 0u;
      const uint32_t hi = s.xcd_claim ? xseg_bound(count, seg + 1) : count;
      uint32_t b = 0xffffffffu;
      if (hi > lo) {
        if (lane == leader) b = atomicAdd(heads + seg * kXHeadStride, batch);
        b = __builtin_amdgcn_readlane(b, leader);
      }
      if (hi > lo && b < hi - lo) {
        base2 = lo + b;
        got2 = min(batch, hi - lo - b);
        return false;
      }
      if (++tries >= kXcds) return true;
      seg = (seg + 1) & (kXcds - 1u);
    }
  }

  // one queue index for every lane in `want`: k is this lane's, ok if it got one
  __device__ __forceinline__ void take(const DevScene &s, uint64_t want, uint32_t lane, uint32_t &k, bool &ok) {
    const uint32_t n = (uint32_t)__popcll(want);
    const uint32_t left = res_hi - res_lo;
    uint32_t base2 = 0, got2 = 0;
    if (left < n && !drained) drained = claim(s, (uint32_t)(__ffsll((unsigned long long)want) - 1), lane, base2, got2);
    const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
    k = 0;
    ok = false;
    if (rk < left) {
      k = res_lo + rk;
      ok = true;
    } else if (rk - left < got2) {
      k = base2 + (rk - left);
      ok = true;
    }
    if (n <= left) {
      res_lo += n;
    } else {
      const uint32_t used2 = min(n - left, got2);
      res_lo = base2 + used2;
      res_hi = base2 + got2;
    }
    exhausted = drained && res_lo >= res_hi;
  }
};

__device__ __forceinline__ void count_wave_iter(uint32_t lane, uint32_t *ctr) {
  const uint64_t m = __ballot(true);
  if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) ++*ctr;
}

// Closest hit on the 4-wide tree: a lane's work item is an inner node to
// visit or a leaf's triangle range; a visit pushes the far hit children
// (three unconditional LDS stores when they fit: dead entries above the new
// top are harmless) and continues with the nearest.
template <bool STATS, class Src>
__device__ __forceinline__ void trace_loop_closest(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                                   int32_t *stk, const int4 *top, uint32_t &nv, uint32_t &tv,
                                                   uint32_t &nr, uint32_t *wave_iters) {
  const uint32_t lane = lane_id();
  int32_t *ovf = reinterpret_cast<int32_t *>(s.stack_ovf) + blockIdx.x * kTraceBlock + threadIdx.x;
  const int lds_n = (int)s.lds_entries, top_n = (int)s.lds_top;
  RayReservoir res;
  if (!res.start(s, heads, count)) return;
  bool has = false;
  typename Src::Payload payload{};
  uint32_t prim = 0xffffffffu;
  TraceRay r;
  float tbest = 0.f, bu = 0.f, bv = 0.f;
  int32_t node = -1;              // >= 0: inner node to visit next
  uint32_t tri = 0, tri_end = 0;  // triangles [tri, tri_end) of the current leaf
  int sp = 0;
  // next work item of a lane from its stack: an inner node, a leaf's
  // triangle range, or nothing (the ray is finished)
  auto pop_next = [&]() {
    node = -1;
    if (sp > 0) {
      --sp;
      const int32_t e = stack_read(stk, ovf, sp, lds_n, s.ovf_threads);
      if (e >= 0) {
        node = e;
      } else {
        uint32_t first, cnt;
        leaf_decode(e, &first, &cnt);
        tri = first;
        tri_end = first + cnt;
      }
    }
  };
  // one inner-node visit of a lane (LDS tree top or global memory)
  auto visit_node = [&]() {
      if (STATS) count_wave_iter(lane, &wave_iters[0]);
      int32_t cr[4];
      ++nv;
      const int n = wide_visit(s, r, node, tbest, cr, top, top_n);
      if (n > 0) {
        const int32_t c1 = cr[1], c2 = cr[2], c3 = cr[3];
        const int32_t e0 = n == 4 ? c3 : (n == 3 ? c2 : c1), e1 = n == 4 ? c2 : c1;
        if (sp + 3 <= lds_n) {
          stk[sp * kTraceBlock] = e0;
          stk[(sp + 1) * kTraceBlock] = e1;
          stk[(sp + 2) * kTraceBlock] = c1;
        } else {
          const int32_t e[3] = {e0, e1, c1};
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if (j < n - 1) {
              const int q = sp + j;
              if (q < lds_n)
                stk[q * kTraceBlock] = e[j];
              else
                ovf[(size_t)(q - lds_n) * s.ovf_threads] = e[j];
            }
        }
        sp += n - 1;
        const int32_t c0 = cr[0];
        if (c0 >= 0) {
          node = c0;
        } else {
          uint32_t first, cnt;
          leaf_decode(c0, &first, &cnt);
          tri = first;
          tri_end = first + cnt;
          node = -1;
        }
      } else {
        pop_next();
      }
  };
  while (true) {
    if (!res.exhausted) {
      const uint64_t idle = __ballot(!has);
      if ((uint32_t)__popcll(idle) >= s.urefill || idle == ~0ull) {
        uint32_t k;
        bool ok;
        res.take(s, idle, lane, k, ok);
        if (!has && ok) {
          src.load(k, r, tbest, payload);
          prim = 0xffffffffu;
          bu = bv = 0.f;
          node = 0;
          tri = tri_end = 0;
          sp = 0;
          has = true;
        }
      }
    }
    if (__ballot(has) == 0) break;
    // ---- one inner-node visit
    if (has && node >= 0) visit_node();
    // ---- one triangle test
    if (has && tri < tri_end) {
      if (STATS) count_wave_iter(lane, &wave_iters[1]);
      const uint32_t pr = tri;
      const TriGeom g = load_tri(s.tri, pr);
      float t, u, v;
      ++tv;
      ++tri;
      if (tri_intersect(r, g.p0, g.e1, g.e2, tbest, &t, &u, &v) && (t < tbest || (t == tbest && pr < prim))) {
        tbest = t;
        prim = pr;
        bu = u;
        bv = v;
      }
      if (tri >= tri_end) pop_next();
    }
    if (has && node < 0 && tri >= tri_end) {
      src.finish(payload, prim != 0xffffffffu, tbest, prim, bu, bv);
      has = false;
      ++nr;
    }
  }
}

// Any hit on the 8-wide occlusion tree: a lane tests its triangle group
// before the next child of its node group; an empty pair pops the next node
// group. The first hit ends the ray.
template <bool STATS, class Src>
__device__ __forceinline__ void trace_loop_occ(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                               uint2 *stk, const int4 *top, uint32_t &nv, uint32_t &tv,
                                               uint32_t &nr, uint32_t *wave_iters) {
  const uint32_t lane = lane_id();
  uint2 *ovf = reinterpret_cast<uint2 *>(s.stack_ovf) + blockIdx.x * kTraceBlock + threadIdx.x;
  const int lds_n = (int)s.occ_lds_entries, top_n = (int)s.occ_lds_top;
  RayReservoir res;
  if (!res.start(s, heads, count)) return;
  bool has = false, hit = false;
  typename Src::Payload payload{};
  TraceRay r;
  float tmax = 0.f;
  uint32_t oct = 0, gbase = 0, ghits = 0, tbase = 0, thits = 0;
  int sp = 0;
  // one node visit: the nearest remaining child of the lane's node group
  auto visit_occ = [&]() {
    if (STATS) count_wave_iter(lane, &wave_iters[0]);
    const uint32_t p = (uint32_t)ctz32(ghits >> 24);
    ghits &= ~(1u << (24 + p));
    const uint32_t node = cw_inner_child(gbase, ghits & 0xffu, oct, p);
    if (ghits >> 24) {
      const uint2 g = make_uint2(gbase, ghits);
      if (sp < lds_n) {
        stk[sp * kTraceBlock] = g;
      } else {
        ovf[(size_t)(sp - lds_n) * s.ovf_threads] = g;
        asm volatile("" ::: "memory");  // keeps the two stores apart (no pointer select + flat store)
      }
      ++sp;
    }
    ++nv;
    const CwVisit v = cw_visit(s, r, oct, node, tmax, top, top_n);
    gbase = v.child_base;
    ghits = (v.hits & 0xff000000u) | v.imask;
    tbase = v.tri_base;
    thits = v.hits & 0x00ffffffu;
  };
  while (true) {
    if (!res.exhausted) {
      const uint64_t idle = __ballot(!has);
      if ((uint32_t)__popcll(idle) >= s.occ_urefill || idle == ~0ull) {
        uint32_t k;
        bool ok;
        res.take(s, idle, lane, k, ok);
        if (!has && ok) {
          src.load(k, r, tmax, payload);
          hit = false;
          oct = ray_octant(r);
          gbase = 0;
          ghits = (1u << (24 + oct)) | 1u;  // the root: node 0 in slot 0
          tbase = thits = 0;
          sp = 0;
          has = true;
        }
      }
    }
    if (__ballot(has) == 0) break;
    // ---- one node visit: the nearest remaining child of the node group
    if (has && thits == 0 && (ghits >> 24) != 0) visit_occ();
    // ---- one triangle test of the triangle group
    if (has && thits != 0) {
      if (STATS) count_wave_iter(lane, &wave_iters[1]);
      const uint32_t pr = tbase + (uint32_t)ctz32(thits);
      thits &= thits - 1u;
      const TriGeom g = load_tri(s.occ_tri, pr);
      float t, u, v;
      ++tv;
      if (tri_intersect(r, g.p0, g.e1, g.e2, tmax, &t, &u, &v)) {
        hit = true;
        thits = 0;
        ghits = 0;
        sp = 0;
      }
    }
    // ---- both groups empty: the next node group, or the ray is done
    if (has && thits == 0 && (ghits >> 24) == 0) {
      if (sp > 0) {
        --sp;
        const uint2 g = stack_read(stk, ovf, sp, lds_n, s.ovf_threads);
        gbase = g.x;
        ghits = g.y;
      } else {
        src.finish(payload, hit, tmax, 0xffffffffu, 0.f, 0.f);
        has = false;
        ++nr;
      }
    }
  }
}

// The persistent traversal of a block: ANY = any hit on the occlusion tree,
// else closest hit on the 4-wide tree. The block's dynamic LDS holds the
// stack columns and then the tree top (persistent_stack_bytes), filled here
// behind a barrier; every thread of the block calls this.
template <bool ANY, bool STATS = false, class Src>
__device__ __forceinline__ void trace_loop(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                           uint32_t &nv, uint32_t &tv, uint32_t &nr,
                                           uint32_t *wave_iters = nullptr) {
  extern __shared__ int4 trace_lds[];
  // a block none of whose waves gets a claim batch (a short queue:
  // RayReservoir::start) exits before it fills its tree top
  {
    const uint32_t n_grid_waves = gridDim.x * (kTraceBlock / 64u);
    const uint32_t batch = max(64u, min(s.trace_batch, (count / n_grid_waves) & ~63u));
    if (blockIdx.x * (kTraceBlock / 64u) >= (count + batch - 1) / batch) return;
  }
  if (ANY) {
    uint2 *cols = reinterpret_cast<uint2 *>(trace_lds);
    int4 *top = reinterpret_cast<int4 *>(cols + s.occ_lds_entries * kTraceBlock);
    for (uint32_t i = threadIdx.x; i < 5 * s.occ_lds_top; i += kTraceBlock) top[i] = s.occ_nodes[i];
    __syncthreads();
    trace_loop_occ<STATS>(s, src, count, heads, cols + threadIdx.x, top, nv, tv, nr, wave_iters);
  } else {
    int32_t *cols = reinterpret_cast<int32_t *>(trace_lds);
    int4 *top = reinterpret_cast<int4 *>(cols + s.lds_entries * kTraceBlock);
    for (uint32_t i = threadIdx.x; i < 4 * s.lds_top; i += kTraceBlock) top[i] = s.nodes[i];
    __syncthreads();
    trace_loop_closest<STATS>(s, src, count, heads, cols + threadIdx.x, top, nv, tv, nr, wave_iters);
  }
}

}  // namespace mtxd
