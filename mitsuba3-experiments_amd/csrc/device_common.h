// device_common.h — device helpers shared by the gfx950 kernel files:
// scene view, wave64 stream compaction, and the BVH2 traversal whose child
// order and tie-breaking match oracle/oracle.cpp:trace_closest exactly.
#pragma once
#include <hip/hip_runtime.h>

#include "mtx_core/bsdf.h"
#include "mtx_core/geometry.h"
#include "mtx_core/interaction.h"
#include "mtx_core/rng.h"
#include "wavefront.h"

namespace mtxd {

using namespace mtx;

// Traversal stacks live in LDS, one column per lane ([entry][lane]); the
// number of entries is the uploaded BVH's depth + 1 (at most
// MTX_BVH_MAX_DEPTH + 1), so shallow trees leave LDS for more waves per CU.
inline size_t stack_bytes(const DevScene &s) { return (size_t)s.stack_entries * kTraceBlock * sizeof(int32_t); }
// The persistent kernels keep only the top s.lds_entries entries in LDS (so
// LDS does not cap occupancy) and spill deeper entries to a per-thread global
// area ([entry - lds_entries][thread], coalesced per depth), rarely touched.
// Behind the stack columns each block holds an LDS copy of the first
// s.lds_top wide nodes (the top of the breadth-first tree, 64 B each).
inline size_t persistent_stack_bytes(const DevScene &s) {
  return (size_t)s.lds_entries * kTraceBlock * sizeof(int32_t) + (size_t)s.lds_top * 64;
}
constexpr int kShadeBlock = 256;

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
  if (prim == 0xffffffffu) return si_invalid(t, prim, ray_d);
#ifdef MTX_DIAG_REC_MASK  // timing diagnostic only (wrong images): records of a few triangles
  const float4 *r = s.shade_rec + 8 * (size_t)(prim & MTX_DIAG_REC_MASK);
#else
  const float4 *r = s.shade_rec + 8 * (size_t)prim;
#endif
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

// Triangle geometry of leaf-order triangle `prim`: 9 packed floats (36 B:
// v0, e1 = v1 - v0, e2 = v2 - v0; mtx_scene_upload drops the ABI's pads),
// three dwordx3 loads.
struct TriGeom {
  V3 p0, e1, e2;
};
__device__ __forceinline__ TriGeom load_tri(const DevScene &s, uint32_t prim) {
  const float *g = s.tri + 9 * (size_t)prim;
  TriGeom t;
  t.p0 = V3{g[0], g[1], g[2]};
  t.e1 = V3{g[3], g[4], g[5]};
  t.e2 = V3{g[6], g[7], g[8]};
  return t;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

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
template <int BLOCK>
__device__ __forceinline__ void block_append2(bool p0, bool p1, uint32_t *c, uint32_t parity, uint32_t &s0,
                                              uint32_t &s1) {
  constexpr int W = BLOCK / 64;
  __shared__ uint32_t wcnt[2][2][W];
  __shared__ uint32_t bbase[2][2];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t m0 = __ballot(p0), m1 = __ballot(p1);
  if (lane == 0) {
    wcnt[parity][0][wave] = (uint32_t)__popcll(m0);
    wcnt[parity][1][wave] = (uint32_t)__popcll(m1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t0 = 0, t1 = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      t0 += wcnt[parity][0][w];
      t1 += wcnt[parity][1][w];
    }
    uint64_t base = 0;
    if (t0 | t1)
      base = atomicAdd(reinterpret_cast<unsigned long long *>(c), ((unsigned long long)t1 << 32) | t0);
    bbase[parity][0] = (uint32_t)base;
    bbase[parity][1] = (uint32_t)(base >> 32);
  }
  __syncthreads();
  uint32_t o0 = bbase[parity][0], o1 = bbase[parity][1];
  for (uint32_t w = 0; w < wave; ++w) {
    o0 += wcnt[parity][0][w];
    o1 += wcnt[parity][1][w];
  }
  s0 = o0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
  s1 = o1 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Child reference of the slot in a sort key, from the 48-B device node's
// bases and per-slot leaf ends (bvh_build.cpp mtx_bvh_device_nodes): end 0 =
// inner child node_base + slot; else the leaf of triangles [tri_base +
// end_{slot-1}, tri_base + end_slot), as the 64-B node's ~(first << 3 | count - 1).
__device__ __forceinline__ int32_t wide_dref(uint32_t key, uint32_t ends, uint32_t node_base, uint32_t tri_base) {
  const uint32_t sh = (key & 3u) * 6u;
  const uint32_t e1 = __builtin_amdgcn_ubfe(ends, sh, 6), e0 = __builtin_amdgcn_ubfe(ends << 6, sh, 6);
  const int32_t leaf = ~(int32_t)(((tri_base + e0) << 3) | (e1 - e0 - 1u));
  return e1 == 0u ? (int32_t)(node_base + (key & 3u)) : leaf;
}

// One visit of a 4-wide node in its 48-B device form: three 16-B loads and
// mtx_core/geometry.h wide_node_order_e. Returns the number of children hit;
// c[0..n) are their references in visit order (the same order and refs as
// the 64-B node gives the oracle).
#ifndef MTX_PAIR_SORT
#define MTX_PAIR_SORT 1  // A/B: 0 = sort the keys, then pick each reference by its key's slot bits
#endif
#ifndef MTX_NODE48
#define MTX_NODE48 0  // A/B: 1 = the 48-B node (three loads, references decoded): slower, DESIGN.md
#endif
__device__ __forceinline__ int wide_visit(const DevScene &s, const TraceRay &r, int32_t node, float tbest,
                                          int32_t c[4], const int4 *top = nullptr, int top_n = 0) {
#if !MTX_NODE48
  {
    // nodes [0, top_n) from the block's LDS copy of the tree top (64 nodes:
    // about half of the visits, tools/top_visits.py), the others from global memory
    // (the LDS reads are inline asm: as plain loads the compiler merges the
    // two branches into flat loads through a selected generic pointer, which
    // take the vector-memory path for every lane)
    int4 a, rf, qa;
    int2 qb;
    if (node < top_n) {
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
    } else {
      const int4 *np = s.nodes + 4 * node;
      a = np[0];
      rf = np[1];
      qa = np[2];
      qb = *reinterpret_cast<const int2 *>(np + 3);
    }
    uint32_t key[4];
    const uint32_t eb = (uint32_t)a.w;
#if MTX_PAIR_SORT
    // the references ride along the compare-exchange network (one compare +
    // four selects per exchange, the keys' dead selects dropped) instead of
    // being picked by the sorted keys' slot bits afterwards: the keys are
    // distinct (slot in the low bits), so the order and the references are
    // those of wide_node_order + wide_ref
    const int n = wide_node_keys_e(r, __int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z),
                                   (int)(int8_t)(uint8_t)(eb & 0xffu), (int)(int8_t)(uint8_t)((eb >> 8) & 0xffu),
                                   (int)(int8_t)(uint8_t)((eb >> 16) & 0xffu), (int)(eb >> 24), (uint32_t)qa.x,
                                   (uint32_t)qa.y, (uint32_t)qa.z, (uint32_t)qa.w, (uint32_t)qb.x, (uint32_t)qb.y,
                                   tbest, key);
    c[0] = rf.x;
    c[1] = rf.y;
    c[2] = rf.z;
    c[3] = rf.w;
#define MTX_CAS2(i, j)                                   \
  {                                                      \
    const bool sw_ = key[j] < key[i];                    \
    const uint32_t ki_ = key[i], kj_ = key[j];           \
    const int32_t ci_ = c[i], cj_ = c[j];                \
    key[i] = sw_ ? kj_ : ki_;                            \
    key[j] = sw_ ? ki_ : kj_;                            \
    c[i] = sw_ ? cj_ : ci_;                              \
    c[j] = sw_ ? ci_ : cj_;                              \
  }
    MTX_CAS2(0, 1) MTX_CAS2(2, 3) MTX_CAS2(0, 2) MTX_CAS2(1, 3) MTX_CAS2(1, 2)
#undef MTX_CAS2
    return n;
#else
    const int n = wide_node_order(r, __int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z), eb,
                                  (uint32_t)qa.x, (uint32_t)qa.y, (uint32_t)qa.z, (uint32_t)qa.w, (uint32_t)qb.x,
                                  (uint32_t)qb.y, tbest, key);
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = wide_ref(key[i], rf.x, rf.y, rf.z, rf.w);
    return n;
#endif
  }
#endif
  const int4 *np = s.nodes + 3 * node;
  const int4 a = np[0], b = np[1], q = np[2];
  const uint32_t w3 = (uint32_t)a.w, w4 = (uint32_t)b.x, w5 = (uint32_t)b.y;
  uint32_t key[4];
  const int n = wide_node_order_e(r, __int_as_float(a.x), __int_as_float(a.y), __int_as_float(a.z),
                                  __builtin_amdgcn_sbfe((int)w3, 0, 6), __builtin_amdgcn_sbfe((int)w3, 6, 6),
                                  __builtin_amdgcn_sbfe((int)w3, 12, 6), (int)__builtin_amdgcn_ubfe(w3, 18, 2) + 1,
                                  (uint32_t)b.z, (uint32_t)b.w, (uint32_t)q.x, (uint32_t)q.y, (uint32_t)q.z,
                                  (uint32_t)q.w, tbest, key);
  const uint32_t ends = (w3 >> 20) | ((w4 >> 24) << 12) | ((w5 >> 24) << 20);
  const uint32_t nb = w4 & 0xffffffu, tb = w5 & 0xffffffu;
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = wide_dref(key[i], ends, nb, tb);
  return n;
}

// ---------------------------------------------------------------------------
// BVH traversal (shared by closest-hit and any-hit). Child order and
// tie-breaking match oracle/oracle.cpp:trace_closest exactly.
// ---------------------------------------------------------------------------
template <bool ANY>
__device__ __forceinline__ bool traverse(const DevScene &s, int32_t *stk, const TraceRay &r, float &tbest,
                                         uint32_t &prim_best, float &bu, float &bv, uint32_t &nv, uint32_t &tv) {
  int sp = 0;
  int32_t node = 0;
  bool hit_any = false;
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
        const TriGeom g = load_tri(s, prim);
        float t, u, v;
        ++tv;
        if (tri_intersect(r, g.p0, g.e1, g.e2, tbest, &t, &u, &v)) {
          if (ANY) {
            hit_any = true;
            break;
          }
          if (t < tbest || (t == tbest && prim < prim_best)) {
            tbest = t;
            prim_best = prim;
            bu = u;
            bv = v;
          }
        }
      }
      if (ANY && hit_any) break;
    }
    if (sp == 0) break;
    --sp;
    node = stk[sp * kTraceBlock];
  }
  return hit_any;
}

}  // namespace mtxd

namespace mtxd {

// ---------------------------------------------------------------------------
// Persistent while-while traversal with per-lane ray replacement.
//
// Every lane owns one ray at a time. A wave alternates an inner-node phase
// (each lane descends until it reaches a leaf or runs out of nodes) with a
// leaf phase (one leaf per lane), so inner-node and triangle code do not
// serialise against each other inside one iteration. When at least
// s.refill_lanes lanes of the wave have finished, their slots are refilled from
// the ray queue with one atomic per wave (ballot + mbcnt). In the STATS
// kernels the visit order of each ray is exactly that of `traverse` above
// (same results and counts, the oracle's order); the production kernels
// speculate (below) and return the same hits with a wave-dependent order.
// ---------------------------------------------------------------------------
#ifndef MTX_PUSH_BRANCHY
#define MTX_PUSH_BRANCHY 0  // A/B: 1 = per-entry conditional pushes only
#endif
constexpr int32_t kTravDone = INT32_MIN;           // never a valid leaf reference
constexpr int32_t kTravLeafTaken = INT32_MIN + 1;  // leaf moved to the leaf phase, pop next

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

// Src provides: a Payload type (what a lane carries for its ray), load(k,
// TraceRay&, float &tmax, Payload &) and finish(const Payload &, bool any_hit,
// float t, uint32_t prim, float u, float v).
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

// Claim of the next queue entries for a wave (wave-uniform; the leader lane
// does the atomic): [base2, base2 + got2) from the own XCD's segment first,
// then the next segments; returns true once every segment is drained.
// (Guided sizes -- each claim its fair share of what the segment has left,
// read with an atomic load before the add -- measured much slower: closest
// 61.3 -> 74.0 ms/step at spp 256, 9.45 -> 15.3 at spp 32)
__device__ __forceinline__ bool claim_rays(const DevScene &s, uint32_t *heads, uint32_t count, uint32_t batch,
                                           uint32_t leader, uint32_t lane, uint32_t &seg, uint32_t &tries,
                                           uint32_t &base2, uint32_t &got2) {
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

// heads: kXcds claim cursors (kXHeadStride words apart), zeroed before the
// launch. A wave claims rays from the queue segment of its own XCD first,
// so the rays an XCD traces come from one band of the (pixel-ordered)
// queue and share BVH nodes in that XCD's L2; exhausted segments send the
// wave on to the next XCD's segment.
template <bool ANY, bool STATS = false, class Src>
__device__ __forceinline__ void trace_loop_ww(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                              int32_t *stk, const int4 *top, uint32_t &nv, uint32_t &tv,
                                              uint32_t &nr, uint32_t *wave_iters = nullptr) {
  const uint32_t lane = lane_id();
  int32_t *ovf = s.stack_ovf + blockIdx.x * kTraceBlock + threadIdx.x;
  const int lds_n = (int)s.lds_entries;
  bool has = false, exhausted = false, hit = false, drained = false;
  uint32_t res_lo = 0, res_hi = 0;
  typename Src::Payload payload{};
  uint32_t prim = 0xffffffffu;
  TraceRay r;
  float tbest = 0.f, bu = 0.f, bv = 0.f;
  int32_t node = kTravDone, leaf = 0;
  bool has_leaf = false;
  const int top_n = (int)s.lds_top;
  int sp = 0;
  const bool spec = !STATS && s.speculate;
  // more waves than batches: the surplus exits at once (a near-empty queue
  // would otherwise cost every wave of the grid its claim atomics)
  // Claim size: s.trace_batch, cut down (to >= 64) when the queue is too
  // short to give every wave of the grid a batch: a small queue then still
  // spreads over the chip instead of running a few long per-lane chains.
  const uint32_t n_grid_waves = gridDim.x * (kTraceBlock / 64u);
  const uint32_t batch = max(64u, min(s.trace_batch, (count / n_grid_waves) & ~63u));
  if ((blockIdx.x * kTraceBlock + threadIdx.x) / 64u >= (count + batch - 1) / batch) return;
  uint32_t seg = s.xcd_claim ? xcc_id() : 0u, tries = s.xcd_claim ? 0u : kXcds - 1u;
  auto pop = [&](int &spr) -> int32_t {
    if (spr == 0) return kTravDone;
    --spr;
    return stack_read(stk, ovf, spr, lds_n, s.ovf_threads);
  };
  while (true) {
    if (!exhausted) {
      // Idle lanes take rays from the wave's reservoir of claimed queue
      // indices [res_lo, res_hi); the reservoir is topped up with one atomic
      // per s.trace_batch rays (contention on the device-scope counter, not
      // the traversal, bounded short batches).
      const uint64_t idle = __ballot(!has);
      if (idle) {
        const uint32_t n = (uint32_t)__popcll(idle);
        const uint32_t left = res_hi - res_lo;
        uint32_t base2 = 0, got2 = 0;
        if (left < n && !drained)
          drained = claim_rays(s, heads, count, batch, (uint32_t)(__ffsll((unsigned long long)idle) - 1), lane, seg,
                               tries, base2, got2);
        const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        uint32_t k = 0;
        bool ok = false;
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
        if (!has && ok) {
          src.load(k, r, tbest, payload);
          prim = 0xffffffffu;
          bu = bv = 0.f;
          hit = false;
          node = 0;
          sp = 0;
          has_leaf = false;
          has = true;
        }
        exhausted = drained && res_lo >= res_hi;
      }
    }
    if (__ballot(has) == 0) break;
    while (true) {
      // inner-node phase. With speculation (Aila & Laine 2009), a lane that
      // reaches a leaf postpones it and keeps descending until every lane
      // still in the phase holds a postponed leaf: the leaf phase then runs
      // with more lanes busy. The hit is unchanged (inclusive culling and the
      // smaller-index tie rule make it order independent); the visit sequence
      // is not, so the STATS kernels (visit counters, tests) do not speculate.
      if (spec && has && !has_leaf && node < 0 && node != kTravDone) {
        leaf = node;
        has_leaf = true;
        node = pop(sp);
      }
      while (has && node >= 0) {
        if (STATS) {
          const uint64_t m = __ballot(true);
          if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) ++wave_iters[0];
        }
        int32_t cr[4];
        ++nv;
        const int n = wide_visit(s, r, node, tbest, cr, top, top_n);
        if (n > 0) {
          // far children pushed farthest first: entries sp .. sp+n-2 hold
          // cr[n-1] .. cr[1]. Branch-free: three stores, the ones beyond
          // the new top are dead (capacity 3*depth+1 covers them).
          const int32_t c1 = cr[1], c2 = cr[2], c3 = cr[3];
          const int32_t e0 = n == 4 ? c3 : (n == 3 ? c2 : c1), e1 = n == 4 ? c2 : c1;
          if (!MTX_PUSH_BRANCHY && sp + 3 <= lds_n) {
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
          node = cr[0];
        } else {
          node = pop(sp);
        }
        if (spec) {
          if (!has_leaf && node < 0 && node != kTravDone) {
            leaf = node;
            has_leaf = true;
            node = pop(sp);
          }
          if (__ballot(!has_leaf) == 0) break;
        }
      }
      // leaf phase: one leaf per lane (the postponed one first)
      if (has && (has_leaf || (node < 0 && node != kTravDone))) {
        if (STATS) {
          const uint64_t m = __ballot(true);
          if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) ++wave_iters[1];
        }
        int32_t lf;
        if (has_leaf) {
          lf = leaf;
          has_leaf = false;
        } else {
          lf = node;
          node = kTravLeafTaken;
        }
        uint32_t first, cnt;
        leaf_decode(lf, &first, &cnt);
        for (uint32_t k = 0; k < cnt; ++k) {
          const uint32_t pr = first + k;
          const TriGeom g = load_tri(s, pr);
          float t, u, v;
          ++tv;
          if (tri_intersect(r, g.p0, g.e1, g.e2, tbest, &t, &u, &v)) {
            if (ANY) {
              hit = true;
              break;
            }
            if (t < tbest || (t == tbest && pr < prim)) {
              tbest = t;
              prim = pr;
              bu = u;
              bv = v;
            }
          }
        }
        if (ANY && hit) {
          node = kTravDone;
        } else if (node == kTravLeafTaken) {
          node = pop(sp);
        }
      }
      if (has && node == kTravDone) {
        src.finish(payload, hit, tbest, prim, bu, bv);
        has = false;
        ++nr;
      }
      const uint64_t idle = __ballot(!has);
      if (idle == ~0ull || (!exhausted && (uint32_t)__popcll(idle) >= s.refill_lanes)) break;
    }
  }
}


// ---------------------------------------------------------------------------
// Unified single-step traversal (A/B against while-while: MTX_TRAV_UNIFIED).
//
// Every iteration each lane with a ray performs one unit of work: one inner
// node visit, then (same iteration) one triangle test if its current leaf
// has triangles left. A lane reaching a leaf starts on its triangles in the
// same iteration; a lane that finishes its ray is refilled once enough lanes
// of the wave are idle. Nothing waits for the slowest lane of the wave to
// reach a leaf (the while-while phase barrier), so more lanes do work per
// wave-instruction; the price is that both code paths run in an iteration
// whenever the wave holds lanes of both kinds. Each ray's visit sequence is
// the plain front-to-back order of `traverse` (the oracle's), with or
// without STATS.
// ---------------------------------------------------------------------------
#ifndef MTX_TRI_MIN
#define MTX_TRI_MIN 0
#endif
// (A per-lane ray prefetch -- the next ray's raw data held in registers so a
// refill starts without a load round trip -- measured slower: closest +2.3 %
// with batched swaps, +16 % swapping every iteration)
template <bool ANY, bool STATS = false, class Src>
__device__ __forceinline__ void trace_loop_u(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                             int32_t *stk, const int4 *top, uint32_t &nv, uint32_t &tv,
                                             uint32_t &nr, uint32_t *wave_iters = nullptr) {
  const uint32_t lane = lane_id();
  int32_t *ovf = s.stack_ovf + blockIdx.x * kTraceBlock + threadIdx.x;
  const int lds_n = (int)s.lds_entries;
  bool has = false, exhausted = false, hit = false, drained = false;
  uint32_t res_lo = 0, res_hi = 0;
  typename Src::Payload payload{};
  uint32_t prim = 0xffffffffu;
  TraceRay r;
  float tbest = 0.f, bu = 0.f, bv = 0.f;
  int32_t node = -1;          // >= 0: inner node to visit next
  const int top_n = (int)s.lds_top;
  uint32_t tri = 0, tri_end = 0;  // triangles [tri, tri_end) of the current leaf
  int sp = 0;
  const uint32_t n_grid_waves = gridDim.x * (kTraceBlock / 64u);
  const uint32_t batch = max(64u, min(s.trace_batch, (count / n_grid_waves) & ~63u));
  if ((blockIdx.x * kTraceBlock + threadIdx.x) / 64u >= (count + batch - 1) / batch) return;
  uint32_t seg = s.xcd_claim ? xcc_id() : 0u, tries = s.xcd_claim ? 0u : kXcds - 1u;
  // next work item of a lane from its stack: an inner node, a leaf's
  // triangle range, or nothing (the ray is finished)
  auto pop_next = [&]() {
    node = -1;
    while (sp > 0) {
      --sp;
      const int32_t e = stack_read(stk, ovf, sp, lds_n, s.ovf_threads);
      if (e >= 0) {
        node = e;
        return;
      }
      uint32_t first, cnt;
      leaf_decode(e, &first, &cnt);
      tri = first;
      tri_end = first + cnt;
      return;
    }
  };
  // claim one queue index for every lane in `want` from the wave's
  // reservoir (topped up by claim_rays): k is this lane's, ok if it got one
  auto take = [&](uint64_t want, uint32_t &k, bool &ok) {
    const uint32_t n = (uint32_t)__popcll(want);
    const uint32_t left = res_hi - res_lo;
    uint32_t base2 = 0, got2 = 0;
    if (left < n && !drained)
      drained = claim_rays(s, heads, count, batch, (uint32_t)(__ffsll((unsigned long long)want) - 1), lane, seg,
                           tries, base2, got2);
    const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
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
  };
  auto begin_ray = [&]() {
    prim = 0xffffffffu;
    bu = bv = 0.f;
    hit = false;
    node = 0;
    tri = tri_end = 0;
    sp = 0;
    has = true;
  };
  while (true) {
    if (!exhausted) {
      const uint64_t idle = __ballot(!has);
      if ((uint32_t)__popcll(idle) >= s.urefill || idle == ~0ull) {
        uint32_t k;
        bool ok;
        take(idle, k, ok);
        if (!has && ok) {
          src.load(k, r, tbest, payload);
          begin_ray();
        }
      }
    }
    if (__ballot(has) == 0) break;
    // ---- one inner-node visit
    if (has && node >= 0) {
      if (STATS) {
        const uint64_t m = __ballot(true);
        if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) ++wave_iters[0];
      }
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
    }
    // ---- one triangle test. Deferred (MTX_TRI_MIN > 0, an A/B build that
    // measured slower at every threshold) until enough lanes wait
    // on a triangle or no lane has a node to visit; every ray's own visit
    // sequence is unchanged.
    bool tri_step = true;
    if (MTX_TRI_MIN) {
      const uint32_t nt = (uint32_t)__popcll(__ballot(has && tri < tri_end));
      tri_step = nt >= MTX_TRI_MIN || __ballot(has && node >= 0) == 0;
    }
    if (tri_step && has && tri < tri_end) {
      if (STATS) {
        const uint64_t m = __ballot(true);
        if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1)) ++wave_iters[1];
      }
      const uint32_t pr = tri;
      const TriGeom g = load_tri(s, pr);
      float t, u, v;
      ++tv;
      ++tri;
      if (tri_intersect(r, g.p0, g.e1, g.e2, tbest, &t, &u, &v)) {
        if (ANY) {
          hit = true;
          tri = tri_end;
          sp = 0;
        } else if (t < tbest || (t == tbest && pr < prim)) {
          tbest = t;
          prim = pr;
          bu = u;
          bv = v;
        }
      }
      if (tri >= tri_end) pop_next();
    }
    if (has && node < 0 && tri >= tri_end) {
      src.finish(payload, hit, tbest, prim, bu, bv);
      has = false;
      ++nr;
    }
  }
}

// bit 0: closest-hit kernels, bit 1: any-hit kernels use trace_loop_u
#ifndef MTX_TRAV_UNIFIED
#define MTX_TRAV_UNIFIED 1
#endif
// stk: this thread's stack column (dynamic LDS + threadIdx.x). Every thread
// of the block calls this (the LDS tree top is filled behind a barrier).
template <bool ANY, bool STATS = false, class Src>
__device__ __forceinline__ void trace_loop(const DevScene &s, const Src &src, uint32_t count, uint32_t *heads,
                                           int32_t *stk, uint32_t &nv, uint32_t &tv, uint32_t &nr,
                                           uint32_t *wave_iters = nullptr) {
  int4 *top = reinterpret_cast<int4 *>(stk - threadIdx.x + s.lds_entries * kTraceBlock);
  for (uint32_t i = threadIdx.x; i < 4 * s.lds_top; i += kTraceBlock) top[i] = s.nodes[i];
  __syncthreads();
  if ((MTX_TRAV_UNIFIED >> (ANY ? 1 : 0)) & 1)
    trace_loop_u<ANY, STATS>(s, src, count, heads, stk, top, nv, tv, nr, wave_iters);
  else
    trace_loop_ww<ANY, STATS>(s, src, count, heads, stk, top, nv, tv, nr, wave_iters);
}

}  // namespace mtxd
