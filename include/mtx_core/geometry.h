// mtx_core/geometry.h — ray/box and ray/triangle tests on the BVH layout of
// mtx.h (4-wide sorted nodes for closest hit, 8-wide compressed nodes for any
// hit, both with 8-bit quantised child boxes). These replace the primitive tests inside Embree's rtcIntersect /
// rtcOccluded and OptiX optixTrace behind Scene.ray_intersect / ray_test
// (path-mis.py:69-71, restirgi.py:320,346). The triangle test is the
// Moeller-Trumbore form of upstream Mesh::ray_intersect_triangle. Closest-hit
// ties on t are broken towards the smaller triangle index, so the result does
// not depend on traversal order.
#pragma once
#include "common.h"

namespace mtx {

struct TraceRay {
  V3 o, d, idir, ooi;  // ooi = o * idir
  float maxt;
};

// Direction components of magnitude < 1e-20 are replaced by +-1e-20 before
// the reciprocal so that the slab test never forms 0*inf.
MTX_HD TraceRay make_trace_ray(V3 o, V3 d, float maxt) {
  TraceRay r;
  r.o = o;
  r.d = d;
  r.maxt = maxt;
  float dx = fabsf(d.x) < 1e-20f ? mulsign(1e-20f, d.x) : d.x;
  float dy = fabsf(d.y) < 1e-20f ? mulsign(1e-20f, d.y) : d.y;
  float dz = fabsf(d.z) < 1e-20f ? mulsign(1e-20f, d.z) : d.z;
  r.idir = V3{1.f / dx, 1.f / dy, 1.f / dz};
  r.ooi = V3{o.x * r.idir.x, o.y * r.idir.y, o.z * r.idir.z};
  return r;
}

// Slab test of one child box; returns the entry distance, or +inf on a miss.
MTX_HD float box_enter(const TraceRay &r, float lox, float hix, float loy, float hiy, float loz, float hiz,
                       float tfar) {
  float tx0 = fmaf(lox, r.idir.x, -r.ooi.x), tx1 = fmaf(hix, r.idir.x, -r.ooi.x);
  float ty0 = fmaf(loy, r.idir.y, -r.ooi.y), ty1 = fmaf(hiy, r.idir.y, -r.ooi.y);
  float tz0 = fmaf(loz, r.idir.z, -r.ooi.z), tz1 = fmaf(hiz, r.idir.z, -r.ooi.z);
  float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
  float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tfar));
  return tmin <= tmax ? tmin : kInf;
}

// Moeller-Trumbore; on a hit with t in (0, tfar] writes t,u,v and returns true.
MTX_HD bool tri_intersect(const TraceRay &r, V3 p0, V3 e1, V3 e2, float tfar, float *t_out, float *u_out,
                          float *v_out) {
  V3 pvec = cross(r.d, e2);
  float inv_det = 1.f / dot(e1, pvec);
  V3 tvec = r.o - p0;
  float u = dot(tvec, pvec) * inv_det;
  V3 qvec = cross(tvec, e1);
  float v = dot(r.d, qvec) * inv_det;
  float t = dot(e2, qvec) * inv_det;
  bool hit = u >= 0.f && u <= 1.f && v >= 0.f && u + v <= 1.f && t > 0.f && t <= tfar;
  *t_out = t;
  *u_out = u;
  *v_out = v;
  return hit;
}

// ---- quantised node frames (both node forms) ------------------------------
// Child box bound = origin + q * 2^e, evaluated in fp32 exactly like this on
// the host (builder) and the device, so the builder's conservative choice of
// q holds for the traversal.
MTX_HD float wide_scale(uint32_t e_byte) {
  const int e = (int)(int8_t)(uint8_t)(e_byte & 0xffu);
  return u2f((uint32_t)(e + 127) << 23);
}
MTX_HD float wide_decode(float origin, float scale, uint32_t q) { return origin + (float)q * scale; }

// 2^e * x, exact (= wide_scale(e) * x): one v_ldexp_f32 on the device.
MTX_HD float wide_ldexp(float x, int e) {
#ifdef MTX_DEVICE_COMPILE
  return __builtin_amdgcn_ldexpf(x, e);
#else
  return ldexpf(x, e);
#endif
}

// ---- 4-wide sorted nodes (closest hit; layout MTX_BVH4 in mtx.h) --------
// Slab tests of a node's children in the node's quantised frame: with
// a = 2^e / d and b = (origin - o) / d per axis, a bound q is at
// t = fma(q, a, b). Children hit within (0, tfar] get the sort key
// (t bits with the 2 low bits cleared) | slot, misses 0x7f800000 | slot; the
// four keys are sorted ascending (5 compare-exchanges), so the visit order is
// by entry distance, near-ties by slot. Returns the number of hits.
// qlx.. hold the four children's 8-bit bounds, child k in bits [8k, 8k+8).
// wide_node_order_e takes the axis exponents and child count decoded (the
// device's 48-B node keeps them in 6-bit fields, mtx_scene_upload).
// wide_node_keys_e: the four keys in slot order (unsorted), for callers that
// sort them together with the child references.
MTX_HD int wide_node_keys_e(const TraceRay &r, float ox, float oy, float oz, int ex, int ey, int ez, int nch,
                            uint32_t qlx, uint32_t qhx, uint32_t qly, uint32_t qhy, uint32_t qlz, uint32_t qhz,
                            float tfar, uint32_t key[4]) {
  const float ax = wide_ldexp(r.idir.x, ex), bx = (ox - r.o.x) * r.idir.x;
  const float ay = wide_ldexp(r.idir.y, ey), by = (oy - r.o.y) * r.idir.y;
  const float az = wide_ldexp(r.idir.z, ez), bz = (oz - r.o.z) * r.idir.z;
  // near / far bound of each axis from the direction's sign: fma(q, a, b)
  // is monotonic in q, so this equals min / max of the two planes (NaN
  // planes of a zero direction component are ignored either way)
  int n = 0;  // children hit (hit keys sort below every miss key)
  const bool nx_ = r.idir.x < 0.f, ny_ = r.idir.y < 0.f, nz_ = r.idir.z < 0.f;
  const uint32_t qnx = nx_ ? qhx : qlx, qfx = nx_ ? qlx : qhx;
  const uint32_t qny = ny_ ? qhy : qly, qfy = ny_ ? qly : qhy;
  const uint32_t qnz = nz_ ? qhz : qlz, qfz = nz_ ? qlz : qhz;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sh = 8 * k;
#ifdef MTX_DEVICE_COMPILE
    // the same six fmas, issued as three packed v_pk_fma_f32
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v tx = __builtin_elementwise_fma(f2v{(float)((qnx >> sh) & 255u), (float)((qfx >> sh) & 255u)},
                                             f2v{ax, ax}, f2v{bx, bx});
    const f2v ty = __builtin_elementwise_fma(f2v{(float)((qny >> sh) & 255u), (float)((qfy >> sh) & 255u)},
                                             f2v{ay, ay}, f2v{by, by});
    const f2v tz = __builtin_elementwise_fma(f2v{(float)((qnz >> sh) & 255u), (float)((qfz >> sh) & 255u)},
                                             f2v{az, az}, f2v{bz, bz});
    const float nx = tx.x, fx = tx.y, ny = ty.x, fy = ty.y, nz = tz.x, fz = tz.y;
#else
    const float nx = fmaf((float)((qnx >> sh) & 255u), ax, bx), fx = fmaf((float)((qfx >> sh) & 255u), ax, bx);
    const float ny = fmaf((float)((qny >> sh) & 255u), ay, by), fy = fmaf((float)((qfy >> sh) & 255u), ay, by);
    const float nz = fmaf((float)((qnz >> sh) & 255u), az, bz), fz = fmaf((float)((qfz >> sh) & 255u), az, bz);
#endif
    const float tmin = fmaxf(fmaxf(fmaxf(nx, ny), nz), 0.f);
    const float tmax = fminf(fminf(fminf(fx, fy), fz), tfar);
    const bool hit = k < nch && tmin <= tmax;
    key[k] = hit ? ((f2u(tmin) & 0x7ffffffcu) | (uint32_t)k) : (0x7f800000u | (uint32_t)k);
    n += hit ? 1 : 0;
  }
  return n;
}

MTX_HD int wide_node_order_e(const TraceRay &r, float ox, float oy, float oz, int ex, int ey, int ez, int nch,
                             uint32_t qlx, uint32_t qhx, uint32_t qly, uint32_t qhy, uint32_t qlz, uint32_t qhz,
                             float tfar, uint32_t key[4]) {
  const int n = wide_node_keys_e(r, ox, oy, oz, ex, ey, ez, nch, qlx, qhx, qly, qhy, qlz, qhz, tfar, key);
#define MTX_CAS(i, j)                                   \
  {                                                     \
    const uint32_t lo_ = key[i] < key[j] ? key[i] : key[j]; \
    const uint32_t hi_ = key[i] < key[j] ? key[j] : key[i]; \
    key[i] = lo_;                                       \
    key[j] = hi_;                                       \
  }
  MTX_CAS(0, 1) MTX_CAS(2, 3) MTX_CAS(0, 2) MTX_CAS(1, 3) MTX_CAS(1, 2)
#undef MTX_CAS
  return n;
}

// The 64-B node form (mtx.h): int8 exponents in eb's bytes 0..2, the child
// count in byte 3.
MTX_HD int wide_node_order(const TraceRay &r, float ox, float oy, float oz, uint32_t eb, uint32_t qlx,
                           uint32_t qhx, uint32_t qly, uint32_t qhy, uint32_t qlz, uint32_t qhz, float tfar,
                           uint32_t key[4]) {
  return wide_node_order_e(r, ox, oy, oz, (int)(int8_t)(uint8_t)(eb & 0xffu), (int)(int8_t)(uint8_t)((eb >> 8) & 0xffu),
                           (int)(int8_t)(uint8_t)((eb >> 16) & 0xffu), (int)(eb >> 24), qlx, qhx, qly, qhy, qlz, qhz,
                           tfar, key);
}

// Child reference of the slot encoded in a sort key.
MTX_HD int32_t wide_ref(uint32_t key, int32_t r0, int32_t r1, int32_t r2, int32_t r3) {
  // two bit selects (no branches on the device)
  const bool b0 = (key & 1u) != 0u, b1 = (key & 2u) != 0u;
  const int32_t lo = b0 ? r1 : r0, hi = b0 ? r3 : r2;
  return b1 ? hi : lo;
}

MTX_HD void leaf_decode(int32_t c, uint32_t *first, uint32_t *count) {
  uint32_t x = (uint32_t)(~c);
  *first = x >> 3;
  *count = (x & 7u) + 1u;
}


// ---- 8-wide compressed nodes (any hit; layout MTX_BVH8 in mtx.h) --------
// Octant of a ray: bit a set when the direction's component a is negative
// (the sign of the clamped reciprocal: -0 counts as negative). A node's slot s
// is visited at position s ^ octant.
MTX_HD uint32_t ray_octant(const TraceRay &r) {
  return (r.idir.x < 0.f ? 1u : 0u) | (r.idir.y < 0.f ? 2u : 0u) | (r.idir.z < 0.f ? 4u : 0u);
}

// Slab tests of one half (slots 4h .. 4h+3) of an 8-wide node in the node's
// quantised frame: with a = 2^e / d and b = (origin - o) / d per axis, a bound
// q lies at t = fma(q, a, b); a child is hit when max(t_near, 0) <=
// min(t_far, tfar). qn* / qf* are the near / far bound bytes of the four
// slots (chosen per axis from the direction's sign), m4 their meta bytes.
// Returns the half's contribution to the hit mask (cw_node_hits).
MTX_HD uint32_t cw_half_hits(float ax, float bx, float ay, float by, float az, float bz, uint32_t qnx, uint32_t qfx,
                             uint32_t qny, uint32_t qfy, uint32_t qnz, uint32_t qfz, uint32_t m4, uint32_t oct4,
                             float tfar) {
  // inner slots have meta 0x38 | s (bits 3 and 4 set); their bit index
  // 24 + s becomes 24 + (s ^ octant), a leaf's (its triangle offset) stays
  const uint32_t inner4 = m4 & (m4 << 1) & 0x10101010u;
  const uint32_t sel4 = (inner4 >> 2) | (inner4 >> 3) | (inner4 >> 4);  // 0x07 in inner bytes
  const uint32_t bidx4 = (m4 ^ (oct4 & sel4)) & 0x1f1f1f1fu;
  const uint32_t cb4 = (m4 >> 5) & 0x07070707u;  // 1 for inner, 1 / 3 / 7 for a leaf of 1 / 2 / 3 triangles
  uint32_t hits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sh = 8 * k;
#ifdef MTX_DEVICE_COMPILE
    // the six fmas as three packed v_pk_fma_f32
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v tx = __builtin_elementwise_fma(f2v{(float)((qnx >> sh) & 255u), (float)((qfx >> sh) & 255u)},
                                             f2v{ax, ax}, f2v{bx, bx});
    const f2v ty = __builtin_elementwise_fma(f2v{(float)((qny >> sh) & 255u), (float)((qfy >> sh) & 255u)},
                                             f2v{ay, ay}, f2v{by, by});
    const f2v tz = __builtin_elementwise_fma(f2v{(float)((qnz >> sh) & 255u), (float)((qfz >> sh) & 255u)},
                                             f2v{az, az}, f2v{bz, bz});
    const float nx = tx.x, fx = tx.y, ny = ty.x, fy = ty.y, nz = tz.x, fz = tz.y;
#else
    const float nx = fmaf((float)((qnx >> sh) & 255u), ax, bx), fx = fmaf((float)((qfx >> sh) & 255u), ax, bx);
    const float ny = fmaf((float)((qny >> sh) & 255u), ay, by), fy = fmaf((float)((qfy >> sh) & 255u), ay, by);
    const float nz = fmaf((float)((qnz >> sh) & 255u), az, bz), fz = fmaf((float)((qfz >> sh) & 255u), az, bz);
#endif
    const float tmin = fmaxf(fmaxf(fmaxf(nx, ny), nz), 0.f);
    const float tmax = fminf(fminf(fminf(fx, fy), fz), tfar);
    const uint32_t bits = ((cb4 >> sh) & 7u) << ((bidx4 >> sh) & 31u);
    hits |= tmin <= tmax ? bits : 0u;
  }
  return hits;
}

// All eight children of a node (words w[0..19] of mtx.h). Returns the hit
// mask: bit 24 + (s ^ oct) for a hit inner child in slot s -- the lowest such
// bit is the nearest child in the octant order -- and bits offset .. offset +
// n - 1 for a hit leaf of n triangles (tri_base + offset ...).
MTX_HD uint32_t cw_node_hits(const TraceRay &r, uint32_t oct, float ox, float oy, float oz, uint32_t w3,
                             uint32_t meta_lo, uint32_t meta_hi, const uint32_t q[12], float tfar) {
  const float ax = wide_ldexp(r.idir.x, (int)(int8_t)(uint8_t)(w3 & 0xffu)), bx = (ox - r.o.x) * r.idir.x;
  const float ay = wide_ldexp(r.idir.y, (int)(int8_t)(uint8_t)((w3 >> 8) & 0xffu)), by = (oy - r.o.y) * r.idir.y;
  const float az = wide_ldexp(r.idir.z, (int)(int8_t)(uint8_t)((w3 >> 16) & 0xffu)), bz = (oz - r.o.z) * r.idir.z;
  // near / far bound of each axis from the direction's sign: fma(q, a, b) is
  // monotonic in q, so this equals min / max of the two planes
  const bool nx_ = (oct & 1u) != 0, ny_ = (oct & 2u) != 0, nz_ = (oct & 4u) != 0;
  const uint32_t oct4 = oct * 0x01010101u;
  uint32_t hits = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t qlx = q[0 + h], qhx = q[2 + h], qly = q[4 + h], qhy = q[6 + h], qlz = q[8 + h], qhz = q[10 + h];
    hits |= cw_half_hits(ax, bx, ay, by, az, bz, nx_ ? qhx : qlx, nx_ ? qlx : qhx, ny_ ? qhy : qly, ny_ ? qly : qhy,
                         nz_ ? qhz : qlz, nz_ ? qlz : qhz, h ? meta_hi : meta_lo, oct4, tfar);
  }
  return hits;
}

// Node index of the inner child at hit-mask bit 24 + p (p = slot ^ oct).
MTX_HD uint32_t cw_inner_child(uint32_t child_base, uint32_t imask, uint32_t oct, uint32_t p) {
  const uint32_t slot = p ^ oct;
  return child_base + (uint32_t)popc32(imask & ((1u << slot) - 1u));
}



}  // namespace mtx
