// mtx_core/geometry.h — ray/box and ray/triangle tests on the BVH layout of
// mtx.h (4-wide nodes with 8-bit quantised child boxes). These replace the primitive tests inside Embree's rtcIntersect /
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

// ---- 4-wide quantised nodes (layout in mtx.h) ----------------------------
// Child box bound = origin + q * 2^e, evaluated in fp32 exactly like this on
// the host (builder, oracle) and the device, so the builder's conservative
// choice of q holds for the traversal.
MTX_HD float wide_scale(uint32_t e_byte) {
  const int e = (int)(int8_t)(uint8_t)(e_byte & 0xffu);
  return u2f((uint32_t)(e + 127) << 23);
}
MTX_HD float wide_decode(float origin, float scale, uint32_t q) { return origin + (float)q * scale; }

// Entry distance of child k (slot 0..3), +inf if missed. qlx.. hold the four
// children's 8-bit bounds, child k in bits [8k, 8k+8).
MTX_HD float wide_child_enter(const TraceRay &r, float ox, float oy, float oz, float sx, float sy, float sz,
                              uint32_t qlx, uint32_t qhx, uint32_t qly, uint32_t qhy, uint32_t qlz, uint32_t qhz,
                              int k, float tfar) {
  const int sh = 8 * k;
  return box_enter(r, wide_decode(ox, sx, (qlx >> sh) & 255u), wide_decode(ox, sx, (qhx >> sh) & 255u),
                   wide_decode(oy, sy, (qly >> sh) & 255u), wide_decode(oy, sy, (qhy >> sh) & 255u),
                   wide_decode(oz, sz, (qlz >> sh) & 255u), wide_decode(oz, sz, (qhz >> sh) & 255u), tfar);
}

// Visit order of a node's children: hits by ascending entry distance, ties by
// slot; rank[k] is child k's position (misses rank after all hits). Returns
// the number of hits. The nearest hit is visited next, the others are pushed
// farthest first.
MTX_HD int wide_ranks(const float t[4], int rank[4]) {
  int n = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int rk = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) rk += (j != k && (t[j] < t[k] || (t[j] == t[k] && j < k))) ? 1 : 0;
    rank[k] = rk;
    n += t[k] != kInf ? 1 : 0;
  }
  return n;
}

MTX_HD int32_t wide_pick(const int rank[4], const int32_t ref[4], int r) {
  int32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v = rank[k] == r ? ref[k] : v;
  return v;
}

MTX_HD void leaf_decode(int32_t c, uint32_t *first, uint32_t *count) {
  uint32_t x = (uint32_t)(~c);
  *first = x >> 3;
  *count = (x & 7u) + 1u;
}

}  // namespace mtx
