// mtx_core/nerad.h — neural radiosity training samples (nerad.py), shared by
// the device kernels and the CPU restatement in oracle/.
//
//   IntersectionSampler.sample (nerad.py:291-310): a shape by surface area
//     (DiscreteDistribution over shape areas, :284-289), a direction sample,
//     then shape.sample_position(0, u2) and a uniform sphere / hemisphere
//     direction for two-sided / one-sided BSDFs (:297-308).
//   Upstream pieces restated (Mitsuba 3 core, unverifiable offline; parity
//   unpinned): DiscreteDistribution::sample / sample_reuse (cdf accumulated
//   in double, stored as float; search restricted to the non-zero range),
//   Mesh::sample_position (triangle by area with the reused sample.y, then
//   warp::square_to_uniform_triangle), warp::square_to_uniform_sphere.
//   Restatement choices: a mesh's triangles are in BVH leaf order (the OBJ
//   face order upstream: same distribution, another u -> triangle map); the
//   sampled point is the surface interaction of a hit at that triangle with
//   barycentrics (b1, b2) (si_from_vertices), so p, n, uv and the shading
//   frame come from the same code as a ray hit.
#pragma once
#include "common.h"
#include "rng.h"
#include "warp.h"

namespace mtx {

// One DiscreteDistribution: pmf[n], cdf[n] (inclusive prefix, double-
// accumulated, stored as float), sum = cdf[n-1], normalization = 1/sum, and
// the first / last index with a non-zero pmf (upstream m_valid).
struct DiscreteDist {
  const float *pmf, *cdf;
  uint32_t n, valid_lo, valid_hi;
  float sum, normalization;
};

// DiscreteDistribution::sample: the first index in [valid_lo, valid_hi]
// whose cdf is not below u * sum.
MTX_HD uint32_t discrete_sample(const DiscreteDist &d, float u) {
  const float value = u * d.sum;
  uint32_t lo = d.valid_lo, hi = d.valid_hi;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (d.cdf[mid] < value)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// DiscreteDistribution::sample_reuse: index and the sample rescaled to
// [0, 1) inside the chosen interval.
MTX_HD uint32_t discrete_sample_reuse(const DiscreteDist &d, float u, float *u_out) {
  const uint32_t i = discrete_sample(d, u);
  const float pmf = d.pmf[i] * d.normalization;
  const float cdf = i > 0 ? d.cdf[i - 1] * d.normalization : 0.f;
  *u_out = (u - cdf) / pmf;
  return i;
}

MTX_HD V2 square_to_uniform_triangle(V2 s) {
  const float t = safe_sqrt(1.f - s.x);
  return V2{1.f - t, t * s.y};
}

// Surface-area tables of a scene (built on the host, mtx/nerad.py): the
// shape distribution and, per shape, the distribution over its triangles
// (tri_dist[shape] views into the concatenated pmf / cdf arrays, whose
// entries map to leaf-order triangles through tri_prim).
struct NeradTables {
  DiscreteDist shape;
  const DiscreteDist *tri_dist;  // per shape
  const uint32_t *tri_off;       // per shape: first entry in tri_prim
  const uint32_t *tri_prim;      // leaf-order triangle of each entry
};

// Mitsuba's BackSide flag: twosided wrappers, dielectrics (transmission)
// and masks (null transmission from both sides).
MTX_HD bool material_two_sided(const mtx_material &m) {
  return (m.flags & (MTX_MF_TWOSIDED | MTX_MF_MASK)) != 0 || m.type == MTX_MAT_DIELECTRIC ||
         m.type == MTX_MAT_ROUGHDIELECTRIC;
}

struct SurfaceSample {
  uint32_t prim;  // leaf-order triangle
  float b1, b2;   // barycentrics of vertices 1 and 2
  V3 wi_local;    // incident direction in the shading frame
};

// IntersectionSampler.sample (nerad.py:291-310), draws in the reference
// order: shape (next_1d), direction (next_2d), position (next_2d).
MTX_HD SurfaceSample nerad_surface_sample(const NeradTables &t, const mtx_shape *shapes,
                                          const mtx_material *materials, Pcg32 &rng) {
  const uint32_t shape = discrete_sample(t.shape, rng.next_1d());
  const V2 dir = rng.next_2d();
  V2 ps = rng.next_2d();
  float y2;
  const uint32_t k = discrete_sample_reuse(t.tri_dist[shape], ps.y, &y2);
  ps.y = y2;
  const V2 b = square_to_uniform_triangle(ps);
  SurfaceSample s;
  s.prim = t.tri_prim[t.tri_off[shape] + k];
  s.b1 = b.x;
  s.b2 = b.y;
  const bool two_sided = material_two_sided(materials[shapes[shape].material]);
  s.wi_local = two_sided ? square_to_uniform_sphere(dir) : square_to_uniform_hemisphere(dir);
  return s;
}

}  // namespace mtx
