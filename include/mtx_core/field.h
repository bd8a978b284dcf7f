// Radiance-field feature encoding (nerad.py:54-106 Field.__call__), shared by
// the device encoder and the CPU reference restatement used by the tests.
//
//   p_norm = (p - bbox.min) / (bbox.max - bbox.min)            nerad.py:92-94
//   p_enc  = multiresolution hash-grid encoding of p_norm        nerad.py:96
//            (drjit.nn.HashGridEncoding; the coopvec-hashgrid branch of
//            Dr.Jit is not available, so this restates the published
//            Instant-NGP / tiny-cuda-nn grid encoding: parity unpinned)
//   wi_enc = real spherical harmonics up to degree `sh_order`     nerad.py:101
//            (dr.sh_eval, Sloan's generated evaluation)
//   features = (p_norm, p_enc, wi, wi_enc) -> fp16                nerad.py:103
#pragma once
#include "common.h"

namespace mtx {

constexpr uint32_t kFieldMaxLevels = 32;

struct FieldEncoding {
  const uint16_t *table;  // fp16 bits, [level][2^log2_table][n_features]
  uint32_t n_levels, n_features, log2_table;
  // per level: scale = base_res * per_level_scale^l - 1 (computed once on the
  // host in double, tiny-cuda-nn grid_scale) and resolution = ceil(scale) + 1
  float level_scale[kFieldMaxLevels];
  uint32_t level_res[kFieldMaxLevels];
  float bbox_min[3], bbox_max[3];
};

constexpr uint32_t kFieldPrimes[3] = {1u, 2654435761u, 805459861u};

// fp16 bits -> float (round-trip exact)
MTX_HD float half_bits_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  if (e == 0) {
    if (m == 0) return u2f(s);
    float f = (float)m * 5.9604644775390625e-08f;  // 2^-24
    return s ? -f : f;
  }
  if (e == 31) return u2f(s | 0x7f800000u | (m << 13));
  return u2f(s | ((e + 112u) << 23) | (m << 13));
}

// float -> fp16 bits, round to nearest even (IEEE binary16, with subnormals)
MTX_HD uint16_t float_to_half_bits(float f) {
  const uint32_t x = f2u(f);
  const uint32_t s = (x >> 16) & 0x8000u;
  const uint32_t a = x & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(s | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);  // >= 65520 rounds to inf
  if (a < 0x38800000u) {                                   // subnormal half (< 2^-14)
    if (a < 0x33000000u) return (uint16_t)s;                // < 2^-25 -> 0
    const uint32_t e = a >> 23, m = (a & 0x7fffffu) | 0x800000u;
    const uint32_t shift = 126u - e;                        // 14 - (e - 127) + 13 - ...
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (r & 1u))) ++r;
    return (uint16_t)(s | r);
  }
  uint32_t r = ((a - 0x38000000u) >> 13);
  const uint32_t rem = a & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) ++r;
  return (uint16_t)(s | r);
}

MTX_HD float round_half(float f) { return half_bits_to_float(float_to_half_bits(f)); }

// Hash-grid encoding of level l of one point (p_norm in [0,1]^3): fp16 bits
// of the level's n_features interpolated features (f32 interpolation, one
// rounding to fp16 per feature).
// Entries (both features, packed) of corners x and x+1 of one (y, z) row.
MTX_HD void field_fetch_pair(const uint32_t *tab, uint32_t i0, uint32_t i1, uint32_t *a, uint32_t *b) {
#ifdef MTX_DEVICE_COMPILE
  // one 8-B gather when the two entries are adjacent (dense levels, and
  // hashed levels whose x-pair differs in bit 0 only): half the requests
  if (i1 == i0 + 1u || i0 == i1 + 1u) {
    const uint32_t lo = i1 == i0 + 1u ? i0 : i1;
    uint2 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(tab + lo, 4), 8);
    *a = i1 == i0 + 1u ? v.x : v.y;
    *b = i1 == i0 + 1u ? v.y : v.x;
    return;
  }
#endif
  *a = tab[i0];
  *b = tab[i1];
}

// Hash-grid encoding of level l of one point (p_norm in [0,1]^3): fp16 bits
// of the level's n_features interpolated features (f32 interpolation, one
// rounding to fp16 per feature).
MTX_HD void field_hashgrid_level(const FieldEncoding &e, V3 pn, uint32_t l, uint16_t *out) {
  const uint32_t T = 1u << e.log2_table;
  const float scale = e.level_scale[l];
  const uint32_t res = e.level_res[l];
  const bool dense = (uint64_t)res * res * res <= (uint64_t)T;
  const float px = fmaf(pn.x, scale, 0.5f), py = fmaf(pn.y, scale, 0.5f), pz = fmaf(pn.z, scale, 0.5f);
  const float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
  const float tx = px - fx, ty = py - fy, tz = pz - fz;
  const uint32_t gx = (uint32_t)(int32_t)fx, gy = (uint32_t)(int32_t)fy, gz = (uint32_t)(int32_t)fz;
  auto index = [&](uint32_t x, uint32_t y, uint32_t z) -> uint32_t {
    const uint32_t idx = dense ? x + y * res + z * res * res
                               : (x * kFieldPrimes[0]) ^ (y * kFieldPrimes[1]) ^ (z * kFieldPrimes[2]);
    return idx & (T - 1u);  // T is a power of two
  };
  float acc0 = 0.f, acc1 = 0.f;
  if (e.n_features == 2) {
    const uint32_t *tab = reinterpret_cast<const uint32_t *>(e.table) + (size_t)l * T;
    uint32_t ent[8];
    for (uint32_t yz = 0; yz < 4; ++yz) {
      const uint32_t y = gy + (yz & 1u), z = gz + (yz >> 1);
      field_fetch_pair(tab, index(gx, y, z), index(gx + 1u, y, z), &ent[2 * yz], &ent[2 * yz + 1]);
    }
    for (uint32_t c = 0; c < 8; ++c) {
      const uint32_t bx = c & 1u, by = (c >> 1) & 1u, bz = (c >> 2) & 1u;
      const float w = (bx ? tx : 1.f - tx) * (by ? ty : 1.f - ty) * (bz ? tz : 1.f - tz);
      acc0 = fmaf(w, half_bits_to_float((uint16_t)(ent[c] & 0xffffu)), acc0);
      acc1 = fmaf(w, half_bits_to_float((uint16_t)(ent[c] >> 16)), acc1);
    }
    out[0] = float_to_half_bits(acc0);
    out[1] = float_to_half_bits(acc1);
    return;
  }
  for (uint32_t c = 0; c < 8; ++c) {
    const uint32_t bx = c & 1u, by = (c >> 1) & 1u, bz = (c >> 2) & 1u;
    const float w = (bx ? tx : 1.f - tx) * (by ? ty : 1.f - ty) * (bz ? tz : 1.f - tz);
    const uint16_t *f = e.table + ((size_t)l * T + index(gx + bx, gy + by, gz + bz)) * e.n_features;
    acc0 = fmaf(w, half_bits_to_float(f[0]), acc0);
  }
  out[0] = float_to_half_bits(acc0);
}

// Corner table indices (within level l) and trilinear weights of one point:
// the same arithmetic as field_hashgrid_level (the backward pass scatters
// d(feature) * weight to these entries).
MTX_HD void field_level_corners(const FieldEncoding &e, V3 pn, uint32_t l, uint32_t idx[8], float w[8]) {
  const uint32_t T = 1u << e.log2_table;
  const float scale = e.level_scale[l];
  const uint32_t res = e.level_res[l];
  const bool dense = (uint64_t)res * res * res <= (uint64_t)T;
  const float px = fmaf(pn.x, scale, 0.5f), py = fmaf(pn.y, scale, 0.5f), pz = fmaf(pn.z, scale, 0.5f);
  const float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
  const float tx = px - fx, ty = py - fy, tz = pz - fz;
  const uint32_t gx = (uint32_t)(int32_t)fx, gy = (uint32_t)(int32_t)fy, gz = (uint32_t)(int32_t)fz;
  for (uint32_t c = 0; c < 8; ++c) {
    const uint32_t bx = c & 1u, by = (c >> 1) & 1u, bz = (c >> 2) & 1u;
    const uint32_t x = gx + bx, y = gy + by, z = gz + bz;
    const uint32_t i = dense ? x + y * res + z * res * res
                             : (x * kFieldPrimes[0]) ^ (y * kFieldPrimes[1]) ^ (z * kFieldPrimes[2]);
    idx[c] = i & (T - 1u);
    w[c] = (bx ? tx : 1.f - tx) * (by ? ty : 1.f - ty) * (bz ? tz : 1.f - tz);
  }
}

// All levels of one point: out[n_features * l + k].
MTX_HD void field_hashgrid(const FieldEncoding &e, V3 pn, uint16_t *out) {
  for (uint32_t l = 0; l < e.n_levels; ++l) field_hashgrid_level(e, pn, l, out + e.n_features * l);
}

// Real spherical harmonics, degrees 0..3 (16 coefficients, index l*(l+1)+m).
MTX_HD void field_sh3(V3 d, float *r) {
  const float x = d.x, y = d.y, z = d.z, z2 = z * z;
  r[0] = 0.28209479177387814f;
  r[2] = z * 0.488602511902919923f;
  r[6] = fmaf(z2, 0.94617469575756008f, -0.315391565252520045f);
  r[12] = z * fmaf(z2, 1.865881662950577f, -1.1195289977703462f);
  float c0 = x, s0 = y;
  float ta = -0.488602511902919978f;
  r[3] = ta * c0;
  r[1] = ta * s0;
  float tb = z * -1.09254843059207896f;
  r[7] = tb * c0;
  r[5] = tb * s0;
  float tc = fmaf(z2, -2.28522899732232876f, 0.457045799464465774f);
  r[13] = tc * c0;
  r[11] = tc * s0;
  float c1 = fmaf(x, c0, -(y * s0)), s1 = fmaf(x, s0, y * c0);
  ta = 0.546274215296039478f;
  r[8] = ta * c1;
  r[4] = ta * s1;
  tb = z * 1.44530572132027735f;
  r[14] = tb * c1;
  r[10] = tb * s1;
  c0 = fmaf(x, c1, -(y * s1));
  s0 = fmaf(x, s1, y * c1);
  tc = -0.590043589926643519f;
  r[15] = tc * c0;
  r[9] = tc * s0;
}

MTX_HD V3 field_pnorm(const FieldEncoding &e, V3 p) {
  return V3{(p.x - e.bbox_min[0]) / (e.bbox_max[0] - e.bbox_min[0]),
            (p.y - e.bbox_min[1]) / (e.bbox_max[1] - e.bbox_min[1]),
            (p.z - e.bbox_min[2]) / (e.bbox_max[2] - e.bbox_min[2])};
}

// Everything of the feature row except the hash-grid block: p_norm(3) at
// 0..2, wi(3) and sh(16) after the L*F grid features, zeros up to n_pad.
// Returns the number of real features.
MTX_HD uint32_t field_features_direct(const FieldEncoding &e, V3 pn, V3 wi, uint16_t *out, uint32_t n_pad) {
  float sh[16];
  field_sh3(wi, sh);
  out[0] = float_to_half_bits(pn.x);
  out[1] = float_to_half_bits(pn.y);
  out[2] = float_to_half_bits(pn.z);
  uint32_t k = 3 + e.n_levels * e.n_features;
  out[k++] = float_to_half_bits(wi.x);
  out[k++] = float_to_half_bits(wi.y);
  out[k++] = float_to_half_bits(wi.z);
  for (int i = 0; i < 16; ++i) out[k++] = float_to_half_bits(sh[i]);
  const uint32_t n = k;
  while (k < n_pad) out[k++] = 0;
  return n;
}

// Feature vector (fp16 bits) of one query: p_norm(3), p_enc(L*F), wi(3),
// sh(16), zero padding up to n_pad. Returns the number of real features.
MTX_HD uint32_t field_features(const FieldEncoding &e, V3 p, V3 wi, uint16_t *out, uint32_t n_pad) {
  const V3 pn = field_pnorm(e, p);
  field_hashgrid(e, pn, out + 3);
  return field_features_direct(e, pn, wi, out, n_pad);
}

}  // namespace mtx
