// mtx_core/dmath.h — deterministic single-precision transcendentals.
//
// Dr.Jit evaluates dr::sin/cos/log/exp/erf/erfinv with its own CEPHES-derived
// polynomial kernels on every backend (upstream drjit/math.h, unverifiable
// offline), not with the platform libm. We restate that design: every function
// below is a fixed sequence of IEEE +,-,*,/,fma,sqrt and bit operations, so it
// returns the same bits on gfx950 and on x86-64. The coefficients are the
// public CEPHES single-precision sets (sinf/cosf, logf, expf), W. J. Cody's
// erfc rational form via Numerical Recipes' Chebyshev fit, and M. Giles'
// single-precision erfinv (2010).
#pragma once
#include "common.h"

namespace mtx {

// Joint sine/cosine, CEPHES sinf/cosf kernels with a 3-part Cody-Waite
// reduction by pi/4 (accurate for |x| < 8192).
MTX_HD void dsincos(float x, float *s_out, float *c_out) {
  float xa = fabsf(x);
  int32_t j = (int32_t)(xa * 1.27323954473516268615f);  // 4/pi
  j = (j + 1) & ~1;
  float y = (float)j;
  uint32_t sign_sin = ((uint32_t)j << 29) ^ f2u(x);
  uint32_t sign_cos = ((uint32_t)(~(j - 2))) << 29;
  y = fmaf(y, -0.78515625f, xa);
  float yy = (float)j;
  y = fmaf(yy, -2.4187564849853515625e-4f, y);
  y = fmaf(yy, -3.77489497744594108e-8f, y);
  float z = y * y;
  float s = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z;
  float c = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f) * z;
  s = fmaf(s, y, y);
  c = fmaf(c, z, fmaf(z, -0.5f, 1.f));
  bool poly = (j & 2) == 0;
  float rs = poly ? s : c;
  float rc = poly ? c : s;
  *s_out = u2f(f2u(rs) ^ (sign_sin & 0x80000000u));
  *c_out = u2f(f2u(rc) ^ (sign_cos & 0x80000000u));
}

// Natural logarithm (CEPHES logf). Returns -inf for 0, NaN for x < 0.
MTX_HD float dlog(float x) {
  if (!(x > 0.f)) return x == 0.f ? -kInf : u2f(0x7fc00000u);
  if (!isfinite_(x)) return x;
  uint32_t bits = f2u(x);
  int32_t e;
  if (bits < 0x00800000u) {  // subnormal: renormalise
    x = x * 8388608.f;       // 2^23
    bits = f2u(x);
    e = (int32_t)(bits >> 23) - 126 - 23;
  } else {
    e = (int32_t)(bits >> 23) - 126;
  }
  float m = u2f((bits & 0x007fffffu) | 0x3f000000u);  // m in [0.5, 1)
  if (m < 0.70710678118654752440f) {
    e -= 1;
    m = m + m - 1.f;
  } else {
    m = m - 1.f;
  }
  float z = m * m;
  float y = 7.0376836292e-2f;
  y = fmaf(y, m, -1.1514610310e-1f);
  y = fmaf(y, m, 1.1676998740e-1f);
  y = fmaf(y, m, -1.2420140846e-1f);
  y = fmaf(y, m, 1.4249322787e-1f);
  y = fmaf(y, m, -1.6668057665e-1f);
  y = fmaf(y, m, 2.0000714765e-1f);
  y = fmaf(y, m, -2.4999993993e-1f);
  y = fmaf(y, m, 3.3333331174e-1f);
  y = y * m * z;
  float fe = (float)e;
  y = fmaf(fe, -2.12194440e-4f, y);
  y = fmaf(z, -0.5f, y);
  float r = m + y;
  r = fmaf(fe, 0.693359375f, r);
  return r;
}

// exp(x), CEPHES expf with a two-part ln2 reduction.
MTX_HD float dexp(float x) {
  if (x != x) return x;
  if (x > 88.7228390f) return kInf;
  if (x < -103.972084f) return 0.f;
  float fx = floorf(fmaf(x, 1.44269504088896341f, 0.5f));
  x = fmaf(fx, -0.693359375f, x);
  x = fmaf(fx, 2.12194440e-4f, x);
  float z = x * x;
  float y = 1.9875691500e-4f;
  y = fmaf(y, x, 1.3981999507e-3f);
  y = fmaf(y, x, 8.3334519073e-3f);
  y = fmaf(y, x, 4.1665795894e-2f);
  y = fmaf(y, x, 1.6666665459e-1f);
  y = fmaf(y, x, 5.0000001201e-1f);
  y = fmaf(y, z, x) + 1.f;
  int32_t n = (int32_t)fx;
  // scale by 2^n in two steps so that subnormal results are reachable
  int32_t n1 = n / 2, n2 = n - n1;
  y = y * u2f((uint32_t)(n1 + 127) << 23);
  y = y * u2f((uint32_t)(n2 + 127) << 23);
  return y;
}

// erfc(x) for x >= 0 (Chebyshev fit, fractional error < 1.2e-7 in exact
// arithmetic), erf(x) = sign(x) * (1 - erfc(|x|)).
MTX_HD float derf(float x) {
  float z = fabsf(x);
  float t = 1.f / fmaf(0.5f, z, 1.f);
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  float erfc = t * dexp(fmaf(-z, z, p));
  float r = 1.f - erfc;
  return mulsign(r, x);
}

// Inverse error function (M. Giles, "Approximating the erfinv function",
// GPU Computing Gems, 2010; single-precision branch set).
MTX_HD float derfinv(float x) {
  float w = -dlog(fmaf(-x, x, 1.f));
  float p;
  if (w < 5.f) {
    w = w - 2.5f;
    p = 2.81022636e-08f;
    p = fmaf(p, w, 3.43273939e-07f);
    p = fmaf(p, w, -3.5233877e-06f);
    p = fmaf(p, w, -4.39150654e-06f);
    p = fmaf(p, w, 0.00021858087f);
    p = fmaf(p, w, -0.00125372503f);
    p = fmaf(p, w, -0.00417768164f);
    p = fmaf(p, w, 0.246640727f);
    p = fmaf(p, w, 1.50140941f);
  } else {
    w = sqrtf(w) - 3.f;
    p = -0.000200214257f;
    p = fmaf(p, w, 0.000100950558f);
    p = fmaf(p, w, 0.00134934322f);
    p = fmaf(p, w, -0.00367342844f);
    p = fmaf(p, w, 0.00573950773f);
    p = fmaf(p, w, -0.0076224613f);
    p = fmaf(p, w, 0.00943887047f);
    p = fmaf(p, w, 1.00167406f);
    p = fmaf(p, w, 2.83297682f);
  }
  return p * x;
}

}  // namespace mtx
