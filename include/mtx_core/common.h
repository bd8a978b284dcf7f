// mtx_core/common.h — scalar/vector arithmetic shared by the HIP kernels and
// the CPU restatement.
//
// These headers restate the *upstream* (Mitsuba 3 / Dr.Jit) per-lane
// primitives that the reference scripts call.
// They are compiled twice: by hipcc for gfx950 device code and by g++ for the
// host (BVH/material precompute and the oracle in oracle/). Both builds use
// -ffp-contract=off and no fast-math, and every fused multiply-add is written
// out explicitly, so a given sequence of operations rounds identically on the
// CPU and on the GPU. The Dr.Jit conventions followed here (upstream,
// unverifiable offline) are:
//   dot(a,b)   = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
//   cross(a,b) = (fmsub(a.y,b.z,a.z*b.y), fmsub(a.z,b.x,a.x*b.z), fmsub(a.x,b.y,a.y*b.x))
//   normalize(v) = v * rsqrt(dot(v,v)),  rsqrt(x) = 1/sqrt(x)  (LLVM backend)
//   mulsign(a,b) = a with b's sign bit xor-ed in
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define MTX_HD __host__ __device__ __forceinline__
#define MTX_DEVICE_COMPILE 1
#else
#define MTX_HD inline
#endif

namespace mtx {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInvTwoPi = 0.15915494309189533577f;
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kFourPi = 12.56637061435917295384f;
constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kInf = __builtin_huge_valf();
// math::RayEpsilon<float> = Epsilon*1500 with Epsilon = 2^-24 (Appendix A)
constexpr float kRayEpsilon = 1500.f * 5.9604644775390625e-8f;
constexpr float kShadowEpsilon = kRayEpsilon * 10.f;
constexpr float kLargest = 3.40282346638528859812e+38f;

MTX_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
MTX_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
MTX_HD int popc32(uint32_t x) { return __builtin_popcount(x); }
MTX_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }  // x != 0

MTX_HD float mulsign(float a, float b) { return u2f(f2u(a) ^ (f2u(b) & 0x80000000u)); }
MTX_HD float mulsign_neg(float a, float b) {
  return u2f(f2u(a) ^ ((~f2u(b)) & 0x80000000u));
}
MTX_HD float sqr(float x) { return x * x; }
MTX_HD float safe_sqrt(float x) { return sqrtf(fmaxf(x, 0.f)); }
MTX_HD float rsqrt_(float x) { return 1.f / sqrtf(x); }
MTX_HD float rcp(float x) { return 1.f / x; }
MTX_HD float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
MTX_HD bool isfinite_(float x) { return (f2u(x) & 0x7f800000u) != 0x7f800000u; }
MTX_HD float lerp(float a, float b, float t) { return fmaf(b, t, fmaf(-a, t, a)); }

struct V2 {
  float x, y;
};
struct V3 {
  float x, y, z;
};

MTX_HD V2 v2(float x, float y) { return V2{x, y}; }
MTX_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
MTX_HD V3 v3s(float s) { return V3{s, s, s}; }
MTX_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MTX_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MTX_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
MTX_HD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MTX_HD V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
MTX_HD V3 operator*(float s, V3 a) { return V3{a.x * s, a.y * s, a.z * s}; }
MTX_HD V3 operator/(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
MTX_HD V3 operator/(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
MTX_HD V3 fma3(V3 a, float b, V3 c) { return V3{fmaf(a.x, b, c.x), fmaf(a.y, b, c.y), fmaf(a.z, b, c.z)}; }
MTX_HD V3 fma3v(V3 a, V3 b, V3 c) { return V3{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z)}; }
MTX_HD float dot(V3 a, V3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
MTX_HD float absdot(V3 a, V3 b) { return fabsf(dot(a, b)); }
MTX_HD V3 cross(V3 a, V3 b) {
  return V3{fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x))};
}
MTX_HD float squared_norm(V3 a) { return dot(a, a); }
MTX_HD float norm(V3 a) { return sqrtf(squared_norm(a)); }
MTX_HD V3 normalize(V3 a) { return a * rsqrt_(squared_norm(a)); }
MTX_HD float hmax(V3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
MTX_HD V3 vabs(V3 a) { return V3{fabsf(a.x), fabsf(a.y), fabsf(a.z)}; }
MTX_HD V3 mulsign3(V3 a, float s) { return V3{mulsign(a.x, s), mulsign(a.y, s), mulsign(a.z, s)}; }
MTX_HD bool all_zero(V3 a) { return a.x == 0.f && a.y == 0.f && a.z == 0.f; }
MTX_HD V3 select3(bool m, V3 a, V3 b) { return m ? a : b; }

// Luminance (Mitsuba mi.luminance for linear sRGB primaries), used by PSSMLT.
MTX_HD float luminance(V3 c) {
  return fmaf(c.z, 0.072169f, fmaf(c.y, 0.715160f, c.x * 0.212671f));
}

// ---- film partial slots (GPU-count-invariant films, DESIGN.md "Film") ----
// A pixel's T = spp_total samples fall into 8 slots: slot k holds the global
// sample indices [floor(k T / 8), floor((k + 1) T / 8)) (empty when T < 8
// leaves it none). The film is the fixed binary tree of the 8 slot films, so
// ranks that each render whole slots and are combined by the top of the same
// tree give the one-device film bit for bit.
struct V4 {
  float x, y, z, w;
};
MTX_HD V4 add4(V4 a, V4 b) { return V4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
MTX_HD uint32_t film_slot_end(uint32_t k, uint32_t T) { return (uint32_t)(((uint64_t)(k + 1) * T) >> 3); }
MTX_HD uint32_t film_slot(uint32_t g, uint32_t T) {
  uint32_t k = 0;
  while (k < 7 && film_slot_end(k, T) <= g) ++k;
  return k;
}
MTX_HD V4 film_tree8(const V4 s[8]) {
  return add4(add4(add4(s[0], s[1]), add4(s[2], s[3])), add4(add4(s[4], s[5]), add4(s[6], s[7])));
}

}  // namespace mtx
