// mtx_core/rng.h — Dr.Jit PCG32 + TEA seeding.
//
// The reference never implements its RNG: every `sampler.next_1d/next_2d`
// (e.g. path-mis.py:97,104-105,147) draws from Mitsuba's IndependentSampler,
// a per-lane Dr.Jit PCG32 whose stream is seeded by `sample_tea_32` (the
// seeding is mirrored in-repo at pssmlt.py:84-93). Restated here:
//   seed(initstate, initseq): state = 0; inc = (initseq << 1) | 1; next();
//                             state += initstate; next()
//   next_u32: old = state; state = old*0x5851f42d4c957f2d + inc;
//             xs = u32(((old >> 18) ^ old) >> 27); rot = u32(old >> 59);
//             return (xs >> rot) | (xs << ((-rot) & 31))
//   next_f32 = bitcast((u >> 9) | 0x3f800000) - 1
// Lane seeding (IndependentSampler::seed, upstream): (v0, v1) =
// sample_tea_32(seed, lane); pcg.seed(v0, v1). The in-repo MLTSampler
// (pssmlt.py:92) passes (lane, seed) instead; mtx fixes the upstream order for
// every integrator and documents it in DESIGN.md.
#pragma once
#include "common.h"

namespace mtx {

constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;

MTX_HD void sample_tea_32(uint32_t v0, uint32_t v1, uint32_t *o0, uint32_t *o1, int rounds = 4) {
  uint32_t sum = 0;
  for (int i = 0; i < rounds; ++i) {
    sum += 0x9e3779b9u;
    v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
    v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
  }
  *o0 = v0;
  *o1 = v1;
}

// PCG32 lane state. `inc` is always (u64(seq) << 1) | 1 for a 32-bit
// sequence id, so only the 32-bit `seq` is stored (12 B of state per lane).
struct Pcg32 {
  uint64_t state;
  uint32_t seq;

  MTX_HD uint64_t inc() const { return ((uint64_t)seq << 1) | 1ULL; }
  MTX_HD uint32_t next_u32() {
    uint64_t old = state;
    state = old * kPcgMult + inc();
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
  }
  MTX_HD float next_1d() { return u2f((next_u32() >> 9) | 0x3f800000u) - 1.f; }
  MTX_HD V2 next_2d() {
    float x = next_1d();
    float y = next_1d();
    return V2{x, y};
  }
  // Advance by `delta` steps in O(log delta) (PCG "advance", Brown 1994).
  MTX_HD void advance(uint64_t delta) {
    uint64_t cur_mult = kPcgMult, cur_plus = inc(), acc_mult = 1, acc_plus = 0;
    while (delta > 0) {
      if (delta & 1) {
        acc_mult *= cur_mult;
        acc_plus = acc_plus * cur_mult + cur_plus;
      }
      cur_plus = (cur_mult + 1) * cur_plus;
      cur_mult *= cur_mult;
      delta >>= 1;
    }
    state = acc_mult * state + acc_plus;
  }
};

MTX_HD Pcg32 pcg32_seed(uint64_t initstate, uint32_t initseq) {
  Pcg32 r;
  r.state = 0;
  r.seq = initseq;
  r.next_u32();
  r.state += initstate;
  r.next_u32();
  return r;
}

// IndependentSampler lane stream: TEA-scrambled (seed, lane) -> PCG32.
MTX_HD Pcg32 sampler_lane(uint32_t seed, uint32_t lane) {
  uint32_t v0, v1;
  sample_tea_32(seed, lane, &v0, &v1);
  return pcg32_seed((uint64_t)v0, v1);
}

}  // namespace mtx
