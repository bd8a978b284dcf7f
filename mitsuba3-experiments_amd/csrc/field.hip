// field.hip — fp16 radiance-field inference on the gfx950 matrix cores
// (nerad.py:54-106 Field: hash-grid + SH encoding, then a 64-wide MLP with
// LeakyReLU, no bias; SURVEY §8f item 3, the cache NRC queries).
//
// k_field_encode  one thread per query: mtx_core/field.h features -> fp16 row
//                 of 64 (p_norm, hash-grid, wi, SH, zero padding)
// k_field_mlp     one wave per 64 queries (two 32-query N-tiles), all layers
//                 fused: activations stay in registers between layers. Every
//                 layer is  Y[64 x 32q] = W[64 x 64] * X[64 x 32q]  with
//                 v_mfma_f32_32x32x16_f16 (A = weights from LDS, B = the
//                 previous accumulator converted to fp16). The accumulator's
//                 rows (output features) sit in registers, so it is the next
//                 layer's B operand with no lane movement; the host prepacks
//                 each weight fragment in that permuted k order
//                 (cdna_hip_programming.md §3, "accumulator tile as the next
//                 MFMA's operand"). f32 accumulation, fp16 activations:
//                 each accumulator pair is rounded with v_cvt_pk_f16_f32 and
//                 LeakyReLU runs packed in fp16 (v_pk_mul_f16 + v_pk_max_f16);
//                 MFMA results stay in VGPRs (-amdgpu-mfma-vgpr-form), so a
//                 layer costs 16 MFMAs + 48 VALU per wave (MFMA-bound).
#include <hip/hip_runtime.h>

#include "mtx.h"
#include "mtx_core/field.h"
#include "prims.h"

void mtx_set_error(const char *fmt, ...);

namespace mtxd {

using namespace mtx;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kFieldPad = 64;     // features per query (padded)
constexpr float kLeakySlope = 0.01f;  // drjit.nn.LeakyReLU default

// One thread per (query, level): the 8 corner gathers of a level are
// independent of the other levels, so a block covers 256 / n_levels queries
// with every thread issuing its own gathers. The rows are assembled in LDS
// and written out as 16-B stores (one 128-B row = 8 lanes).
constexpr uint32_t kEncodeBlock = 256;

// xcd_split (rows grouped by region, k_cache_bucket_*): the blocks that
// share an XCD (equal blockIdx % 8 under the observed round-robin placement,
// MI355X_MICROARCH.md "Workgroup dispatch") take one contiguous eighth of the
// rows, i.e. one eighth of the space, so each XCD's 4 MiB L2 holds the table
// entries of its own region instead of all of them. Speed only: any
// placement gives the same rows.
__global__ __launch_bounds__(kEncodeBlock) void k_field_encode(FieldEncoding e, const float4 *qp, const float4 *qd,
                                                               const uint32_t *count, uint32_t n_max,
                                                               uint16_t *feat, const uint32_t *perm, int xcd_split) {
  extern __shared__ uint4 rows[];  // 256 / n_levels rows of 128 B
  const uint32_t n = count ? min(*count, n_max) : n_max;
  const uint32_t L = e.n_levels, qpb = kEncodeBlock / L;
  uint16_t *row_h = reinterpret_cast<uint16_t *>(rows);
  const uint32_t ql = threadIdx.x / L, l = threadIdx.x - ql * L;
  uint32_t lo = 0, hi = n, first = blockIdx.x, stride = gridDim.x;
  if (xcd_split) {
    const uint32_t g = blockIdx.x & 7u;
    lo = (uint32_t)(((uint64_t)n * g) >> 3);
    hi = (uint32_t)(((uint64_t)n * (g + 1)) >> 3);
    first = blockIdx.x >> 3;
    stride = gridDim.x >> 3;
  }
  for (uint32_t q0 = lo + first * qpb; q0 < hi; q0 += stride * qpb) {
    const uint32_t q = q0 + ql;
    if (ql < qpb && q < hi) {
      const uint32_t qs = perm ? perm[q] : q;  // Morton-ordered rows: neighbouring threads share table lines
      const float4 p = qp[qs];
      const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
      uint16_t *row = row_h + (size_t)kFieldPad * ql;
      field_hashgrid_level(e, pn, l, row + 3 + e.n_features * l);
      if (l == 0) {
        const float4 d = qd[qs];
        field_features_direct(e, pn, V3{d.x, d.y, d.z}, row, kFieldPad);
      }
    }
    __syncthreads();
    const uint32_t nq = min(qpb, hi - q0);
    for (uint32_t c = threadIdx.x; c < nq * (kFieldPad / 8); c += kEncodeBlock)
      reinterpret_cast<uint4 *>(feat + (size_t)kFieldPad * q0)[c] = rows[c];
    __syncthreads();
  }
}

// Level-major encoder (round 5): a block takes 64 queries; 64 threads first
// compute each query's p_norm (once, not once per level) and its direct
// features (p_norm, wi, SH, padding), then the block's 256 threads walk the
// 64 x n_levels (query, level) items with the query fastest, so the 64 lanes
// of a wave gather from ONE level's table at 64 queries: with the rows
// grouped by region (MTX_CACHE_SORT=2) the coarse levels' corners of nearby
// queries share lines (the TA prices a gather by the distinct lines it
// touches), where the query-major mapping above spreads a wave over 16
// tables. Same arithmetic per feature: the same rows.
constexpr uint32_t kEncQ = 64;
__global__ __launch_bounds__(256) void k_field_encode_lm(FieldEncoding e, const float4 *qp, const float4 *qd,
                                                         const uint32_t *count, uint32_t n_max, uint16_t *feat,
                                                         const uint32_t *perm, int xcd_split) {
  __shared__ uint4 rows[kEncQ * kFieldPad / 8];
  __shared__ float4 pn_s[kEncQ];
  uint16_t *row_h = reinterpret_cast<uint16_t *>(rows);
  const uint32_t n = count ? min(*count, n_max) : n_max;
  const uint32_t L = e.n_levels, F = e.n_features;
  uint32_t lo = 0, hi = n, first = blockIdx.x, stride = gridDim.x;
  if (xcd_split) {
    const uint32_t g = blockIdx.x & 7u;
    lo = (uint32_t)(((uint64_t)n * g) >> 3);
    hi = (uint32_t)(((uint64_t)n * (g + 1)) >> 3);
    first = blockIdx.x >> 3;
    stride = gridDim.x >> 3;
  }
  for (uint32_t q0 = lo + first * kEncQ; q0 < hi; q0 += stride * kEncQ) {
    const uint32_t nq = min(kEncQ, hi - q0);
    if (threadIdx.x < nq) {
      const uint32_t qs = perm ? perm[q0 + threadIdx.x] : q0 + threadIdx.x;
      const float4 p = qp[qs], d = qd[qs];
      const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
      pn_s[threadIdx.x] = make_float4(pn.x, pn.y, pn.z, 0.f);
      field_features_direct(e, pn, V3{d.x, d.y, d.z}, row_h + (size_t)kFieldPad * threadIdx.x, kFieldPad);
    }
    __syncthreads();
    const uint32_t items = kEncQ * L;
#pragma unroll 4
    for (uint32_t it = threadIdx.x; it < items; it += 256) {
      const uint32_t q = it & (kEncQ - 1u), l = it / kEncQ;
      if (q < nq) {
        const float4 pn = pn_s[q];
        field_hashgrid_level(e, V3{pn.x, pn.y, pn.z}, l, row_h + (size_t)kFieldPad * q + 3 + F * l);
      }
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < nq * (kFieldPad / 8); c += 256)
      reinterpret_cast<uint4 *>(feat + (size_t)kFieldPad * q0)[c] = rows[c];
    __syncthreads();
  }
}

typedef _Float16 half2v __attribute__((ext_vector_type(2)));

// Accumulator -> next layer's B operand: round to fp16, then LeakyReLU in
// fp16 as max(h, h * 0.01) (the activation of a Float16 network; packed
// v_cvt_pk_f16_f32 / v_pk_mul_f16 / v_pk_max_f16, 1.5 VALU per element).
__device__ __forceinline__ half8 leaky_pack(const f32x16 &acc, int s) {
  half8 r;
  const half2v slope = {(_Float16)kLeakySlope, (_Float16)kLeakySlope};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    half2v h = {(_Float16)acc[8 * s + 2 * j], (_Float16)acc[8 * s + 2 * j + 1]};
    h = __builtin_elementwise_max(h, h * slope);
    r[2 * j] = h.x;
    r[2 * j + 1] = h.y;
  }
  return r;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// wfrag: prepacked fragments [frag][64 lanes] (see field_prepack); n_hidden
// hidden 64x64 layers after the input layer; out: 3 floats per query
// (fp16-rounded, the reference's Float16 network output cast to Color3f).
__global__ __launch_bounds__(256) void k_field_mlp(const uint16_t *feat, const uint32_t *count, uint32_t n_max,
                                                   const half8 *wfrag, uint32_t n_frag, uint32_t n_hidden,
                                                   float *out) {
  extern __shared__ half8 w[];
  for (uint32_t i = threadIdx.x; i < n_frag * 64; i += blockDim.x) w[i] = wfrag[i];
  __syncthreads();
  const uint32_t n = count ? min(*count, n_max) : n_max;
  const uint32_t lane = threadIdx.x & 63, h = lane >> 5, col = lane & 31;
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint32_t wave = blockIdx.x * waves_per_block + (threadIdx.x >> 6);
  const uint32_t n_waves = gridDim.x * waves_per_block;
  // input-layer B fragments of a tile (natural k order), zero past n
  auto load_in = [&](uint32_t tile, half8 (&b)[2][4]) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const uint32_t q = tile * 64 + nt * 32 + col;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (q < n) {
          b[nt][ks] = *reinterpret_cast<const half8 *>(feat + (size_t)kFieldPad * q + ks * 16 + h * 8);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) b[nt][ks][j] = (_Float16)0.f;
        }
      }
    }
  };
  half8 bin[2][4];
  if (wave * 64 < n) load_in(wave, bin);
  for (uint32_t tile = wave; tile * 64 < n; tile += n_waves) {
    const uint32_t q0 = tile * 64;
    f32x16 acc[2][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const half8 a = w[(mt * 4 + ks) * 64 + lane];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bin[nt][ks], ks == 0 ? zero16() : acc[mt][nt], 0, 0,
                                                                0);
      }
    uint32_t base = 8;
    for (uint32_t layer = 0; layer < n_hidden; ++layer, base += 8) {
      half8 bf[2][4];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int s = 0; s < 2; ++s) bf[nt][2 * mt + s] = leaky_pack(acc[mt][nt], s);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const half8 a = w[(base + mt * 4 + ks) * 64 + lane];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bf[nt][ks], ks == 0 ? zero16() : acc[mt][nt], 0,
                                                                  0, 0);
        }
    }
    // output layer (3 rows of one 32-row M tile)
    half8 bf[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) bf[nt][2 * mt + s] = leaky_pack(acc[mt][nt], s);
    f32x16 o[2] = {zero16(), zero16()};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const half8 a = w[(base + ks) * 64 + lane];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) o[nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bf[nt][ks], o[nt], 0, 0, 0);
    }
    // C/D rows 0..2 = registers 0..2 of the lanes with h = 0
    if (h == 0) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint32_t q = q0 + nt * 32 + col;
        if (q < n) {
#pragma unroll
          for (int c = 0; c < 3; ++c) out[3 * (size_t)q + c] = (float)(_Float16)o[nt][c];
        }
      }
    }
    // (loading the next tile's features at the top of the tile instead took
    // 180 VGPRs, 2 waves/SIMD: slower)
    if ((tile + n_waves) * 64 < n) load_in(tile + n_waves, bin);
  }
}

// ---- the NRC cache pass fused: encode + MLP + apply (round 5) -----------
// One block of 512 threads (8 waves) takes 256 cache queries at a time:
// their feature rows are assembled in LDS (level-major lanes as in
// k_field_encode_lm), each wave runs the fused MLP of k_field_mlp on 32 of
// them (one 32-query N-tile) straight from LDS, and the lanes holding the
// outputs add T * out to the path's L (k_cache_apply). The 128 B of features
// and 12 B of outputs per query no longer go through HBM, and two launches
// go. Every query's features, MLP column and L update are those of the
// three-kernel path (MFMA output columns do not depend on their tile), so
// the films are the same bits.
constexpr uint32_t kFusedQ = 256;
__global__ __launch_bounds__(512) void k_field_cache_fused(FieldEncoding e, const float4 *qp, const float4 *qd,
                                                           const float4 *qt, const uint32_t *count, uint32_t n_max,
                                                           const uint32_t *perm, int xcd_split, const half8 *wfrag,
                                                           uint32_t n_frag, uint32_t n_hidden, float4 *L_final) {
  extern __shared__ half8 fused_lds[];
  half8 *w = fused_lds;                                                // n_frag x 64 fragments
  uint16_t *row_h = reinterpret_cast<uint16_t *>(w + n_frag * 64);     // kFusedQ rows of 64 halfs
  float4 *pn_s = reinterpret_cast<float4 *>(row_h + kFusedQ * kFieldPad);
  for (uint32_t i = threadIdx.x; i < n_frag * 64; i += blockDim.x) w[i] = wfrag[i];
  const uint32_t n = count ? min(*count, n_max) : n_max;
  const uint32_t L = e.n_levels, F = e.n_features;
  uint32_t lo = 0, hi = n, first = blockIdx.x, stride = gridDim.x;
  if (xcd_split) {
    const uint32_t g = blockIdx.x & 7u;
    lo = (uint32_t)(((uint64_t)n * g) >> 3);
    hi = (uint32_t)(((uint64_t)n * (g + 1)) >> 3);
    first = blockIdx.x >> 3;
    stride = gridDim.x >> 3;
  }
  const uint32_t lane = threadIdx.x & 63u, h = lane >> 5, col = lane & 31u, wave = threadIdx.x >> 6;
  __syncthreads();
  for (uint32_t q0 = lo + first * kFusedQ; q0 < hi; q0 += stride * kFusedQ) {
    const uint32_t nq = min(kFusedQ, hi - q0);
    // ---- encode: direct features per query, then the (query, level) items
    if (threadIdx.x < kFusedQ) {
      uint16_t *row = row_h + (size_t)kFieldPad * threadIdx.x;
      if (threadIdx.x < nq) {
        const uint32_t qs = perm ? perm[q0 + threadIdx.x] : q0 + threadIdx.x;
        const float4 p = qp[qs], d = qd[qs];
        const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
        pn_s[threadIdx.x] = make_float4(pn.x, pn.y, pn.z, 0.f);
        field_features_direct(e, pn, V3{d.x, d.y, d.z}, row, kFieldPad);
      } else {
        for (uint32_t k = 0; k < kFieldPad; ++k) row[k] = 0;  // rows past n: zero MLP inputs
      }
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t it = threadIdx.x; it < kFusedQ * L; it += 512) {
      const uint32_t q = it & (kFusedQ - 1u), l = it / kFusedQ;
      if (q < nq) {
        const float4 pn = pn_s[q];
        field_hashgrid_level(e, V3{pn.x, pn.y, pn.z}, l, row_h + (size_t)kFieldPad * q + 3 + F * l);
      }
    }
    __syncthreads();
    // ---- MLP: wave w on rows [32w, 32w + 32) (k_field_mlp with one N-tile)
    if (wave * 32 < nq) {
      const uint16_t *rb = row_h + (size_t)kFieldPad * (wave * 32 + col);
      half8 bin[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) bin[ks] = *reinterpret_cast<const half8 *>(rb + ks * 16 + h * 8);
      f32x16 acc[2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[(mt * 4 + ks) * 64 + lane], bin[ks],
                                                           ks == 0 ? zero16() : acc[mt], 0, 0, 0);
      uint32_t base = 8;
      for (uint32_t layer = 0; layer < n_hidden; ++layer, base += 8) {
        half8 bf[4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int sgl = 0; sgl < 2; ++sgl) bf[2 * mt + sgl] = leaky_pack(acc[mt], sgl);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[(base + mt * 4 + ks) * 64 + lane], bf[ks],
                                                             ks == 0 ? zero16() : acc[mt], 0, 0, 0);
      }
      half8 bf[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int sgl = 0; sgl < 2; ++sgl) bf[2 * mt + sgl] = leaky_pack(acc[mt], sgl);
      f32x16 o = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) o = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[(base + ks) * 64 + lane], bf[ks], o, 0, 0, 0);
      // ---- apply (k_cache_apply): C/D rows 0..2 in registers 0..2 of h = 0
      const uint32_t q = wave * 32 + col;
      if (h == 0 && q < nq) {
        const uint32_t qs = perm ? perm[q0 + q] : q0 + q;
        const float4 t = qt[qs];
        const uint32_t path = __float_as_uint(t.w);
        float4 Lp = L_final[path];
        Lp.x = Lp.x + t.x * (float)(_Float16)o[0];
        Lp.y = Lp.y + t.y * (float)(_Float16)o[1];
        Lp.z = Lp.z + t.z * (float)(_Float16)o[2];
        L_final[path] = Lp;
      }
    }
    __syncthreads();
  }
}

int field_cache_fused(const FieldEncoding &e, const float4 *qp, const float4 *qd, const float4 *qt,
                      const uint32_t *count, uint32_t n_max, const uint32_t *perm, int xcd_split, const void *wfrag,
                      uint32_t n_hidden, float4 *L_final, int n_cu, hipStream_t st) {
  if (n_max == 0) return MTX_OK;
  if (e.n_levels == 0 || e.n_levels > kFieldMaxLevels) {
    mtx_set_error("field_cache_fused: unsupported n_levels %u", e.n_levels);
    return MTX_E_ARG;
  }
  const uint32_t n_frag = field_frag_count(n_hidden);
  const size_t lds = field_cache_fused_lds(n_hidden);
  unsigned blocks = (unsigned)std::max<uint64_t>(
      1, std::min<uint64_t>((n_max + kFusedQ - 1) / kFusedQ, (uint64_t)n_cu * 2));
  if (xcd_split) blocks = (blocks + 7u) & ~7u;
  hipLaunchKernelGGL(k_field_cache_fused, dim3(blocks), dim3(512), lds, st, e, qp, qd, qt, count, n_max, perm,
                     xcd_split, (const half8 *)wfrag, n_frag, n_hidden, L_final);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    mtx_set_error("field_cache_fused: launch failed (%zu B of LDS): %s", lds, hipGetErrorString(err));
    return MTX_E_HIP;
  }
  return MTX_OK;
}

uint32_t field_frag_count(uint32_t n_hidden) { return 8 * (1 + n_hidden) + 4; }

// Dynamic LDS of k_field_cache_fused: the prepacked weight fragments + the
// block's 256 feature rows + their T / path records (n_hidden 15 / 16 need
// more than the 160 KB a workgroup may hold: run_cache then takes the
// three-kernel path).
size_t field_cache_fused_lds(uint32_t n_hidden) {
  return (size_t)field_frag_count(n_hidden) * 64 * sizeof(half8) + (size_t)kFusedQ * kFieldPad * 2 +
         kFusedQ * sizeof(float4);
}

// Host: weight matrices (fp16 bits, W[out][in] row-major per layer: input
// n_in -> 64, n_hidden x 64 -> 64, 64 -> 3) -> MFMA A fragments.
void field_prepack(const uint16_t *weights, uint32_t n_in, uint32_t n_hidden, uint16_t *frag) {
  const uint32_t n_layers = n_hidden + 2;
  size_t woff = 0;
  uint32_t f = 0;
  for (uint32_t l = 0; l < n_layers; ++l) {
    const uint32_t in = l == 0 ? n_in : 64, out = l == n_layers - 1 ? 3 : 64;
    const uint32_t n_mt = l == n_layers - 1 ? 1 : 2;
    for (uint32_t mt = 0; mt < n_mt; ++mt)
      for (uint32_t ks = 0; ks < 4; ++ks, ++f)
        for (uint32_t lane = 0; lane < 64; ++lane)
          for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t row = 32 * mt + (lane & 31), h = lane >> 5;
            const uint32_t k = l == 0 ? 16 * ks + 8 * h + j
                                      : 32 * (ks >> 1) + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
            frag[((size_t)f * 64 + lane) * 8 + j] = (row < out && k < in) ? weights[woff + (size_t)row * in + k] : 0;
          }
    woff += (size_t)in * out;
  }
}

// 8-bit-per-axis Morton code of the query position in the field's box (the
// encoder's locality order: queries close in space share hash-grid lines).
__device__ __forceinline__ uint32_t morton_spread8(uint32_t x) {
  x = (x | (x << 8)) & 0x0300F00Fu;
  x = (x | (x << 4)) & 0x030C30C3u;
  x = (x | (x << 2)) & 0x09249249u;
  return x;
}
__global__ void k_morton_keys(FieldEncoding e, const float4 *qp, uint32_t n, uint32_t *keys) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const float4 p = qp[q];
  const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
  auto cell = [](float v) { return (uint32_t)fminf(fmaxf(v * 256.f, 0.f), 255.f); };
  keys[q] = morton_spread8(cell(pn.x)) | (morton_spread8(cell(pn.y)) << 1) | (morton_spread8(cell(pn.z)) << 2);
}

void field_morton_keys(const FieldEncoding &e, const float4 *qp, uint32_t n, uint32_t *keys, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_morton_keys, dim3((n + 255) / 256), dim3(256), 0, st, e, qp, n, keys);
}

// ---- region bucketing of the cache queries (no host round trip) -------
// Bucket = 3-bit-per-axis Morton cell of the query in the field's box (512
// regions); rows are grouped by bucket (order inside a bucket arbitrary: a
// row's features and MLP column depend on its query only, and each path has
// at most one query, so the film is unchanged).
#ifndef MTX_CACHE_AXIS_BITS
#define MTX_CACHE_AXIS_BITS 4  // Morton bits per axis of the cache-query regions (4: 4096; 3 and 5 measured slower)
#endif
constexpr uint32_t kCacheAxisBits = MTX_CACHE_AXIS_BITS;
constexpr uint32_t kCacheBuckets = 1u << (3 * kCacheAxisBits);
constexpr uint32_t kBucketTile = 4096;  // queries per block of the scatter

__device__ __forceinline__ uint32_t cache_bucket(const FieldEncoding &e, float4 p) {
  const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
  constexpr float kCells = (float)(1u << kCacheAxisBits);
  auto c = [](float v) { return (uint32_t)fminf(fmaxf(v * kCells, 0.f), kCells - 1.f); };
  const uint32_t x = c(pn.x), y = c(pn.y), z = c(pn.z);
  uint32_t m = 0;
#pragma unroll
  for (int b = 0; b < (int)kCacheAxisBits; ++b) m |= (((x >> b) & 1u) << (3 * b)) | (((y >> b) & 1u) << (3 * b + 1)) | (((z >> b) & 1u) << (3 * b + 2));
  return m;
}

// counts per bucket (cursor[0..511], zeroed by the caller)
__global__ __launch_bounds__(256) void k_cache_bucket_count(FieldEncoding e, const float4 *qp, const uint32_t *count,
                                                            uint32_t n_max, uint32_t *cursor) {
  __shared__ uint32_t h[kCacheBuckets];
  for (uint32_t i = threadIdx.x; i < kCacheBuckets; i += 256) h[i] = 0;
  __syncthreads();
  const uint32_t n = min(*count, n_max);
  for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256) atomicAdd(&h[cache_bucket(e, qp[q])], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kCacheBuckets; i += 256)
    if (h[i]) atomicAdd(&cursor[i], h[i]);
}

// counts -> exclusive offsets, in place (one block of 512 threads, each
// owning kCacheBuckets / 512 consecutive counts)
constexpr uint32_t kScanPer = kCacheBuckets >= 512 ? kCacheBuckets / 512 : 1;
__global__ __launch_bounds__(512) void k_cache_bucket_scan(uint32_t *cursor) {
  __shared__ uint32_t v[512];
  const uint32_t i = threadIdx.x;
  uint32_t x[kScanPer], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    const uint32_t j = i * kScanPer + k;
    x[k] = j < kCacheBuckets ? cursor[j] : 0u;
    sum += x[k];
  }
  v[i] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 512; off <<= 1) {
    const uint32_t y = i >= off ? v[i - off] : 0u;
    __syncthreads();
    v[i] += y;
    __syncthreads();
  }
  uint32_t run = v[i] - sum;
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    const uint32_t j = i * kScanPer + k;
    if (j < kCacheBuckets) cursor[j] = run;
    run += x[k];
  }
}

// perm[row] = query: per block tile, LDS counts, one reservation per
// (block, bucket), LDS cursors for the positions
__global__ __launch_bounds__(256) void k_cache_bucket_scatter(FieldEncoding e, const float4 *qp, const uint32_t *count,
                                                              uint32_t n_max, uint32_t *cursor, uint32_t *perm) {
  __shared__ uint32_t h[kCacheBuckets];
  constexpr uint32_t kPer = kBucketTile / 256;
  const uint32_t n = min(*count, n_max);
  for (uint32_t t0 = blockIdx.x * kBucketTile; t0 < n; t0 += gridDim.x * kBucketTile) {
    for (uint32_t i = threadIdx.x; i < kCacheBuckets; i += 256) h[i] = 0;
    __syncthreads();
    uint32_t bk[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      const uint32_t q = t0 + k * 256 + threadIdx.x;
      bk[k] = q < n ? cache_bucket(e, qp[q]) : 0xffffffffu;
      if (q < n) atomicAdd(&h[bk[k]], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kCacheBuckets; i += 256)
      if (h[i]) h[i] = atomicAdd(&cursor[i], h[i]);
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      if (bk[k] != 0xffffffffu) perm[atomicAdd(&h[bk[k]], 1u)] = t0 + k * 256 + threadIdx.x;
    __syncthreads();
  }
}

void field_bucket_queries(const FieldEncoding &e, const float4 *qp, const uint32_t *count, uint32_t n_max,
                          uint32_t *cursor, uint32_t *perm, int n_cu, hipStream_t st) {
  if (n_max == 0) return;
  hipMemsetAsync(cursor, 0, 4 * kCacheBuckets, st);
  const unsigned g1 = (unsigned)std::min<uint64_t>((n_max + 255) / 256, (uint64_t)n_cu * 4);
  hipLaunchKernelGGL(k_cache_bucket_count, dim3(std::max(1u, g1)), dim3(256), 0, st, e, qp, count, n_max, cursor);
  hipLaunchKernelGGL(k_cache_bucket_scan, dim3(1), dim3(512), 0, st, cursor);
  const unsigned g2 = (unsigned)std::min<uint64_t>((n_max + kBucketTile - 1) / kBucketTile, (uint64_t)n_cu * 4);
  hipLaunchKernelGGL(k_cache_bucket_scatter, dim3(std::max(1u, g2)), dim3(256), 0, st, e, qp, count, n_max, cursor,
                     perm);
}

int field_encode(const FieldEncoding &e, const float4 *qp, const float4 *qd, const uint32_t *count, uint32_t n_max,
                 uint16_t *feat, hipStream_t st, const uint32_t *perm, int xcd_split, int level_major) {
  if (n_max == 0) return MTX_OK;
  if (level_major && e.n_levels >= 1 && e.n_levels <= kFieldMaxLevels) {
    unsigned blocks = (unsigned)std::min<uint64_t>((n_max + kEncQ - 1) / kEncQ, 256ull * 32);
    if (xcd_split) blocks = (blocks + 7u) & ~7u;
    hipLaunchKernelGGL(k_field_encode_lm, dim3(blocks), dim3(256), 0, st, e, qp, qd, count, n_max, feat, perm,
                       xcd_split);
    return MTX_OK;
  }
  if (e.n_levels == 0 || e.n_levels > kEncodeBlock) {
    mtx_set_error("field_encode: unsupported n_levels %u", e.n_levels);
    return MTX_E_ARG;
  }
  const uint32_t qpb = kEncodeBlock / e.n_levels;
  unsigned blocks = (unsigned)std::min<uint64_t>((n_max + qpb - 1) / qpb, 256ull * 64);
  if (xcd_split) blocks = (blocks + 7u) & ~7u;  // whole groups of 8
  hipLaunchKernelGGL(k_field_encode, dim3(blocks), dim3(kEncodeBlock), (size_t)qpb * kFieldPad * 2, st, e, qp, qd,
                     count, n_max, feat, perm, xcd_split);
  return MTX_OK;
}

int field_mlp(const uint16_t *feat, const uint32_t *count, uint32_t n_max, const void *wfrag, uint32_t n_hidden,
              float *out, int n_cu, hipStream_t st) {
  if (n_max == 0) return MTX_OK;
  const uint32_t n_frag = field_frag_count(n_hidden);
  const size_t lds = (size_t)n_frag * 64 * sizeof(half8);
  const uint64_t tiles = (n_max + 63) / 64;
  const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((tiles + 3) / 4, (uint64_t)n_cu * 3));
  hipLaunchKernelGGL(k_field_mlp, dim3(blocks), dim3(256), lds, st, feat, count, n_max, (const half8 *)wfrag, n_frag,
                     n_hidden, out);
  return MTX_OK;
}

}  // namespace mtxd
