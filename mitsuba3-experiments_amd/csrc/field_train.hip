// field_train.hip — training of the radiance field (nerad.py:336-400):
// loss = mean((L_lhs - detach(L_rhs))^2) (:370), dr.backward(scaler.scale(
// loss)) through the fp16 MLP and the hash-grid table (:372), then
// scaler.step(opt) -- GradScaler + Adam on fp32 master copies of the table
// and the weights, re-cast to the fp16 field after the step (:389-390).
//
// k_field_train     one block per 64 training points (lane = point). The
//                   forward keeps every layer's fp16 input tile in LDS
//                   (64 rows x 64 points); the backward runs layer by layer:
//                   dY = dX(next) * LeakyReLU'(h), partial dW = dY X^T
//                   (lane = input feature), dX = W^T dY (lane = point), in
//                   fp32 (gradients of the fp16 network are not rounded).
//                   A 16 K-point batch is 0.8 GFLOP: latency-bound tiles,
//                   LDS broadcasts + FMA, no MFMA tiling needed.
// k_wgrad_reduce    per-wave partial weight gradients summed in wave order
//                   (deterministic).
// k_field_encode_bwd  d(grid features) -> table gradient: one thread per
//                   (point, level), 8 corners x trilinear weight, f32
//                   atomics (the table is 2^19 entries per level).
// k_grad_check / k_adam / k_field_prepack_dev  GradScaler's finite check,
//                   the Adam step (Dr.Jit drjit.opt.Adam form, upstream,
//                   parity unpinned) writing the fp16 table and weights, and
//                   the MFMA fragment prepack of field.hip on the device.
#include <hip/hip_runtime.h>

#include "mtx.h"
#include "mtx_core/field.h"
#include "prims.h"

void mtx_set_error(const char *fmt, ...);

namespace mtxd {

using namespace mtx;

constexpr int kTQ = 64;     // points per block (lane = point)
constexpr int kTW = 4;      // waves per block: each owns 16 of the 64 rows of a layer
constexpr int kTB = 64 * kTW;
constexpr int kXS = 66;     // fp16 row stride of the activation tiles (column reads conflict-free)
constexpr int kDS = 65;     // f32 row stride of the gradient tile
constexpr float kSlope = 0.01f;

__device__ __forceinline__ float h2f(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }

// Layer l of the network: in = n_in (l = 0) or 64, out = 64 or 3 (last).
struct TrainShape {
  uint32_t n_in, n_hidden;
  __host__ __device__ uint32_t layers() const { return n_hidden + 2; }
  __host__ __device__ uint32_t in(uint32_t l) const { return l == 0 ? n_in : 64u; }
  __host__ __device__ uint32_t out(uint32_t l) const { return l == n_hidden + 1 ? 3u : 64u; }
  __host__ __device__ uint32_t woff(uint32_t l) const { return l == 0 ? 0u : 64u * n_in + (l - 1) * 4096u; }
  __host__ __device__ uint32_t n_weights() const { return 64u * n_in + n_hidden * 4096u + 3u * 64u; }
};

// Layer l's weights into LDS (64 x 64, zero padded): W[o][k] (transpose =
// false, rows contiguous for dX) or W[k][o] (transpose = true: a wave's 16
// output rows are contiguous for the forward).
__device__ __forceinline__ void load_layer(float *W, const uint16_t *w16, const TrainShape &t, uint32_t l,
                                           bool transpose) {
  const uint32_t in = t.in(l), out = t.out(l), off = t.woff(l);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 4096; i += kTB) {
    const uint32_t o = i >> 6, k = i & 63u;
    const float w = (o < out && k < in) ? h2f(w16[off + o * in + k]) : 0.f;
    W[transpose ? k * 64 + o : i] = w;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kTB) void k_field_train(const uint16_t *feat, uint32_t n, const uint16_t *w16,
                                                      TrainShape t, const float *target, float gscale, float *out,
                                                      float *wave_loss, float *wpart, float *dfeat,
                                                      uint32_t n_grid) {
  extern __shared__ float lds[];
  float *W = lds;                                            // 64 x 64
  float *D = W + 4096;                                       // 64 x kDS
  _Float16 *X = reinterpret_cast<_Float16 *>(D + 64 * kDS);  // layers x 64 x kXS
  const uint32_t q = threadIdx.x & 63u, wave = threadIdx.x >> 6, r0 = 16 * wave;
  const uint32_t gq = blockIdx.x * kTQ + q;
  const bool live = gq < n;
  const uint32_t NL = t.layers(), n_w = t.n_weights();
  for (uint32_t k = r0; k < r0 + 16; ++k)
    X[k * kXS + q] = live ? __builtin_bit_cast(_Float16, feat[(size_t)gq * 64 + k]) : (_Float16)0.f;
  // ------------------------------------------------------------ forward
  float o3[3] = {0.f, 0.f, 0.f};
  for (uint32_t l = 0; l < NL; ++l) {
    load_layer(W, w16, t, l, true);
    const _Float16 *Xl = X + l * 64 * kXS;
    if (l + 1 < NL) {
      float y[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) y[j] = 0.f;
      for (uint32_t k = 0; k < 64; ++k) {
        const float x = (float)Xl[k * kXS + q];
        const float4 *wr = reinterpret_cast<const float4 *>(W + k * 64 + r0);
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const float4 w = wr[j4];
          y[4 * j4 + 0] = fmaf(w.x, x, y[4 * j4 + 0]);
          y[4 * j4 + 1] = fmaf(w.y, x, y[4 * j4 + 1]);
          y[4 * j4 + 2] = fmaf(w.z, x, y[4 * j4 + 2]);
          y[4 * j4 + 3] = fmaf(w.w, x, y[4 * j4 + 3]);
        }
      }
      _Float16 *Xn = X + (l + 1) * 64 * kXS;
      const _Float16 slope = (_Float16)kSlope;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const _Float16 h = (_Float16)y[j];
        const _Float16 hs = h * slope;
        Xn[(r0 + j) * kXS + q] = h > hs ? h : hs;  // max(h, 0.01 h) in fp16 (field.hip leaky_pack)
      }
    } else if (wave == 0) {
      for (uint32_t k = 0; k < 64; ++k) {
        const float x = (float)Xl[k * kXS + q];
#pragma unroll
        for (int c = 0; c < 3; ++c) o3[c] = fmaf(W[k * 64 + c], x, o3[c]);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) o3[c] = (float)(_Float16)o3[c];  // Float16 network output
    }
  }
  // ---------------------------------------------------- loss, dL/dout
  if (wave == 0) {
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float d = 0.f;
      if (live) {
        d = o3[c] - target[3 * (size_t)gq + c];
        sq = fmaf(d, d, sq);
        out[3 * (size_t)gq + c] = o3[c];
      }
      D[c * kDS + q] = gscale * d;
    }
    for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
    if (q == 0) wave_loss[blockIdx.x] = sq;
  }
  // ----------------------------------------------------------- backward
  float *wp = wpart + (size_t)blockIdx.x * n_w;
  for (int l = (int)NL - 1; l >= 0; --l) {
    load_layer(W, w16, t, (uint32_t)l, false);
    const uint32_t in = t.in(l), out = t.out(l), woff = t.woff(l);
    if (l + 1 < (int)NL) {  // through the LeakyReLU of this layer's output
      const _Float16 *Xn = X + (l + 1) * 64 * kXS;
      for (uint32_t o = r0; o < r0 + 16; ++o)
        if (!((float)Xn[o * kXS + q] > 0.f)) D[o * kDS + q] *= kSlope;
    }
    __syncthreads();
    const _Float16 *Xl = X + l * 64 * kXS;
    // partial dW[o][i] = sum_q dY[o][q] X[i][q]   (lane = i, wave = 16 rows o)
    const uint32_t i = q;
    if (out == 64) {
      float acc[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      for (uint32_t qq = 0; qq < 64; ++qq) {
        const float x = (float)Xl[i * kXS + qq];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(D[(r0 + j) * kDS + qq], x, acc[j]);
      }
      if (i < in) {
#pragma unroll
        for (int j = 0; j < 16; ++j) wp[woff + (r0 + j) * in + i] = acc[j];
      }
    } else if (wave == 0) {
      float acc[3] = {0.f, 0.f, 0.f};
      for (uint32_t qq = 0; qq < 64; ++qq) {
        const float x = (float)Xl[i * kXS + qq];
#pragma unroll
        for (int o = 0; o < 3; ++o) acc[o] = fmaf(D[o * kDS + qq], x, acc[o]);
      }
      if (i < in) {
#pragma unroll
        for (int o = 0; o < 3; ++o) wp[woff + o * in + i] = acc[o];
      }
    }
    if (l == 0 && !dfeat) break;
    // dX[k][q] = sum_o W[o][k] dY[o][q]   (lane = q, wave = 16 rows k)
    float g[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) g[j] = 0.f;
    for (uint32_t o = 0; o < out; ++o) {
      const float dy = D[o * kDS + q];
      const float4 *wr = reinterpret_cast<const float4 *>(W + o * 64 + r0);
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const float4 w = wr[j4];
        g[4 * j4 + 0] = fmaf(w.x, dy, g[4 * j4 + 0]);
        g[4 * j4 + 1] = fmaf(w.y, dy, g[4 * j4 + 1]);
        g[4 * j4 + 2] = fmaf(w.z, dy, g[4 * j4 + 2]);
        g[4 * j4 + 3] = fmaf(w.w, dy, g[4 * j4 + 3]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) D[(r0 + j) * kDS + q] = g[j];
  }
  __syncthreads();
  // d(hash-grid features): rows 3 .. 3 + n_grid of dX0
  if (dfeat && live) {
    for (uint32_t k = wave; k < n_grid; k += kTW) dfeat[(size_t)gq * n_grid + k] = D[(3 + k) * kDS + q];
  }
}

__global__ void k_wgrad_reduce(const float *wpart, uint32_t n_blocks, uint32_t n_w, float *grad_w) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_w) return;
  float s = 0.f;
  for (uint32_t b = 0; b < n_blocks; ++b) s += wpart[(size_t)b * n_w + j];
  grad_w[j] = s;
}

// One thread per (point, level).
__global__ void k_field_encode_bwd(FieldEncoding e, const float4 *qp, uint32_t n, const float *dfeat, float *gtab) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t L = e.n_levels, F = e.n_features;
  if (tid >= (uint64_t)n * L) return;
  const uint32_t q = (uint32_t)(tid / L), l = (uint32_t)(tid - (uint64_t)q * L);
  const float4 p = qp[q];
  const V3 pn = field_pnorm(e, V3{p.x, p.y, p.z});
  uint32_t idx[8];
  float w[8];
  field_level_corners(e, pn, l, idx, w);
  const size_t T = (size_t)1 << e.log2_table;
  for (uint32_t f = 0; f < F; ++f) {
    const float d = dfeat[(size_t)q * (L * F) + l * F + f];
    if (d == 0.f) continue;
    for (int c = 0; c < 8; ++c) atomicAdd(gtab + ((size_t)l * T + idx[c]) * F + f, w[c] * d);
  }
}

__global__ void k_grad_check(const float *g, uint64_t n, uint32_t *flag) {
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i]);
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

struct AdamStep {
  float lr_t, b1, b2, eps, inv_scale;
};

// drjit.opt.Adam (upstream): m = fma(b1, m, (1-b1) g), v = fma(b2, v, (1-b2) g^2),
// p -= lr_t m / (sqrt(v) + eps), lr_t = lr sqrt(1 - b2^t) / (1 - b1^t); g are
// the unscaled gradients (GradScaler). Skipped when a gradient is non-finite.
__global__ void k_adam(float *p, float *m, float *v, const float *g, uint64_t n, AdamStep a, const uint32_t *flag,
                       uint16_t *tab16, uint64_t n_tab, uint16_t *w16) {
  if (*flag) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * a.inv_scale;
    const float mi = fmaf(a.b1, m[i], (1.f - a.b1) * gi);
    const float vi = fmaf(a.b2, v[i], (1.f - a.b2) * (gi * gi));
    const float pi = p[i] - a.lr_t * mi / (sqrtf(vi) + a.eps);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    const uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)pi);
    if (i < n_tab)
      tab16[i] = h;
    else
      w16[i - n_tab] = h;
  }
}

__global__ void k_half_to_float(const uint16_t *h, uint64_t n, float *f) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] = h2f(h[i]);
}

// field_prepack (field.hip) on the device: thread per (fragment, lane, j).
__global__ void k_field_prepack_dev(const uint16_t *w, TrainShape t, uint16_t *frag, uint32_t n_frag) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n_frag * 64 * 8) return;
  const uint32_t f = tid / 512, lane = (tid / 8) & 63u, j = tid & 7u;
  const uint32_t n_mid = 8 * (t.n_hidden + 1);
  uint32_t l, mt, ks;
  if (f < n_mid) {
    l = f / 8;
    mt = (f % 8) / 4;
    ks = f % 4;
  } else {
    l = t.n_hidden + 1;
    mt = 0;
    ks = f - n_mid;
  }
  const uint32_t in = t.in(l), out = t.out(l);
  const uint32_t row = 32 * mt + (lane & 31), h = lane >> 5;
  const uint32_t k = l == 0 ? 16 * ks + 8 * h + j : 32 * (ks >> 1) + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
  frag[tid] = (row < out && k < in) ? w[t.woff(l) + (size_t)row * in + k] : 0;
}

// ------------------------------------------------------------- launchers --
size_t field_train_lds(uint32_t n_hidden) {
  return (4096 + 64 * kDS) * sizeof(float) + (size_t)(n_hidden + 2) * 64 * kXS * sizeof(_Float16);
}

int field_train_launch(const uint16_t *feat, uint32_t n, const uint16_t *w16, uint32_t n_in, uint32_t n_hidden,
                       const float *target, float gscale, float *out, float *wave_loss, float *wpart, float *grad_w,
                       float *dfeat, uint32_t n_grid, hipStream_t st) {
  const TrainShape t{n_in, n_hidden};
  const uint32_t blocks = (n + kTQ - 1) / kTQ;
  const size_t lds = field_train_lds(n_hidden);
  if (hipFuncSetAttribute((const void *)k_field_train, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess) {
    mtx_set_error("field_train: %zu B of LDS per block not available", lds);
    return MTX_E_HIP;
  }
  hipLaunchKernelGGL(k_field_train, dim3(blocks), dim3(kTB), lds, st, feat, n, w16, t, target,
                     gscale, out, wave_loss, wpart, dfeat, n_grid);
  const uint32_t n_w = t.n_weights();
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((n_w + 255) / 256), dim3(256), 0, st, wpart, blocks, n_w, grad_w);
  return MTX_OK;
}

void field_encode_bwd_launch(const FieldEncoding &e, const float4 *qp, uint32_t n, const float *dfeat, float *gtab,
                             hipStream_t st) {
  const uint64_t th = (uint64_t)n * e.n_levels;
  hipLaunchKernelGGL(k_field_encode_bwd, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, e, qp, n, dfeat, gtab);
}

void grad_check_launch(const float *g, uint64_t n, uint32_t *flag, hipStream_t st) {
  hipLaunchKernelGGL(k_grad_check, dim3(2048), dim3(256), 0, st, g, n, flag);
}

void adam_launch(float *p, float *m, float *v, const float *g, uint64_t n, float lr_t, float b1, float b2, float eps,
                 float inv_scale, const uint32_t *flag, uint16_t *tab16, uint64_t n_tab, uint16_t *w16,
                 hipStream_t st) {
  const AdamStep a{lr_t, b1, b2, eps, inv_scale};
  hipLaunchKernelGGL(k_adam, dim3(4096), dim3(256), 0, st, p, m, v, g, n, a, flag, tab16, n_tab, w16);
}

void half_to_float_launch(const uint16_t *h, uint64_t n, float *f, hipStream_t st) {
  hipLaunchKernelGGL(k_half_to_float, dim3(4096), dim3(256), 0, st, h, n, f);
}

void field_prepack_launch(const uint16_t *w16, uint32_t n_in, uint32_t n_hidden, uint16_t *frag, hipStream_t st) {
  const TrainShape t{n_in, n_hidden};
  const uint32_t n_frag = field_frag_count(n_hidden);
  hipLaunchKernelGGL(k_field_prepack_dev, dim3((n_frag * 512 + 255) / 256), dim3(256), 0, st, w16, t, frag, n_frag);
}

}  // namespace mtxd
