// prims.hip — GPU primitives of the reference repository, MI355X-native.
//
// * scan_u32: prefix_sum.py:9-36 on u32 as a single-pass decoupled look-back
//   scan (Merrill & Garland 2016): 256 threads x 16 items per tile, dynamic
//   tile tickets, one 8-byte {status, value} granule per tile published with
//   agent-scope (sc1) stores and polled with sc1 loads; 8 B of HBM traffic
//   per element instead of the reference's floor(log2 n)+1 full passes.
// * scan_f32_hs: prefix_sum.py:9-36 on f32 in exactly the reference's
//   Hillis-Steele summation order (bit-identical results): the first 11
//   passes run in LDS on a tile plus its 2047-element halo, the remaining
//   passes (offsets >= 2048) as coalesced full-array passes.
// * hashgrid_build: hashgrid.py:16-90 — scalar bbox reduction, cell hash,
//   then the cell grouping as one stable radix sort of (cell, sample index)
//   pairs: sample_idx is the sorted index column, so within a cell the
//   samples come in ascending index order (one valid outcome of the
//   reference's race-defined winner election, :52-63, and the exact order of
//   the CPU restatement); cell_offset (:65-76) and cell_size come from the
//   run boundaries of the sorted cells. Sequential passes replace the
//   random-address rank atomics and scatter.
// * scatter_reduce_f32: reductions.py:12-54 — the reference serialises each
//   target with host-synchronised winner-election rounds (race-defined
//   order). Here: one stable radix sort of (index, value) pairs (rocPRIM,
//   header-only), segment bounds from the sorted keys, then one thread per
//   target folds its segment in ascending original position — every target
//   receives its values in ascending index order (deterministic), with no
//   host round trips.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "mtx.h"
#include "prims.h"

void mtx_set_error(const char *fmt, ...);

namespace mtxd {

namespace {

// Large tiles: the tile ticket is one same-address atomic per tile (~90 per
// microsecond chip-wide), so 16K-element tiles keep it off the critical path.
constexpr int kScanBlock = 512;
constexpr int kScanItems = 32;
constexpr uint32_t kScanTile = kScanBlock * kScanItems;


__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ws layout (u64 words): [0] tile ticket (low 32 bits), [1] give-up flag,
// [2 + t] status of tile t: (status << 32) | value; 1 = aggregate,
// 2 = inclusive prefix.
__global__ __launch_bounds__(kScanBlock) void k_scan_u32(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                         uint64_t n, int inclusive, unsigned long long *ws) {
  __shared__ uint32_t s_tile, s_prefix;
  __shared__ uint32_t s_wave[kScanBlock / 64];
  const uint32_t tid = threadIdx.x, wid = tid >> 6, ln = tid & 63;
  if (tid == 0) s_tile = atomicAdd(reinterpret_cast<unsigned int *>(ws), 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  unsigned long long *status = ws + 2;
  const uint64_t tile0 = (uint64_t)tile * kScanTile;
  const bool full = tile0 + kScanTile <= n;
  // Coalesced 16-B loads (consecutive lanes, consecutive 16 B), transposed
  // through LDS to kScanItems consecutive items per thread. One padding
  // dword per kScanItems keeps the blocked accesses conflict-free.
  __shared__ uint32_t s_x[kScanTile + kScanTile / kScanItems];
#pragma unroll
  for (int q = 0; q < kScanItems / 4; ++q) {
    const uint32_t i = (uint32_t)q * (kScanBlock * 4) + tid * 4;
    uint4 x;
    if (full) {
      x = *reinterpret_cast<const uint4 *>(in + tile0 + i);
    } else {
      x.x = tile0 + i < n ? in[tile0 + i] : 0u;
      x.y = tile0 + i + 1 < n ? in[tile0 + i + 1] : 0u;
      x.z = tile0 + i + 2 < n ? in[tile0 + i + 2] : 0u;
      x.w = tile0 + i + 3 < n ? in[tile0 + i + 3] : 0u;
    }
    const uint32_t pi = i + i / kScanItems;
    s_x[pi] = x.x;
    s_x[pi + 1] = x.y;
    s_x[pi + 2] = x.z;
    s_x[pi + 3] = x.w;
  }
  __syncthreads();
  uint32_t v[kScanItems];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) v[k] = s_x[tid * (kScanItems + 1) + k];
#pragma unroll
  for (int k = 1; k < kScanItems; ++k) v[k] += v[k - 1];
  const uint32_t total = v[kScanItems - 1];
  uint32_t x = total;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off);
    if (ln >= (uint32_t)off) x += y;
  }
  const uint32_t thread_excl = x - total;
  if (ln == 63) s_wave[wid] = x;
  __syncthreads();
  uint32_t wave_prefix = 0, tile_total = 0;
#pragma unroll
  for (int w = 0; w < kScanBlock / 64; ++w) {
    if ((uint32_t)w < wid) wave_prefix += s_wave[w];
    tile_total += s_wave[w];
  }
  if (wid == 0) {
    uint32_t prefix = 0;
    if (tile == 0) {
      if (ln == 0) st_agent(&status[0], (2ull << 32) | tile_total);
    } else {
      if (ln == 0) st_agent(&status[tile], (1ull << 32) | tile_total);
      int64_t pos = (int64_t)tile - 1;
      while (true) {
        const int64_t idx = pos - (int64_t)ln;
        unsigned long long w = 2ull << 32;
        if (idx >= 0) {
          uint32_t spins = 0;
          w = ld_agent(&status[idx]);
          while ((w >> 32) == 0) {
            __builtin_amdgcn_s_sleep(1);
            w = ld_agent(&status[idx]);
            if (++spins > (1u << 26)) {  // never expected: record and give up
              ws[1] = 1;
              w = 2ull << 32;
              break;
            }
          }
        }
        const uint32_t st = (uint32_t)(w >> 32), val = (uint32_t)w;
        const uint64_t incl = __ballot(st == 2);
        if (incl) {
          const uint32_t k = (uint32_t)(__ffsll((unsigned long long)incl) - 1);
          prefix += wave_sum(ln <= k ? val : 0u);
          break;
        }
        prefix += wave_sum(val);
        pos -= 64;
      }
      if (ln == 0) st_agent(&status[tile], (2ull << 32) | (uint32_t)(prefix + tile_total));
    }
    if (ln == 0) s_prefix = prefix;
  }
  __syncthreads();
  const uint32_t off = s_prefix + wave_prefix + thread_excl;
  // results back through LDS (each thread rewrites only its own slots, so
  // no barrier is needed before the writes), then coalesced 16-B stores
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) s_x[tid * (kScanItems + 1) + k] = (inclusive ? v[k] : (k ? v[k - 1] : 0u)) + off;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kScanItems / 4; ++q) {
    const uint32_t i = (uint32_t)q * (kScanBlock * 4) + tid * 4;
    const uint32_t pi = i + i / kScanItems;
    const uint4 x = make_uint4(s_x[pi], s_x[pi + 1], s_x[pi + 2], s_x[pi + 3]);
    if (full) {
      *reinterpret_cast<uint4 *>(out + tile0 + i) = x;
    } else {
      if (tile0 + i < n) out[tile0 + i] = x.x;
      if (tile0 + i + 1 < n) out[tile0 + i + 1] = x.y;
      if (tile0 + i + 2 < n) out[tile0 + i + 2] = x.z;
      if (tile0 + i + 3 < n) out[tile0 + i + 3] = x.w;
    }
  }
}

// Hillis-Steele in LDS: passes 0..k-1 for a tile of kHsTile outputs.
constexpr int kHsLog = 11;
constexpr int kHsTile = 2048;
constexpr int kHsHalo = (1 << kHsLog) - 1;
constexpr int kHsSpan = kHsTile + kHsHalo;

__global__ __launch_bounds__(256) void k_hs_local(const float *__restrict__ x, float *__restrict__ y, uint64_t n,
                                                  int passes) {
  __shared__ float buf[2][kHsSpan + 1];
  const int64_t a = (int64_t)blockIdx.x * kHsTile;
  for (int l = threadIdx.x; l < kHsSpan; l += blockDim.x) {
    const int64_t g = a - kHsHalo + l;
    buf[0][l] = (g >= 0 && g < (int64_t)n) ? x[g] : 0.f;
  }
  int cur = 0;
  for (int i = 0; i < passes; ++i) {
    __syncthreads();
    const int s = 1 << i;
    for (int l = threadIdx.x; l < kHsSpan; l += blockDim.x) {
      const int64_t g = a - kHsHalo + l;
      float v = buf[cur][l];
      if (g >= s && l >= s) v = buf[cur][l] + buf[cur][l - s];
      buf[cur ^ 1][l] = v;
    }
    cur ^= 1;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < kHsTile; t += blockDim.x) {
    const int64_t g = a + t;
    if (g < (int64_t)n) y[g] = buf[cur][kHsHalo + t];
  }
}

__global__ void k_hs_pass(const float *__restrict__ x, float *__restrict__ y, uint64_t n, uint64_t s) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  y[j] = j >= s ? x[j] + x[j - s] : x[j];
}

// ----------------------------- hash grid ----------------------------------
__global__ void k_minmax(const float *__restrict__ p, uint64_t n3, float2 *partial) {
  __shared__ float smin[256], smax[256];
  float lo = INFINITY, hi = -INFINITY;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x, t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float4 *p4 = reinterpret_cast<const float4 *>(p);  // 256-B aligned device buffer
  for (uint64_t i = t0; i < n3 / 4; i += stride) {
    const float4 v = p4[i];
    lo = fminf(lo, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
    hi = fmaxf(hi, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
  }
  for (uint64_t i = n3 / 4 * 4 + t0; i < n3; i += stride) {
    lo = fminf(lo, p[i]);
    hi = fmaxf(hi, p[i]);
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = make_float2(smin[0], smax[0]);
}

__global__ void k_minmax_final(float2 *partial, int m) {
  __shared__ float smin[256], smax[256];
  float lo = INFINITY, hi = -INFINITY;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    lo = fminf(lo, partial[i].x);
    hi = fmaxf(hi, partial[i].y);
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[m] = make_float2(smin[0], smax[0]);
}

__global__ void k_hash_cells(const float *__restrict__ p, uint64_t n, uint32_t res, uint32_t n_cells,
                             const float2 *bbox, uint32_t *cell) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float2 bb = *bbox;
  const float bbmin = bb.x, ext = bb.y - bb.x, fres = (float)res;
  const uint32_t x = (uint32_t)((p[i] - bbmin) / ext * fres);
  const uint32_t y = (uint32_t)((p[n + i] - bbmin) / ext * fres);
  const uint32_t z = (uint32_t)((p[2 * n + i] - bbmin) / ext * fres);
  cell[i] = ((x * 73856093u) ^ (y * 19349663u) ^ (z * 83492791u)) % n_cells;
}

// cell_offset[c] = number of samples with cell < c and cell_size[c], from
// the sorted cells. Block b holds keys [i0, i1) (kHashTile of them) in LDS
// and owns the cells (key[i0-1], key[i1-1]] (the first block from cell 0,
// the last up to n_cells - 1): each cell is written once, coalesced, with a
// binary search in LDS for its first position in the tile, a short walk to
// the run's end (and a search in global memory for a run that continues
// past the tile).
constexpr int kHashTile = 2048;
__global__ __launch_bounds__(256) void k_hash_ranges(const uint32_t *__restrict__ key, uint64_t n, uint32_t n_cells,
                                                      uint32_t *__restrict__ cell_offset,
                                                      uint32_t *__restrict__ cell_size) {
  __shared__ uint32_t tk[kHashTile];
  const uint64_t i0 = (uint64_t)blockIdx.x * kHashTile;
  const uint32_t cnt = (uint32_t)min((uint64_t)kHashTile, n - i0);
  {  // eight independent loads in flight (clamped index: no branch between them)
    uint32_t v[kHashTile / 256];
#pragma unroll
    for (int r = 0; r < kHashTile / 256; ++r) v[r] = key[i0 + min(threadIdx.x + 256u * r, cnt - 1u)];
#pragma unroll
    for (int r = 0; r < kHashTile / 256; ++r) tk[threadIdx.x + 256u * r] = v[r];
  }
  __syncthreads();
  // cells are < n_cells <= 2^32 - 1, so c + 1 fits in 32 bits
  const uint32_t lo = i0 == 0 ? 0u : key[i0 - 1] + 1u;
  const uint32_t hi = i0 + cnt == n ? n_cells - 1u : tk[cnt - 1];
  if (hi < lo) return;
  for (uint32_t c = lo + threadIdx.x; c <= hi && c >= lo; c += 256) {
    uint32_t l = 0, h = cnt;  // first tile position with key >= c
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if (tk[m] < c)
        l = m + 1;
      else
        h = m;
    }
    uint32_t e = l;
    while (e < cnt && tk[e] == c) ++e;
    uint64_t ge = i0 + e;
    if (e == cnt && ge < n && key[ge] == c) {  // the run of c continues past the tile:
      uint64_t last = ge, step = 1, probe = ge + 1;  // gallop, then bisect: O(log run) loads
      while (probe < n && key[probe] == c) {
        last = probe;
        step *= 2;
        probe = last + step;
      }
      uint64_t gl = last + 1, gh = min(probe, (uint64_t)n);  // first key > c in [gl, gh]
      while (gl < gh) {
        const uint64_t m = (gl + gh) >> 1;
        if (key[m] <= c)
          gl = m + 1;
        else
          gh = m;
      }
      ge = gl;
    }
    cell_offset[c] = (uint32_t)(i0 + l);
    cell_size[c] = (uint32_t)(ge - (i0 + l));
  }
}

// Sparse case (n_cells > 4 n): lower bounds of c and c + 1 in the sorted
// cells, one thread per cell.
__global__ void k_hash_offsets_search(const uint32_t *__restrict__ key, uint64_t n, uint32_t n_cells,
                                      uint32_t *__restrict__ cell_offset, uint32_t *__restrict__ cell_size) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cells) return;
  auto lower = [&](uint64_t v) -> uint64_t {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if ((uint64_t)key[mid] < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  const uint64_t b = lower(c);
  cell_offset[c] = (uint32_t)b;
  cell_size[c] = (uint32_t)(lower(c + 1) - b);
}

// --------------------------- scatter reduce -------------------------------
__global__ void k_sr_bounds(const uint32_t *keys, uint64_t n, uint32_t *seg_start, uint32_t *seg_end) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t key = keys[k];
  if (k == 0 || keys[k - 1] != key) seg_start[key] = (uint32_t)k;
  if (k == n - 1 || keys[k + 1] != key) seg_end[key] = (uint32_t)(k + 1);
}

__global__ void k_sr_fold(int op, float *target, uint64_t nt, const float *vals, const uint32_t *seg_start,
                          const uint32_t *seg_end) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;
  const uint32_t b = seg_start[t], e = seg_end[t];
  if (b >= e) return;
  float acc = target[t];
  for (uint32_t k = b; k < e; ++k) {
    const float v = vals[k];
    acc = op == 0 ? acc + v : (op == 1 ? fminf(acc, v) : fmaxf(acc, v));
  }
  target[t] = acc;
}



inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

size_t scan_workspace_bytes(uint64_t n) { return 8ull * (2 + (n + kScanTile - 1) / kScanTile); }

int scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, int inclusive, void *ws, hipStream_t st) {
  if (n == 0) return MTX_OK;
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  if (tiles >= (1ull << 31)) {
    mtx_set_error("scan_u32: too many tiles");
    return MTX_E_ARG;
  }
  if (hipMemsetAsync(ws, 0, scan_workspace_bytes(n), st) != hipSuccess) {
    mtx_set_error("scan_u32: memset failed");
    return MTX_E_HIP;
  }
  hipLaunchKernelGGL(k_scan_u32, dim3((unsigned)tiles), dim3(kScanBlock), 0, st, in, out, n, inclusive,
                     (unsigned long long *)ws);
  return MTX_OK;
}

int scan_f32_hs(float *a, float *b, uint64_t n, float **result, hipStream_t st) {
  *result = a;
  if (n == 0) return MTX_OK;
  int passes = 0;  // number of passes with 2^i < n
  while ((1ull << passes) < n) ++passes;
  const int local = passes < kHsLog ? passes : kHsLog;
  hipLaunchKernelGGL(k_hs_local, dim3(nblk(n, kHsTile)), dim3(256), 0, st, a, b, n, local);
  float *x = b, *y = a;
  for (int i = local; i < passes; ++i) {
    hipLaunchKernelGGL(k_hs_pass, dim3(nblk(n, 256)), dim3(256), 0, st, x, y, n, 1ull << i);
    float *t = x;
    x = y;
    y = t;
  }
  *result = x;
  return MTX_OK;
}

static unsigned key_bits(uint64_t n_target);

static size_t hash_sort_temp_bytes(uint64_t n, uint32_t n_cells) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                            rocprim::counting_iterator<uint32_t>(0u), (uint32_t *)nullptr, (size_t)n, 0u,
                            key_bits(n_cells));
  return bytes;
}

size_t hashgrid_workspace_bytes(uint64_t n, uint32_t n_cells) {
  return 8ull * 1025 + 4ull * n + hash_sort_temp_bytes(n, n_cells) + 512;
}

int hashgrid_build(const float *p, uint64_t n, uint32_t res, uint32_t n_cells, uint32_t *cell, uint32_t *cell_size,
                   uint32_t *cell_offset, uint32_t *sample_idx, void *ws, hipStream_t st) {
  char *w = (char *)ws;
  float2 *partial = (float2 *)w;
  uint32_t *keys = (uint32_t *)(w + 8 * 1025);
  void *temp = (void *)(((uintptr_t)(keys + n) + 255) & ~(uintptr_t)255);
  size_t temp_bytes = hash_sort_temp_bytes(n, n_cells);
  const int m = 1024;
  hipLaunchKernelGGL(k_minmax, dim3(m), dim3(256), 0, st, p, 3 * n, partial);
  hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(256), 0, st, partial, m);
  hipLaunchKernelGGL(k_hash_cells, dim3(nblk(n, 256)), dim3(256), 0, st, p, n, res, n_cells, partial + m, cell);
  if (rocprim::radix_sort_pairs(temp, temp_bytes, cell, keys, rocprim::counting_iterator<uint32_t>(0u), sample_idx,
                                (size_t)n, 0u, key_bits(n_cells), st) != hipSuccess) {
    mtx_set_error("hashgrid: radix sort failed");
    return MTX_E_HIP;
  }
  if ((uint64_t)n_cells > 4 * n)
    hipLaunchKernelGGL(k_hash_offsets_search, dim3(nblk(n_cells, 256)), dim3(256), 0, st, keys, n, n_cells,
                       cell_offset, cell_size);
  else
    hipLaunchKernelGGL(k_hash_ranges, dim3(nblk(n, kHashTile)), dim3(256), 0, st, keys, n, n_cells, cell_offset,
                       cell_size);
  return MTX_OK;
}

static unsigned key_bits(uint64_t n_target) {
  unsigned b = 1;
  while (b < 32 && (1ull << b) < n_target) ++b;
  return b;
}

static size_t sort_temp_bytes(uint64_t n_value, uint64_t n_target) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, (const float *)nullptr,
                            (float *)nullptr, (size_t)n_value, 0u, key_bits(n_target));
  return bytes;
}

size_t scatter_workspace_bytes(uint64_t n_target, uint64_t n_value) {
  return 8ull * n_value + 8ull * n_target + sort_temp_bytes(n_value, n_target) + 256;
}

int scatter_reduce_f32(int op, float *target, uint64_t n_target, const float *value, const uint32_t *index,
                       uint64_t n_value, void *ws, hipStream_t st) {
  uint32_t *keys = (uint32_t *)ws;
  float *vals = (float *)(keys + n_value);
  uint32_t *seg_start = (uint32_t *)(vals + n_value), *seg_end = seg_start + n_target;
  void *temp = (void *)(((uintptr_t)(seg_end + n_target) + 255) & ~(uintptr_t)255);
  size_t temp_bytes = sort_temp_bytes(n_value, n_target);
  if (rocprim::radix_sort_pairs(temp, temp_bytes, index, keys, value, vals, (size_t)n_value, 0u,
                                key_bits(n_target), st) != hipSuccess) {
    mtx_set_error("scatter_reduce: radix sort failed");
    return MTX_E_HIP;
  }
  if (hipMemsetAsync(seg_start, 0, 8ull * n_target, st) != hipSuccess) return MTX_E_HIP;
  hipLaunchKernelGGL(k_sr_bounds, dim3(nblk(n_value, 256)), dim3(256), 0, st, keys, n_value, seg_start, seg_end);
  hipLaunchKernelGGL(k_sr_fold, dim3(nblk(n_target, 256)), dim3(256), 0, st, op, target, n_target, vals, seg_start,
                     seg_end);
  return MTX_OK;
}

}  // namespace mtxd
