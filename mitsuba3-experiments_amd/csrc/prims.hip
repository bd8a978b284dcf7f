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
// * hashgrid_build: hashgrid.py:16-90 — bbox reduction, then the cell
//   grouping as a hand-written stable counting multisplit (see "stable
//   group-by" below): per-tile histograms of the top cell digit fused with
//   the hash, a scan, a stable split into buckets, and one workgroup per
//   bucket that counts its cells in LDS, writes cell_size / cell_offset
//   (:65-76) and places sample_idx. Within a cell the samples come in
//   ascending index order (one valid outcome of the reference's
//   race-defined winner election, :52-63, and the oracle's order).
// * scatter_reduce_f32: reductions.py:12-54 — the reference serialises each
//   target with host-synchronised winner-election rounds (race-defined
//   order). Here the same stable group-by by target index, then one ordered
//   fold per target in LDS-bucket order: every target receives its values
//   in ascending index order (deterministic), with no host round trips and
//   no global atomics.
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdlib.h>

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
  const uint64_t n4 = n3 / 4;
  uint64_t i = t0;
  for (; i + 3 * stride < n4; i += 4 * stride) {  // four loads in flight per thread (eight: 42.7 -> 46.5 us)
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p4[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lo = fminf(lo, fminf(fminf(v[k].x, v[k].y), fminf(v[k].z, v[k].w)));
      hi = fmaxf(hi, fmaxf(fmaxf(v[k].x, v[k].y), fmaxf(v[k].z, v[k].w)));
    }
  }
  for (; i < n4; i += stride) {
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

// Bounding interval of k_minmax's m partials, reduced by the first 256
// threads of the block in a fixed tree (every caller gets the same floats;
// larger blocks' other threads only take the barriers).
__device__ __forceinline__ float2 minmax_reduce(const float2 *partial, int m) {
  __shared__ float smin[256], smax[256];
  if (threadIdx.x < 256) {
    float lo = INFINITY, hi = -INFINITY;
    for (int i = threadIdx.x; i < m; i += 256) {
      lo = fminf(lo, partial[i].x);
      hi = fmaxf(hi, partial[i].y);
    }
    smin[threadIdx.x] = lo;
    smax[threadIdx.x] = hi;
  }
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + s]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + s]);
    }
    __syncthreads();
  }
  return make_float2(smin[0], smax[0]);
}

__global__ __launch_bounds__(256) void k_minmax_final(float2 *partial, int m) {
  const float2 bb = minmax_reduce(partial, m);
  if (threadIdx.x == 0) partial[m] = bb;
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

// ------------------ stable group-by (hashgrid, scatter-reduce) -------------
// hashgrid.py:52-84 and reductions.py:23-54 both group elements by a u32 key
// (cell / target index) and, for determinism, keep ascending element index
// inside a key (one of the reference's race-defined outcomes, and the
// oracle's order). Hand-written counting multisplits, no global atomics:
// * keys < 2^24 (two levels): k_tile_split sorts every tile stably by the
//   top digit (key >> s, at most 12 bits) in LDS and writes it back
//   contiguously with a per-tile digit table; k_bucket_fast gives each
//   bucket one workgroup that gathers its runs from all tiles into LDS,
//   counts its 2^s keys, writes their cell_size / cell_offset (or folds
//   their values) and places every element at its final position. HBM
//   traffic: the keys/points read once, one 4-8 B record written and
//   gathered back, the outputs written once.
// * wider keys: LSD passes of k_ms_place over 12-bit digits, then the run
//   bounds of the sorted keys.
// Stability comes from one construction: a wave owns a contiguous run of
// elements and a private LDS counter row; inside a 64-element round, lanes
// with equal digits are found with one ballot per digit bit (a match mask)
// and ranked in lane order; the waves' bases for a digit are prefix sums
// over the waves in order. A wave's own LDS reads and writes complete in
// program order, so the read-then-bump of a counter needs no atomic.
constexpr int kMsWaves = 8;
constexpr int kMsThreads = 64 * kMsWaves;
constexpr int kMsRounds = 32;
constexpr uint32_t kMsSub = 64u * kMsRounds;     // elements per wave
constexpr uint32_t kMsTile = kMsSub * kMsWaves;  // elements per workgroup
constexpr int kMsMaxBits = 12;                   // 8 waves x 4096 counters x 4 B = 128 KB of LDS

// Tile of a workgroup: consecutive tiles on one XCD (workgroups are dealt to
// the 8 XCDs round robin), so the [digit][tile] table's columns share lines
// inside one L2. A bijection of [0, tiles).
__device__ __forceinline__ uint32_t ms_tile(uint32_t blk, uint32_t tiles) {
  const uint32_t x = blk & 7u, j = blk >> 3, q = tiles >> 3, r = tiles & 7u;
  return x * q + min(x, r) + j;
}

// Lanes of `active` whose digit equals this lane's (bits ballots).
__device__ __forceinline__ uint64_t ms_match(uint32_t d, int bits, uint64_t active) {
  uint64_t m = active;
  for (int j = 0; j < bits; ++j) {
    const uint32_t bit = (d >> j) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

__device__ __forceinline__ uint32_t hg_cell(const float *__restrict__ p, uint64_t n, uint64_t i, float bbmin,
                                            float ext, float fres, uint32_t n_cells) {
  // hashgrid.py:86-90 with hash :8-12 (u32 wraparound); the oracle's exact
  // operation order (orc_hashgrid)
  const uint32_t x = (uint32_t)((p[i] - bbmin) / ext * fres);
  const uint32_t y = (uint32_t)((p[n + i] - bbmin) / ext * fres);
  const uint32_t z = (uint32_t)((p[2 * n + i] - bbmin) / ext * fres);
  return ((x * 73856093u) ^ (y * 19349663u) ^ (z * 83492791u)) % n_cells;
}

// Per-tile digit histogram: hist[digit * tiles + tile]. HASH: the keys are
// the hash-grid cells, computed here from the points and stored to `cell`.
template <bool HASH>
__global__ __launch_bounds__(kMsThreads) void k_ms_hist(const uint32_t *__restrict__ keys,
                                                        const float *__restrict__ p, uint64_t n, uint32_t res,
                                                        uint32_t n_cells, const float2 *__restrict__ bbox,
                                                        uint32_t *__restrict__ cell, int shift, int bits,
                                                        uint32_t *__restrict__ hist, uint32_t tiles) {
  extern __shared__ uint32_t s_cnt[];
  const uint32_t B = 1u << bits, t = ms_tile(blockIdx.x, tiles);
  for (uint32_t b = threadIdx.x; b < B; b += kMsThreads) s_cnt[b] = 0;
  float bbmin = 0.f, ext = 1.f;
  if (HASH) {
    const float2 bb = *bbox;
    bbmin = bb.x;
    ext = bb.y - bb.x;
  }
  __syncthreads();
  const uint64_t t0 = (uint64_t)t * kMsTile;
#pragma unroll 8
  for (uint32_t r = 0; r < kMsTile / kMsThreads; ++r) {
    const uint64_t e = t0 + r * kMsThreads + threadIdx.x;
    if (e < n) {
      uint32_t k;
      if (HASH) {
        k = hg_cell(p, n, e, bbmin, ext, (float)res, n_cells);
        cell[e] = k;
      } else {
        k = keys[e];
      }
      atomicAdd(&s_cnt[(k >> shift) & (B - 1u)], 1u);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < B; b += kMsThreads) hist[(uint64_t)b * tiles + t] = s_cnt[b];
}

// Stable multisplit of one tile by digit = (key >> shift) & (2^bits - 1):
// element e goes to base[digit][tile] + (number of the tile's earlier
// elements with that digit); base = exclusive scan of k_ms_hist's table.
// The payload is the element index (INDEX) or pay[e].
template <bool INDEX>
__global__ __launch_bounds__(kMsThreads) void k_ms_place(const uint32_t *__restrict__ keys,
                                                         const uint32_t *__restrict__ pay, uint64_t n, int shift,
                                                         int bits, const uint32_t *__restrict__ base, uint32_t tiles,
                                                         uint32_t *__restrict__ keys_out,
                                                         uint32_t *__restrict__ pay_out) {
  extern __shared__ uint32_t s_cnt[];  // [kMsWaves][2^bits]
  const uint32_t B = 1u << bits, t = ms_tile(blockIdx.x, tiles);
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t *cnt = s_cnt + w * B;
  for (uint32_t b = lane; b < B; b += 64) cnt[b] = 0;
  const uint64_t s0 = (uint64_t)t * kMsTile + (uint64_t)w * kMsSub;
  uint32_t k[kMsRounds], v[kMsRounds];
#pragma unroll
  for (int r = 0; r < kMsRounds; ++r) {
    const uint64_t e = s0 + (uint32_t)r * 64u + lane;
    k[r] = e < n ? keys[e] : 0u;
    if (!INDEX) v[r] = e < n ? pay[e] : 0u;
  }
#pragma unroll
  for (int r = 0; r < kMsRounds; ++r)
    if (s0 + (uint32_t)r * 64u + lane < n) atomicAdd(&cnt[(k[r] >> shift) & (B - 1u)], 1u);
  // the tile's column of bases: all loads in flight before the LDS work
  constexpr int kCol = (1 << kMsMaxBits) / kMsThreads;
  uint32_t col[kCol];
#pragma unroll
  for (int i = 0; i < kCol; ++i) {
    const uint32_t b = threadIdx.x + (uint32_t)i * kMsThreads;
    col[i] = b < B ? base[(uint64_t)b * tiles + t] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kCol; ++i) {
    const uint32_t b = threadIdx.x + (uint32_t)i * kMsThreads;
    if (b < B) {
      uint32_t run = col[i];
#pragma unroll
      for (int q = 0; q < kMsWaves; ++q) {
        const uint32_t c = s_cnt[q * B + b];
        s_cnt[q * B + b] = run;
        run += c;
      }
    }
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < kMsRounds; ++r) {
    const uint64_t e = s0 + (uint32_t)r * 64u + lane;
    const bool ok = e < n;
    const uint32_t d = (k[r] >> shift) & (B - 1u);
    const uint64_t peers = ms_match(d, bits, __ballot(ok));
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    const uint32_t p0 = cnt[d];
    if (ok && rank == 0) cnt[d] = p0 + (uint32_t)__popcll(peers);
    if (ok) {
      keys_out[p0 + rank] = k[r];
      pay_out[p0 + rank] = INDEX ? (uint32_t)e : v[r];
    }
  }
}

__device__ __forceinline__ float sr_apply(int op, float a, float b) {
  switch (op) {
    case 0: return a + b;
    case 1: return fminf(a, b);
    case 2: return fmaxf(a, b);
    default: return a * b;
  }
}

// ---- two-level path (keys < 2^24) ----
// Level 1, k_tile_split: one workgroup per tile of T elements sorts the tile
// stably by the top digit d = key >> s in LDS and writes it back
// contiguously (no scattered stores: a 4096-way global split of 4-byte
// elements wrote 12x its bytes to the fabric as partial lines), with the
// tile's digit table tab[tile][d] = start | end << 16. Level 2,
// k_bucket_fast: one workgroup per bucket d gathers the bucket's runs from
// every tile (tile order = element order) into registers, sorts them stably
// by the 2^s local keys with the same per-wave-row construction, and writes
// the bucket's slice of the output contiguously (hashgrid: cell_size,
// cell_offset, sample_idx) or folds each key's run in order (scatter-reduce).
// Adjacent buckets run on one XCD, so neighbouring digits' runs share L2
// lines. Records: hashgrid (local key << 14 | position in tile), T = 16384;
// scatter-reduce {value bits, local key}, T = 8192.
template <int MODE>
struct SplitCfg;
template <>
struct SplitCfg<0> {
  static constexpr uint32_t T = 16384, Tiles = 1024;  // Tiles: tile runs level 2 holds in LDS per pass
  using Rec = uint32_t;
};
template <>
struct SplitCfg<1> {
  static constexpr uint32_t T = 8192, Tiles = 2048;
  using Rec = uint2;
};
constexpr int kSplitMaxTop = 12;  // level-1 LDS: 8 waves x 4096 digits x u16 + the staged tile
constexpr int kBkWaves = 4, kBkThreads = 64 * kBkWaves;
constexpr uint32_t kBkCap = 5120;                    // records per level-2 chunk (20 per thread)
constexpr uint32_t kBkRounds = kBkCap / kBkThreads;  // rounds of 64 per wave

// Exclusive scan of one value per thread over a workgroup of NW waves.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_wsum, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= (uint32_t)off) x += y;
  }
  __syncthreads();  // s_wsum free
  if (lane == 63) s_wsum[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t sq = s_wsum[q];
    pre += (uint32_t)q < w ? sq : 0u;
    tot += sq;
  }
  *total = tot;
  return pre + x - v;
}

// Cells of the points, grid-stride; every block first reduces k_minmax's m
// partials itself (8 KB from L2, the tree of k_minmax_final: no separate
// launch for the final bbox).
__global__ __launch_bounds__(256) void k_hash_cells(const float *__restrict__ p, uint64_t n, uint32_t res,
                                                    uint32_t n_cells, const float2 *__restrict__ partial, int m,
                                                    uint32_t *__restrict__ cell) {
  const float2 bb = minmax_reduce(partial, m);
  const float ext = bb.y - bb.x, fres = (float)res;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    cell[i] = hg_cell(p, n, i, bb.x, ext, fres, n_cells);
}

// Persistent (round 5): a workgroup takes tiles blockIdx.x, + gridDim.x, ...
// and issues the next tile's loads before it sorts the current one, so that
// with one 128-KB workgroup per CU the HBM reads overlap the LDS work instead
// of alternating with it.
template <int MODE, bool RANK>
__global__ __launch_bounds__(512) void k_tile_split(const uint32_t *__restrict__ keys, const float *__restrict__ value,
                                                    uint64_t n, int s, int top, uint32_t tiles,
                                                    uint32_t *__restrict__ tab,
                                                    typename SplitCfg<MODE>::Rec *__restrict__ out1,
                                                    uint32_t *__restrict__ slow) {
  if (blockIdx.x == 0 && threadIdx.x == 0) slow[0] = 0;  // level 2's slow-bucket count
  using Rec = typename SplitCfg<MODE>::Rec;
  constexpr uint32_t T = SplitCfg<MODE>::T, R = T / 512;  // rounds of 64 per wave
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t s_wsum[8];
  const uint32_t B = 1u << top, L1 = (1u << s) - 1u;
  uint32_t *rows = lds;  // [8][B] u16 counters, two per word
  Rec *stage = (Rec *)(lds + 4 * B);
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t *row = rows + w * (B / 2);
  uint16_t *row16 = (uint16_t *)row;
  uint32_t tile = blockIdx.x;
  if (tile >= tiles) return;
  // the current tile's keys and the next tile's, in flight during this
  // tile's sort
  uint32_t key[R], val[R], nk[R], nv[R];
  auto fetch = [&](uint32_t t, uint32_t *k, uint32_t *v) {
    const uint64_t t0 = (uint64_t)t * T;
    const uint32_t ts = (uint32_t)min((uint64_t)T, n - t0);
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t j = w * (T / 8) + r * 64 + lane;
      const bool ok = j < ts;
      k[r] = ok ? keys[t0 + j] : 0u;
      if (MODE == 1) v[r] = ok ? __float_as_uint(value[t0 + j]) : 0u;
    }
  };
  fetch(tile, key, val);
  while (true) {
    const uint64_t t0 = (uint64_t)tile * T;
    const uint32_t tsize = (uint32_t)min((uint64_t)T, n - t0);
    const uint32_t next = tile + gridDim.x;
    if (next < tiles) fetch(next, nk, nv);
    for (uint32_t i = lane; i < B / 2; i += 64) row[i] = 0;
    __syncthreads();  // the previous tile's stage has left LDS; rows zeroed
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t d = key[r] >> s;
      if (w * (T / 8) + r * 64 + lane < tsize) atomicAdd(&row[d >> 1], 1u << ((d & 1u) << 4));
    }
    __syncthreads();
    // digits [8 tid, 8 tid + 8): totals over the waves, tile-level exclusive
    // scan, the table row, then each wave's base per digit (u16)
    const uint32_t d0 = threadIdx.x * 8;
    const bool mine = d0 < B;
    uint32_t tot[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (mine) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 c = *(const uint4 *)&rows[q * (B / 2) + d0 / 2];
        const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tot[2 * i] += cw[i] & 0xFFFFu;
          tot[2 * i + 1] += cw[i] >> 16;
        }
      }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) sum += tot[i];
    uint32_t all;
    uint32_t run = block_excl_scan<8>(sum, s_wsum, &all);
    if (mine) {
      uint32_t st[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        st[i] = run;
        run += tot[i];
      }
      uint4 *trow = (uint4 *)&tab[(uint64_t)tile * B + d0];
      trow[0] = make_uint4(st[0] | (st[1] << 16), st[1] | (st[2] << 16), st[2] | (st[3] << 16), st[3] | (st[4] << 16));
      trow[1] = make_uint4(st[4] | (st[5] << 16), st[5] | (st[6] << 16), st[6] | (st[7] << 16), st[7] | (run << 16));
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 *cp = (uint4 *)&rows[q * (B / 2) + d0 / 2];
        const uint4 c = *cp;
        const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
        uint32_t nw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          nw[i] = st[2 * i] | (st[2 * i + 1] << 16);
          st[2 * i] += cw[i] & 0xFFFFu;
          st[2 * i + 1] += cw[i] >> 16;
        }
        *cp = make_uint4(nw[0], nw[1], nw[2], nw[3]);
      }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t j = w * (T / 8) + r * 64 + lane;
      const bool ok = j < tsize;
      const uint32_t d = key[r] >> s;
      uint32_t pos;
      if constexpr (RANK) {
        // same-address LDS atomics of one wave return in lane order (checked
        // once per device, lds_lane_order()): the old value is the position
        pos = ok ? (atomicAdd(&row[d >> 1], 1u << ((d & 1u) << 4)) >> ((d & 1u) << 4)) & 0xFFFFu : 0u;
      } else {
        const uint64_t peers = ms_match(d, top, __ballot(ok));
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t p0 = row16[d];
        if (ok && rank == 0) row16[d] = (uint16_t)(p0 + (uint32_t)__popcll(peers));
        pos = p0 + rank;
      }
      if (ok) {
        if constexpr (MODE == 0)
          stage[pos] = ((key[r] & L1) << 14) | j;
        else
          stage[pos] = make_uint2(val[r], key[r] & L1);
      }
    }
    __syncthreads();
    // the sorted tile leaves as 16-B stores
    constexpr uint32_t per = 16 / sizeof(Rec);
    for (uint32_t j = threadIdx.x * per; j < tsize; j += 512 * per) {
      if (j + per <= tsize) {
        *(uint4 *)&out1[t0 + j] = *(const uint4 *)&stage[j];
      } else {
        for (uint32_t i = j; i < tsize; ++i) out1[t0 + i] = stage[i];
      }
    }
    if (next >= tiles) break;
    tile = next;
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      key[r] = nk[r];
      if (MODE == 1) val[r] = nv[r];
    }
  }
}

// Exclusive scan of two values per thread at once (one barrier pair).
template <int NW>
__device__ __forceinline__ uint2 block_excl_scan2(uint2 v, uint32_t (*s_wsum)[NW], uint2 *total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint2 x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t ya = __shfl_up(x.x, off), yb = __shfl_up(x.y, off);
    if (lane >= (uint32_t)off) {
      x.x += ya;
      x.y += yb;
    }
  }
  __syncthreads();
  if (lane == 63) {
    s_wsum[0][w] = x.x;
    s_wsum[1][w] = x.y;
  }
  __syncthreads();
  uint2 pre = make_uint2(0, 0), tot = make_uint2(0, 0);
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t a = s_wsum[0][q], c = s_wsum[1][q];
    if ((uint32_t)q < w) {
      pre.x += a;
      pre.y += c;
    }
    tot.x += a;
    tot.y += c;
  }
  *total = tot;
  return make_uint2(pre.x + x.x - v.x, pre.y + x.y - v.y);
}

// KPT u16 counters of row q for keys [k0, k0 + KPT) (vector LDS access).
template <int KPT>
__device__ __forceinline__ void rows_read(const uint16_t *p, uint32_t *c) {
  if constexpr (KPT >= 8) {
#pragma unroll
    for (int v = 0; v < KPT / 8; ++v) {
      const uint4 x = ((const uint4 *)p)[v];
      const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        c[8 * v + 2 * i] = wv[i] & 0xFFFFu;
        c[8 * v + 2 * i + 1] = wv[i] >> 16;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < KPT; ++i) c[i] = p[i];
  }
}
template <int KPT>
__device__ __forceinline__ void rows_write(uint16_t *p, const uint32_t *c) {
  if constexpr (KPT >= 8) {
#pragma unroll
    for (int v = 0; v < KPT / 8; ++v)
      ((uint4 *)p)[v] = make_uint4(c[8 * v] | (c[8 * v + 1] << 16), c[8 * v + 2] | (c[8 * v + 3] << 16),
                                   c[8 * v + 4] | (c[8 * v + 5] << 16), c[8 * v + 6] | (c[8 * v + 7] << 16));
  } else {
#pragma unroll
    for (int i = 0; i < KPT; ++i) p[i] = (uint16_t)c[i];
  }
}

// Per-key pass over the bucket's 2^s local keys, KPT consecutive keys per
// thread: the per-wave u16 counts in rows become per-wave bases. ABS: base =
// chunk start of the key + the earlier waves' counts (staging positions of
// the chunk's stable order); else the earlier waves' counts only (ranks
// relative to the key's running position). Returns the chunk totals of the
// thread's keys (tot) and their chunk starts (cst).
template <int KPT>
__device__ __forceinline__ void bk_keys(uint16_t *rows16, uint32_t L, uint32_t Lr, bool abs,
                                        uint32_t (*s_wsum)[kBkWaves], uint32_t *tot, uint32_t *cst) {
  const uint32_t k0 = threadIdx.x * KPT;
  const bool mine = k0 < L;
  const uint32_t kr = mine ? k0 : 0u;
  uint32_t c[kBkWaves][KPT];
#pragma unroll
  for (int q = 0; q < kBkWaves; ++q) rows_read<KPT>(rows16 + q * Lr + kr, c[q]);
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    tot[i] = 0;
#pragma unroll
    for (int q = 0; q < kBkWaves; ++q) tot[i] += mine ? c[q][i] : 0u;
    sum += tot[i];
  }
  uint2 all;
  uint32_t run = block_excl_scan2<kBkWaves>(make_uint2(sum, 0), s_wsum, &all).x;
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    cst[i] = run;
    run += tot[i];
  }
  if (mine) {
    uint32_t bse[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) bse[i] = abs ? cst[i] : 0u;
#pragma unroll
    for (int q = 0; q < kBkWaves; ++q) {
      rows_write<KPT>(rows16 + q * Lr + k0, bse);
#pragma unroll
      for (int i = 0; i < KPT; ++i) bse[i] += c[q][i];
    }
  }
}

// Lanes of `active` whose local key equals this lane's (s <= 12 bits).
__device__ __forceinline__ uint64_t bk_match(uint32_t k, int s, uint64_t active) {
  uint64_t m = active;
#pragma unroll
  for (int j = 0; j < kSplitMaxTop; ++j)
    if (j < s) {  // uniform
      const uint32_t bit = (k >> j) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
  return m;
}

// Level-2 runs of tile group g of bucket b into LDS: s_pre (prefix in the
// bucket's element sequence, from `base`), s_src (record address of the
// run). Returns {group element count, sum of the run starts}.
template <int MODE>
__device__ __forceinline__ uint2 bk_load_runs(const uint32_t *__restrict__ tab, uint32_t n_tiles, uint32_t B,
                                              uint32_t b, uint32_t g, uint32_t base, uint32_t *s_pre,
                                              uint32_t *s_src, uint32_t (*s_wsum)[kBkWaves]) {
  constexpr uint32_t T = SplitCfg<MODE>::T, kTiles = SplitCfg<MODE>::Tiles, TPT = kTiles / kBkThreads;
  uint32_t rs[TPT], rl[TPT], sum = 0, ssum = 0;
#pragma unroll
  for (uint32_t i = 0; i < TPT; ++i) {
    const uint32_t t = g * kTiles + threadIdx.x * TPT + i;
    const uint32_t e = t < n_tiles ? tab[(uint64_t)t * B + b] : 0u;
    rs[i] = e & 0xFFFFu;
    rl[i] = (e >> 16) - rs[i];
    sum += rl[i];
    ssum += rs[i];
  }
  uint2 tot;
  const uint2 ex = block_excl_scan2<kBkWaves>(make_uint2(sum, ssum), s_wsum, &tot);
  uint32_t run = base + ex.x;
#pragma unroll
  for (uint32_t i = 0; i < TPT; ++i) {
    const uint32_t t = g * kTiles + threadIdx.x * TPT + i;
    s_pre[threadIdx.x * TPT + i] = run;
    s_src[threadIdx.x * TPT + i] = t * T + rs[i];
    run += rl[i];
  }
  if (threadIdx.x == 0) s_pre[kTiles] = base + tot.x;
  return tot;
}

// Records [c0, c0 + cl) of the bucket sequence (inside the loaded group) into
// registers: wave w holds [w*Q, (w+1)*Q), round r lane l = w*Q + 64r + l.
// All rounds search (branch-free, fixed steps) and load together.
template <int MODE>
__device__ __forceinline__ void bk_gather(const typename SplitCfg<MODE>::Rec *__restrict__ out1,
                                          const uint32_t *s_pre, const uint32_t *s_src, uint32_t c0, uint32_t cl,
                                          uint32_t Q, uint32_t *key, uint32_t *pay) {
  using Rec = typename SplitCfg<MODE>::Rec;
  constexpr uint32_t T = SplitCfg<MODE>::T, kTiles = SplitCfg<MODE>::Tiles;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t j[kBkRounds], lo[kBkRounds];
#pragma unroll
  for (uint32_t r = 0; r < kBkRounds; ++r) {
    j[r] = c0 + min(w * Q + r * 64 + lane, cl - 1u);
    lo[r] = 0;
  }
#pragma unroll
  for (uint32_t step = kTiles / 2; step > 0; step >>= 1)
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r) lo[r] += s_pre[lo[r] + step] <= j[r] ? step : 0u;
  Rec rc[kBkRounds];
  uint32_t src[kBkRounds];
#pragma unroll
  for (uint32_t r = 0; r < kBkRounds; ++r) {
    src[r] = s_src[lo[r]] + (j[r] - s_pre[lo[r]]);
    rc[r] = out1[src[r]];  // clamped index: always a valid record of the chunk
  }
#pragma unroll
  for (uint32_t r = 0; r < kBkRounds; ++r) {
    if constexpr (MODE == 0) {
      key[r] = rc[r] >> 14;
      pay[r] = (src[r] / T) * T + (rc[r] & 0x3FFFu);
    } else {
      key[r] = rc[r].y;
      pay[r] = rc[r].x;
    }
  }
}

// Level 2, common case: one workgroup per bucket whose elements fit one
// chunk (kBkCap) and whose tiles fit one group; others are listed in
// `slow` for k_bucket_slow. 2^s = KPT * 256 local keys (KPT = 1: up to 256).
template <int MODE, int KPT, bool RANK>
__global__ __launch_bounds__(kBkThreads, 3) void k_bucket_fast(const typename SplitCfg<MODE>::Rec *__restrict__ out1,
                                                            const uint32_t *__restrict__ tab, uint32_t n_tiles, int s,
                                                            int top, uint32_t n_keys, uint32_t nb,
                                                            uint32_t *__restrict__ cell_size,
                                                            uint32_t *__restrict__ cell_offset,
                                                            uint32_t *__restrict__ sample_idx,
                                                            float *__restrict__ target, int op,
                                                            uint32_t *__restrict__ slow) {
  using Rec = typename SplitCfg<MODE>::Rec;
  constexpr uint32_t T = SplitCfg<MODE>::T, kTiles = SplitCfg<MODE>::Tiles, TPT = kTiles / kBkThreads;
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t s_wsum[2][kBkWaves];
  const uint32_t L = 1u << s, B = 1u << top, Lr = L < 2u ? 2u : L;  // row stride: u16 pairs share a word
  const uint32_t b = ms_tile(blockIdx.x, nb);
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint16_t *rows16 = (uint16_t *)lds;           // [kBkWaves][Lr]
  uint32_t *stage = lds + (kBkWaves / 2) * Lr;  // [kBkCap]
  // the bucket's runs (TPT consecutive tiles per thread) and their prefix
  uint32_t rs[TPT], rl[TPT], sum = 0, ssum = 0;
#pragma unroll
  for (uint32_t i = 0; i < TPT; ++i) {
    const uint32_t t = threadIdx.x * TPT + i;
    const uint32_t e = t < n_tiles ? tab[(uint64_t)t * B + b] : 0u;
    rs[i] = e & 0xFFFFu;
    rl[i] = (e >> 16) - rs[i];
    sum += rl[i];
    ssum += rs[i];
  }
  uint2 rt;
  const uint32_t ex = block_excl_scan2<kBkWaves>(make_uint2(sum, ssum), s_wsum, &rt).x;
  const uint32_t len = rt.x, start = rt.y;  // start: elements of smaller digits in every tile
  if (len > kBkCap) {  // uniform
    if (threadIdx.x == 0) slow[1 + atomicAdd(&slow[0], 1u)] = b;
    return;
  }
  // record address of every element of the bucket sequence, written by the
  // thread owning its tile (runs are short: 2-4 records on average)
  {
    uint32_t q = ex;
#pragma unroll
    for (uint32_t i = 0; i < TPT; ++i) {
      const uint32_t a = (threadIdx.x * TPT + i) * T + rs[i];
      for (uint32_t m = 0; m < rl[i]; ++m) stage[q + m] = a + m;
      q += rl[i];
    }
  }
  for (uint32_t i = threadIdx.x; i < (kBkWaves / 2) * Lr; i += kBkThreads) lds[i] = 0;
  __syncthreads();
  const uint32_t Q = ((len + kBkWaves * 64 - 1) / (kBkWaves * 64)) * 64;
  uint32_t key[kBkRounds], pay[kBkRounds];
  {
    uint32_t src[kBkRounds];
    Rec rc[kBkRounds];
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r) {
      const uint32_t jj = w * Q + r * 64 + lane;
      src[r] = stage[jj < len ? jj : 0u];
    }
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r)
      if (r * 64 < Q && w * Q + r * 64 + lane < len) rc[r] = out1[src[r]];
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r) {
      if constexpr (MODE == 0) {
        key[r] = rc[r] >> 14;
        pay[r] = (src[r] / T) * T + (rc[r] & 0x3FFFu);
      } else {
        key[r] = rc[r].y;
        pay[r] = rc[r].x;
      }
    }
  }
  __syncthreads();  // stage is reused for the placement
#pragma unroll
  for (uint32_t r = 0; r < kBkRounds; ++r)
    if (w * Q + r * 64 + lane < len && r * 64 < Q)
      atomicAdd((uint32_t *)&rows16[w * Lr + (key[r] & ~1u)], 1u << ((key[r] & 1u) << 4));
  __syncthreads();
  uint32_t tot[KPT], cst[KPT];
  bk_keys<KPT>(rows16, L, Lr, true, s_wsum, tot, cst);
  const uint32_t k0 = threadIdx.x * KPT;
  if (MODE == 0 && cell_size && k0 < L) {
    const uint32_t kk = b * L + k0;
    if constexpr (KPT >= 4) {
      if (kk + KPT <= n_keys) {
#pragma unroll
        for (int v = 0; v < KPT / 4; ++v) {
          ((uint4 *)&cell_size[kk])[v] = make_uint4(tot[4 * v], tot[4 * v + 1], tot[4 * v + 2], tot[4 * v + 3]);
          ((uint4 *)&cell_offset[kk])[v] = make_uint4(start + cst[4 * v], start + cst[4 * v + 1],
                                                      start + cst[4 * v + 2], start + cst[4 * v + 3]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < KPT; ++i)
          if (kk + i < n_keys) {
            cell_size[kk + i] = tot[i];
            cell_offset[kk + i] = start + cst[i];
          }
      }
    } else {
#pragma unroll
      for (int i = 0; i < KPT; ++i)
        if (kk + i < n_keys) {
          cell_size[kk + i] = tot[i];
          cell_offset[kk + i] = start + cst[i];
        }
    }
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (uint32_t r = 0; r < kBkRounds; ++r) {
    if (r * 64 < Q) {  // uniform
      const bool ok = w * Q + r * 64 + lane < len;
      const uint32_t k = key[r];
      if constexpr (RANK) {  // lane-ordered LDS atomics (see k_tile_split)
        if (ok) {
          const uint32_t sh = (k & 1u) << 4;
          const uint32_t pos = (atomicAdd((uint32_t *)&rows16[w * Lr + (k & ~1u)], 1u << sh) >> sh) & 0xFFFFu;
          stage[pos] = pay[r];
        }
      } else {
        const uint64_t peers = bk_match(k, s, __ballot(ok));
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t p0 = rows16[w * Lr + k];
        if (ok && rank == 0) rows16[w * Lr + k] = (uint16_t)(p0 + (uint32_t)__popcll(peers));
        if (ok) stage[p0 + rank] = pay[r];
      }
    }
  }
  __syncthreads();
  if (MODE == 0) {
    for (uint32_t i = threadIdx.x; i < len; i += kBkThreads) sample_idx[start + i] = stage[i];
  } else if (k0 < L) {
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const uint32_t kk = b * L + k0 + i;
      if (kk >= n_keys || tot[i] == 0) continue;
      float acc = target[kk];
      for (uint32_t m = cst[i]; m < cst[i] + tot[i]; ++m) acc = sr_apply(op, acc, __uint_as_float(stage[m]));
      target[kk] = acc;
    }
  }
}

// Level 2, general case: the buckets k_bucket_fast listed (or every bucket
// when the tiles exceed one group: list == nullptr), in chunks of kBkCap
// records in sequence order, group by group. MODE 0: a counting pass for the
// bucket offsets, then stable placement straight to the output; MODE 1:
// chunk-wise stable order in LDS, folded into per-key accumulators in order.
// one bucket of k_bucket_slow
template <int MODE, int KPT>
__device__ __forceinline__ void bk_slow_one(const typename SplitCfg<MODE>::Rec *__restrict__ out1,
                                            const uint32_t *__restrict__ tab, uint32_t n_tiles, int s, int top,
                                            uint32_t n_keys, uint32_t b, uint32_t *__restrict__ cell_size,
                                            uint32_t *__restrict__ cell_offset, uint32_t *__restrict__ sample_idx,
                                            float *__restrict__ target, int op, uint32_t *lds,
                                            uint32_t (*s_wsum)[kBkWaves], uint32_t *s_pre, uint32_t *s_src) {
  constexpr uint32_t kTiles = SplitCfg<MODE>::Tiles;
  const uint32_t L = 1u << s, B = 1u << top, Lr = L < 2u ? 2u : L;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint16_t *rows16 = (uint16_t *)lds;           // [kBkWaves][Lr]
  uint32_t *stage = lds + (kBkWaves / 2) * Lr;  // [kBkCap]
  uint32_t *cnt = stage + kBkCap;               // [L]: positions (MODE 0) / accumulators (MODE 1)
  const uint32_t ngroups = (n_tiles + kTiles - 1) / kTiles;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t k0 = threadIdx.x * KPT;
  uint32_t key[kBkRounds], pay[kBkRounds], tot[KPT], cst[KPT];
  auto chunk_rows = [&](uint32_t c0, uint32_t cl, uint32_t Q, bool abs) {
    bk_gather<MODE>(out1, s_pre, s_src, c0, cl, Q, key, pay);
    for (uint32_t i = threadIdx.x; i < (kBkWaves / 2) * Lr; i += kBkThreads) lds[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r)
      if (w * Q + r * 64 + lane < cl && r * 64 < Q)
        atomicAdd((uint32_t *)&rows16[w * Lr + (key[r] & ~1u)], 1u << ((key[r] & 1u) << 4));
    __syncthreads();
    bk_keys<KPT>(rows16, L, Lr, abs, s_wsum, tot, cst);
    __syncthreads();
  };
  auto place = [&](uint32_t cl, uint32_t Q, auto &&dst) {
#pragma unroll
    for (uint32_t r = 0; r < kBkRounds; ++r) {
      if (r * 64 < Q) {
        const bool ok = w * Q + r * 64 + lane < cl;
        const uint32_t k = key[r];
        const uint64_t peers = bk_match(k, s, __ballot(ok));
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t p0 = rows16[w * Lr + k];
        if (ok && rank == 0) rows16[w * Lr + k] = (uint16_t)(p0 + (uint32_t)__popcll(peers));
        if (ok) dst(k, p0 + rank, pay[r]);
      }
    }
    __syncthreads();
  };
  if (MODE == 0) {
    for (uint32_t i = threadIdx.x; i < L; i += kBkThreads) cnt[i] = 0;
    uint32_t base = 0, startsum = 0;
    for (uint32_t g = 0; g < ngroups; ++g) {  // pass A: per-key counts
      const uint2 rt = bk_load_runs<MODE>(tab, n_tiles, B, b, g, base, s_pre, s_src, s_wsum);
      __syncthreads();
      startsum += rt.y;
      for (uint32_t c0 = base; c0 < base + rt.x; c0 += kBkCap) {
        const uint32_t cl = min(kBkCap, base + rt.x - c0);
        const uint32_t Q = ((cl + kBkWaves * 64 - 1) / (kBkWaves * 64)) * 64;
        bk_gather<MODE>(out1, s_pre, s_src, c0, cl, Q, key, pay);
#pragma unroll
        for (uint32_t r = 0; r < kBkRounds; ++r)
          if (r * 64 < Q && w * Q + r * 64 + lane < cl) atomicAdd(&cnt[key[r]], 1u);
      }
      base += rt.x;
      __syncthreads();
    }
    {  // bucket offsets and the per-key outputs
      uint32_t sum = 0;
      if (k0 < L)
#pragma unroll
        for (int i = 0; i < KPT; ++i) sum += cnt[k0 + i];
      uint2 all;
      uint32_t run = startsum + block_excl_scan2<kBkWaves>(make_uint2(sum, 0), s_wsum, &all).x;
      if (k0 < L)
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
          const uint32_t kk = b * L + k0 + i, c = cnt[k0 + i];
          if (kk < n_keys && cell_size) {
            cell_size[kk] = c;
            cell_offset[kk] = run;
          }
          cnt[k0 + i] = run;
          run += c;
        }
      __syncthreads();
    }
    base = 0;
    for (uint32_t g = 0; g < ngroups; ++g) {  // pass B: placement
      const uint2 rt = bk_load_runs<MODE>(tab, n_tiles, B, b, g, base, s_pre, s_src, s_wsum);
      __syncthreads();
      for (uint32_t c0 = base; c0 < base + rt.x; c0 += kBkCap) {
        const uint32_t cl = min(kBkCap, base + rt.x - c0);
        const uint32_t Q = ((cl + kBkWaves * 64 - 1) / (kBkWaves * 64)) * 64;
        chunk_rows(c0, cl, Q, false);
        place(cl, Q, [&](uint32_t k, uint32_t pos, uint32_t v) { sample_idx[cnt[k] + pos] = v; });
        if (k0 < L)
#pragma unroll
          for (int i = 0; i < KPT; ++i) cnt[k0 + i] += tot[i];
        __syncthreads();
      }
      base += rt.x;
    }
    return;
  }
  for (uint32_t i = threadIdx.x; i < L; i += kBkThreads) {
    const uint32_t kk = b * L + i;
    cnt[i] = kk < n_keys ? __float_as_uint(target[kk]) : 0u;
  }
  uint32_t base = 0;
  for (uint32_t g = 0; g < ngroups; ++g) {
    const uint2 rt = bk_load_runs<MODE>(tab, n_tiles, B, b, g, base, s_pre, s_src, s_wsum);
    __syncthreads();
    for (uint32_t c0 = base; c0 < base + rt.x; c0 += kBkCap) {
      const uint32_t cl = min(kBkCap, base + rt.x - c0);
      const uint32_t Q = ((cl + kBkWaves * 64 - 1) / (kBkWaves * 64)) * 64;
      chunk_rows(c0, cl, Q, true);
      place(cl, Q, [&](uint32_t, uint32_t pos, uint32_t v) { stage[pos] = v; });
      if (k0 < L)
#pragma unroll
        for (int i = 0; i < KPT; ++i) {
          float acc = __uint_as_float(cnt[k0 + i]);
          for (uint32_t m = cst[i]; m < cst[i] + tot[i]; ++m) acc = sr_apply(op, acc, __uint_as_float(stage[m]));
          cnt[k0 + i] = __float_as_uint(acc);
        }
      __syncthreads();
    }
    base += rt.x;
  }
  for (uint32_t i = threadIdx.x; i < L; i += kBkThreads) {
    const uint32_t kk = b * L + i;
    if (kk < n_keys) target[kk] = __uint_as_float(cnt[i]);
  }
}

template <int MODE, int KPT>
__global__ __launch_bounds__(kBkThreads) void k_bucket_slow(const typename SplitCfg<MODE>::Rec *__restrict__ out1,
                                                            const uint32_t *__restrict__ tab, uint32_t n_tiles, int s,
                                                            int top, uint32_t n_keys, uint32_t nb,
                                                            uint32_t *__restrict__ cell_size,
                                                            uint32_t *__restrict__ cell_offset,
                                                            uint32_t *__restrict__ sample_idx,
                                                            float *__restrict__ target, int op,
                                                            const uint32_t *__restrict__ list) {
  constexpr uint32_t kTiles = SplitCfg<MODE>::Tiles;
  extern __shared__ uint32_t lds[];
  __shared__ uint32_t s_wsum[2][kBkWaves];
  __shared__ uint32_t s_pre[kTiles + 1], s_src[kTiles];
  const uint32_t n_work = list ? list[0] : nb;
  for (uint32_t item = blockIdx.x; item < n_work; item += gridDim.x) {
    bk_slow_one<MODE, KPT>(out1, tab, n_tiles, s, top, n_keys, list ? list[1 + item] : item, cell_size, cell_offset,
                           sample_idx, target, op, lds, s_wsum, s_pre, s_src);
    __syncthreads();
  }
}

// Keys >= 2^24 after the LSD passes (keys sorted): fold every run into its
// target (reductions.py:53 in ascending element order).
__global__ void k_sorted_fold(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ sorted, uint64_t n,
                              float *__restrict__ target, int op) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t t = keys[k];
  if (k > 0 && keys[k - 1] == t) return;  // not a run start
  float acc = target[t];
  for (uint64_t m = k; m < n && keys[m] == t; ++m) acc = sr_apply(op, acc, __uint_as_float(sorted[m]));
  target[t] = acc;
}

// Self-check of the lane-ordered LDS atomic property the RANK kernels use, in
// their exact access pattern: per-wave rows of u16 counters packed two per
// word (digits d and d^1 share a word), up to 4096 digits, random keys with
// 2..4096 distinct values per wave instruction (many same-word collisions).
// Counts returns whose u16 half differs from (first return of the key + number
// of lower lanes with the same key).
__global__ __launch_bounds__(512) void k_lds_order_probe(uint32_t seed, uint32_t *bad) {
  __shared__ uint32_t cnt[8][2048];  // [wave][4096 digits / 2]
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  for (uint32_t i = lane; i < 2048; i += 64) cnt[w][i] = 0;
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t x = seed ^ (blockIdx.x * 7919u + threadIdx.x * 104729u);
  constexpr uint32_t kinds[6] = {2u, 3u, 16u, 64u, 512u, 4096u};
  for (int r = 0; r < 60; ++r) {  // <= 60 * 64 increments per digit: no u16 carry
    x = x * 1664525u + 1013904223u;
    const uint32_t K = kinds[r % 6];
    const uint32_t k = (x >> 8) % K;
    const uint32_t sh = (k & 1u) << 4;
    const uint32_t old = (atomicAdd(&cnt[w][k >> 1], 1u << sh) >> sh) & 0xFFFFu;
    const uint64_t m = ms_match(k, 12, ~0ull);
    const uint32_t base = __shfl(old, __ffsll((unsigned long long)m) - 1);
    if (old != base + (uint32_t)__popcll(m & lt)) atomicAdd(bad, 1u);
  }
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

// The same passes from a read-only input into `out`, with `tmp` as the
// ping-pong partner: the LDS pass writes whichever of the two makes the
// last global pass land in `out` (device-pointer entry points: the caller's
// input is not clobbered and no copy-back is needed).
int scan_f32_hs_to(const float *in, float *out, float *tmp, uint64_t n, hipStream_t st) {
  if (n == 0) return MTX_OK;
  int passes = 0;
  while ((1ull << passes) < n) ++passes;
  const int local = passes < kHsLog ? passes : kHsLog;
  const int global = passes - local;
  float *x = (global & 1) ? tmp : out, *y = (global & 1) ? out : tmp;
  hipLaunchKernelGGL(k_hs_local, dim3(nblk(n, kHsTile)), dim3(256), 0, st, in, x, n, local);
  for (int i = local; i < passes; ++i) {
    hipLaunchKernelGGL(k_hs_pass, dim3(nblk(n, 256)), dim3(256), 0, st, x, y, n, 1ull << i);
    float *t = x;
    x = y;
    y = t;
  }
  return MTX_OK;
}

static int bits_for(uint64_t k) {
  int b = 0;
  while (b < 32 && (1ull << b) < k) ++b;
  return b;
}

// Workspace carving (256-B aligned pieces).
namespace {
struct Carve {
  char *base;
  size_t off = 0;
  template <class T>
  T *take(uint64_t count) {
    off = (off + 255) & ~(size_t)255;
    T *r = (T *)(base + off);
    off += count * sizeof(T);
    return r;
  }
};

struct GbPlan {
  int bits;      // key bits
  bool msd;      // two-level path (bits <= 24)
  int top, s;    // two-level: tile-table digit bits (3..12), bucket-local key bits
  uint32_t tiles;  // LSD tiles
};

GbPlan gb_plan(uint64_t n, uint64_t n_keys) {
  GbPlan g;
  g.bits = bits_for(n_keys);
  g.msd = g.bits <= 2 * kSplitMaxTop;
  g.top = g.bits < 3 ? 3 : (g.bits > kSplitMaxTop ? kSplitMaxTop : g.bits);
  g.s = g.bits > g.top ? g.bits - g.top : 0;
  g.tiles = (uint32_t)((n + kMsTile - 1) / kMsTile);
  return g;
}

template <int MODE>
uint32_t split_tiles(uint64_t n) {
  return (uint32_t)((n + SplitCfg<MODE>::T - 1) / SplitCfg<MODE>::T);
}

// two-level: digit table, level-1 records, (MODE 1) the placed values;
// LSD: digit histogram + scan + two key/payload buffer pairs.
template <int MODE>
size_t gb_bytes(uint64_t n, uint64_t n_keys, const GbPlan &g) {
  size_t bytes = 8 * 1025 + 256;
  if (g.msd) {
    bytes += 4 * ((uint64_t)split_tiles<MODE>(n) << g.top) + 256;
    bytes += sizeof(typename SplitCfg<MODE>::Rec) * n + 256;
    bytes += 4 * ((n_keys >> g.s) + 2) + 256;  // level-2 slow-bucket list
  } else {
    const uint64_t hn = ((uint64_t)1 << kMsMaxBits) * g.tiles;
    bytes += 2 * (4 * hn + 256) + scan_workspace_bytes(hn) + 256 + 4 * (4 * n + 256);
  }
  return bytes;
}

template <int MODE>
uint32_t split_lds(int top) {
  return (16u << top) + (uint32_t)(SplitCfg<MODE>::T * sizeof(typename SplitCfg<MODE>::Rec));
}
uint32_t bucket_lds(int s, bool slow) {
  const uint32_t Lr = s ? 1u << s : 2u;
  return 2u * kBkWaves * Lr + 4u * kBkCap + (slow ? 4u << s : 0u);
}

// One-time check per device that same-address LDS atomics of a wave return
// in ascending lane order (observed on gfx950; not a documented guarantee):
// the RANK kernels rely on it, the ballot-match kernels do not.
bool lds_lane_order(hipStream_t st) {
  static std::atomic<int> state[64];  // 0 unknown, 1 holds, 2 fails (a racing first call probes twice: same answer)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  const int known = state[dev].load(std::memory_order_acquire);
  if (known) return known == 1;
  const char *env = getenv("MTX_LDS_RANK");  // "0": always the ballot-match kernels
  if (env && env[0] == '0') {
    state[dev].store(2, std::memory_order_release);
    return false;
  }
  uint32_t *d_bad = nullptr, bad = 1;
  if (hipMalloc(&d_bad, 4) == hipSuccess) {
    if (hipMemsetAsync(d_bad, 0, 4, st) == hipSuccess) {
      hipLaunchKernelGGL(k_lds_order_probe, dim3(256), dim3(512), 0, st, 12345u, d_bad);
      if (hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        bad = 1;
    }
    hipFree(d_bad);
  }
  state[dev].store(bad == 0 ? 1 : 2, std::memory_order_release);
  return bad == 0;
}

int gb_attrs() {  // per call: the attribute belongs to the current device
  const int place = kMsWaves * (4 << kMsMaxBits);
  if (hipFuncSetAttribute((const void *)k_ms_place<true>, hipFuncAttributeMaxDynamicSharedMemorySize, place) ||
      hipFuncSetAttribute((const void *)k_ms_place<false>, hipFuncAttributeMaxDynamicSharedMemorySize, place) ||
      hipFuncSetAttribute((const void *)k_tile_split<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)split_lds<0>(kSplitMaxTop)) ||
      hipFuncSetAttribute((const void *)k_tile_split<1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)split_lds<1>(kSplitMaxTop)) ||
      hipFuncSetAttribute((const void *)k_tile_split<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)split_lds<0>(kSplitMaxTop)) ||
      hipFuncSetAttribute((const void *)k_tile_split<1, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)split_lds<1>(kSplitMaxTop))) {
    mtx_set_error("group-by: LDS attribute rejected");
    return MTX_E_HIP;
  }
  return MTX_OK;
}

// Level 1 launch: persistent k_tile_split, as many workgroups as fit on the
// device at once (at most one per tile).
template <int MODE>
void tile_split_launch(const uint32_t *keys, const float *value, uint64_t n, int s, int top, uint32_t tiles,
                       uint32_t *tab, typename SplitCfg<MODE>::Rec *out1, uint32_t *slow, hipStream_t st) {
  const bool rank = lds_lane_order(st);
  const uint32_t lds = split_lds<MODE>(top);
  int dev = 0, ncu = 256, per = 1;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  auto kern = rank ? k_tile_split<MODE, true> : k_tile_split<MODE, false>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 512, lds) != hipSuccess || per < 1) per = 1;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, (uint64_t)ncu * (uint32_t)per);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, keys, value, n, s, top, tiles, tab, out1, slow);
}

// Level 2 for 2^s local keys: k_bucket_fast over every bucket, then
// k_bucket_slow over the buckets it listed (long buckets); with more tiles
// than one level-2 group, k_bucket_slow over every bucket.
template <int MODE, int KPT>
int bk_launch_k(const typename SplitCfg<MODE>::Rec *out1, const uint32_t *tab, uint32_t tiles, int s, int top,
                uint32_t n_keys, uint32_t *cs, uint32_t *co, uint32_t *si, float *tgt, int op, uint32_t *slow,
                hipStream_t st) {
  const bool rank = lds_lane_order(st);
  const uint32_t nb = (uint32_t)(((uint64_t)n_keys + (1ull << s) - 1) >> s);
  const int lf = (int)bucket_lds(s, false), ls = (int)bucket_lds(s, true);
  if (hipFuncSetAttribute((const void *)k_bucket_fast<MODE, KPT, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          lf) ||
      hipFuncSetAttribute((const void *)k_bucket_fast<MODE, KPT, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          lf) ||
      hipFuncSetAttribute((const void *)k_bucket_slow<MODE, KPT>, hipFuncAttributeMaxDynamicSharedMemorySize, ls)) {
    mtx_set_error("group-by: LDS attribute rejected");
    return MTX_E_HIP;
  }
  if (tiles <= SplitCfg<MODE>::Tiles) {
    if (rank)
      hipLaunchKernelGGL((k_bucket_fast<MODE, KPT, true>), dim3(nb), dim3(kBkThreads), lf, st, out1, tab, tiles, s,
                         top, n_keys, nb, cs, co, si, tgt, op, slow);
    else
      hipLaunchKernelGGL((k_bucket_fast<MODE, KPT, false>), dim3(nb), dim3(kBkThreads), lf, st, out1, tab, tiles, s,
                         top, n_keys, nb, cs, co, si, tgt, op, slow);
    hipLaunchKernelGGL((k_bucket_slow<MODE, KPT>), dim3(nb < 256u ? nb : 256u), dim3(kBkThreads), ls, st, out1, tab,
                       tiles, s, top, n_keys, nb, cs, co, si, tgt, op, (const uint32_t *)slow);
  } else {
    hipLaunchKernelGGL((k_bucket_slow<MODE, KPT>), dim3(nb), dim3(kBkThreads), ls, st, out1, tab, tiles, s, top,
                       n_keys, nb, cs, co, si, tgt, op, (const uint32_t *)nullptr);
  }
  return MTX_OK;
}
template <int MODE>
int bk_launch(const typename SplitCfg<MODE>::Rec *out1, const uint32_t *tab, uint32_t tiles, int s, int top,
              uint32_t n_keys, uint32_t *cs, uint32_t *co, uint32_t *si, float *tgt, int op, uint32_t *slow,
              hipStream_t st) {
  const uint32_t L = 1u << s, kpt = L > (uint32_t)kBkThreads ? L / kBkThreads : 1u;
  switch (kpt) {
    case 1: return bk_launch_k<MODE, 1>(out1, tab, tiles, s, top, n_keys, cs, co, si, tgt, op, slow, st);
    case 2: return bk_launch_k<MODE, 2>(out1, tab, tiles, s, top, n_keys, cs, co, si, tgt, op, slow, st);
    case 4: return bk_launch_k<MODE, 4>(out1, tab, tiles, s, top, n_keys, cs, co, si, tgt, op, slow, st);
    case 8: return bk_launch_k<MODE, 8>(out1, tab, tiles, s, top, n_keys, cs, co, si, tgt, op, slow, st);
    default: return bk_launch_k<MODE, 16>(out1, tab, tiles, s, top, n_keys, cs, co, si, tgt, op, slow, st);
  }
}

// One stable multisplit pass (LSD path): histogram (of keys, or of the
// hash-grid cells computed from the points when hp != nullptr), scan, place.
struct HashIn {
  const float *p;
  uint32_t res, n_cells;
  const float2 *bbox;
};
int ms_pass(const uint32_t *keys, const uint32_t *pay, uint64_t n, int shift, int bits, uint32_t tiles,
            uint32_t *hist, uint32_t *hscan, void *scan_ws, uint32_t *keys_out, uint32_t *pay_out,
            const HashIn *hp, uint32_t *cell, hipStream_t st) {
  const uint64_t hn = ((uint64_t)1 << bits) * tiles;
  if (hp)
    hipLaunchKernelGGL(k_ms_hist<true>, dim3(tiles), dim3(kMsThreads), 4u << bits, st, nullptr, hp->p, n, hp->res,
                       hp->n_cells, hp->bbox, cell, shift, bits, hist, tiles);
  else
    hipLaunchKernelGGL(k_ms_hist<false>, dim3(tiles), dim3(kMsThreads), 4u << bits, st, keys, nullptr, n, 0u, 1u,
                       nullptr, nullptr, shift, bits, hist, tiles);
  int rc = scan_u32(hist, hscan, hn, 0, scan_ws, st);
  if (rc) return rc;
  const uint32_t lds = (uint32_t)kMsWaves * (4u << bits);
  if (hp)
    hipLaunchKernelGGL(k_ms_place<true>, dim3(tiles), dim3(kMsThreads), lds, st, cell, nullptr, n, shift, bits, hscan,
                       tiles, keys_out, pay_out);
  else if (!pay)
    hipLaunchKernelGGL(k_ms_place<true>, dim3(tiles), dim3(kMsThreads), lds, st, keys, nullptr, n, shift, bits, hscan,
                       tiles, keys_out, pay_out);
  else
    hipLaunchKernelGGL(k_ms_place<false>, dim3(tiles), dim3(kMsThreads), lds, st, keys, pay, n, shift, bits, hscan,
                       tiles, keys_out, pay_out);
  return MTX_OK;
}
}  // namespace

size_t hashgrid_workspace_bytes(uint64_t n, uint32_t n_cells) { return gb_bytes<0>(n, n_cells, gb_plan(n, n_cells)); }


int hashgrid_build(const float *p, uint64_t n, uint32_t res, uint32_t n_cells, uint32_t *cell, uint32_t *cell_size,
                   uint32_t *cell_offset, uint32_t *sample_idx, void *ws, hipStream_t st) {
  if (int e = gb_attrs()) return e;
  const GbPlan g = gb_plan(n, n_cells);
  Carve cv{(char *)ws};
  float2 *partial = cv.take<float2>(1025);
  const int m = 1024;
  hipLaunchKernelGGL(k_minmax, dim3(m), dim3(256), 0, st, p, 3 * n, partial);
  if (!g.msd) hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(256), 0, st, partial, m);
  if (g.msd) {
    // cells; level 1: per-tile stable split by the top digit; level 2: buckets
    const uint32_t tiles = split_tiles<0>(n);
    uint32_t *tab = cv.take<uint32_t>((uint64_t)tiles << g.top);
    uint32_t *out1 = cv.take<uint32_t>(n);
    uint32_t *slow = cv.take<uint32_t>(1 + (((uint64_t)n_cells + (1ull << g.s) - 1) >> g.s));
    const uint32_t hb = (uint32_t)std::min<uint64_t>(nblk(n, 256), 2048);  // 8 blocks per CU
    hipLaunchKernelGGL(k_hash_cells, dim3(hb), dim3(256), 0, st, p, n, res, n_cells, partial, m, cell);
    tile_split_launch<0>(cell, nullptr, n, g.s, g.top, tiles, tab, out1, slow, st);
    return bk_launch<0>(out1, tab, tiles, g.s, g.top, n_cells, cell_size, cell_offset, sample_idx, nullptr, 0, slow,
                        st);
  }
  // LSD: 12-bit digit passes (the first one hashes), then the run bounds
  const uint64_t hn = ((uint64_t)1 << kMsMaxBits) * g.tiles;
  uint32_t *hist = cv.take<uint32_t>(hn), *hscan = cv.take<uint32_t>(hn);
  void *scan_ws = cv.take<char>(scan_workspace_bytes(hn));
  uint32_t *ka = cv.take<uint32_t>(n), *pa = cv.take<uint32_t>(n), *kb = cv.take<uint32_t>(n),
           *pb = cv.take<uint32_t>(n);
  const HashIn hin{p, res, n_cells, partial + m};
  const uint32_t *kin = nullptr, *pin = nullptr;
  uint32_t *kbuf[2] = {ka, kb}, *pbuf[2] = {pa, pb};
  int cur = 0, rc;
  for (int shift = 0; shift < g.bits; shift += kMsMaxBits) {
    const int bits = g.bits - shift < kMsMaxBits ? g.bits - shift : kMsMaxBits;
    const bool last = shift + kMsMaxBits >= g.bits;
    uint32_t *pout = last ? sample_idx : pbuf[cur];
    if ((rc = ms_pass(kin, pin, n, shift, bits, g.tiles, hist, hscan, scan_ws, kbuf[cur], pout,
                      shift == 0 ? &hin : nullptr, cell, st)))
      return rc;
    kin = kbuf[cur];
    pin = pout;
    cur ^= 1;
  }
  if ((uint64_t)n_cells > 4 * n)
    hipLaunchKernelGGL(k_hash_offsets_search, dim3(nblk(n_cells, 256)), dim3(256), 0, st, kin, n, n_cells,
                       cell_offset, cell_size);
  else
    hipLaunchKernelGGL(k_hash_ranges, dim3(nblk(n, kHashTile)), dim3(256), 0, st, kin, n, n_cells, cell_offset,
                       cell_size);
  return MTX_OK;
}

// Device-side key check of mtx_group_by_u32_dev: *bad becomes non-zero when
// any key is >= n_keys (one ballot per wave, one store by the wave's first
// lane; no kernel reads a key out of range afterwards).
__global__ __launch_bounds__(256) void k_keys_in_range(const uint32_t *__restrict__ keys, uint64_t n, uint32_t n_keys,
                                                       uint32_t *bad) {
  bool any = false;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull)
    any = any || keys[i] >= n_keys;
  if (__ballot(any) != 0 && (threadIdx.x & 63u) == 0) *bad = 1u;
}
int keys_in_range(const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *bad, hipStream_t st) {
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_keys_in_range, dim3((unsigned)(blocks < 4096 ? (blocks ? blocks : 1) : 4096)), dim3(256), 0, st,
                     keys, n, n_keys, bad);
  return MTX_OK;
}

// Stable group-by of n keys < n_keys (the hash grid's machinery without the
// hashing): key_size, exclusive key_offset and order (element indices grouped
// by key, ascending index inside a key).
int group_by_u32(const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size, uint32_t *key_offset,
                 uint32_t *order, void *ws, hipStream_t st) {
  if (int e = gb_attrs()) return e;
  const GbPlan g = gb_plan(n, n_keys);
  Carve cv{(char *)ws};
  cv.take<float2>(1025);
  if (g.msd) {
    const uint32_t tiles = split_tiles<0>(n);
    uint32_t *tab = cv.take<uint32_t>((uint64_t)tiles << g.top);
    uint32_t *out1 = cv.take<uint32_t>(n);
    uint32_t *slow = cv.take<uint32_t>(1 + (((uint64_t)n_keys + (1ull << g.s) - 1) >> g.s));
    tile_split_launch<0>(keys, nullptr, n, g.s, g.top, tiles, tab, out1, slow, st);
    return bk_launch<0>(out1, tab, tiles, g.s, g.top, n_keys, key_size, key_offset, order, nullptr, 0, slow, st);
  }
  const uint64_t hn = ((uint64_t)1 << kMsMaxBits) * g.tiles;
  uint32_t *hist = cv.take<uint32_t>(hn), *hscan = cv.take<uint32_t>(hn);
  void *scan_ws = cv.take<char>(scan_workspace_bytes(hn));
  uint32_t *ka = cv.take<uint32_t>(n), *pa = cv.take<uint32_t>(n), *kb = cv.take<uint32_t>(n),
           *pb = cv.take<uint32_t>(n);
  const uint32_t *kin = keys, *pin = nullptr;
  uint32_t *kbuf[2] = {ka, kb}, *pbuf[2] = {pa, pb};
  int cur = 0, rc;
  for (int shift = 0; shift < g.bits; shift += kMsMaxBits) {
    const int bits = g.bits - shift < kMsMaxBits ? g.bits - shift : kMsMaxBits;
    const bool last = shift + kMsMaxBits >= g.bits;
    uint32_t *pout = last ? order : pbuf[cur];
    if ((rc = ms_pass(kin, pin, n, shift, bits, g.tiles, hist, hscan, scan_ws, kbuf[cur], pout, nullptr, nullptr,
                      st)))
      return rc;
    kin = kbuf[cur];
    pin = pout;
    cur ^= 1;
  }
  if ((uint64_t)n_keys > 4 * n)
    hipLaunchKernelGGL(k_hash_offsets_search, dim3(nblk(n_keys, 256)), dim3(256), 0, st, kin, n, n_keys, key_offset,
                       key_size);
  else
    hipLaunchKernelGGL(k_hash_ranges, dim3(nblk(n, kHashTile)), dim3(256), 0, st, kin, n, n_keys, key_offset,
                       key_size);
  return MTX_OK;
}

size_t sort24_workspace_bytes(uint64_t n) { return gb_bytes<0>(n, 1u << 24, gb_plan(n, 1u << 24)); }

// Stable sort permutation of n keys < 2^24 (the hash grid's two levels
// without the per-key outputs): perm[i] = index of the i-th smallest key.
int sort24(const uint32_t *keys, uint64_t n, uint32_t *perm, void *ws, hipStream_t st) {
  if (n == 0) return MTX_OK;
  if (int e = gb_attrs()) return e;
  const GbPlan g = gb_plan(n, 1u << 24);
  Carve cv{(char *)ws};
  cv.take<float2>(1025);
  const uint32_t tiles = split_tiles<0>(n);
  uint32_t *tab = cv.take<uint32_t>((uint64_t)tiles << g.top);
  uint32_t *out1 = cv.take<uint32_t>(n);
  uint32_t *slow = cv.take<uint32_t>(1 + ((1ull << 24) >> g.s));
  tile_split_launch<0>(keys, nullptr, n, g.s, g.top, tiles, tab, out1, slow, st);
  return bk_launch<0>(out1, tab, tiles, g.s, g.top, 1u << 24, nullptr, nullptr, perm, nullptr, 0, slow, st);
}

size_t scatter_workspace_bytes(uint64_t n_target, uint64_t n_value) {
  return gb_bytes<1>(n_value, n_target, gb_plan(n_value, n_target));
}

int scatter_reduce_f32(int op, float *target, uint64_t n_target, const float *value, const uint32_t *index,
                       uint64_t n_value, void *ws, hipStream_t st) {
  if (int e = gb_attrs()) return e;
  const uint64_t n = n_value;
  const GbPlan g = gb_plan(n, n_target);
  Carve cv{(char *)ws};
  cv.take<float2>(1025);
  if (g.msd) {
    const uint32_t tiles = split_tiles<1>(n);
    uint32_t *tab = cv.take<uint32_t>((uint64_t)tiles << g.top);
    uint2 *out1 = cv.take<uint2>(n);
    uint32_t *slow = cv.take<uint32_t>(1 + ((n_target + (1ull << g.s) - 1) >> g.s));
    tile_split_launch<1>(index, value, n, g.s, g.top, tiles, tab, out1, slow, st);
    return bk_launch<1>(out1, tab, tiles, g.s, g.top, (uint32_t)n_target, nullptr, nullptr, nullptr, target, op, slow,
                        st);
  }
  const uint64_t hn = ((uint64_t)1 << kMsMaxBits) * g.tiles;
  uint32_t *hist = cv.take<uint32_t>(hn), *hscan = cv.take<uint32_t>(hn);
  void *scan_ws = cv.take<char>(scan_workspace_bytes(hn));
  uint32_t *ka = cv.take<uint32_t>(n), *pa = cv.take<uint32_t>(n), *kb = cv.take<uint32_t>(n),
           *pb = cv.take<uint32_t>(n);
  const uint32_t *kin = index, *pin = (const uint32_t *)value;
  uint32_t *kbuf[2] = {ka, kb}, *pbuf[2] = {pa, pb};
  int cur = 0, rc;
  for (int shift = 0; shift < g.bits; shift += kMsMaxBits) {
    const int bits = g.bits - shift < kMsMaxBits ? g.bits - shift : kMsMaxBits;
    if ((rc = ms_pass(kin, pin, n, shift, bits, g.tiles, hist, hscan, scan_ws, kbuf[cur], pbuf[cur], nullptr, nullptr,
                      st)))
      return rc;
    kin = kbuf[cur];
    pin = pbuf[cur];
    cur ^= 1;
  }
  hipLaunchKernelGGL(k_sorted_fold, dim3(nblk(n, 256)), dim3(256), 0, st, kin, pin, n, target, op);
  return MTX_OK;
}

}  // namespace mtxd
