// ta_rate.hip — vector-memory (TA/TCP) issue cost of wave64 gathers on gfx950,
// by address pattern: how many cycles one global_load costs a CU when the
// 64 lanes hit 1, 16 or 64 distinct 128-B lines, L1- or L2-resident, 4/8/16-B
// per lane; and a scalar (s_load) fetch of the same 64 B for comparison.
// Informs the traversal's node-fetch design. Standalone:
//   hipcc --offload-arch=gfx950 -O3 ta_rate.hip -o ta_rate && ./ta_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

constexpr int kIters = 4096;

// PAT: 0 all lanes one address, 1 four lanes per 64-B node, 16 nodes in 16
// lines, 2 one line per lane (64 lines), 3 coalesced (lane-contiguous),
// 4 one line per lane, lanes of a 4-lane group read the 4 16-B parts of one
// 64-B node (16 nodes, 8 lines). W: bytes per lane (4, 8, 16).
template <int PAT, int W, int ACTIVE = 64>
__global__ __launch_bounds__(256) void k_gather(const uint4 *__restrict__ buf, uint32_t mask16, uint4 *out) {
  const uint32_t lane = threadIdx.x & 63u;
  if (lane >= (uint32_t)ACTIVE) return;  // partial waves: exec mask of the first ACTIVE lanes
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t acc = 0;
  uint32_t base = wave * 1021u;
#pragma unroll 8
  for (int i = 0; i < kIters; ++i) {
    uint32_t idx;  // in 16-B units
    if (PAT == 0) idx = base;
    else if (PAT == 1) idx = base + (lane >> 2) * 8u;
    else if (PAT == 2) idx = base + lane * 8u;
    else if (PAT == 3) idx = base + lane;
    else idx = base + (lane >> 2) * 4u + (lane & 3u);
    idx &= mask16;
    if (W == 16) {
      const uint4 v = buf[idx];
      acc += v.x ^ v.y ^ v.z ^ v.w;
    } else if (W == 8) {
      const uint2 v = reinterpret_cast<const uint2 *>(buf)[2 * idx];
      acc += v.x ^ v.y;
    } else {
      acc += reinterpret_cast<const uint32_t *>(buf)[4 * idx];
    }
    base += 8u * 67u;
  }
  if (acc == 0x12345678u) out[0] = make_uint4(acc, 0, 0, 0);
}

// scalar fetch of a 64-B node per iteration (wave-uniform address)
__global__ __launch_bounds__(256) void k_scalar(const uint4 *__restrict__ buf, uint32_t mask16, uint4 *out) {
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t acc = 0;
  uint32_t base = __builtin_amdgcn_readfirstlane(wave * 1021u);
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(4))) u4v *cb = (const __attribute__((address_space(4))) u4v *)buf;
#pragma unroll 8
  for (int i = 0; i < kIters; ++i) {
    const uint32_t idx = (base & mask16) & ~3u;
    const u4v a = cb[idx], b = cb[idx + 1], c = cb[idx + 2], d = cb[idx + 3];
    acc += a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x;
    base += 8u * 67u;
  }
  acc += threadIdx.x;
  if (acc == 0x12345678u) out[0] = make_uint4(acc, 0, 0, 0);
}

template <class K>
static float run(K kern, const uint4 *buf, uint32_t mask16, uint4 *out, int grid, hipEvent_t e0, hipEvent_t e1) {
  kern<<<grid, 256>>>(buf, mask16, out);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) kern<<<grid, 256>>>(buf, mask16, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 3.f;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const double ghz = p.clockRate / 1e6;
  const size_t bytes = 64ull << 20;
  uint4 *buf, *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 16));
  CK(hipMemset(buf, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = ncu * 8;  // 8 x 256 threads = 32 waves / CU
  const double waves_per_cu = grid * 4.0 / ncu;
  printf("CUs %d, clock %.2f GHz (reported), %d waves, %d loads per wave\n", ncu, ghz, grid * 4, kIters);
  printf("%-28s %-10s %10s %14s\n", "pattern", "footprint", "ms", "CU-cycles/load");
  struct Fp {
    const char *name;
    uint32_t mask16;
  } fps[] = {{"16KB(L1)", (16u << 10) / 16 - 1}, {"2MB(L2)", (2u << 20) / 16 - 1}, {"64MB", (64u << 20) / 16 - 1}};
  auto report = [&](const char *name, const Fp &f, float ms) {
    const double cyc = ms * 1e-3 * ghz * 1e9 / (waves_per_cu * kIters);
    printf("%-28s %-10s %10.3f %14.2f\n", name, f.name, ms, cyc);
  };
  for (const Fp &f : fps) {
    report("x16 same address", f, run(k_gather<0, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 16 nodes/16 lines", f, run(k_gather<1, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 64 lines", f, run(k_gather<2, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 coalesced (8 lines)", f, run(k_gather<3, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 4 lanes/node (8 lines)", f, run(k_gather<4, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x8 64 lines", f, run(k_gather<2, 8>, buf, f.mask16, out, grid, e0, e1));
    report("x4 64 lines", f, run(k_gather<2, 4>, buf, f.mask16, out, grid, e0, e1));
    report("x4 same address", f, run(k_gather<0, 4>, buf, f.mask16, out, grid, e0, e1));
    report("x8 16 lines", f, run(k_gather<1, 8>, buf, f.mask16, out, grid, e0, e1));
    report("scalar 64-B node (4 x s_load_x4)", f, run(k_scalar, buf, f.mask16, out, grid, e0, e1));
    report("x16 coalesced, 48 lanes", f, run(k_gather<3, 16, 48>, buf, f.mask16, out, grid, e0, e1));
    report("x16 coalesced, 16 lanes", f, run(k_gather<3, 16, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 same address, 16 lanes", f, run(k_gather<0, 16, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 64 lines, 48 lanes", f, run(k_gather<2, 16, 48>, buf, f.mask16, out, grid, e0, e1));
    report("x16 64 lines, 16 lanes", f, run(k_gather<2, 16, 16>, buf, f.mask16, out, grid, e0, e1));
    report("x16 16 lines, 16 lanes", f, run(k_gather<1, 16, 16>, buf, f.mask16, out, grid, e0, e1));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
