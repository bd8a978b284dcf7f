// Probe: do same-address LDS atomics of one wave instruction return their
// old values in ascending lane order? (answers whether ds_add_rtn could rank
// equal keys stably). Random key patterns with many collisions; prints the
// number of violations.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_probe(const unsigned *keys, unsigned *bad, int rounds, int nkeys) {
  __shared__ unsigned cnt[8][256];
  const unsigned w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = lane; i < 256; i += 64) cnt[w][i] = 0;
  __syncthreads();
  for (int r = 0; r < rounds; ++r) {
    const unsigned k = keys[(blockIdx.x * rounds + r) * blockDim.x + threadIdx.x] % nkeys;
    const unsigned old = atomicAdd(&cnt[w][k], 1u);
    // expected: number of lower lanes with the same key (+ previous rounds)
    unsigned long long m = 0;
    for (int j = 0; j < 8; ++j) {
      const unsigned bit = (k >> j) & 1u;
      const unsigned long long bal = __ballot(bit);
      m = j ? (m & (bit ? bal : ~bal)) : (bit ? bal : ~bal);
    }
    const unsigned rank = __popcll(m & ((1ull << lane) - 1));
    const unsigned total = __popcll(m);
    // previous value is the same for all peers: recover it from the leader
    const unsigned leader = __ffsll((long long)m) - 1;
    const unsigned base = __shfl(old, leader);
    if (old != base + rank) atomicAdd(bad, 1u);
    (void)total;
  }
}

int main() {
  const int blocks = 2048, threads = 512, rounds = 64;
  const size_t n = (size_t)blocks * threads * rounds;
  unsigned *h = (unsigned *)malloc(n * 4);
  srand(1);
  for (size_t i = 0; i < n; ++i) h[i] = (unsigned)rand();
  unsigned *dk, *dbad, bad = 0;
  hipMalloc(&dk, n * 4);
  hipMalloc(&dbad, 4);
  hipMemcpy(dk, h, n * 4, hipMemcpyHostToDevice);
  const int nk[] = {1, 2, 4, 16, 64, 256};
  for (int t = 0; t < 6; ++t) {
    hipMemset(dbad, 0, 4);
    hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(threads), 0, 0, dk, dbad, rounds, nk[t]);
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("keys %3d: %u violations of lane-order returns over %zu atomics\n", nk[t], bad, n);
  }
  return 0;
}
