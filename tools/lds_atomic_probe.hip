// LDS bit-set throughput probe (dev tool): random-address ORs into a 2048-word chunk per block, in the shapes the roaring
// decode issues them.  Modes: 0 atomicOr, 1 plain RMW (racy), 2 plain store, 3 atomicOr under a divergent branch
// (~60 % of lanes), 4 as 3 plus an LDS read used after every 8 ORs (lgkmcnt waits on the ORs), 5 as 0 with 36 KB of LDS
// per block (4 blocks per CU, the index kernel's residency).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t iters) {
  __shared__ uint32_t ch[MODE == 5 ? 9216 : 2048];
  __shared__ uint32_t aux[256];
  for (int i = threadIdx.x; i < 2048; i += 256) ch[i] = 0;
  aux[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x, s = 0;
  for (uint32_t i = 0; i < iters; i++) {
    x = x * 1664525u + 1013904223u;
    const uint32_t w = (x >> 16) & 2047u, b = 1u << (x & 31u);
    if (MODE == 0 || MODE == 5) atomicOr(&ch[w], b);
    else if (MODE == 1) ch[w] |= b;
    else if (MODE == 2) ch[w] = b;
    else {
      if ((x >> 8) % 10u < 6u) atomicOr(&ch[w], b);
      if (MODE == 4 && (i & 7u) == 7u) s += aux[(s + x) & 255u];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 256) s ^= ch[i];
  atomicXor(out, s);
}
int main() {
  uint32_t* o;
  if (hipMalloc(&o, 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t iters = 4096, blocks = 256 * 8;
  for (int m = 0; m < 6; m++) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(a);
      switch (m) {
        case 0: k<0><<<blocks, 256>>>(o, iters); break;
        case 1: k<1><<<blocks, 256>>>(o, iters); break;
        case 2: k<2><<<blocks, 256>>>(o, iters); break;
        case 3: k<3><<<blocks, 256>>>(o, iters); break;
        case 4: k<4><<<blocks, 256>>>(o, iters); break;
        default: k<5><<<blocks, 256>>>(o, iters); break;
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double ops = (double)blocks * 256 * iters * (m == 3 || m == 4 ? 0.6 : 1.0);
      if (rep) printf("mode %d: %.3f ms, %.2f lane-ops/cycle/CU (2.4 GHz)\n", m, ms, ops / (ms * 1e-3 * 2.4e9) / 256);
    }
  }
  return 0;
}
