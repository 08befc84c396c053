// Probe: can config 4's DISTINCTCOUNT state be aggregated by global atomics on a cache-resident state slice?
// (VERDICT r05 "next" #3, option 1: level-1 partitions OR-ed straight into a per-XCD state slice.)
// Measures no-return 32-bit global atomicOr at random word addresses (one bit per doc, as the value-bitmap update
// would be) over footprints from an L2-sized slice per XCD up to the full 1.28 GB state, 2^30 atomics per launch
// (config 4's doc count).  xcd = 1: each XCD's blocks (blockIdx % 8) address only their own slice of the footprint.
// Build: hipcc --offload-arch=gfx950 -O3 tools/l2_atomic_probe.hip -o tools/l2_atomic_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                       \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } \
  } while (0)

__global__ __launch_bounds__(256) void or_probe(uint32_t* state, uint32_t slice_words, uint32_t per_thread, int xcd) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x = gtid * 2654435761u + 0x9E3779B9u;
  const uint32_t base = xcd ? (blockIdx.x & 7u) * slice_words : 0u;
  const uint32_t span = xcd ? slice_words : 8u * slice_words;
  for (uint32_t i = 0; i < per_thread; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    // word index from the lane's own random stream (never wave-uniform): vector atomics only
    atomicOr(&state[base + (x % span)], 1u << (x >> 27));
  }
}

// the same addresses with plain loads (a gather of the footprint at the same rate of requests) for comparison
__global__ __launch_bounds__(256) void load_probe(const uint32_t* state, uint32_t slice_words, uint32_t per_thread,
                                                  int xcd, uint32_t* sink) {
  const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x = gtid * 2654435761u + 0x9E3779B9u, acc = 0;
  const uint32_t base = xcd ? (blockIdx.x & 7u) * slice_words : 0u;
  const uint32_t span = xcd ? slice_words : 8u * slice_words;
  for (uint32_t i = 0; i < per_thread; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    acc += state[base + (x % span)];
  }
  if (acc == 0x12345678u) sink[gtid & 1023u] = acc;
}

int main() {
  const uint64_t total = 1ull << 30;
  const uint32_t threads = 256, blocks = 256 * 8;  // 8 blocks of 256 threads per CU
  const uint32_t per_thread = (uint32_t)(total / ((uint64_t)threads * blocks));
  const uint64_t footprints_mb[] = {16, 32, 64, 256, 1280};
  uint32_t* state;
  uint32_t* sink;
  CK(hipMalloc(&state, 1280ull << 20));
  CK(hipMalloc(&sink, 4096));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (uint64_t mb : footprints_mb) {
    const uint32_t slice_words = (uint32_t)((mb << 20) / 4 / 8);
    for (int xcd = 0; xcd < 2; xcd++) {
      for (int kind = 0; kind < 2; kind++) {
        CK(hipMemset(state, 0, mb << 20));
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
          CK(hipEventRecord(a));
          if (kind == 0) hipLaunchKernelGGL(or_probe, dim3(blocks), dim3(threads), 0, 0, state, slice_words, per_thread, xcd);
          else hipLaunchKernelGGL(load_probe, dim3(blocks), dim3(threads), 0, 0, state, slice_words, per_thread, xcd, sink);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (ms < best) best = ms;
        }
        printf("{\"op\": \"%s\", \"footprint_MB\": %llu, \"per_xcd_slice_MB\": %.1f, \"xcd_local\": %d, "
               "\"ops\": %llu, \"ms\": %.3f, \"Gops_per_s\": %.1f}\n",
               kind ? "load" : "atomic_or", (unsigned long long)mb, xcd ? mb / 8.0 : (double)mb, xcd,
               (unsigned long long)total, best, total / (best * 1e6));
        fflush(stdout);
      }
    }
  }
  CK(hipFree(state));
  CK(hipFree(sink));
  return 0;
}
