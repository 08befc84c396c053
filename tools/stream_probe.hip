// stream_probe.hip -- dev micro-benchmark (not product code): how fast can one gfx950 kernel stream a bit-packed
// column and test each value against an IN-set?  The config-2 driving leaf: accountId, 20 bits/value, 1 B values
// (2.5 GB), IN (1 000 ids) over a 1 M dictionary, tested through a 16 KB LDS bitmap over dictId >> 3 (+ the exact
// LUT for candidates).  Variants:
//   A<R>  per-doc 64-bit window loads (buffer_load_dwordx2), interleaved docs (lane l of a wave: doc base + j*64 + l),
//         R docs per lane in flight per batch
//   D<K>  LDS-DMA staging of 8192-doc tiles (1 KiB pieces), ring of K buffers (K-1 tiles in flight per block)
//   C     thread-contiguous 32 docs, dwordx4 loads to registers, bit width a template parameter
// Every variant writes the number of matches; all must agree.
// build: hipcc --offload-arch=gfx950 -O3 -o stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                  \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t B = 20;
constexpr uint32_t SHIFT = 3;
constexpr uint32_t NBW = ((1u << 20) >> SHIFT) / 32 + 1;  // filter bitmap words

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}

__global__ void fill_kernel(uint32_t* w, uint64_t nwords) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x)
    w[i] = hash32((uint32_t)i * 2654435761u + 17u);
}

__device__ __forceinline__ void load_set(uint32_t* lds, const uint32_t* g) {
  for (uint32_t i = threadIdx.x; i < NBW; i += blockDim.x) lds[i] = g[i];
  __syncthreads();
}
__device__ __forceinline__ uint32_t test(const uint32_t* bm, const uint32_t* lut, uint32_t v) {
  const uint32_t x = v >> SHIFT;
  if (!((bm[x >> 5] >> (x & 31)) & 1u)) return 0;
  return (lut[v >> 5] >> (v & 31)) & 1u;
}

// ---- A: per-doc windows
template <int R>
__global__ __launch_bounds__(256) void kA(const uint32_t* words, uint32_t wbytes, uint64_t n, const uint32_t* set,
                                          const uint32_t* lut, unsigned long long* out) {
  __shared__ uint32_t bm[NBW];
  load_set(bm, set);
  const rsrc_t r = make_rsrc(words, wbytes);
  uint32_t cnt = 0;
  const uint64_t step = (uint64_t)gridDim.x * 256 * R;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * R; base < n; base += step) {
    uint64_t win[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
      const uint64_t d = base + (uint64_t)j * 256 + threadIdx.x;
      const uint64_t p = d * B;
      const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)(p >> 5) << 2, 0, 0);
      win[j] = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
    }
#pragma unroll
    for (int j = 0; j < R; j++) {
      const uint64_t d = base + (uint64_t)j * 256 + threadIdx.x;
      const uint32_t sh = (uint32_t)(d * B) & 31u;
      const uint64_t w = (win[j] << 32) | (win[j] >> 32);  // word order: first word most significant
      const uint32_t v = (uint32_t)(w >> (64u - sh - B)) & ((1u << B) - 1u);
      if (d < n) cnt += test(bm, lut, v);
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// ---- D: LDS-DMA staging ring of K tiles of 8192 docs
template <int K>
__global__ __launch_bounds__(256) void kD(const uint32_t* words, uint32_t wbytes, uint64_t ntiles, const uint32_t* set,
                                          const uint32_t* lut, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* bm = smem;
  uint32_t* ring = smem + ((NBW + 3) & ~3u) + 4;  // +16 B: st[-1]
  load_set(bm, set);
  const rsrc_t r = make_rsrc(words, wbytes);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr uint32_t TW = 8192 / 32 * B;  // words per tile
  auto issue = [&](uint64_t tile, uint32_t slot) {
    const uint32_t tb = (uint32_t)(tile * TW * 4);
    for (uint32_t c = wave; c < B; c += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ring + slot * TW + c * 256), 16,
                                               tb + (c * 64 + lane) * 16, 0, 0, 0);
  };
  uint32_t cnt = 0;
  // tiles of this block: t = blockIdx.x + i * gridDim.x
  uint64_t t0 = blockIdx.x;
  int issued = 0;
  for (int k = 0; k < K - 1; k++)
    if (t0 + (uint64_t)k * gridDim.x < ntiles) { issue(t0 + (uint64_t)k * gridDim.x, k); issued++; }
  uint32_t slot = 0;
  for (uint64_t t = t0; t < ntiles; t += gridDim.x) {
    // wait for this tile: all but the (K-2) younger tiles' pieces of this wave
    const uint32_t mine = (B - wave + 3) / 4;  // pieces of this wave per tile
    const uint64_t later = t + (uint64_t)(K - 1) * gridDim.x;
    if (K == 2 || mine == 0) __builtin_amdgcn_s_waitcnt(0);
    else {
      // pieces younger than this tile's: (number of later tiles issued) * mine; K==3 -> at most 1 tile
      if (t + gridDim.x < ntiles) {
        if (mine == 5) __builtin_amdgcn_s_waitcnt(0x0F70 | 5);  // vmcnt(5): see gfx9 encoding (lgkm=15 exp=7)
        else __builtin_amdgcn_s_waitcnt(0x0F70 | 4);
      } else __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
    if (later < ntiles) issue(later, (slot + K - 1) % K);
    const uint32_t* st = ring + slot * TW;
#pragma unroll 8
    for (int j = 0; j < 32; j++) {
      const uint32_t rel = j * 256 + threadIdx.x;
      const uint32_t e = rel * B + B - 1;
      const uint32_t kk = e >> 5;
      const uint32_t v = __builtin_amdgcn_alignbit(st[kk - 1], st[kk], ~e) & ((1u << B) - 1u);
      cnt += test(bm, lut, v);
    }
    __syncthreads();
    slot = (slot + 1) % K;
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// ---- C: thread-contiguous 32 docs, B dwords per thread via dwordx4 (B = 20 -> 5 loads)
__global__ __launch_bounds__(256) void kC(const uint32_t* words, uint32_t wbytes, uint64_t n, const uint32_t* set,
                                          const uint32_t* lut, unsigned long long* out) {
  __shared__ uint32_t bm[NBW];
  load_set(bm, set);
  uint32_t cnt = 0;
  const uint64_t groups = n / 32;  // 32-doc groups = B words each
  for (uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x; gi < groups; gi += (uint64_t)gridDim.x * 256) {
    const uint4* p = (const uint4*)(words + gi * B);  // 80-byte groups: 16-byte aligned
    uint32_t w[B + 1];
#pragma unroll
    for (int k = 0; k < (int)B / 4; k++) {
      const uint4 x = p[k];
      w[4 * k] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
    }
    w[B] = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t s = j * B;  // first bit
      const uint32_t k = s >> 5, o = s & 31;
      const uint32_t v = (o + B <= 32) ? (w[k] >> (32 - o - B)) & ((1u << B) - 1u)
                                       : __builtin_amdgcn_alignbit(w[k], w[k + 1], 64 - o - B) & ((1u << B) - 1u);
      cnt += test(bm, lut, v);
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// ---- C variants: G groups per thread per iteration (G*5 dwordx4 loads issued before use); RANGE = no LDS test
template <int G, bool RANGE>
__global__ __launch_bounds__(256) void kCG(const uint32_t* words, uint32_t wbytes, uint64_t n, const uint32_t* set,
                                           const uint32_t* lut, unsigned long long* out) {
  __shared__ uint32_t bm[NBW];
  if (!RANGE) load_set(bm, set);
  uint32_t cnt = 0;
  const uint64_t groups = n / 32;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t g0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; g0 < groups; g0 += stride * G) {
    uint32_t w[G][B + 1];
#pragma unroll
    for (int g = 0; g < G; g++) {
      const uint64_t gi = g0 + (uint64_t)g * stride;
      const uint4* p = (const uint4*)(words + (gi < groups ? gi : 0) * B);
#pragma unroll
      for (int k = 0; k < (int)B / 4; k++) {
        const uint4 x = p[k];
        w[g][4 * k] = x.x; w[g][4 * k + 1] = x.y; w[g][4 * k + 2] = x.z; w[g][4 * k + 3] = x.w;
      }
      w[g][B] = 0;
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      if (g0 + (uint64_t)g * stride >= groups) break;
#pragma unroll
      for (int j = 0; j < 32; j++) {
        const uint32_t s = j * B;
        const uint32_t k = s >> 5, o = s & 31;
        const uint32_t v = (o + B <= 32) ? (w[g][k] >> (32 - o - B)) & ((1u << B) - 1u)
                                         : __builtin_amdgcn_alignbit(w[g][k], w[g][k + 1], 64 - o - B) & ((1u << B) - 1u);
        if (RANGE) cnt += (v - 1000u) < 4000u;
        else cnt += test(bm, lut, v);
      }
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// exact 1 M-bit bitmap in LDS (128 KiB): one 1024-thread block per CU, no candidate step
__global__ __launch_bounds__(1024) void kCX(const uint32_t* words, uint64_t n, const uint32_t* lut,
                                            unsigned long long* out) {
  extern __shared__ uint32_t ex[];
  for (uint32_t i = threadIdx.x; i < (1u << 20) / 32; i += blockDim.x) ex[i] = lut[i];
  __syncthreads();
  uint32_t cnt = 0;
  const uint64_t groups = n / 32;
  for (uint64_t gi = (uint64_t)blockIdx.x * 1024 + threadIdx.x; gi < groups; gi += (uint64_t)gridDim.x * 1024) {
    const uint4* p = (const uint4*)(words + gi * B);
    uint32_t w[B + 1];
#pragma unroll
    for (int k = 0; k < (int)B / 4; k++) {
      const uint4 x = p[k];
      w[4 * k] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
    }
    w[B] = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t s = j * B;
      const uint32_t k = s >> 5, o = s & 31;
      const uint32_t v = (o + B <= 32) ? (w[k] >> (32 - o - B)) & ((1u << B) - 1u)
                                       : __builtin_amdgcn_alignbit(w[k], w[k + 1], 64 - o - B) & ((1u << B) - 1u);
      cnt += (ex[v >> 5] >> (v & 31)) & 1u;
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// shifted LDS bitmap, candidates collected into a 32-bit mask and resolved in one batch per group
__global__ __launch_bounds__(256) void kCB(const uint32_t* words, uint64_t n, const uint32_t* set, const uint32_t* lut,
                                           unsigned long long* out) {
  __shared__ uint32_t bm[NBW];
  load_set(bm, set);
  uint32_t cnt = 0;
  const uint64_t groups = n / 32;
  for (uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x; gi < groups; gi += (uint64_t)gridDim.x * 256) {
    const uint4* p = (const uint4*)(words + gi * B);
    uint32_t w[B + 1];
#pragma unroll
    for (int k = 0; k < (int)B / 4; k++) {
      const uint4 x = p[k];
      w[4 * k] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
    }
    w[B] = 0;
    uint32_t cand = 0;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t s = j * B;
      const uint32_t k = s >> 5, o = s & 31;
      const uint32_t v = (o + B <= 32) ? (w[k] >> (32 - o - B)) & ((1u << B) - 1u)
                                       : __builtin_amdgcn_alignbit(w[k], w[k + 1], 64 - o - B) & ((1u << B) - 1u);
      const uint32_t x = v >> SHIFT;
      cand |= ((bm[x >> 5] >> (x & 31)) & 1u) << j;
    }
    while (cand) {  // rare: resolve through the exact LUT
      const uint32_t j = __ffs(cand) - 1;
      cand &= cand - 1;
      const uint32_t s = j * B, k = s >> 5, o = s & 31;
      const uint32_t v = (uint32_t)((((uint64_t)w[k] << 32) | w[k + 1]) >> (64 - o - B)) & ((1u << B) - 1u);
      cnt += (lut[v >> 5] >> (v & 31)) & 1u;
    }
  }
  atomicAdd(out, (unsigned long long)cnt);
}

// raw read bandwidth: dwordx4 loads, xor-reduce
__global__ __launch_bounds__(256) void kCopy(const uint4* p, uint64_t n16, unsigned long long* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 122070ull * 8192;
  const uint64_t nwords = (n * B + 31) / 32 + 8;
  uint32_t* words;
  CHECK(hipMalloc(&words, nwords * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, words, nwords);
  // set: 1000 ids; filter bitmap + exact lut
  std::vector<uint32_t> hb(NBW, 0), hl((1u << 20) / 32 + 1, 0);
  for (int i = 0; i < 1000; i++) {
    const uint32_t id = (uint32_t)((i * 7919 + 13) % 1000000);
    hl[id >> 5] |= 1u << (id & 31);
    const uint32_t x = id >> SHIFT;
    hb[x >> 5] |= 1u << (x & 31);
  }
  uint32_t *set, *lut;
  unsigned long long* out;
  CHECK(hipMalloc(&set, hb.size() * 4));
  CHECK(hipMalloc(&lut, hl.size() * 4));
  CHECK(hipMalloc(&out, 8));
  CHECK(hipMemcpy(set, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(lut, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
  const uint32_t wbytes = (uint32_t)std::min<uint64_t>(nwords * 4, 0xFFFFFFF0ull);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double gb = (double)n * B / 8 / 1e9;
  auto run = [&](const char* name, auto launch) {
    float best = 1e9;
    unsigned long long h = 0;
    for (int rep = 0; rep < 6; rep++) {
      CHECK(hipMemset(out, 0, 8));
      CHECK(hipEventRecord(e0));
      launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) best = std::min(best, ms);
      CHECK(hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost));
    }
    printf("%-14s %8.3f ms  %7.2f TB/s  matches %llu\n", name, best, gb / best, h);
    fflush(stdout);
  };
  const uint64_t ntiles = n / 8192;
  const uint32_t lds_bm = ((NBW + 3) & ~3u) * 4 + 16;
  CHECK(hipFuncSetAttribute((const void*)kCX, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  run("CX  1x1024", [&] { hipLaunchKernelGGL(kCX, dim3(256), dim3(1024), 131072, 0, words, n, lut, out); });
  run("CX  2x1024", [&] { hipLaunchKernelGGL(kCX, dim3(512), dim3(1024), 131072, 0, words, n, lut, out); });
  for (int bpc : {8, 16}) {
    char nm[64];
    snprintf(nm, sizeof nm, "CB  g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL(kCB, dim3(256 * bpc), dim3(256), 0, 0, words, n, set, lut, out); });
  }
  for (int bpc : {8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL(kCopy, dim3(256 * bpc), dim3(256), 0, 0, (const uint4*)words, (uint64_t)(n * B / 128), out); });
    snprintf(nm, sizeof nm, "CR1 g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL((kCG<1, true>), dim3(256 * bpc), dim3(256), 0, 0, words, wbytes, n, set, lut, out); });
    snprintf(nm, sizeof nm, "CR2 g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL((kCG<2, true>), dim3(256 * bpc), dim3(256), 0, 0, words, wbytes, n, set, lut, out); });
    snprintf(nm, sizeof nm, "C1 g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL((kCG<1, false>), dim3(256 * bpc), dim3(256), 0, 0, words, wbytes, n, set, lut, out); });
    snprintf(nm, sizeof nm, "C2 g%dx", bpc);
    run(nm, [&] { hipLaunchKernelGGL((kCG<2, false>), dim3(256 * bpc), dim3(256), 0, 0, words, wbytes, n, set, lut, out); });
  }
  return 0;
}
