// pg_index.hip -- the fused index count (gfx950): COUNT / COUNTMV under a filter made only of index leaves.
//
// The reference answers such a query per segment with BitmapBasedFilterOperator (the OR of the selected dictIds'
// RoaringBitmaps, filter/BitmapBasedFilterOperator.java:66-155), SortedIndexBasedFilterOperator (doc ranges),
// AndFilterOperator / OrFilterOperator / NotFilterOperator over their doc id sets (AndDocIdSet.java:60-150,
// OrDocIdSet.java:58-114) and CountMVAggregationFunction over the matching docs' value counts
// (CountMVAggregationFunction.java:64-95).  The general device path materialises each inverted leaf as a doc bitmap in
// HBM (roaring_keys_kernel) and scans those bitmaps tile by tile (pg_scan.hip).  Here one workgroup owns one 64 K-doc
// key of a segment's doc range: it decodes every inverted leaf's containers of that key into an 8 KB LDS chunk
// (pg_roaring.h), evaluates the filter on the chunk words together with the doc-range and constant leaves, counts the
// matching docs and adds their value counts from a 4-bit count column -- the only HBM bytes are the containers and
// directory entries the leaves select and the count words of the matched docs.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pg_aux.h"
#include "pg_roaring.h"
#if PG_IDX_PROF
#include <cstdio>
#include <cstring>
#endif

namespace pg {

#ifndef PG_IDX_NT
#define PG_IDX_NT 256
#endif
constexpr int kIdxNT = PG_IDX_NT;  // threads per (segment, key) block
static_assert(kIdxNT % 64 == 0 && 2048 % kIdxNT == 0 && kIdxNT <= 1024, "whole waves, whole chunk words per thread");

// docs [a, b) of a 32-doc word (bit 31 - j <-> doc j), clamped to the word
__device__ __forceinline__ uint32_t word_range(int64_t a, int64_t b) {
  a = a < 0 ? 0 : a;
  b = b > 32 ? 32 : b;
  if (a >= b) return 0u;
  const uint32_t hi = a >= 32 ? 0u : (0xFFFFFFFFu >> (uint32_t)a);
  const uint32_t lo = b >= 32 ? 0u : (0xFFFFFFFFu >> (uint32_t)b);
  return hi & ~lo;
}

#if PG_IDX_PROF
// per-block sums of thread 0's phase cycles: 0 setup, 1-4 the decode's phases (pg_roaring.h), 5 filter + count,
// 6 reduce; 7 block wall-clock ticks (start to end); g_idx_span: min start, max end of the launch (wall clock)
__device__ unsigned long long g_idx_prof[8], g_idx_span[2];
#endif

#ifndef PG_IDX_LATE_COUNT  // 1: the count words are loaded after the decode (32 fewer VGPRs held across it)
#define PG_IDX_LATE_COUNT 1
#endif
#ifndef PG_IDX_WAVES
#define PG_IDX_WAVES 4  // waves per SIMD the register budget is cut for (4: <= 128 VGPRs)
#endif
__global__ __launch_bounds__(kIdxNT, PG_IDX_WAVES) void index_count_kernel(IdxSpec p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t chunks[];  // [num_chunks][2048]
  __shared__ RoaringLds<kIdxNT> S;
  __shared__ RoarView V[kIdxMaxLeaves];
  __shared__ uint4 D[kIdxMaxLeaves];  // leaf l for the filter: (kind | negate << 8, lo, hi, chunk word offset)
  __shared__ uint32_t nv;
  __shared__ unsigned long long red[2][kIdxNT / 64];
  static_assert(kIdxMaxLeaves <= kRoarMaxViews && kIdxMaxLeaves <= 64, "one view per inverted leaf");
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_ = PG_IDX_PROF ? prof_clk() : 0ull;
  const unsigned long long w0 = PG_IDX_PROF ? wall_clock64() : 0ull;
  // the block's segment from the host's block -> segment table (one load), then its descriptor and its leaves' (in
  // parallel: the leaves are [segment][leaf] in one array)
  const uint32_t si = ld_global(p.blk_seg + blockIdx.x);
  const IdxSeg G = ld_global(p.segs + si);
  IdxLeaf L{};
  if (tid < p.num_leaves) L = ld_global(p.leaves + (uint64_t)si * p.num_leaves + tid);
  const uint32_t key = G.key0 + (blockIdx.x - G.first_block);
  const uint32_t nd = G.num_docs;
  // COUNTMV from the 4-bit count column: this thread's count words of all its chunk words are loaded up front, before
  // the decode (they do not depend on it: one latency hidden under the directory loads; most words hold a match at
  // config 5's 5.6 % pass).  Unconditional loads (a word past the segment reads word 0): a select between a load and
  // zero would wait for the load right here.
  constexpr uint32_t kWpt = 2048u / kIdxNT;
  uint4 cwp[kWpt];
#pragma unroll
  for (uint32_t k = 0; k < kWpt; k++) cwp[k] = make_uint4(0u, 0u, 0u, 0u);
  auto load_counts = [&]() {
    if (p.cntmv_slot != 0xFFFFFFFFu && G.mv_cnt && !(PG_IDX_SKIP & 8)) {
#pragma unroll
      for (uint32_t k = 0; k < kWpt; k++) {
        const uint64_t d0 = (uint64_t)key * 65536u + 32u * (tid + k * kIdxNT);
        cwp[k] = ld_global((const uint4*)(G.mv_cnt + (d0 < nd ? d0 / 8 : 0)));
      }
    }
  };
  if (!PG_IDX_LATE_COUNT) load_counts();
  for (uint32_t w = tid; w < p.num_chunks * 512u; w += kIdxNT) ((uint4*)chunks)[w] = make_uint4(0u, 0u, 0u, 0u);
  // every inverted leaf of the segment, decoded together into its chunk: the views compacted by wave 0
  if (tid < 64) {
    const bool on = tid < p.num_leaves && L.kind == IL_ROARING && L.nids;
    const unsigned long long b = __ballot(on);
    if (on) {
      const uint32_t at = (uint32_t)__popcll(b & ((1ull << tid) - 1ull));
      V[at] = RoarView{L.roaring, L.cs, L.dir, L.keydir, L.ids, p.chunk_of[tid] * 2048u, L.nids, L.card};
    }
    if (tid < p.num_leaves)
      D[tid] = make_uint4(L.kind | L.negate << 8, (uint32_t)L.lo, (uint32_t)L.hi,
                          L.kind == IL_ROARING ? p.chunk_of[tid] * 2048u : 0u);
    if (tid == 0) nv = (uint32_t)__popcll(b);
  }
  lds_barrier();
  if (PG_IDX_PROF && tid == 0) { const unsigned long long n_ = prof_clk(); prof[0] += n_ - t_; t_ = n_; }
  roaring_key_chunks<kIdxNT>(V, nv, key, S, chunks, PG_IDX_PROF ? prof : nullptr);
  if (PG_IDX_PROF && tid == 0) t_ = prof_clk();
  if (PG_IDX_LATE_COUNT) load_counts();
  // the filter over this thread's kWpt chunk words at once: wave-uniform loops over the (at most two-level) item list,
  // each leaf's descriptor read once per item (an LDS broadcast), not once per word
  const int64_t dbase = (int64_t)key * 65536 + 32 * (int64_t)tid;  // doc of word 0's bit 31; word k: + 32 k NT
  auto leafw = [&](uint32_t l, uint32_t* out) {
    const uint4 d = D[l];
    const uint32_t kind = d.x & 0xFFu;
    if (kind == IL_ROARING) {
      const uint32_t neg = (d.x >> 8) ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (uint32_t k = 0; k < kWpt; k++) out[k] = chunks[d.w + tid + k * kIdxNT] ^ neg;
    } else if (kind == IL_DOCRANGE) {
#pragma unroll
      for (uint32_t k = 0; k < kWpt; k++) {
        const int64_t d0 = dbase + 32 * (int64_t)(k * kIdxNT);
        out[k] = word_range((int64_t)(int32_t)d.y - d0, (int64_t)(int32_t)d.z - d0);
      }
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kWpt; k++) out[k] = kind == IL_ALL ? 0xFFFFFFFFu : 0u;
    }
  };
  uint32_t m[kWpt];
#pragma unroll
  for (uint32_t k = 0; k < kWpt; k++) m[k] = p.root_or ? 0u : 0xFFFFFFFFu;
  for (uint32_t i = 0; i < p.num_items; i++) {
    const uint32_t it = p.item[i];
    uint32_t v[kWpt];
    if (it & 0x40000000u) {
      const uint32_t g = it & 0xFFu;
      const bool gor = p.group_or[g] != 0;
#pragma unroll
      for (uint32_t k = 0; k < kWpt; k++) v[k] = gor ? 0u : 0xFFFFFFFFu;
      for (uint32_t j = 0; j < p.gn[g]; j++) {
        const uint32_t gl = p.gleaf[p.gfirst[g] + j];
        uint32_t x[kWpt];
        leafw(gl & 0xFFu, x);
        const uint32_t neg = (gl & 0x80000000u) ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (uint32_t k = 0; k < kWpt; k++) v[k] = gor ? (v[k] | (x[k] ^ neg)) : (v[k] & (x[k] ^ neg));
      }
    } else {
      leafw(it & 0xFFu, v);
    }
    const uint32_t neg = (it & 0x80000000u) ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kWpt; k++) m[k] = p.root_or ? (m[k] | (v[k] ^ neg)) : (m[k] & (v[k] ^ neg));
  }
  unsigned long long cnt = 0, cmv = 0;
#pragma unroll
  for (uint32_t k = 0; k < kWpt; k++) {
    const uint64_t d0 = (uint64_t)key * 65536u + 32u * (tid + k * kIdxNT);
    const uint32_t valid = d0 >= nd ? 0u : d0 + 32 <= nd ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (uint32_t)(nd - d0));
    const uint32_t mk = m[k] & valid;
    cnt += (uint32_t)__popc(mk);
    if (p.cntmv_slot != 0xFFFFFFFFu && mk && !(PG_IDX_SKIP & 8)) {
      if (G.mv_cnt) {  // 4-bit counts: docs d0 .. d0 + 31 are the 4 count words at d0 / 8
        // count word q holds docs 8 q + j at nibble 7 - j; mask byte (mk >> 24 - 8 q) holds them at bit 7 - j: spread
        // the byte's bit i to nibble i, mask the counts with it, add the nibbles (no per-doc loop, no divergence)
        const uint4 cw = cwp[k];
        const uint32_t c4[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          uint32_t x = (mk >> (24u - 8u * q)) & 0xFFu;
          x = (x | (x << 12)) & 0x000F000Fu;
          x = (x | (x << 6)) & 0x03030303u;
          x = (x | (x << 3)) & 0x11111111u;
          const uint32_t v = c4[q] & (x * 15u);
          const uint32_t b = (v & 0x0F0F0F0Fu) + ((v >> 4) & 0x0F0F0F0Fu);
          cmv += (b * 0x01010101u) >> 24;
        }
      } else {
        for (uint32_t r = mk; r; ) {
          const uint32_t j = (uint32_t)__builtin_clz(r);
          r &= ~(0x80000000u >> j);
          cmv += ld_global(G.mv_offsets + d0 + j + 1) - ld_global(G.mv_offsets + d0 + j);
        }
      }
    }
  }
  if (PG_IDX_PROF && tid == 0) { const unsigned long long n_ = prof_clk(); prof[5] += n_ - t_; t_ = n_; }
  // block sums -> one atomic per value
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_down(cnt, o);
    cmv += __shfl_down(cmv, o);
  }
  if (lane == 0) { red[0][wave] = cnt; red[1][wave] = cmv; }
  lds_barrier();
  if (tid == 0) {
    unsigned long long c = 0, v = 0;
    for (uint32_t k = 0; k < kIdxNT / 64; k++) { c += red[0][k]; v += red[1][k]; }
    if (c) {
      atomicAdd(&p.i64[0], c);
      atomicAdd(&p.seg_matched[si], c);
      if (p.cntmv_slot != 0xFFFFFFFFu) atomicAdd(&p.i64[p.cntmv_slot], v);
    }
  }
#if PG_IDX_PROF
  if (tid == 0) {
    prof[6] += prof_clk() - t_;
    const unsigned long long w1 = wall_clock64();
    prof[7] = w1 - w0;
    for (int i = 0; i < 8; i++) atomicAdd(&g_idx_prof[i], prof[i]);
    atomicMax(&g_idx_span[0], ~w0);
    atomicMax(&g_idx_span[1], w1);
  }
#endif
}

hipError_t launch_index_count(const IdxSpec& p, uint32_t blocks, hipStream_t s) {
  if (!blocks) return hipSuccess;
#ifndef PG_IDX_LDS_PAD  // dev: extra dynamic LDS per block (fewer blocks per CU: the contention experiment)
#define PG_IDX_LDS_PAD 0
#endif
  const size_t lds = (size_t)p.num_chunks * 2048 * 4 + PG_IDX_LDS_PAD;
  if (lds > 64 * 1024) {
    static bool attr = false;  // > 64 KiB of dynamic LDS is opted into once per process
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)index_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)std::min<size_t>(kIdxMaxLeaves * 2048 * 4 + PG_IDX_LDS_PAD, 160 * 1024 - 12 * 1024));
      attr = true;
    }
  }
  hipLaunchKernelGGL(index_count_kernel, dim3(blocks), dim3(kIdxNT), lds, s, p);
#if PG_IDX_PROF
  {
    unsigned long long h[8], sp[2];
    int khz = 0;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    if (hipDeviceSynchronize() == hipSuccess && hipMemcpyFromSymbol(h, HIP_SYMBOL(g_idx_prof), sizeof(h)) == hipSuccess &&
        hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_idx_span), sizeof(sp)) == hipSuccess) {
      fprintf(stderr, "[idx_prof] blocks=%u lds=%zu per-block kcycles:", blocks, lds);
      for (int i = 0; i < 7; i++) fprintf(stderr, " %.2f", h[i] / 1e3 / (double)blocks);
      fprintf(stderr, " | block us %.2f | span us %.2f\n", h[7] / (double)blocks / (khz / 1e3),
              (double)(sp[1] - ~sp[0]) / (khz / 1e3));
      memset(h, 0, sizeof(h));
      memset(sp, 0, sizeof(sp));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_idx_prof), h, sizeof(h));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_idx_span), sp, sizeof(sp));
    }
  }
#endif
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ the count column

// word w <- docs 8w .. 8w + 7, doc 8w + j in bits [28 - 4j, 32 - 4j): the 4-bit packed column order
__global__ void mv_counts_kernel(const uint32_t* __restrict__ off, uint32_t num_docs, uint32_t* __restrict__ out,
                                 unsigned int* over) {
  const uint32_t nw = (num_docs + 7) / 8 + 4;  // + 4 zero words: a 16-byte read at the last doc word stays inside
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
    uint32_t v = 0;
    bool big = false;
    for (uint32_t j = 0; j < 8; j++) {
      const uint32_t d = 8 * w + j;
      const uint32_t c = d < num_docs ? off[d + 1] - off[d] : 0u;
      big |= c > 15u;
      v |= (c > 15u ? 15u : c) << (28u - 4u * j);
    }
    out[w] = v;
    if (big) atomicOr(over, 1u);
  }
}

hipError_t launch_mv_counts(const uint32_t* offsets, uint32_t num_docs, uint32_t* out, unsigned int* over, hipStream_t s) {
  const uint32_t nw = (num_docs + 7) / 8 + 4;
  const uint32_t blocks = (nw + 255) / 256 < 4096 ? (nw + 255) / 256 : 4096;
  hipLaunchKernelGGL(mv_counts_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, s, offsets, num_docs, out, over);
  return hipGetLastError();
}

}  // namespace pg
