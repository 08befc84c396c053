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

#include "pg_aux.h"
#include "pg_roaring.h"

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

__global__ __launch_bounds__(kIdxNT) void index_count_kernel(IdxSpec p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t chunks[];  // [num_chunks][2048]
  __shared__ RoaringLds<kIdxNT> S;
  __shared__ RoarView V[kIdxMaxLeaves];
  __shared__ uint32_t nv;
  __shared__ unsigned long long red[2][kIdxNT / 64];
  static_assert(kIdxMaxLeaves <= kRoarMaxViews, "one view per inverted leaf");
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t lo = 0, hi = p.num_segs;  // the segment whose block range holds this block
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (p.segs[mid].first_block <= blockIdx.x) lo = mid; else hi = mid;
  }
  const uint32_t si = lo;
  const IdxSeg G = p.segs[si];
  const uint32_t key = G.key0 + (blockIdx.x - G.first_block);
  for (uint32_t w = tid; w < p.num_chunks * 2048u; w += kIdxNT) chunks[w] = 0u;
  // every inverted leaf of the segment, decoded together into its chunk: leaf l's descriptor read by lane l (one
  // latency), the views compacted by wave 0
  if (tid < 64) {
    IdxLeaf L{};
    if (tid < p.num_leaves) L = G.leaves[tid];
    const bool on = tid < p.num_leaves && L.kind == IL_ROARING && L.nids;
    const unsigned long long b = __ballot(on);
    if (on) {
      const uint32_t at = (uint32_t)__popcll(b & ((1ull << tid) - 1ull));
      V[at] = RoarView{L.roaring, L.cs, L.dir, L.keydir, L.ids, chunks + p.chunk_of[tid] * 2048u, L.nids, L.card};
    }
    if (tid == 0) nv = (uint32_t)__popcll(b);
  }
  __syncthreads();
  roaring_key_chunks<kIdxNT>(V, nv, key, S);
  const uint32_t nd = G.num_docs;
  unsigned long long cnt = 0, cmv = 0;
  // COUNTMV from the 4-bit count column: this thread's count words of all its chunk words are loaded up front (one
  // latency, not one per word; most words hold a match at config 5's 5.6 % pass)
  constexpr uint32_t kWpt = 2048u / kIdxNT;
  uint4 cwp[kWpt];
  const bool pre_cnt = p.cntmv_slot != 0xFFFFFFFFu && G.mv_cnt;
#pragma unroll
  for (uint32_t k = 0; k < kWpt; k++) {
    const uint64_t d0 = (uint64_t)key * 65536u + 32u * (tid + k * kIdxNT);
    cwp[k] = pre_cnt && d0 < nd ? *(const uint4*)(G.mv_cnt + d0 / 8) : make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (uint32_t k = 0; k < kWpt; k++) {
    const uint32_t w = tid + k * kIdxNT;
    const uint64_t d0 = (uint64_t)key * 65536u + 32u * w;
    if (d0 >= nd) break;
    const uint32_t valid = d0 + 32 <= nd ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (uint32_t)(nd - d0));
    auto leaf = [&](uint32_t l) -> uint32_t {
      const IdxLeaf& L = G.leaves[l];
      switch (L.kind) {
        case IL_ALL: return 0xFFFFFFFFu;
        case IL_NONE: return 0u;
        case IL_DOCRANGE: return word_range((int64_t)L.lo - (int64_t)d0, (int64_t)L.hi - (int64_t)d0);
        default: {
          const uint32_t v = chunks[p.chunk_of[l] * 2048u + w];
          return L.negate ? ~v : v;
        }
      }
    };
    uint32_t m = p.root_or ? 0u : 0xFFFFFFFFu;
    for (uint32_t i = 0; i < p.num_items; i++) {  // wave-uniform loops over the (at most two-level) filter
      const uint32_t it = p.item[i];
      uint32_t v;
      if (it & 0x40000000u) {
        const uint32_t g = it & 0xFFu;
        v = p.group_or[g] ? 0u : 0xFFFFFFFFu;
        for (uint32_t k = 0; k < p.gn[g]; k++) {
          const uint32_t gl = p.gleaf[p.gfirst[g] + k];
          uint32_t x = leaf(gl & 0xFFu);
          if (gl & 0x80000000u) x = ~x;
          v = p.group_or[g] ? (v | x) : (v & x);
        }
      } else {
        v = leaf(it & 0xFFu);
      }
      if (it & 0x80000000u) v = ~v;
      m = p.root_or ? (m | v) : (m & v);
    }
    m &= valid;
    cnt += (uint32_t)__popc(m);
    if (p.cntmv_slot != 0xFFFFFFFFu && m) {
      if (G.mv_cnt) {  // 4-bit counts: docs d0 .. d0 + 31 are the 4 count words at d0 / 8
        const uint4 cw = cwp[k];
        const uint32_t c4[4] = {cw.x, cw.y, cw.z, cw.w};
        for (uint32_t r = m; r; ) {
          const uint32_t j = (uint32_t)__builtin_clz(r);
          r &= ~(0x80000000u >> j);
          cmv += (c4[j >> 3] >> (28u - 4u * (j & 7u))) & 15u;
        }
      } else {
        for (uint32_t r = m; r; ) {
          const uint32_t j = (uint32_t)__builtin_clz(r);
          r &= ~(0x80000000u >> j);
          cmv += G.mv_offsets[d0 + j + 1] - G.mv_offsets[d0 + j];
        }
      }
    }
  }
  // block sums -> one atomic per value
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_down(cnt, o);
    cmv += __shfl_down(cmv, o);
  }
  if (lane == 0) { red[0][wave] = cnt; red[1][wave] = cmv; }
  __syncthreads();
  if (tid == 0) {
    unsigned long long c = 0, v = 0;
    for (uint32_t k = 0; k < kIdxNT / 64; k++) { c += red[0][k]; v += red[1][k]; }
    if (c) {
      atomicAdd(&p.i64[0], c);
      atomicAdd(&p.seg_matched[si], c);
      if (p.cntmv_slot != 0xFFFFFFFFu) atomicAdd(&p.i64[p.cntmv_slot], v);
    }
  }
}

hipError_t launch_index_count(const IdxSpec& p, uint32_t blocks, hipStream_t s) {
  if (!blocks) return hipSuccess;
  const size_t lds = (size_t)p.num_chunks * 2048 * 4;
  if (lds > 64 * 1024) {
    static bool attr = false;  // > 64 KiB of dynamic LDS is opted into once per process
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)index_count_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kIdxMaxLeaves * 2048 * 4);
      attr = true;
    }
  }
  hipLaunchKernelGGL(index_count_kernel, dim3(blocks), dim3(kIdxNT), lds, s, p);
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
