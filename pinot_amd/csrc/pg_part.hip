// pg_part.hip -- radix-partitioned dense group-by of libpinot_gpu (gfx950): the device form of
// DictionaryBasedGroupKeyGenerator + the DISTINCTCOUNT / COUNT result holders for key spaces whose group state is far
// larger than any cache (config 4: 10 M userId groups x a 1 000-bit itemId value set = 1.36 GB of state).
//
// Reference per-doc work (query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:384-463 IntMapBasedHolder
// -> DefaultGroupByExecutor.aggregate -> DistinctCountAggregationFunction.aggregateGroupBySV, :131-190: one
// RoaringBitmap add per doc in the group's holder) is a random update of a huge table.  On MI355X a global atomic
// executes at the memory side (MI355X_MICROARCH.md, Global atomics), so one random atomic per doc runs at the
// atomic rate, not at HBM bandwidth (r02_v1: 90.7 ms for 1 B docs).  Instead the docs are radix-partitioned by key
// with plain, coalescable stores and each bucket is aggregated in LDS:
//
//   scan pass 1 (pg_scan.hip, GM_PART_COUNT)   per (level-1 partition, block): matched-doc counts   (LDS atomics)
//   exclusive scan                              -> every block's private range of every partition
//   scan pass 2 (GM_PART_SCATTER)               32-bit entry (key low bits | value id) per matched doc, appended
//                                               to its block's range of its partition (LDS-atomic cursor)
//   part_count2 / exclusive scan / part_scatter2   the same one level down: kPartNB blocks per level-1 partition
//   part_aggregate                              one workgroup per bucket of 2^shift2 groups: count + value bitmap
//                                               in LDS (LDS atomics), then the bucket's rows of the dense state
//                                               written once, coalesced (every slot, so no state memset is needed)
//
// Bytes per matched doc: key + value columns once per scan pass (the key column twice), then 4 B written / 4 B read
// per level, + the state rows once.  No global atomics anywhere; no MFMA (nothing is a contraction).
#include <hip/hip_runtime.h>

#include "pg_internal.h"

namespace pg {

// Entries of level-1 partition p handled by level-2 block j (of kPartNB): [lo, hi).
__device__ __forceinline__ void l2_range(const PartSpec& P, uint32_t p, uint32_t j, uint64_t& lo, uint64_t& hi) {
  const uint64_t s = P.off1[(uint64_t)p * P.blocks1], e = P.off1[(uint64_t)(p + 1) * P.blocks1];
  const uint64_t n = e - s;
  lo = s + n * j / kPartNB;
  hi = s + n * (j + 1) / kPartNB;
}

// Level-2 digit of an entry: key bits [shift2, shift1) (the entry keeps the key below the level-1 digit).
__device__ __forceinline__ uint32_t digit2(const PartSpec& P, uint32_t e) {
  return (e >> (P.vbits + P.shift2)) & (P.nparts2 - 1u);
}

// Counts of the level-2 digits in block (j, p)'s range -> hist2[(p * nparts2 + digit) * kPartNB + j].
__global__ __launch_bounds__(256) void part_count2_kernel(PartSpec P) {
  extern __shared__ uint32_t h[];  // [nparts2]
  const uint32_t j = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
  for (uint32_t i = tid; i < P.nparts2; i += 256) h[i] = 0;
  __syncthreads();
  uint64_t lo, hi;
  l2_range(P, p, j, lo, hi);
  const uint32_t* __restrict__ in = P.in1;
  uint64_t i = lo + tid;
  for (; i + 768 < hi; i += 1024) {  // four independent loads in flight per lane
    const uint32_t e0 = in[i], e1 = in[i + 256], e2 = in[i + 512], e3 = in[i + 768];
    atomicAdd(&h[digit2(P, e0)], 1u);
    atomicAdd(&h[digit2(P, e1)], 1u);
    atomicAdd(&h[digit2(P, e2)], 1u);
    atomicAdd(&h[digit2(P, e3)], 1u);
  }
  for (; i < hi; i += 256) atomicAdd(&h[digit2(P, in[i])], 1u);
  __syncthreads();
  for (uint32_t d = tid; d < P.nparts2; d += 256) P.hist2[((uint64_t)p * P.nparts2 + d) * kPartNB + j] = h[d];
}

// The same ranges again: every entry to its block's next position of its bucket (offsets = exclusive scan of hist2).
__global__ __launch_bounds__(256) void part_scatter2_kernel(PartSpec P) {
  extern __shared__ uint32_t cur[];  // [nparts2]
  const uint32_t j = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
  for (uint32_t d = tid; d < P.nparts2; d += 256)
    cur[d] = (uint32_t)P.off2[((uint64_t)p * P.nparts2 + d) * kPartNB + j];
  __syncthreads();
  uint64_t lo, hi;
  l2_range(P, p, j, lo, hi);
  const uint32_t* __restrict__ in = P.in1;
  uint32_t* __restrict__ out = P.out2;
  uint64_t i = lo + tid;
  for (; i + 768 < hi; i += 1024) {
    const uint32_t e0 = in[i], e1 = in[i + 256], e2 = in[i + 512], e3 = in[i + 768];
    out[atomicAdd(&cur[digit2(P, e0)], 1u)] = e0;
    out[atomicAdd(&cur[digit2(P, e1)], 1u)] = e1;
    out[atomicAdd(&cur[digit2(P, e2)], 1u)] = e2;
    out[atomicAdd(&cur[digit2(P, e3)], 1u)] = e3;
  }
  for (; i < hi; i += 256) {
    const uint32_t e = in[i];
    out[atomicAdd(&cur[digit2(P, e)], 1u)] = e;
  }
}

// One workgroup per bucket b (groups g = b << shift2 | gl): doc count and value bitmap of each group in LDS, then the
// bucket's slice of the dense state (i64 slot 0 = doc count, the bitmap row) written whole.
__global__ __launch_bounds__(256) void part_aggregate_kernel(PartSpec P) {
  extern __shared__ uint32_t lds[];
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  const uint32_t ng = 1u << P.shift2, dw = P.dc_words;
  uint32_t* cnt = lds;        // [ng]
  uint32_t* bm = lds + ng;    // [ng][dw]
  for (uint32_t i = tid; i < ng * (1u + dw); i += 256) lds[i] = 0;
  __syncthreads();
  const uint64_t lo = P.off2[(uint64_t)b * kPartNB], hi = P.off2[(uint64_t)(b + 1) * kPartNB];
  const uint32_t gm = ng - 1u, vm = (1u << P.vbits) - 1u, vb = P.vbits;
  const uint32_t* __restrict__ in = P.out2;
  uint64_t i = lo + tid;
  if (dw) {
    for (; i + 256 < hi; i += 512) {
      const uint32_t e0 = in[i], e1 = in[i + 256];
      const uint32_t g0 = (e0 >> vb) & gm, v0 = e0 & vm, g1 = (e1 >> vb) & gm, v1 = e1 & vm;
      atomicAdd(&cnt[g0], 1u);
      atomicOr(&bm[g0 * dw + (v0 >> 5)], 1u << (v0 & 31u));
      atomicAdd(&cnt[g1], 1u);
      atomicOr(&bm[g1 * dw + (v1 >> 5)], 1u << (v1 & 31u));
    }
    for (; i < hi; i += 256) {
      const uint32_t e = in[i];
      const uint32_t g = (e >> vb) & gm, v = e & vm;
      atomicAdd(&cnt[g], 1u);
      atomicOr(&bm[g * dw + (v >> 5)], 1u << (v & 31u));
    }
  } else {
    for (; i < hi; i += 256) atomicAdd(&cnt[(in[i] >> vb) & gm], 1u);
  }
  __syncthreads();
  const uint64_t g0 = (uint64_t)b << P.shift2;
  const uint32_t n = (uint32_t)(g0 + ng <= P.num_groups ? ng : (g0 < P.num_groups ? P.num_groups - g0 : 0));
  for (uint32_t gl = tid; gl < n; gl += 256) P.i64[(g0 + gl) * P.n_i64] = cnt[gl];
  if (P.row_words) {
    const uint32_t rw = P.row_words;
    uint32_t* __restrict__ dst = P.bits + g0 * rw;
    for (uint32_t w = tid; w < n * rw; w += 256) {
      const uint32_t gl = w / rw, k = w - gl * rw;
      dst[w] = (k >= P.dc_word && k < P.dc_word + dw) ? bm[gl * dw + (k - P.dc_word)] : 0u;
    }
  }
}

hipError_t launch_part_count2(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_count2_kernel, dim3(kPartNB, p.nparts1), dim3(256), p.nparts2 * 4, s, p);
  return hipGetLastError();
}
hipError_t launch_part_scatter2(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_scatter2_kernel, dim3(kPartNB, p.nparts1), dim3(256), p.nparts2 * 4, s, p);
  return hipGetLastError();
}
hipError_t launch_part_aggregate(const PartSpec& p, hipStream_t s) {
  const size_t lds = (size_t)(1u << p.shift2) * (1u + p.dc_words) * 4u;
  hipLaunchKernelGGL(part_aggregate_kernel, dim3(p.nparts1 * p.nparts2), dim3(256), lds, s, p);
  return hipGetLastError();
}

}  // namespace pg
