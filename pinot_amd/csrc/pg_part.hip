// pg_part.hip -- radix-partitioned dense group-by of libpinot_gpu (gfx950): the device form of
// DictionaryBasedGroupKeyGenerator + the DISTINCTCOUNT / COUNT result holders for key spaces whose group state is far
// larger than any cache (config 4: 10 M userId groups x a 1 000-bit itemId value set = 1.36 GB of state).
//
// Reference per-doc work (query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:384-463 IntMapBasedHolder
// -> DefaultGroupByExecutor.aggregate -> DistinctCountAggregationFunction.aggregateGroupBySV, :131-190: one
// RoaringBitmap add per doc in the group's holder) is a random update of a huge table.  On MI355X a global atomic
// executes at the memory side (MI355X_MICROARCH.md, Global atomics), so one random atomic per doc runs at the
// atomic rate, not at HBM bandwidth (r02_v1: 90.7 ms for 1 B docs), and scattered 4-byte stores are bound by the
// request rate the same way.  So every pass here moves whole runs:
//
//   scan (pg_scan.hip, GM_PART)  one 64-bit entry (key << vbits | value id) per matched doc appended to its block's
//                                region (consecutive words per wave) + the block's level-1 histogram (LDS atomics)
//   exclusive scan               -> each block's output range in every level-1 partition
//   part_split1                  per scan block, chunks of kSplitChunk entries counting-sorted by level-1 digit in
//                                LDS, each digit's run written at once (32-bit entries: key below the digit | value)
//   part_count2 / scan / part_split2   the same one level down, kPartNB blocks per level-1 partition
//   part_aggregate               one workgroup per bucket of 2^shift2 groups: count + value bitmap in LDS (LDS
//                                atomics), then the bucket's rows of the dense state written once, coalesced (every
//                                slot is written, so the state needs no memset)
//
// No global atomics anywhere; no MFMA (nothing is a contraction).  Bytes per matched doc: the key + value columns
// once (scan) + 8 written / 8 read (scan entries) + 4 / 4 twice (levels 1, 2) + 4 read (count2) + state rows once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pg_aux.h"

namespace pg {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
#define PG_CONST __attribute__((address_space(4)))

// A wave-uniform struct read through the scalar cache (s_load: descriptors live in SGPRs, not 64 lanes' VGPRs).
template <class T> __device__ __forceinline__ T ldcf(const T* p, uint64_t i) {
  const PG_CONST uint32_t* src = (const PG_CONST uint32_t*)(p + i);
  T v;
  uint32_t* dst = (uint32_t*)&v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = src[k];
  return v;
}

#ifndef PG_SPLIT_CHUNK
#define PG_SPLIT_CHUNK 16384
#endif
#ifndef PG_SPLIT_THREADS
#define PG_SPLIT_THREADS 1024
#endif
constexpr uint32_t kST = PG_SPLIT_THREADS;  // threads of a split block
#ifndef PG_SPLIT_WAVES
#define PG_SPLIT_WAVES (PG_SPLIT_THREADS / 256)  // register budget: one resident block per CU
#endif
#ifndef PG_SPLIT2_DIG
#define PG_SPLIT2_DIG 0
#endif
#ifndef PG_AGG_THREADS
#define PG_AGG_THREADS 1024
#endif
constexpr uint32_t kAT = PG_AGG_THREADS;  // threads of a part_aggregate block
constexpr uint32_t kSplitChunk = PG_SPLIT_CHUNK;
#ifndef PG_AGG_BATCH
#define PG_AGG_BATCH 16
#endif
constexpr int kAggB = PG_AGG_BATCH;  // entries per lane per load batch of the bucket pass  // entries counting-sorted per LDS round (16 per thread): longer runs per digit
// (16 384 x 1 024 threads, one block per CU: split1 4.08 -> 3.10 ms, split2 2.71 -> 2.15 ms on config 4 vs 4 096 x 256)

// The compile-time knobs (tools/variant.sh pg_part builds variants with -D) and what they size.  split_round scans the
// digit counts with one thread per digit (<= 256 digits) in whole waves, each thread holds E = chunk / threads
// entries in registers, and the chunk's sorted entries + digits live in the kernel's static LDS next to cnt / start /
// cur; part_aggregate and part_direct stride their LDS tables by their thread counts.  A combination outside these
// bounds would index past an LDS array (the r03 sweep's illegal access came from an ablation build whose flags were
// not recorded: variant.sh now writes them next to the library).
static_assert(kST % 64 == 0 && kST >= 256 && kST <= 1024, "split blocks: whole waves, one thread per digit (<= 256)");
static_assert(kSplitChunk % kST == 0 && kSplitChunk / kST >= 1 && kSplitChunk / kST <= 32,
              "split chunk: E = chunk / threads entries per thread, held in registers");
static_assert(4ull * kSplitChunk + kSplitChunk + 2 * 4 * 256 + 8 * 256 <= 160 * 1024,
              "split1's static LDS (sorted entries + digits + cnt / start / cur) must fit a CU");
static_assert(PG_SPLIT_WAVES >= 1 && PG_SPLIT_WAVES * 256 >= kST / 4, "split register budget: >= one block per CU");
static_assert(kAT % 64 == 0 && kAT >= 64 && kAT <= 1024, "part_aggregate blocks: whole waves");
static_assert(kPartLdsBytes <= 160 * 1024, "one bucket's LDS state must fit a CU");

__device__ __forceinline__ rsrc_t part_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// ---- dev instrumentation (PG_PART_PROF=1 variant builds only: tools/variant.sh pg_part): lane 0 of every block sums
// clock64() deltas per phase in registers and adds them to g_part_prof[kernel][phase] once at its end; the launch
// functions synchronise and print the per-block averages to stderr.  Kernels: 0 part_direct, 1 split2s, 2 aggregate.
#ifndef PG_PART_PROF
#define PG_PART_PROF 0
#endif
#if PG_PART_PROF
__device__ unsigned long long g_part_prof[3][8];
#define PROF_NOW() (threadIdx.x == 0 ? (uint64_t)clock64() : 0ull)
#define PROF_LAP(acc, ph, t) do { if (threadIdx.x == 0) { const uint64_t n_ = clock64(); (acc)[ph] += n_ - (t); (t) = n_; } } while (0)
#define PROF_FLUSH(k, acc) do { if (threadIdx.x == 0) for (int i_ = 0; i_ < 8; i_++) atomicAdd(&g_part_prof[k][i_], (acc)[i_]); } while (0)
static void prof_report(const char* name, int k, uint64_t blocks) {
  unsigned long long h[3][8];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_part_prof), sizeof(h)) != hipSuccess) return;
  fprintf(stderr, "[part_prof] %s blocks=%llu per-block kcycles:", name, (unsigned long long)blocks);
  for (int i = 0; i < 8; i++) fprintf(stderr, " %.1f", h[k][i] / 1e3 / (double)blocks);
  fprintf(stderr, "\n");
  memset(h, 0, sizeof(h));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_part_prof), h, sizeof(h));
}
#else
#define PROF_NOW() 0ull
#define PROF_LAP(acc, ph, t) do { } while (0)
#define PROF_FLUSH(k, acc) do { } while (0)
#endif

// Entries of level-1 partition p handled by level-2 block j (of kPartNB): [lo, hi).
__device__ __forceinline__ void l2_range(const PartSpec& P, uint32_t p, uint32_t j, uint64_t& lo, uint64_t& hi) {
  const uint64_t s = P.off1[(uint64_t)p * P.blocks1], e = P.off1[(uint64_t)(p + 1) * P.blocks1];
  const uint64_t n = e - s;
  lo = s + n * j / kPartNB;
  hi = s + n * (j + 1) / kPartNB;
}

// Level-2 digit of a 32-bit entry: key bits [shift2, shift1).
__device__ __forceinline__ uint32_t digit2(const PartSpec& P, uint32_t e) {
  return (e >> (P.vbits + P.shift2)) & (P.nparts2 - 1u);
}

// One LDS counting-sort round of an NT-thread block: the block's `n` (<= NT * E) entries `e[k]` with digits `dg[k]`
// (thread t holds round entries t + NT k) go out as one run per digit.  LDS: cnt/start [ndig] + sorted entries + their
// digits.  DIG = false: the digit is recomputable from the sorted entry itself, (e >> dsh) & (ndig - 1), so sdig is not
// used.  Output cursors:
//   RES = false: cur[d] = the block's next output position of digit d (exact offsets from a histogram; advanced here);
//   RES = true:  each run is reserved in digit d's fixed-capacity region by one global atomic on fill[d]: the run lands
//                at region0 + d * cap + (entries reserved before it); a run that would pass the region's capacity is
//                dropped and raises err bit 4 (the runtime reruns the query with exact offsets).  Run order within a
//                region is not deterministic; what is aggregated from it (counts, value sets) does not depend on it.
// `after_reserve()` runs once the runs are reserved (the caller's prefetch of its next round: issued there, its loads
// are not waited on by the reservations' returned values).
struct NoPrefetch {
  __device__ void operator()() const {}
};
template <int NT, int E, class Out, bool DIG, bool RES, class F = NoPrefetch>
__device__ __forceinline__ void split_round(uint32_t (&e)[E], uint32_t (&dg)[E], uint32_t n, uint32_t ndig,
                                            uint32_t* cnt, uint32_t* start, unsigned long long* cur, uint32_t* sbuf,
                                            uint8_t* sdig, Out* out, uint32_t dsh = 0, unsigned int* fill = nullptr,
                                            uint64_t region0 = 0, uint64_t cap = 0, unsigned int* err = nullptr,
                                            F after_reserve = F(), uint64_t* prof = nullptr) {
  // a dropped run's cursor: never a (run start - sort position) value, which lies in (-2^15, 2^40) mod 2^64
  constexpr unsigned long long kDrop = 1ull << 63;
  [[maybe_unused]] uint64_t pt = PROF_NOW();
  const uint32_t tid = threadIdx.x;
  uint32_t rank[E];
#pragma unroll
  for (int k = 0; k < E; k++) {
    const uint32_t d = DIG ? dg[k] : ((e[k] >> dsh) & (ndig - 1u));  // !DIG: recomputed, dg[] is never held
    rank[k] = tid + NT * k < n ? atomicAdd(&cnt[d], 1u) : 0u;
  }
  __syncthreads();
  if (prof) PROF_LAP(prof, 1, pt);
  // exclusive scan of cnt over the digits (ndig <= 256 <= NT: one per thread) -> start; reserve the runs
  {
    uint32_t c = tid < ndig ? cnt[tid] : 0u, x = c;
    const uint32_t lane = tid & 63u, wave = tid >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    __shared__ uint32_t wsum[NT / 64];
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (uint32_t w = 0; w < wave; w++) wb += wsum[w];
    if (tid < ndig) {
      start[tid] = wb + x - c;
      cnt[tid] = 0;
      if (RES && c) {
        const uint32_t old = atomicAdd(&fill[tid], c);
        if ((uint64_t)old + c <= cap) {
          cur[tid] = region0 + (uint64_t)tid * cap + old - (wb + x - c);  // run start - its sort position
        } else {
          cur[tid] = kDrop;
          atomicOr(err, 16u);
        }
      }
    }
  }
  __syncthreads();
  if (prof) PROF_LAP(prof, 2, pt);
  after_reserve();
#pragma unroll
  for (int k = 0; k < E; k++)
    if (tid + NT * k < n) {
      const uint32_t at = start[DIG ? dg[k] : ((e[k] >> dsh) & (ndig - 1u))] + rank[k];
      sbuf[at] = e[k];
      if (DIG) sdig[at] = (uint8_t)dg[k];
    }
  __syncthreads();
  if (prof) PROF_LAP(prof, 3, pt);
  for (uint32_t i = tid; i < n; i += NT) {
    const uint32_t x = sbuf[i];
    const uint32_t d = DIG ? (uint32_t)sdig[i] : (x >> dsh) & (ndig - 1u);
    // RES: cur[d] holds the run's start minus its sort position (one LDS read per entry); else the cursor
    const unsigned long long c0 = cur[d];
    if (!RES || c0 != kDrop) {
      out[RES ? c0 + i : c0 + (i - start[d])] = (Out)x;
    }
  }
  __syncthreads();
  if (prof) PROF_LAP(prof, 4, pt);
  if (!RES) {  // advance the cursors by this round's run lengths (start[d+1] - start[d])
    if (tid < ndig) cur[tid] += (tid + 1 < ndig ? start[tid + 1] : n) - start[tid];
    __syncthreads();
  }
}

// Level 1: scan block b's entries -> level-1 partitions (its range of each starts at off1[p * blocks1 + b]).
__global__ __launch_bounds__(kST) void part_split1_kernel(PartSpec P) {
  constexpr int E = kSplitChunk / kST;
  __shared__ uint32_t cnt[kPartL1], start[kPartL1], sbuf[kSplitChunk];
  __shared__ unsigned long long cur[kPartL1];
  __shared__ uint8_t sdig[kSplitChunk];  // digits < 256: one byte each
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  if (tid < P.nparts1) {
    cnt[tid] = 0;
    cur[tid] = P.off1[(uint64_t)tid * P.blocks1 + b];
  }
  __syncthreads();
  const unsigned long long* __restrict__ in = P.in0 + P.base0[b];
  const uint32_t n = P.count0[b];
  const uint32_t sh = P.vbits + P.shift1;
  const uint64_t lmask = (1ull << P.shift1) - 1ull, vmask = (1ull << P.vbits) - 1ull;
  for (uint32_t c0 = 0; c0 < n; c0 += kSplitChunk) {
    const uint32_t m = min(kSplitChunk, n - c0);
    uint32_t e[E], dg[E];
#pragma unroll
    for (int k = 0; k < E; k++) {
      const uint32_t i = tid + kST * k;
      const uint64_t x = i < m ? in[c0 + i] : 0ull;
      dg[k] = (uint32_t)(x >> sh);
      e[k] = (uint32_t)((((x >> P.vbits) & lmask) << P.vbits) | (x & vmask));
    }
    split_round<kST, E, uint32_t, true, false>(e, dg, m, P.nparts1, cnt, start, cur, sbuf, sdig, P.in1);
  }
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

// Level 2: the same ranges, counting-sorted by level-2 digit into buckets (bucket p * nparts2 + d).
__global__ __launch_bounds__(kST) void part_split2_kernel(PartSpec P) {
  constexpr int E = kSplitChunk / kST;
  __shared__ uint32_t cnt[256], start[256], sbuf[kSplitChunk];
  __shared__ unsigned long long cur[256];
  __shared__ uint8_t sdig[PG_SPLIT2_DIG ? kSplitChunk : 1];  // the digit is recomputed from the entry when !PG_SPLIT2_DIG
  const uint32_t j = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
  if (tid < P.nparts2) {
    cnt[tid] = 0;
    cur[tid] = P.off2[((uint64_t)p * P.nparts2 + tid) * kPartNB + j];
  }
  __syncthreads();
  uint64_t lo, hi;
  l2_range(P, p, j, lo, hi);
  const uint32_t* __restrict__ in = P.in1;
  for (uint64_t c0 = lo; c0 < hi; c0 += kSplitChunk) {
    const uint32_t m = (uint32_t)min((uint64_t)kSplitChunk, hi - c0);
    uint32_t e[E], dg[E];
#pragma unroll
    for (int k = 0; k < E; k++) {
      const uint32_t i = tid + kST * k;
      e[k] = i < m ? in[c0 + i] : 0u;
      dg[k] = digit2(P, e[k]);
    }
    split_round<kST, E, uint32_t, PG_SPLIT2_DIG, false>(e, dg, m, P.nparts2, cnt, start, cur, sbuf, sdig, P.out2,
                                                      P.vbits + P.shift2);
  }
}

#ifndef PG_SPLIT2S_PREFETCH
#define PG_SPLIT2S_PREFETCH 1  // the next chunk's loads issued while this one is sorted (registers: 1 block per CU)
#endif
// Level 2, speculative layout: entries [lo, hi) of level-1 partition p (its region starts at s0 and holds n entries),
// counting-sorted by level-2 digit in LDS rounds of kSplitChunk, each run reserved in its bucket's fixed-capacity
// region (bucket d at region0 + d * cap2, reservations on fill[d]; no count pass).  cnt must be zero on entry (it is
// again on exit).
__device__ __forceinline__ void split2s_range(const PartSpec& P, uint64_t s0, uint64_t n, uint64_t lo, uint64_t hi,
                                              unsigned int* fill, uint64_t region0, uint32_t* cnt, uint32_t* start,
                                              unsigned long long* cur, uint32_t* sbuf, uint64_t* prof = nullptr) {
  constexpr int E = kSplitChunk / kST;
  const uint32_t tid = threadIdx.x;
  uint32_t e[E], ne[E];
  // buffer loads relative to the partition (one 32-bit lane offset, the k stride as a scalar offset, reads past the
  // block's range return 0): no 64-bit address per load in flight
  const rsrc_t rin = part_rsrc(P.in1 + s0, (uint32_t)(4ull * n));
  // (no select on the loaded value: split_round skips the round's entries past n itself, so the loads stay in flight
  // until the round that consumes them -- a `cond ? v : 0` here waited for them where they were issued)
  auto load = [&](uint64_t c0, uint32_t (&x)[E]) {
    const uint32_t vo = 4u * (uint32_t)(c0 - s0 + tid);
#pragma unroll
    for (int k = 0; k < E; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b32(rin, vo, 4u * kST * k, 0);
  };
  if (lo < hi) load(lo, e);
  for (uint64_t c0 = lo; c0 < hi; c0 += kSplitChunk) {
    const uint32_t m = (uint32_t)min((uint64_t)kSplitChunk, hi - c0);
    [[maybe_unused]] uint64_t pt = PROF_NOW();
    uint32_t dg[E];
#pragma unroll
    for (int k = 0; k < E; k++) dg[k] = digit2(P, e[k]);
    if (prof) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (profile build only: the loads' wait shows up here)
      PROF_LAP(prof, 0, pt);
      if (threadIdx.x == 0) prof[7]++;
    }
    const uint64_t c1 = c0 + kSplitChunk;
    auto pre = [&]() { if (PG_SPLIT2S_PREFETCH && c1 < hi) load(c1, ne); };
    split_round<kST, E, uint32_t, false, true>(e, dg, m, P.nparts2, cnt, start, cur, sbuf, nullptr, P.out2,
                                               P.vbits + P.shift2, fill, region0, P.cap2, P.err, pre, prof);
    if (!PG_SPLIT2S_PREFETCH && c1 < hi) load(c1, ne);
#pragma unroll
    for (int k = 0; k < E; k++) e[k] = ne[k];
  }
}

// Level 2 as its own launch: level-1 partition p's entries (min(fill1[p], cap1) of them) split over kPartNB blocks,
// buckets at b * cap2 for every bucket b of the plan.
__global__ __launch_bounds__(kST, PG_SPLIT_WAVES) void part_split2s_kernel(PartSpec P) {
  __shared__ uint32_t cnt[256], start[256], sbuf[kSplitChunk];
  __shared__ unsigned long long cur[256];
  const uint32_t j = blockIdx.x, p = blockIdx.y, tid = threadIdx.x;
  if (tid < P.nparts2) cnt[tid] = 0;
  __syncthreads();
  const uint64_t n = min((uint64_t)P.fill1[p], P.cap1), s0 = (uint64_t)p * P.cap1;
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  split2s_range(P, s0, n, s0 + n * j / kPartNB, s0 + n * (j + 1) / kPartNB, P.fill2 + (uint64_t)p * P.nparts2,
                (uint64_t)p * P.nparts2 * P.cap2, cnt, start, cur, sbuf, PG_PART_PROF ? prof : nullptr);
  PROF_FLUSH(1, prof);
}

// Bucket b (groups g = b << shift2 | gl), entries [lo, hi) of out2: doc count and value bitmap of each group in LDS
// (lds: (1 + dc_words) words per group, zeroed here), then the bucket's slice of the dense state (i64 slot 0 = doc
// count, the bitmap row) written whole.
template <uint32_t NT>  // threads of the workgroup
__device__ __forceinline__ void aggregate_bucket(const PartSpec& P, uint32_t b, uint64_t lo, uint64_t hi, uint32_t* lds) {
  const uint32_t tid = threadIdx.x;
  const uint32_t ng = 1u << P.shift2, dw = P.dc_words;
  uint32_t* cnt = lds;        // [ng]
  uint32_t* bm = lds + ng;    // [ng][dw]
  [[maybe_unused]] uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  [[maybe_unused]] uint64_t pt = PROF_NOW();
  for (uint32_t i = tid; i < ng * (1u + dw); i += NT) lds[i] = 0;
  __syncthreads();
  PROF_LAP(prof, 0, pt);
  const uint32_t gm = ng - 1u, vm = (1u << P.vbits) - 1u, vb = P.vbits;
  // the bucket's entries by buffer loads relative to lo (reads past the bucket's region return 0), kAggB per lane in
  // flight and the next batch issued before this one is counted: the pass is bound by load latency otherwise
  // (4 loads per lane: 66k cycles per 51k-entry bucket on config 4, r05 PG_PART_PROF)
  constexpr int B = kAggB;
  const uint64_t n = hi - lo;
  const rsrc_t rin = part_rsrc(P.out2 + lo, (uint32_t)(4ull * n));
  uint32_t e[B], ne[B];
  auto load = [&](uint32_t base, uint32_t (&x)[B]) {
#pragma unroll
    for (int k = 0; k < B; k++) x[k] = __builtin_amdgcn_raw_buffer_load_b32(rin, 4u * (base + tid), 4u * NT * k, 0);
  };
  load(0, e);
  for (uint32_t base = 0; base < n; base += B * NT) {
    // issued whatever remains (reads past the region return 0): a conditional load here made the compiler wait for
    // every outstanding load at the first use below, which undid the prefetch
    load(base + B * NT, ne);
#pragma unroll
    for (int k = 0; k < B; k++) {
      if (base + tid + NT * k < n) {
        const uint32_t g = (e[k] >> vb) & gm;
        if (P.count_docs) atomicAdd(&cnt[g], 1u);
        if (dw) {
          const uint32_t v = e[k] & vm;
          atomicOr(&bm[g * dw + (v >> 5)], 1u << (v & 31u));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < B; k++) e[k] = ne[k];
  }
  __syncthreads();
  PROF_LAP(prof, 1, pt);
  const uint64_t g0 = (uint64_t)b << P.shift2;
  const uint32_t ng_out = (uint32_t)(g0 + ng <= P.num_groups ? ng : (g0 < P.num_groups ? P.num_groups - g0 : 0));
  const bool want_pop = dw && (P.dc_pop || !P.count_docs);
  if (want_pop && dw == 32 && NT >= 2 * 512 && ng <= NT / 2) {
    // the group's set size (extractFinalResult) while its bitmap is in LDS: two lanes per group, 16 words each as four
    // 16-B reads (a wave reads 32 whole rows per instruction), halves combined across the lane pair
    const uint32_t gl = tid >> 1, h = tid & 1u;
    uint32_t pc = 0;
    if (gl < ng) {
      const uint4* row = (const uint4*)(bm + gl * 32u + h * 16u);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint4 x = row[k];
        pc += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
      }
    }
    pc += __shfl_xor(pc, 1);
    if (gl < ng_out && h == 0) {
      // slot 0: the doc count, or with no COUNT aggregation (count_docs 0) the set size -- nonzero exactly for the
      // groups that have a doc, which is all a DISTINCTCOUNT-only state reads from it
      P.i64[(g0 + gl) * P.n_i64] = P.count_docs ? cnt[gl] : pc;
      if (P.dc_pop) P.dc_pop[g0 + gl] = pc;
    }
  } else {
    for (uint32_t gl = tid; gl < ng_out; gl += NT) {
      uint32_t pc = 0;
      if (want_pop)
        for (uint32_t k = 0, r = gl % dw; k < dw; k++, r = r + 1 == dw ? 0 : r + 1) pc += __popc(bm[gl * dw + r]);  // lanes on distinct banks
      P.i64[(g0 + gl) * P.n_i64] = P.count_docs ? cnt[gl] : pc;
      if (P.dc_pop && dw) P.dc_pop[g0 + gl] = pc;
    }
  }
  if (P.row_words) {
    const uint32_t rw = P.row_words;
    uint32_t* __restrict__ dst = P.bits + g0 * rw;
    for (uint32_t w = tid; w < ng_out * rw; w += NT) {
      const uint32_t gl = w / rw, k = w - gl * rw;
      dst[w] = (k >= P.dc_word && k < P.dc_word + dw) ? bm[gl * dw + (k - P.dc_word)] : 0u;
    }
  }
  if (PG_PART_PROF) {
    __syncthreads();
    PROF_LAP(prof, 2, pt);
    PROF_FLUSH(2, prof);
  }
}

// One workgroup per bucket b: its entries at [off2[b * kPartNB], off2[(b + 1) * kPartNB]) (exact layout) or
// [b * cap2, b * cap2 + min(fill2[b], cap2)) (speculative).
__global__ __launch_bounds__(kAT) void part_aggregate_kernel(PartSpec P) {
  extern __shared__ uint32_t lds[];
  const uint32_t b = blockIdx.x;
  uint64_t lo, hi;
  if (P.fill2) {
    lo = (uint64_t)b * P.cap2;
    hi = lo + min((uint64_t)P.fill2[b], P.cap2);
  } else {
    lo = P.off2[(uint64_t)b * kPartNB];
    hi = P.off2[(uint64_t)(b + 1) * kPartNB];
  }
  aggregate_bucket<kAT>(P, b, lo, hi, lds);
}

// ------------------------------------------------------------------------------------------ level 1 from the columns

// FixedBitIntReader.readUnchecked on the native-word image (columns keep 4 zero words of tail padding).
__device__ __forceinline__ uint32_t col_unpack(const uint32_t* __restrict__ w, uint32_t idx, uint32_t b) {
  const uint64_t p = (uint64_t)idx * b;
  const uint64_t k = p >> 5;
  const uint64_t win = ((uint64_t)w[k] << 32) | (uint64_t)w[k + 1];
  return (uint32_t)(win >> (64u - ((uint32_t)p & 31u) - b)) & (0xFFFFFFFFu >> (32u - b));
}

// table-global id of dictId `id` (the scan's key_of): value offset through the dictionary / decoded image, or keymap
__device__ __forceinline__ uint64_t col_key_of(uint32_t kind, int64_t base, const ColDesc& c, uint32_t id) {
  if (id >= c.card) return ~0ull;
  if (kind == PG_KEY_KEYMAP) return (uint64_t)(uint32_t)c.keymap[id];
  int64_t v;
  if (c.decoded) v = c.vbase + (int64_t)id;
  else v = c.dtype == PG_INT ? (int64_t)((const int32_t*)c.dict)[id] : ((const int64_t*)c.dict)[id];
  return (uint64_t)(v - base);
}

// The level-1 digits and 32-bit entries of the round's docs r0 + tid + kST * j (j < E, those < m valid), every key
// and value column's window loads issued before any is consumed.  The segment's key / value descriptors are held in
// registers for the whole item (NK: compile-time bound on the keys).  A key or value outside its space (never
// expected: the host proved the ranges) reports an error bit and lands in partition 0; hist and scatter agree.
template <int NK, int E, int J0, int JN>  // docs j in [J0, J0 + JN) of the round's E
__device__ __forceinline__ void part_entries(const PartScanSpec& P, const ColDesc (&kc)[NK], const ColDesc& vc,
                                             uint32_t r0, uint32_t m, uint32_t (&dg)[E], uint32_t (&ent)[E]) {
  const uint32_t tid = threadIdx.x;
  const bool has_val = P.val_agg != (uint32_t)kNoSlot;
  uint32_t raw[NK][JN], vraw[JN];
#pragma unroll
  for (int k = 0; k < NK; k++)
#pragma unroll
    for (int jj = 0; jj < JN; jj++) {
      const uint32_t i = tid + kST * (J0 + jj);
      raw[k][jj] = (i < m && (uint32_t)k < P.num_keys) ? col_unpack(kc[k].words, r0 + i, kc[k].bits) : 0u;
    }
#pragma unroll
  for (int jj = 0; jj < JN; jj++) {
    const uint32_t i = tid + kST * (J0 + jj);
    vraw[jj] = (i < m && has_val) ? col_unpack(vc.words, r0 + i, vc.bits) : 0u;
  }
#pragma unroll
  for (int jj = 0; jj < JN; jj++) {
    const int j = J0 + jj;
    uint64_t g = 0;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < NK; k++) {
      if ((uint32_t)k >= P.num_keys) break;
      const uint64_t kid = col_key_of(P.key_kind[k], P.key_base[k], kc[k], raw[k][jj]);
      bad |= kid >= P.key_card[k];
      g += kid * P.key_stride[k];
    }
    uint32_t vid = 0;
    if (has_val) {
      const uint64_t v = col_key_of(P.val.key_kind, P.val.key_base, vc, vraw[jj]);
      if (v < P.val.key_card) vid = (uint32_t)v;
      else if (tid + kST * j < m) atomicOr(P.err, 2u);
    }
    if (bad) {
      if (tid + kST * j < m) atomicOr(P.err, 1u);
      g = 0;
    }
    dg[j] = (uint32_t)(g >> P.shift1);
    ent[j] = (uint32_t)(((g & ((1ull << P.shift1) - 1ull)) << P.vbits) | vid);
  }
}

template <int NK>
__device__ __forceinline__ void item_cols(const PartScanSpec& P, const SegDesc& sd, ColDesc (&kc)[NK], ColDesc& vc) {
#pragma unroll
  for (int k = 0; k < NK; k++)
    if ((uint32_t)k < P.num_keys) kc[k] = sd.keycols[k];
  if (P.val_agg != (uint32_t)kNoSlot) vc = sd.aggcols[2 * P.val_agg];
}

template <int NK>
__global__ __launch_bounds__(kST) void part_hist_kernel(PartScanSpec P) {
  constexpr int E = kSplitChunk / kST;
  __shared__ uint32_t h[kPartL1];
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  for (uint32_t i = tid; i < kPartL1; i += kST) h[i] = 0;
  __syncthreads();
  const uint64_t i0 = (uint64_t)b * P.num_items / P.blocks, i1 = (uint64_t)(b + 1) * P.num_items / P.blocks;
  for (uint64_t it = i0; it < i1; it++) {
    const WorkItem w = P.items[it];
    const SegDesc sd = P.segs[w.seg];
    ColDesc kc[NK], vc;
    item_cols<NK>(P, sd, kc, vc);
    const uint32_t d0 = w.tile_begin * (uint32_t)kTileDocs, d1 = min(w.tile_end * (uint32_t)kTileDocs, sd.num_docs);
    for (uint32_t r0 = d0; r0 < d1; r0 += kSplitChunk) {  // the scatter's rounds
      const uint32_t m = min(kSplitChunk, d1 - r0);
      uint32_t dg[E], e[E];
      part_entries<NK, E, 0, E / 2>(P, kc, vc, r0, m, dg, e);
      part_entries<NK, E, E / 2, E / 2>(P, kc, vc, r0, m, dg, e);
#pragma unroll
      for (int j = 0; j < E; j++)
        if (tid + kST * j < m) atomicAdd(&h[dg[j]], 1u);
    }
  }
  __syncthreads();
  for (uint32_t p = tid; p < P.nparts1; p += kST) P.hist1[(uint64_t)p * P.blocks + b] = h[p];
}

template <int NK>
__global__ __launch_bounds__(kST) void part_scatter_kernel(PartScanSpec P) {
  constexpr int E = kSplitChunk / kST;
  __shared__ uint32_t cnt[kPartL1], start[kPartL1], sbuf[kSplitChunk];
  __shared__ unsigned long long cur[kPartL1];
  __shared__ uint8_t sdig[kSplitChunk];
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  if (tid < P.nparts1) {
    cnt[tid] = 0;
    cur[tid] = P.off1[(uint64_t)tid * P.blocks + b];
  }
  __syncthreads();
  const uint64_t i0 = (uint64_t)b * P.num_items / P.blocks, i1 = (uint64_t)(b + 1) * P.num_items / P.blocks;
  for (uint64_t it = i0; it < i1; it++) {
    const WorkItem w = P.items[it];
    const SegDesc sd = P.segs[w.seg];
    ColDesc kc[NK], vc;
    item_cols<NK>(P, sd, kc, vc);
    const uint32_t d0 = w.tile_begin * (uint32_t)kTileDocs, d1 = min(w.tile_end * (uint32_t)kTileDocs, sd.num_docs);
    for (uint32_t r0 = d0; r0 < d1; r0 += kSplitChunk) {
      const uint32_t m = min(kSplitChunk, d1 - r0);
      uint32_t e[E], dg[E];
      part_entries<NK, E, 0, E / 2>(P, kc, vc, r0, m, dg, e);
      part_entries<NK, E, E / 2, E / 2>(P, kc, vc, r0, m, dg, e);
      split_round<kST, E, uint32_t, true, false>(e, dg, m, P.nparts1, cnt, start, cur, sbuf, sdig, P.out1);
    }
  }
}

// ------------------------------------------------------------------------------------------ level 1, speculative

// 512 threads x 16 docs, two resident blocks per CU (their sort and write phases overlap each other's loads): 3.06 ms
// on config 4 vs 3.65 for one 1 024-thread block per CU with the next tile prefetched into registers (r03_v3)
#ifndef PG_DIRECT_THREADS
#define PG_DIRECT_THREADS 512
#endif
constexpr uint32_t kDT = PG_DIRECT_THREADS;   // threads of a part_direct block
constexpr uint32_t kDE = kTileDocs / kDT;     // docs per thread per round (a round is one tile)
static_assert(kDE * kDT == kTileDocs && kDT >= kPartL1, "one digit per thread in the run scan");
static_assert(kDT % 64 == 0 && kDT <= 1024 && kDE <= 32, "part_direct blocks: whole waves, <= 32 docs per thread");

// The tile's word range [w0, w0 + nw) of a packed column into LDS (16-byte loads; reads past the column return 0).
// nw is a multiple of 4 plus the 4 words of padding the unpack's 64-bit window may touch.
// Every pass's load is issued before the first is stored (a load-store loop waited for each load in turn); passes are
// skipped by a block-uniform test, lanes past nw load a few words they do not store.
constexpr uint32_t kStageQ = ((256u * 32u + 4u) / 4u + kDT - 1u) / kDT;  // uint4 passes for a 32-bit column
__device__ __forceinline__ void stage_words(rsrc_t r, uint32_t w0, uint32_t nw, uint32_t* lds) {
  uint4 x[kStageQ];
#pragma unroll
  for (uint32_t k = 0; k < kStageQ; k++)
    if (kDT * k < nw / 4) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (w0 + 4u * (threadIdx.x + kDT * k)) * 4u, 0, 0);
      x[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
  for (uint32_t k = 0; k < kStageQ; k++) {
    const uint32_t q = threadIdx.x + kDT * k;
    if (q < nw / 4) *(uint4*)(lds + 4u * q) = x[k];
  }
}

// The same word range into LDS by LDS-DMA (buffer_load_dwordx4 ... lds: no registers, reads past the column return 0):
// wave v's pass r covers uint4s q = r * kDT + 64 v + lane, landing at lds + 4 q.  Waited for by vmcnt, not lgkmcnt.
__device__ __forceinline__ void dma_words(rsrc_t r, uint32_t w0, uint32_t nw, uint32_t* lds) {
  const uint32_t lane = threadIdx.x & 63u, q0w = (threadIdx.x >> 6) * 64u;
  for (uint32_t q0 = q0w; q0 < nw / 4; q0 += kDT)
    if (q0 + lane < nw / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 4u * q0), 16,
                                               (w0 + 4u * (q0 + lane)) * 4u, 0, 0, 0);
}

// the b-bit value at bit p of a packed run staged at lds (FixedBitIntReader: MSB first)
__device__ __forceinline__ uint32_t lds_unpack(const uint32_t* lds, uint32_t p, uint32_t b) {
  const uint32_t k = p >> 5, o = p & 31u;
  const uint64_t win = ((uint64_t)lds[k] << 32) | (uint64_t)lds[k + 1];
  return (uint32_t)(win >> (64u - o - b)) & (0xFFFFFFFFu >> (32u - b));
}


// Table-global id of a raw (dictId / decoded) value: M = 0 decoded image (vbase + raw - base), 1 gather from an int32
// array (`tab` = the int32 dictionary with `base`, or the keymap with base 0), 2 int64 dictionary (not taken by the
// direct path: the runtime uses the exact one).  Ids outside [0, card) come back as ~0 (the caller's range check).
template <int M>
__device__ __forceinline__ uint64_t id_of(const ColDesc& c, const int32_t* tab, int64_t base, uint32_t raw) {
  if (M == 0) return raw < c.card ? (uint64_t)(c.vbase + (int64_t)raw - base) : ~0ull;
  // (an unconditional global load at a clamped index: a load under the range check, or through the generic table
  // pointer -- a flat load, counted in lgkmcnt -- would be waited for by the caller's next LDS atomic)
  const int32_t x = ld_global(tab + (raw < c.card ? raw : 0u));
  return raw < c.card ? (uint64_t)((int64_t)x - base) : ~0ull;
}
__host__ __device__ __forceinline__ int id_mode(uint32_t key_kind, const ColDesc& c) {
  if (key_kind == PG_KEY_KEYMAP) return 1;
  if (c.decoded) return 0;
  return c.dtype == PG_INT ? 1 : 2;
}

// Round body: 32 docs per thread (doc tid + 256 j) -> level-1 digit + 32-bit entry, ranked within its digit right
// away (LDS atomic; docs past the segment go to the spare digit kPartL1).  Returns the error bits seen.
template <int KM, int VM>  // VM = -1: no value column (COUNTs only)
__device__ __forceinline__ uint32_t direct_unpack(const PartDirectSpec& P, const ColDesc& kc, const ColDesc& vc,
                                                  const int32_t* ktab, int64_t kbase, const int32_t* vtab, int64_t vbase,
                                                  const uint32_t* stk, const uint32_t* stv, uint32_t kb, uint32_t vb,
                                                  uint32_t m, uint32_t* cnt, uint32_t (&dr)[kDE], uint32_t (&e)[kDE]) {
  const uint32_t tid = threadIdx.x;
  const uint64_t lmask = (1ull << P.shift1) - 1ull;
  uint32_t bad = 0;
  // bit positions of doc tid, advanced by 256 docs per j; opaque to the optimiser so that the 64 positions are not
  // hoisted out of the round loop as invariants (they would pin 64+ registers for the whole kernel)
  uint32_t pk = tid * kb, pv = tid * vb;
  asm volatile("" : "+v"(pk), "+v"(pv));
  const uint32_t sk = kDT * kb, sv = kDT * vb;
#pragma unroll
  for (int j = 0; j < (int)kDE; j++) {
    const uint32_t i = tid + kDT * j;
    const bool ok = i < m;
    uint64_t g = id_of<KM>(kc, ktab, kbase, lds_unpack(stk, pk + sk * j, kb));
    uint32_t vid = 0;
    if constexpr (VM >= 0) {
      const uint64_t v = id_of<VM>(vc, vtab, vbase, lds_unpack(stv, pv + sv * j, vb));
      const bool vbad = v >= P.val_card;
      bad |= (ok && vbad) ? 2u : 0u;
      vid = vbad ? 0u : (uint32_t)v;
    }
    const bool kbad = g >= P.key_card;
    bad |= (ok && kbad) ? 1u : 0u;
    g = kbad ? 0ull : g;
    const uint32_t d = ok ? (uint32_t)(g >> P.shift1) : kPartL1;
    e[j] = (uint32_t)(((g & lmask) << P.vbits) | vid);
    dr[j] = (d << 16) | atomicAdd(&cnt[d], 1u);
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // at most 4 docs in flight (loads, 64-bit gather addresses)
  }
  return bad;
}

// KM / VM: the id modes of the key / value column, uniform over the plan's segments (runtime-checked).  W: waves per
// SIMD the register budget is cut for (PG_DIRECT_WAVES).  PRE: the stage has LDS of its own, and the next tile's words
// are DMA'd into it while this tile is sorted and written (issued after the reservations -- a returned atomic waits
// for every older vector-memory op -- and carried across raw barriers, which do not drain vmcnt); else the stage and
// the sort buffer share LDS and each tile's words are loaded when it starts.
//
// LDS (one dynamic array, 16-B aligned carve): stage [stage_words] | sort: sbuf [kTileDocs] + sdig [kTileDocs bytes]
// (PRE: after the stage; else over it) | cnt [kPartL1 + 4] | start [kPartL1] | cur [kPartL1] (8 B) | wsum [16].
template <int KM, int VM, int W, bool PRE>
__global__ __launch_bounds__(kDT, W) void part_direct_kernel(PartDirectSpec P) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dl[];
  const uint32_t sw = P.stage_words;
  const uint32_t so = PRE ? sw : 0u, sort_words = kTileDocs + kTileDocs / 4;
  const uint32_t mo = PRE ? sw + sort_words : (sw > sort_words ? sw : sort_words);
  uint32_t* sbuf = dl + so;
  uint8_t* sdig = (uint8_t*)(dl + so + kTileDocs);
  uint32_t* cnt = dl + mo;                   // [kPartL1 + 1] (+ pad)
  uint32_t* start = cnt + kPartL1 + 4;       // [kPartL1]
  unsigned long long* cur = (unsigned long long*)(start + kPartL1);  // [kPartL1]
  uint32_t* wsum = (uint32_t*)(cur + kPartL1);                       // [kDT / 64]
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  if (tid < kPartL1) cnt[tid] = 0;
  if (tid == 0) cnt[kPartL1] = 0;  // the spare digit of docs past the segment
  __syncthreads();
  uint32_t bad = 0;
  [[maybe_unused]] uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t i0 = (uint64_t)b * P.num_items / P.blocks, i1 = (uint64_t)(b + 1) * P.num_items / P.blocks;
  for (uint64_t it = i0; it < i1; it++) {
    const WorkItem w = ldcf(P.items, it);
    const SegDesc sd = ldcf(P.segs, w.seg);
    const ColDesc kc = ldcf(sd.keycols, 0);
    const ColDesc vc = P.has_val ? ldcf(sd.aggcols, 2ull * P.val_agg) : kc;
    const uint32_t kb = __builtin_amdgcn_readfirstlane(kc.bits);
    const uint32_t vb = P.has_val ? __builtin_amdgcn_readfirstlane(vc.bits) : 0u;
    const uint32_t nwk = 256u * kb + 4u, nwv = P.has_val ? 256u * vb + 4u : 0u;
    const rsrc_t rk = part_rsrc(kc.words, kc.wbytes);
    const rsrc_t rv = part_rsrc(vc.words, vc.wbytes);
    const bool kmap = P.key_kind == PG_KEY_KEYMAP, vmap = P.val_kind == PG_KEY_KEYMAP;
    const int32_t* ktab = kmap ? kc.keymap : (const int32_t*)kc.dict;
    const int32_t* vtab = vmap ? vc.keymap : (const int32_t*)vc.dict;
    const int64_t kbase = kmap ? 0 : P.key_base, vbase = vmap ? 0 : P.val_base;
    const uint32_t num_docs = __builtin_amdgcn_readfirstlane(sd.num_docs);
    const uint32_t t_end = min(w.tile_end, (num_docs + (uint32_t)kTileDocs - 1u) / (uint32_t)kTileDocs);
    bool staged = false;  // this tile's words already DMA'd into the stage during the previous tile (PRE)
    for (uint32_t t = w.tile_begin; t < t_end; t++) {
      const uint32_t r0 = t * (uint32_t)kTileDocs;
      const uint32_t m = min((uint32_t)kTileDocs, num_docs - r0);
      [[maybe_unused]] uint64_t pt = PROF_NOW();
      // 1. the tile's words of both columns, coalesced, into LDS
      if (staged) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed; the barrier: every wave's
        __syncthreads();
      } else {
        stage_words(rk, t * 256u * kb, nwk, dl);
        if (P.has_val) stage_words(rv, t * 256u * vb, nwv, dl + nwk);
        __syncthreads();
      }
      PROF_LAP(prof, 0, pt);
      // 2. entries + ranks ((digit << 16 | rank) and the entry are all a thread keeps)
      uint32_t dr[kDE], e[kDE];
      bad |= direct_unpack<KM, VM>(P, kc, vc, ktab, kbase, vtab, vbase, dl, dl + nwk, kb, vb, m, cnt, dr, e);
      __syncthreads();  // every rank taken; the stage is dead (!PRE: its LDS becomes the sort buffer)
      PROF_LAP(prof, 1, pt);
      // 3. run starts (exclusive scan of the digit counts) and one reservation per non-empty run
      {
        const uint32_t c = tid < P.nparts1 ? cnt[tid] : 0u;
        uint32_t x = c;
        const uint32_t lane = tid & 63u, wave = tid >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o);
          if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t wb = 0;
        for (uint32_t w2 = 0; w2 < wave; w2++) wb += wsum[w2];
        if (tid < P.nparts1) {
          start[tid] = wb + x - c;
          cnt[tid] = 0;
          if (c) {
            const uint32_t old = atomicAdd(&P.fill1[tid], c);
            if ((uint64_t)old + c <= P.cap1) {
              cur[tid] = (uint64_t)tid * P.cap1 + old - (wb + x - c);  // run start - its sort position
            } else {
              cur[tid] = 1ull << 63;  // dropped (never a run start - sort position value)
              atomicOr(P.err, 16u);
            }
          }
        }
        if (tid == 0) cnt[kPartL1] = 0;
      }
      __syncthreads();
      PROF_LAP(prof, 2, pt);
      // PRE: the next tile's words go out now, into the stage (dead since step 2's barrier)
      const bool pre = PRE && t + 1 < t_end;
      if (pre) {
        dma_words(rk, (t + 1) * 256u * kb, nwk, dl);
        if (P.has_val) dma_words(rv, (t + 1) * 256u * vb, nwv, dl + nwk);
      }
#pragma unroll
      for (int j = 0; j < (int)kDE; j++) {
        const uint32_t d = dr[j] >> 16;
        if (d < kPartL1) {
          const uint32_t at = start[d] + (dr[j] & 0xFFFFu);
          sbuf[at] = e[j];
          sdig[at] = (uint8_t)d;
        }
      }
      if (PRE) {  // a raw barrier: __syncthreads() would drain the DMA in flight (vmcnt(0))
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        __syncthreads();
      }
      PROF_LAP(prof, 3, pt);
      // 4. the runs, written out whole
      for (uint32_t i = tid; i < m; i += kDT) {  // cur[d] already holds the run's start minus its sort position
        const unsigned long long c0 = cur[sdig[i]];
        if (c0 != (1ull << 63)) P.out1[c0 + i] = sbuf[i];
      }
      // PRE: the next tile's first barrier (or the next item's stage barrier) orders these reads before the sort
      // buffer's next writes; !PRE: the next stage overwrites the sort buffer
      if (!PRE) __syncthreads();
      else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      PROF_LAP(prof, 4, pt);
      if (PG_PART_PROF && tid == 0) prof[7]++;
      staged = pre;
    }
  }
  if (bad) atomicOr(P.err, bad);
  PROF_FLUSH(0, prof);
}

static void prof_report_direct(uint64_t blocks) {
#if PG_PART_PROF
  prof_report("part_direct", 0, blocks);
#endif
}
hipError_t launch_part_direct(const PartDirectSpec& p_in, uint32_t key_bits, uint32_t val_bits, int key_mode, int val_mode,
                              hipStream_t s) {
  PartDirectSpec p = p_in;
  // stage words of the widest key / value column (a multiple of 4: 16-B aligned carve)
  p.stage_words = (uint32_t)((256ull * key_bits + 4) + (p.has_val ? 256ull * val_bits + 4 : 0));
  const uint32_t sort_words = kTileDocs + kTileDocs / 4, misc_words = (kPartL1 + 4) + kPartL1 + 2 * kPartL1 + 16;
  // PRE when stage + sort + misc leave two resident blocks per CU (config 4: 79.9 KB per block); PG_DIRECT_PRE=0 off
  const size_t pre_bytes = 4ull * (p.stage_words + sort_words + misc_words);
  const char* pe = getenv("PG_DIRECT_PRE");
  const bool pre = pre_bytes <= 80 * 1024 && !(pe && atoi(pe) == 0);
  const size_t lds = pre ? pre_bytes : 4ull * (std::max(p.stage_words, sort_words) + misc_words);
  const dim3 g(p.blocks), b(kDT);
#ifndef PG_DIRECT_WAVES2
#define PG_DIRECT_WAVES2 (3 * PG_DIRECT_THREADS / 256)
#endif
  // register budget: two resident blocks per CU (default) or PG_DIRECT_WAVES2 waves per SIMD
  constexpr int kW0 = 2 * kDT / 256, kW1 = PG_DIRECT_WAVES2;
  static const int waves = getenv("PG_DIRECT_WAVES") ? atoi(getenv("PG_DIRECT_WAVES")) : kW0;
#define PG_DIRECT(K, V)                                                                                 \
  if (key_mode == (K) && val_mode == (V)) {                                                             \
    if (pre) hipLaunchKernelGGL((part_direct_kernel<K, V, kW0, true>), g, b, lds, s, p);                \
    else if (waves == kW1) hipLaunchKernelGGL((part_direct_kernel<K, V, kW1, false>), g, b, lds, s, p); \
    else hipLaunchKernelGGL((part_direct_kernel<K, V, kW0, false>), g, b, lds, s, p);                   \
    if (PG_PART_PROF) prof_report_direct(p.blocks);                                                     \
    return hipGetLastError();                                                                           \
  }
  PG_DIRECT(0, -1) PG_DIRECT(0, 0) PG_DIRECT(0, 1) PG_DIRECT(1, -1) PG_DIRECT(1, 0) PG_DIRECT(1, 1)
#undef PG_DIRECT
  return hipErrorInvalidValue;
}
int part_id_mode(uint32_t key_kind, const ColDesc& c) { return id_mode(key_kind, c); }
hipError_t launch_part_split2s(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_split2s_kernel, dim3(kPartNB, p.nparts1), dim3(kST), 0, s, p);
#if PG_PART_PROF
  prof_report("split2s", 1, (uint64_t)kPartNB * p.nparts1);
#endif
  return hipGetLastError();
}
hipError_t launch_part_hist(const PartScanSpec& p, hipStream_t s) {
  if (p.num_keys <= 1) hipLaunchKernelGGL(part_hist_kernel<1>, dim3(p.blocks), dim3(kST), 0, s, p);
  else hipLaunchKernelGGL(part_hist_kernel<kMaxKeys>, dim3(p.blocks), dim3(kST), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_part_scatter(const PartScanSpec& p, hipStream_t s) {
  if (p.num_keys <= 1) hipLaunchKernelGGL(part_scatter_kernel<1>, dim3(p.blocks), dim3(kST), 0, s, p);
  else hipLaunchKernelGGL(part_scatter_kernel<kMaxKeys>, dim3(p.blocks), dim3(kST), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_part_split1(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_split1_kernel, dim3(p.blocks1), dim3(kST), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_part_count2(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_count2_kernel, dim3(kPartNB, p.nparts1), dim3(256), p.nparts2 * 4, s, p);
  return hipGetLastError();
}
hipError_t launch_part_split2(const PartSpec& p, hipStream_t s) {
  hipLaunchKernelGGL(part_split2_kernel, dim3(kPartNB, p.nparts1), dim3(kST), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_part_aggregate(const PartSpec& p, hipStream_t s) {
  const size_t lds = (size_t)(1u << p.shift2) * (1u + p.dc_words) * 4u;
  hipLaunchKernelGGL(part_aggregate_kernel, dim3(p.nparts1 * p.nparts2), dim3(kAT), lds, s, p);
#if PG_PART_PROF
  prof_report("aggregate", 2, (uint64_t)p.nparts1 * p.nparts2);
#endif
  return hipGetLastError();
}

}  // namespace pg
