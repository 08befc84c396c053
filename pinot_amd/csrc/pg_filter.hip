// pg_filter.hip -- the streaming pre-filter of the segment query hot path (gfx950).
//
// The selective leaves of a query's root AND (ScanBasedFilterOperator leaves over bit-packed forward indexes, doc
// ranges, index bitmaps) are evaluated here by a lean kernel into one doc bitmap per segment; the fused scan
// (pg_scan.hip) then reads that bitmap as a 1-bit column and does projection / aggregation for the survivors only.
// This is SVScanDocIdIterator (dociditerators/SVScanDocIdIterator.java:67-125) with AndDocIdSet's scan-children
// order (docidsets/AndDocIdSet.java:60-150): each later leaf is tested only on docs the earlier ones accepted.
//
// Why a separate kernel: the fused scan carries every query shape's registers (3-4 waves/SIMD) and stages packed
// columns through LDS-DMA, which streamed a 20-bit column at ~1.9 TB/s; this kernel holds ~60 VGPRs (8 waves/SIMD)
// and loads each thread's 32 consecutive values straight into registers with 16-byte loads, the bit width a
// template parameter so unpacking is static register arithmetic: 5.5-5.9 TB/s on the same column (tools/stream_probe).
//
// Thread t of a block takes 32-doc groups; group g of a segment = docs [32g, 32g+32) = packed words [g*b, (g+1)*b),
// so the group's bits start word-aligned.  Output word g: bit 31-j <-> doc 32g+j (the packed 1-bit column order).
#include <hip/hip_runtime.h>

#include "pg_aux.h"
#include "pg_dict.h"

namespace pg {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
#define PG_CONST __attribute__((address_space(4)))

template <class T> __device__ __forceinline__ T ldcf(const T* p, uint64_t i) {
  const PG_CONST uint32_t* src = (const PG_CONST uint32_t*)(p + i);
  T v;
  uint32_t* dst = (uint32_t*)&v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = src[k];
  return v;
}

__device__ __forceinline__ rsrc_t rsrc_of(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

#ifndef PG_STREAM_CPOL
#define PG_STREAM_CPOL 0  // cache policy of the stream's group loads (gfx950 aux bits: 1 sc0, 2 nt, 16 sc1); 0 = default
#endif

// The B words of a 32-doc group into registers (buffer loads: reads past the column return 0).
template <int B>
__device__ __forceinline__ void load_group(rsrc_t r, uint64_t g, uint32_t (&w)[B + 1]) {
  const uint32_t off = (uint32_t)(g * B * 4u);
#pragma unroll
  for (int k = 0; k + 4 <= B; k += 4) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off + 4u * k, 0, PG_STREAM_CPOL);
    w[k] = x[0]; w[k + 1] = x[1]; w[k + 2] = x[2]; w[k + 3] = x[3];
  }
  constexpr int R = B & 3, K0 = B & ~3;
  if constexpr (R == 1) {
    w[K0] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u * K0, 0, PG_STREAM_CPOL);
  } else if constexpr (R == 2) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, off + 4u * K0, 0, PG_STREAM_CPOL);
    w[K0] = x[0]; w[K0 + 1] = x[1];
  } else if constexpr (R == 3) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b96(r, off + 4u * K0, 0, PG_STREAM_CPOL);
    w[K0] = x[0]; w[K0 + 1] = x[1]; w[K0 + 2] = x[2];
  }
  w[B] = 0;
}

// value j (0..31) of the group: bits [j*B, j*B+B) of w, most significant first (FixedBitIntReader)
template <int B>
__device__ __forceinline__ uint32_t value_at(const uint32_t (&w)[B + 1], int j) {
  constexpr uint32_t M = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
  const uint32_t s = (uint32_t)j * B, k = s >> 5, o = s & 31u;
  if (o + B <= 32) return (w[k] >> (32u - o - B)) & M;
  return __builtin_amdgcn_alignbit(w[k], w[k + 1], 64u - o - B) & M;
}

// value j of the group in the low B bits, with whatever bits precede it above them (no mask): for lookups that mask
// the index themselves and bit tests whose offset is taken mod 32
template <int B>
__device__ __forceinline__ uint32_t value_raw(const uint32_t (&w)[B + 1], int j) {
  const uint32_t s = (uint32_t)j * B, k = s >> 5, o = s & 31u;
  if (o + B <= 32) return w[k] >> (32u - o - B);
  return __builtin_amdgcn_alignbit(w[k], w[k + 1], 64u - o - B);
}

typedef const __attribute__((address_space(3))) uint32_t* lds_cptr;

// value `idx` of a `b`-bit packed column through its buffer descriptor (a 64-bit window of two words)
__device__ __forceinline__ uint32_t unpack_win(rsrc_t r, uint32_t idx, uint32_t b) {
  const uint64_t pbit = (uint64_t)idx * b;
  const uint32_t off = (uint32_t)(pbit >> 5) << 2;
  const uint32_t sh = (uint32_t)pbit & 31u;
  const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0);
  const uint64_t win = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)(win >> (64u - sh - b)) & (0xFFFFFFFFu >> (32u - b));
}

// One leaf over one group for the docs in `need`: bit j <-> doc 32g + j.
template <int B>
__device__ __forceinline__ uint32_t test_group(const LeafDesc& L, const uint32_t* lds_sets, uint64_t g, uint32_t need,
                                               bool exact, const uint32_t (&w)[B + 1]);

template <int B>
__device__ __forceinline__ uint32_t eval_group(const LeafDesc& L, const uint32_t* lds_sets, uint64_t g, uint32_t need,
                                               bool exact = false) {
  uint32_t w[B + 1];
  load_group<B>(rsrc_of(L.words, L.wbytes), g, w);
  return test_group<B>(L, lds_sets, g, need, exact, w);
}

// The leaf's test over a group whose words `w` are in registers.
template <int B>
__device__ __forceinline__ uint32_t test_group(const LeafDesc& L, const uint32_t* lds_sets, uint64_t g, uint32_t need,
                                               bool exact, const uint32_t (&w)[B + 1]) {
  uint32_t m = 0;
  if (exact) {
    // SET_LDS with its exact LUT over dictIds staged at lds_sets[0], which is LDS address 0 (stream_kernel has no
    // static LDS; checked at its start): the word's byte address is the LDS address itself, and v_bfe_u32 takes the
    // bit offset mod 32 -- per value one extract, two ops of address, the read, v_bfe_u32 and v_lshl_or_b32
    constexpr uint32_t M = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
#pragma unroll
    for (int j0 = 0; j0 < 32; j0 += 8) {  // 8 reads in flight per wait
      uint32_t r[8], word[8];
#pragma unroll
      for (int x = 0; x < 8; x++) {
        r[x] = value_raw<B>(w, j0 + x);
        word[x] = *(lds_cptr)(uintptr_t)(((r[x] & M) >> 5) << 2);
      }
#pragma unroll
      for (int x = 0; x < 8; x++) m |= __builtin_amdgcn_ubfe(word[x], r[x], 1u) << (j0 + x);
    }
  } else if (L.kind == LK_RANGE) {
    const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll
    for (int j = 0; j < 32; j++) m |= (uint32_t)((value_at<B>(w, j) - lo) < span) << j;
  } else if (L.kind == LK_SET_LDS) {
    const uint32_t* bm = lds_sets + L.lds_off;
    const uint32_t sh = L.shift;
#pragma unroll
    for (int j = 0; j < 32; j++) {
      const uint32_t x = value_at<B>(w, j) >> sh;
      m |= ((bm[x >> 5] >> (x & 31u)) & 1u) << j;
    }
    if (sh) {
      // candidates of the coarse filter bitmap, resolved through the exact LUT in rounds of up to 4 per lane with
      // their loads in flight together.  The candidate's value is re-read from memory (its line was just loaded):
      // picking it out of w[] by a per-lane index would be a waterfall loop over the lanes' indices.
      const rsrc_t rs = rsrc_of(L.words, L.wbytes);
      const uint32_t d0 = (uint32_t)(g * 32);
      uint32_t cand = m & need;
      m = 0;
      while (__ballot(cand != 0)) {
        uint32_t jj[4], v[4], lw[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
          jj[x] = cand ? (uint32_t)__ffs(cand) - 1u : 32u;
          cand &= cand - 1u;
          v[x] = jj[x] < 32u ? unpack_win(rs, d0 + jj[x], B) : 0u;
        }
#pragma unroll
        for (int x = 0; x < 4; x++) lw[x] = jj[x] < 32u ? L.lut[v[x] >> 5] : 0u;
#pragma unroll
        for (int x = 0; x < 4; x++)
          if (jj[x] < 32u) m |= ((lw[x] >> (v[x] & 31u)) & 1u) << jj[x];
      }
    }
  } else {  // LK_SET_LUT: a global bitmap over dictIds, 8 lookups in flight at a time
#pragma unroll
    for (int j0 = 0; j0 < 32; j0 += 8) {
      uint32_t lw[8];
#pragma unroll
      for (int r = 0; r < 8; r++) lw[r] = ((need >> (j0 + r)) & 1u) ? L.aux[value_at<B>(w, j0 + r) >> 5] : 0u;
#pragma unroll
      for (int r = 0; r < 8; r++) m |= ((lw[r] >> (value_at<B>(w, j0 + r) & 31u)) & 1u) << (j0 + r);
    }
  }
  return m;
}

// One leaf of the root AND over the work items of the segments whose form of the leaf reads B-bit values (or a
// doc range / constant): the first leaf writes each group's word, later ones AND into it and load their column
// only for lanes whose word still has a doc.
template <int B>
__global__ __launch_bounds__(256) void prefilter_kernel(PreSpec p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_sets[];
  const uint32_t tid = threadIdx.x;
  const uint32_t i0 = (uint32_t)((uint64_t)blockIdx.x * p.num_items / gridDim.x);
  const uint32_t i1 = (uint32_t)(((uint64_t)blockIdx.x + 1) * p.num_items / gridDim.x);
  uint32_t cur_seg = 0xFFFFFFFFu;
  LeafDesc L;
  uint32_t nd = 0;
  for (uint32_t it = i0; it < i1; it++) {
    const WorkItem wi = ldcf(p.items, it);  // tile_begin / tile_end count 32-doc groups here
    if (wi.seg != cur_seg) {
      const SegDesc sd = ldcf(p.segs, wi.seg);
      L = ldcf(sd.leaves, p.leaf);
      nd = sd.num_docs;
      if (L.kind == LK_SET_LDS) {
        __syncthreads();  // every thread is done with the previous segment's set
        for (uint32_t k = tid; k < L.set_ints; k += 256) lds_sets[L.lds_off + k] = L.aux[k];
        __syncthreads();
      }
      cur_seg = wi.seg;
    }
    uint32_t* out = ldcf(p.out, wi.seg);
    for (uint64_t g = wi.tile_begin + tid; g < wi.tile_end; g += 256) {
      const uint64_t d0 = g * 32;
      uint32_t m = d0 + 32 <= nd ? 0xFFFFFFFFu : (d0 < nd ? (0xFFFFFFFFu >> (32u - (uint32_t)(nd - d0))) : 0u);
      if (!p.first) m &= __builtin_bitreverse32(out[g]);
      uint32_t r = 0;
      if (m) {
        switch (L.kind) {
          case LK_ALL: r = 0xFFFFFFFFu; break;
          case LK_NONE: r = 0u; break;
          case LK_DOCRANGE: {  // docs [lo, hi) within [d0, d0 + 32)
            const int64_t lo = std::max<int64_t>((int64_t)L.lo - (int64_t)d0, 0);
            const int64_t hi = std::min<int64_t>((int64_t)L.hi - (int64_t)d0, 32);
            const uint32_t below_hi = hi >= 32 ? 0xFFFFFFFFu : (hi <= 0 ? 0u : ((1u << hi) - 1u));
            r = lo >= 32 ? 0u : below_hi & ~((1u << lo) - 1u);
            break;
          }
          default: r = eval_group<B>(L, lds_sets, g, m); break;
        }
        if (L.excl) r = ~r;
      }
      const uint32_t nm = m & r;
      if (p.first || nm != m) out[g] = __builtin_bitreverse32(nm);
    }
  }
}

// A further leaf of the root AND on the docs `need` of the group at doc d0 (AndDocIdSet: later children see only the
// survivors): per needed doc a window read, rounds of up to 4 docs per lane with their loads in flight together.
__device__ __forceinline__ uint32_t eval_extra(const LeafDesc& X, const uint32_t* lds_sets, uint32_t d0, uint32_t need) {
  uint32_t r = 0;
  switch (X.kind) {
    case LK_ALL: r = 0xFFFFFFFFu; break;
    case LK_NONE: break;
    case LK_DOCRANGE: {
      const int64_t lo = std::max<int64_t>((int64_t)X.lo - (int64_t)d0, 0);
      const int64_t hi = std::min<int64_t>((int64_t)X.hi - (int64_t)d0, 32);
      const uint32_t below_hi = hi >= 32 ? 0xFFFFFFFFu : (hi <= 0 ? 0u : ((1u << hi) - 1u));
      r = lo >= 32 ? 0u : below_hi & ~((1u << lo) - 1u);
      break;
    }
    default: {  // RANGE / SET_LDS / SET_LUT on a packed column (doc bitmaps: RANGE [1, 2) on 1 bit)
      const rsrc_t rs = rsrc_of(X.words, X.wbytes);
      uint32_t rem = need;
      while (__ballot(rem != 0)) {
        uint32_t jj[4], v[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
          jj[x] = rem ? (uint32_t)__ffs(rem) - 1u : 32u;
          rem &= rem - 1u;
          v[x] = unpack_win(rs, d0 + (jj[x] < 32u ? jj[x] : 0u), X.bits);
        }
#pragma unroll
        for (int x = 0; x < 4; x++) {
          if (jj[x] >= 32u) continue;
          bool hit;
          if (X.kind == LK_RANGE) {
            hit = (v[x] - (uint32_t)X.lo) < (uint32_t)(X.hi - X.lo);
          } else if (X.kind == LK_SET_LDS) {
            const uint32_t y = v[x] >> X.shift;
            hit = (lds_sets[X.lds_off + (y >> 5)] >> (y & 31u)) & 1u;
            if (hit && X.shift) hit = (X.lut[v[x] >> 5] >> (v[x] & 31u)) & 1u;
          } else {
            hit = (X.aux[v[x] >> 5] >> (v[x] & 31u)) & 1u;
          }
          r |= (uint32_t)hit << jj[x];
        }
      }
    }
  }
  return X.excl ? ~r : r;
}

// The same test from the wave's LDS slice: the words of its 64 consecutive groups (lane l's group = words
// [l * B, l * B + B) of the slice), staged by stage_slice.
__device__ __forceinline__ uint32_t eval_staged(const LeafDesc& X, const uint32_t* lds_sets, const uint32_t* slice,
                                                uint32_t lane, uint32_t need) {
  const uint32_t b = X.bits, mask = 0xFFFFFFFFu >> (32u - b);
  uint32_t r = 0;
  for (uint32_t rem = need; rem; rem &= rem - 1u) {
    const uint32_t j = (uint32_t)__ffs(rem) - 1u;
    const uint32_t bit = (lane * 32u + j) * b, k = bit >> 5;
    const uint64_t win = ((uint64_t)slice[k] << 32) | (uint64_t)slice[k + 1];
    const uint32_t v = (uint32_t)(win >> (64u - (bit & 31u) - b)) & mask;
    bool hit;
    if (X.kind == LK_RANGE) {
      hit = (v - (uint32_t)X.lo) < (uint32_t)(X.hi - X.lo);
    } else if (X.kind == LK_SET_LDS) {
      const uint32_t y = v >> X.shift;
      hit = (lds_sets[X.lds_off + (y >> 5)] >> (y & 31u)) & 1u;
      if (hit && X.shift) hit = (X.lut[v >> 5] >> (v & 31u)) & 1u;
    } else {
      hit = (X.aux[v >> 5] >> (v & 31u)) & 1u;
    }
    r |= (uint32_t)hit << j;
  }
  return X.excl ? ~r : r;
}

// The wave's 64 groups [wg0, wg0 + 64) of a b-bit column into its slice: 64 * b words + 4 of window padding, 16-byte
// loads (reads past the column return 0).  Wave-local: the same wave reads the slice back.
__device__ __forceinline__ void stage_slice(const LeafDesc& X, uint32_t wg0, uint32_t* slice, uint32_t lane) {
  const rsrc_t rs = rsrc_of(X.words, X.wbytes);
  const uint32_t nq = 16u * X.bits + 1u, w0 = wg0 * X.bits;
  for (uint32_t q = lane; q < nq; q += 64u) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (w0 + 4u * q) * 4u, 0, 0);
    *(uint4*)(slice + 4u * q) = make_uint4(v[0], v[1], v[2], v[3]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef PG_STREAM_STAGE_BOTH
#define PG_STREAM_STAGE_BOTH 0  // 1 (dev variant): the first two further leaves' slices (<= 8 bits) loaded together
#endif

// The first two further leaves' slices of the wave's 64 groups (<= 8 bits: <= 129 quads, 3 loads per lane each), every
// load issued before any is stored, so the two slices cost one memory latency instead of two (PG_STREAM_STAGE_BOTH).
__device__ __forceinline__ void stage_two(const LeafDesc& A, const LeafDesc& B, uint32_t wg0, uint32_t* sa, uint32_t* sb,
                                          uint32_t lane) {
  const rsrc_t ra = rsrc_of(A.words, A.wbytes), rb = rsrc_of(B.words, B.wbytes);
  const uint32_t na = 16u * A.bits + 1u, nb = 16u * B.bits + 1u, wa = wg0 * A.bits, wb = wg0 * B.bits;
  uint4 va[3], vb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t q = lane + 64u * k;
    va[k] = vb[k] = make_uint4(0u, 0u, 0u, 0u);
    if (q < na) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(ra, (wa + 4u * q) * 4u, 0, 0);
      va[k] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    if (q < nb) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(rb, (wb + 4u * q) * 4u, 0, 0);
      vb[k] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t q = lane + 64u * k;
    if (q < na) *(uint4*)(sa + 4u * q) = va[k];
    if (q < nb) *(uint4*)(sb + 4u * q) = vb[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The selective stream: the driving leaf of the root AND over the block's items (32-doc groups, thread-contiguous
// 16-byte loads, 6 waves per SIMD so ~120 KiB per CU are in flight), survivors appended to the item's region in group
// order within each wave: one wave prefix sum + one LDS cursor atomic per wave and group round that has a survivor.
// This is SVScanDocIdIterator over the first AND child, the compacted output playing the role of its docId batches.
// EXTRA: further AND leaves tested on the survivors (their code costs registers: 71 VGPRs at 7 waves per SIMD with,
// 72 / 7 without).  Items: contiguous ranges per block (block_first), or with `interleave` item b + k * gridDim.x.
// NT: threads per block.  NT = 1024 is exact mode (p.exact): one block per CU holding the exact LUT.
constexpr uint32_t kExactLutWords = 32768;  // 128 KiB: the exact LUT of a <= 1 M-entry dictionary

// Words of dynamic LDS the stream's sets / LUT / slices take; the block's append cursor is the word after them (no
// static LDS in the kernel, so the exact LUT sits at LDS address 0).
__host__ __device__ __forceinline__ uint32_t stream_lds_words(const StreamSpec& p, bool exact) {
  return exact ? kExactLutWords
               : p.set_lds_ints + (p.num_extra ? 4u * p.stage_words * ((p.stage_pre || PG_STREAM_STAGE_BOTH) ? p.num_extra : 1u) : 0u);
}

#ifndef PG_STREAM_PIPE_EXTRA
#define PG_STREAM_PIPE_EXTRA 0  // 1: the variant with further leaves pipelines the driving leaf's loads too (5 waves / SIMD; config 3 stream 0.713 vs 0.596 ms, r04d)
#endif

template <int B, bool EXTRA, int NT>
#ifndef PG_STREAM_EXTRA_WAVES
#define PG_STREAM_EXTRA_WAVES 7  // waves / SIMD the further-leaf variant's register budget allows (71 VGPRs, no scratch; config 3 stream 0.579 vs 0.595 ms at 6, 0.631 at 8)
#endif
__global__ __launch_bounds__(NT, NT == 1024 ? 4 : (EXTRA ? (PG_STREAM_PIPE_EXTRA && B <= 20 ? 5 : PG_STREAM_EXTRA_WAVES) : 7)) void stream_kernel(StreamSpec p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_sets[];
  constexpr bool EXACT = NT == 1024;
  constexpr bool PIPE = EXACT || (EXTRA && PG_STREAM_PIPE_EXTRA && B <= 20);
  uint32_t& cursor = lds_sets[stream_lds_words(p, EXACT)];
  // the exact LUT's lookups address LDS absolutely (eval_group): the dynamic LDS must start at address 0
  if (EXACT && threadIdx.x == 0 && (uint32_t)(uintptr_t)(lds_cptr)lds_sets != 0u) atomicOr(p.err, 64u);
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  if (p.stamp && tid == 0) atomicMax(&p.stamp[0], ~(unsigned long long)wall_clock64());
  const uint32_t i0 = p.interleave ? ldcf(p.block_first, 0) + blockIdx.x : ldcf(p.block_first, blockIdx.x);
  const uint32_t i1 = ldcf(p.block_first, p.interleave ? gridDim.x : blockIdx.x + 1);
  const uint32_t istep = p.interleave ? gridDim.x : 1u;
  uint32_t cur_seg = 0xFFFFFFFFu;
  LeafDesc L;
  const LeafDesc* seg_leaves = nullptr;
  uint32_t nd = 0;
  for (uint32_t it = i0; it < i1; it += istep) {
    const WorkItem wi = ldcf(p.items, it);
    if (wi.seg != cur_seg) {
      const SegDesc sd = ldcf(p.segs, wi.seg);
      seg_leaves = sd.leaves;
      L = ldcf(sd.leaves, p.leaf);
      nd = sd.num_docs;
      if (EXACT) {
        __syncthreads();  // every thread is done with the previous segment's LUT
        const ExactSet es = ldcf(p.exact, wi.seg);
        if (L.kind == LK_SET_LDS && (es.ids || es.vals)) {
          // the segment's exact LUT built in LDS from its IN list: each thread resolves its dictIds (values mode: the
          // literal's dictionary lookup, PredicateUtils.getDictIdSet) while the LUT's words are zeroed (16-byte
          // stores), then one LDS atomic per dictId -- no global LUT, no set_lut_bits launch, no 128 KiB staging read
          const uint32_t nq = (es.nwords + 3u) / 4u, lim = 32u * es.nwords;
          auto id_at = [&](uint32_t k) -> int32_t {
            return es.ids ? es.ids[k] : dict_find_typed(es.dict, es.card, es.dtype, es.vals, k);
          };
          const int32_t id0 = tid < es.n ? id_at(tid) : -1;
          for (uint32_t q0 = tid; q0 < nq; q0 += NT) ((uint4*)lds_sets)[q0] = make_uint4(0u, 0u, 0u, 0u);
          __syncthreads();
          if (id0 >= 0 && (uint32_t)id0 < lim) atomicOr(&lds_sets[(uint32_t)id0 >> 5], 1u << (id0 & 31));
          for (uint32_t k = tid + NT; k < es.n; k += NT) {
            const int32_t v = id_at(k);
            if (v >= 0 && (uint32_t)v < lim) atomicOr(&lds_sets[(uint32_t)v >> 5], 1u << (v & 31));
          }
        } else if (L.kind == LK_SET_LDS) {
          // the segment's exact LUT (up to 128 KiB) into LDS: 16-byte buffer loads, 8 per thread issued before any is
          // stored (one load latency per segment change instead of one per word; reads past the LUT return 0)
          const uint32_t nw = es.nwords, nq = (nw + 3u) / 4u;
          const rsrc_t rl = rsrc_of(L.lut, 4u * nw);
          constexpr uint32_t kU = 8;
          for (uint32_t q0 = tid; q0 < nq; q0 += NT * kU) {
            uint4 v[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
              const auto x = __builtin_amdgcn_raw_buffer_load_b128(rl, (q0 + u * NT) * 16u, 0, 0);
              v[u] = make_uint4(x[0], x[1], x[2], x[3]);
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++)
              if (q0 + u * NT < nq) ((uint4*)lds_sets)[q0 + u * NT] = v[u];
          }
        }
      } else if (p.set_lds_ints) {
        __syncthreads();  // every thread is done with the previous segment's sets
        for (uint32_t x = 0; x <= (EXTRA ? p.num_extra : 0u); x++) {
          const LeafDesc S = x ? ldcf(sd.leaves, p.extra[x - 1]) : L;
          if (S.kind != LK_SET_LDS) continue;
          for (uint32_t k = tid; k < S.set_ints; k += NT) lds_sets[S.lds_off + k] = S.aux[k];
        }
      }
      cur_seg = wi.seg;
    }
    if (tid == 0) cursor = 0u;
    __syncthreads();  // set staged, cursor reset
    uint32_t* out = p.docs + (uint64_t)it * p.cap;
    if (L.kind != LK_NONE) {
      // exact mode is software-pipelined: the next group's words are loaded before this group is tested, so each lane
      // keeps two groups' loads in flight (160 KiB per CU at B = 20; 96 VGPRs of the 128 its 4 waves / SIMD allow --
      // the 256-thread variants run 6-7 waves / SIMD and would spill)
      const rsrc_t rs = rsrc_of(L.words, L.wbytes);
      uint32_t w[B + 1];
      if (PIPE && wi.tile_begin + tid < wi.tile_end) load_group<B>(rs, wi.tile_begin + tid, w);
      for (uint32_t g0 = wi.tile_begin; g0 < wi.tile_end; g0 += NT) {
        const uint32_t g = g0 + tid;
        const uint64_t d0 = (uint64_t)g * 32;
        uint32_t m = 0;
        if (EXTRA && p.stage_pre) {
          // the further leaves' slices of this wave's 64 groups, DMA'd into LDS (buffer_load ... lds) before the driving
          // leaf's loads: both in flight together, no registers held (reads past a column return 0)
          for (uint32_t x = 0; x < p.num_extra; x++) {
            const LeafDesc X = ldcf(seg_leaves, p.extra[x]);
            const bool packed = X.kind == LK_RANGE || X.kind == LK_SET_LDS || X.kind == LK_SET_LUT;
            if (!packed || X.bits * 64u + 4u > p.stage_words) continue;
            uint32_t* slice = lds_sets + p.set_lds_ints + ((tid >> 6) * p.num_extra + x) * p.stage_words;
            const rsrc_t rx = rsrc_of(X.words, X.wbytes);
            const uint32_t nq = 16u * X.bits + 1u, w0 = (g0 + (tid & ~63u)) * X.bits;
            for (uint32_t q0 = 0; q0 < nq; q0 += 64u)
              if (q0 + lane < nq)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(slice + 4u * q0), 16,
                                                         (w0 + 4u * (q0 + lane)) * 4u, 0, 0, 0);
          }
        }
        if (PIPE) {
          uint32_t wn[B + 1];
          if (g + NT < wi.tile_end) load_group<B>(rs, g + NT, wn);
          if (g < wi.tile_end && d0 < nd) {
            const uint32_t valid = d0 + 32 <= nd ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32u - (uint32_t)(nd - d0)));
            uint32_t r = test_group<B>(L, lds_sets, g, valid, EXACT && L.kind == LK_SET_LDS, w);
            if (L.excl) r = ~r;
            m = r & valid;
          }
#pragma unroll
          for (int k = 0; k <= B; k++) w[k] = wn[k];
        } else if (g < wi.tile_end && d0 < nd) {
          const uint32_t valid = d0 + 32 <= nd ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32u - (uint32_t)(nd - d0)));
          uint32_t r = eval_group<B>(L, lds_sets, g, valid, EXACT && L.kind == LK_SET_LDS);
          if (L.excl) r = ~r;
          m = r & valid;
        }
        bool staged2 = false;  // PG_STREAM_STAGE_BOTH: extras 0 and 1 already in their slices
        if (EXTRA && PG_STREAM_STAGE_BOTH && !p.stage_pre && p.stage_words && p.num_extra >= 2 && __ballot(m != 0)) {
          const LeafDesc X0 = ldcf(seg_leaves, p.extra[0]), X1 = ldcf(seg_leaves, p.extra[1]);
          auto two_ok = [](const LeafDesc& X) {
            return (X.kind == LK_RANGE || X.kind == LK_SET_LDS || X.kind == LK_SET_LUT) && X.bits <= 8u;
          };
          if (two_ok(X0) && two_ok(X1)) {
            uint32_t* s0 = lds_sets + p.set_lds_ints + ((tid >> 6) * p.num_extra) * p.stage_words;
            stage_two(X0, X1, g0 + (tid & ~63u), s0, s0 + p.stage_words, lane);
            staged2 = true;
          }
        }
        for (uint32_t x = 0; x < (EXTRA ? p.num_extra : 0u); x++) {
          if (__ballot(m != 0) == 0) break;
          const LeafDesc X = ldcf(seg_leaves, p.extra[x]);
          const bool packed = X.kind == LK_RANGE || X.kind == LK_SET_LDS || X.kind == LK_SET_LUT;
          if (EXTRA && p.stage_words && packed && X.bits * 64u + 4u <= p.stage_words) {
            uint32_t* slice = lds_sets + p.set_lds_ints +
                              ((p.stage_pre || PG_STREAM_STAGE_BOTH) ? (tid >> 6) * p.num_extra + x : (tid >> 6)) * p.stage_words;
            if (p.stage_pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slice's DMA has landed
            else if (!(staged2 && x < 2)) stage_slice(X, g0 + (tid & ~63u), slice, lane);
            if (m) m &= eval_staged(X, lds_sets, slice, lane, m);
          } else if (m) {
            m &= eval_extra(X, lds_sets, (uint32_t)d0, m);
          }
        }
        if (__ballot(m != 0) == 0) continue;
        const uint32_t cnt = __popc(m);
        uint32_t x = cnt;  // inclusive prefix over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o);
          if (lane >= (uint32_t)o) x += y;
        }
        uint32_t base = 0;
        if (lane == 63) base = __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)&cursor, x,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        base = __builtin_amdgcn_readlane(base, 63);
        uint32_t pos = base + x - cnt;
        for (uint32_t r = m; r; r &= r - 1u, pos++)
          if (pos < p.cap) out[pos] = (uint32_t)d0 + (uint32_t)(__ffs(r) - 1);
      }
    }
    __syncthreads();  // every append of this item is counted
    if (tid == 0) {
      const uint32_t n = cursor;
      p.counts[it] = n < p.cap ? n : p.cap;
      if (n > p.cap) atomicOr(p.err, 8u);
    }
  }
  if (p.stamp && tid == 0) atomicMax(&p.stamp[1], (unsigned long long)wall_clock64());
}

hipError_t launch_stream(const StreamSpec& p, uint32_t bits, uint32_t blocks, hipStream_t s) {
  if (!p.num_items || !blocks) return hipSuccess;
  const size_t lds = 4ull * stream_lds_words(p, p.exact != nullptr) + 16;  // + the cursor word
  if (p.exact) {
    static bool attr = false;  // >64 KiB of dynamic LDS must be opted into per kernel (once per process)
    if (!attr) {
#define PG_A(b)                                                                                                 \
  (void)hipFuncSetAttribute((const void*)stream_kernel<b, false, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                            4 * kExactLutWords + 16);                                                            \
  (void)hipFuncSetAttribute((const void*)stream_kernel<b, true, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                            4 * kExactLutWords + 16);
      PG_A(1) PG_A(2) PG_A(3) PG_A(4) PG_A(5) PG_A(6) PG_A(7) PG_A(8) PG_A(9) PG_A(10) PG_A(11) PG_A(12) PG_A(13)
      PG_A(14) PG_A(15) PG_A(16) PG_A(17) PG_A(18) PG_A(19) PG_A(20) PG_A(21) PG_A(22) PG_A(23) PG_A(24) PG_A(25)
      PG_A(26) PG_A(27) PG_A(28) PG_A(29) PG_A(30) PG_A(31) PG_A(32)
#undef PG_A
      attr = true;
    }
  }
  switch (bits) {
#define PG_B(b)                                                                                              \
  case b:                                                                                                    \
    if (p.exact && p.num_extra) hipLaunchKernelGGL((stream_kernel<b, true, 1024>), dim3(blocks), dim3(1024), lds, s, p); \
    else if (p.exact) hipLaunchKernelGGL((stream_kernel<b, false, 1024>), dim3(blocks), dim3(1024), lds, s, p); \
    else if (p.num_extra) hipLaunchKernelGGL((stream_kernel<b, true, 256>), dim3(blocks), dim3(256), lds, s, p); \
    else hipLaunchKernelGGL((stream_kernel<b, false, 256>), dim3(blocks), dim3(256), lds, s, p);                \
    break;
    PG_B(1) PG_B(2) PG_B(3) PG_B(4) PG_B(5) PG_B(6) PG_B(7) PG_B(8) PG_B(9) PG_B(10) PG_B(11) PG_B(12) PG_B(13)
    PG_B(14) PG_B(15) PG_B(16) PG_B(17) PG_B(18) PG_B(19) PG_B(20) PG_B(21) PG_B(22) PG_B(23) PG_B(24) PG_B(25)
    PG_B(26) PG_B(27) PG_B(28) PG_B(29) PG_B(30) PG_B(31) PG_B(32)
#undef PG_B
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_prefilter(const PreSpec& p, uint32_t bits, uint32_t blocks, hipStream_t s) {
  if (!p.num_items || !blocks) return hipSuccess;
  const size_t lds = (size_t)p.set_lds_ints * 4;
  switch (bits) {
#define PG_B(b) case b: hipLaunchKernelGGL(prefilter_kernel<b>, dim3(blocks), dim3(256), lds, s, p); break;
    PG_B(1) PG_B(2) PG_B(3) PG_B(4) PG_B(5) PG_B(6) PG_B(7) PG_B(8) PG_B(9) PG_B(10) PG_B(11) PG_B(12) PG_B(13)
    PG_B(14) PG_B(15) PG_B(16) PG_B(17) PG_B(18) PG_B(19) PG_B(20) PG_B(21) PG_B(22) PG_B(23) PG_B(24) PG_B(25)
    PG_B(26) PG_B(27) PG_B(28) PG_B(29) PG_B(30) PG_B(31) PG_B(32)
#undef PG_B
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pg
