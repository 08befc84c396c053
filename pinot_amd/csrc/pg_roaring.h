// pg_roaring.h -- device-side decoding of one 64 K-doc key of inverted-index leaves (BitmapBasedFilterOperator's OR of
// the selected dictIds' RoaringBitmaps, restricted to one high-16-bit key) into LDS chunks of 2 048 words, shared by
// the index pre-pass (pg_kernels.hip roaring_keys_kernel: one leaf) and the fused index count (pg_index.hip: every
// inverted leaf of the filter at once).
//
// Chunk word w, bit 31 - j <-> doc key * 65 536 + 32 w + j (the packed 1-bit column order).  Containers follow the
// RoaringBitmap portable format (RoaringBitmap 0.9.28): array (sorted uint16), bitmap (1 024 little-endian uint64) and
// run ((start, length - 1) uint16 pairs) containers, re-laid 8-byte aligned and key-major (by key, then dictId) at upload,
// the payload region padded to whole 8-byte words (pg_runtime.hip parse_inverted), so an array container is read as
// 8-byte quads of 4 entries.
#pragma once
#include <hip/hip_runtime.h>

#include "pg_aux.h"

namespace pg {

// dictIds per thread per round: a round issues its R container lookups per thread before any is consumed (config 5's
// 2 022 selected dictIds: two rounds at 256 threads)
#ifndef PG_ROAR_R
#define PG_ROAR_R 4
#endif
#ifndef PG_ROAR_Q
#define PG_ROAR_Q 4
#endif
#ifndef PG_ROAR_BIG  // large-array list entries per round, in threads (1 or 2)
#define PG_ROAR_BIG 2
#endif
#ifndef PG_ROAR_OWN  // owner-table windows (8 quads each)
#define PG_ROAR_OWN 1024
#endif
#ifndef PG_ROAR_SB  // 1: a scheduling barrier after each container's ORs (bounds the addresses live at once)
#define PG_ROAR_SB 1
#endif
#ifndef PG_ROAR_MASKED  // 1: an array entry slot past the container's end ORs 0 instead of branching around its OR
#define PG_ROAR_MASKED 0
#endif
constexpr int kRoarR = PG_ROAR_R;
constexpr int kRoarQ = PG_ROAR_Q;  // quads of the large array containers per thread per step (loads in flight together)
constexpr uint32_t kRoarSmall = 8;  // array containers of <= 8 entries: expanded by the thread that found them
constexpr uint32_t kRoarMaxViews = 8;
static_assert(kRoarR >= 1 && kRoarR <= 16 && kRoarQ >= 1 && kRoarQ <= 32, "roaring decode knobs");

// dev instrumentation (PG_IDX_PROF=1 variant builds only: tools/variant.sh pg_index): thread 0 of a block adds cycle
// deltas per decode phase into prof[1..4] (directory lookups, classify + lists, array quads, bitmap containers)
#ifndef PG_IDX_PROF
#define PG_IDX_PROF 0
#endif
// dev ablation (variant builds only, wrong results): skip 1 small arrays, 2 large arrays, 4 bitmaps, 8 the COUNTMV
// count words, 16 the directory loads, 32 / 64 the small / large arrays' ORs (their loads kept) -- the kernel-time
// deltas price each part
#ifndef PG_IDX_SKIP
#define PG_IDX_SKIP 0
#endif
// clock64 (s_memtime).  It perturbs what it measures: its result waits on lgkmcnt, and the lap accumulators live in
// scratch, whose stores wait on vmcnt -- the laps rank the phases, the absolute times run ~2x long.  (The 20-bit
// SHADER_CYCLES register would avoid the waits, but reads 0 on these boxes.)
__device__ __forceinline__ unsigned long long prof_clk() { return (unsigned long long)clock64(); }
#define ROAR_LAP(ph)                                                              \
  do {                                                                            \
    if (PG_IDX_PROF && prof && threadIdx.x == 0) {                                \
      const unsigned long long n_ = prof_clk();                                    \
      prof[ph] += n_ - t_;                                                        \
      t_ = n_;                                                                    \
    }                                                                             \
  } while (0)

// A block barrier that orders LDS only: __syncthreads() also waits for every outstanding global load (vmcnt(0)), which
// would drain the prefetches this decode keeps in flight across its phases (the count words, the small containers).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One inverted leaf to decode: its column's containers, the selected dictIds, the LDS chunk it is OR-ed into.
struct RoarView {
  const uint8_t* roaring;
  const RoaringContainer* cs;
  const uint32_t* dir;
  const uint2* keydir;      // optional key-major directory: [key * card + dictId] = keydir_entry or ~0 ~0
  const int32_t* ids;
  uint32_t chunk;           // its LDS chunk: word offset in the decode's `lds` array (an offset, not a pointer kept in
  uint32_t nids, card;      //   LDS: a pointer read back from LDS is generic, and its atomics compile to flat atomics)
};

// LDS scratch of one decode (besides the chunks and the views)
template <int NT>
struct RoaringLds {
  static constexpr uint32_t kBig = PG_ROAR_BIG * NT;  // large array containers listed per round (more: the finder
                                                      // expands it)
  static constexpr uint32_t kOwn = PG_ROAR_OWN;  // 8-quad windows the owner table covers (more: a binary search)
  uint32_t bml[NT];            // bitmap containers of this round (payload offsets), OR-ed by the whole block
  uint8_t bview[NT];           //   and their views (more than NT in a round: the finder ORs it in by itself)
  uint32_t nbml[2];            //   (counters double-buffered by round parity: reset a round ahead, no barrier of their own)
  uint32_t goff[kBig];         // array containers of more than kRoarSmall entries: payload offset,
  uint16_t gcard[kBig];        //   cardinality,
  uint8_t gview[kBig];         //   view,
  uint32_t gpre[kBig + 1];     //   first quad among the round's (exclusive prefix; [ng] = the total)
  uint16_t gown[kOwn];         // the entry holding quad 8 j (the quads' owner search starts there: <= 3 steps)
  uint32_t ng[2];
  uint32_t wsum[NT / 64];
  uint32_t vpre[kRoarMaxViews + 1];  // prefix of the views' dictId counts
};

// OR one array container's entries (8-byte quads of 4 uint16 at `src`) into `chunk`, quad by quad (the rare path: a
// round with more large containers than the list holds)
__device__ __forceinline__ void roaring_array_or(const uint8_t* src, uint32_t card, uint32_t* __restrict__ chunk) {
  for (uint32_t q = 0; 4 * q < card; q++) {
    const uint2 w = ld_global((const uint2*)(src + 8u * q));
    const uint32_t v4[4] = {w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16};
#pragma unroll
    for (uint32_t h = 0; h < 4; h++)
      if (4 * q + h < card) atomicOr(&chunk[v4[h] >> 5], 0x80000000u >> (v4[h] & 31u));
  }
}

// OR the containers of `key` of every view's selected dictIds into the view's chunk (zeroed by the caller).  The views'
// dictIds are taken as one list, so a round's lookups span the leaves (config 5: 4 leaves of 1 + 20 + 1 + 2 000 ids
// decode in two rounds of NT * kRoarR).  Per round, three dependent global loads: the dictIds, the directory entries,
// then every small array container's two quads (its finder, no LDS hand-off), every large array container's quads
// (the whole block, kRoarQ per thread per step, each quad's owner from the 8-quad-window table) and the first bitmap
// container's words; runs are expanded by their finder.  Every bit is set by an LDS atomic, so no barrier orders the
// kinds.  `V` (nv <= kRoarMaxViews entries) is visible to the whole block; starts and ends with a
// block barrier.  `lds`: the chunks' array, a __shared__ array of the caller (so the ORs compile to LDS atomics).
template <int NT>
__device__ __forceinline__ void roaring_key_chunks(const RoarView* V, uint32_t nv, uint32_t key, RoaringLds<NT>& S,
                                                   uint32_t* lds, unsigned long long* prof = nullptr) {
  constexpr int R = kRoarR;
  constexpr uint32_t kBig = RoaringLds<NT>::kBig;
  unsigned long long t_ = PG_IDX_PROF ? prof_clk() : 0ull;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t sink = 0;  // (PG_IDX_SKIP 32 / 64: the loads kept alive without their ORs)
  if (tid == 0) {
    S.nbml[0] = S.nbml[1] = 0;
    S.ng[0] = S.ng[1] = 0;
    uint32_t a = 0;
    for (uint32_t l = 0; l < nv; l++) { S.vpre[l] = a; a += V[l].nids; }
    S.vpre[nv] = a;
  }
  lds_barrier();
  const uint32_t nids = S.vpre[nv];
  const uint8_t* const base0 = V[0].roaring;  // a harmless address for the loads of lanes with nothing to load
  uint32_t vp[kRoarMaxViews];  // view j's first index in the combined list (~0 past the last view): selects by compares
#pragma unroll
  for (uint32_t j = 0; j < kRoarMaxViews; j++) vp[j] = j < nv ? S.vpre[j] : 0xFFFFFFFFu;
  for (uint32_t r0 = 0, par = 0; r0 < nids; r0 += NT * R, par ^= 1u) {
    // 1. the container of `key` of each of this thread's dictIds: the views (LDS), then the R dictIds, then the R
    //    key-major directory entries (one 8-byte load each: the descriptor itself) -- each set of R loads in flight
    //    together, as straight-line code with no branch between a load and the next one (a load under a per-lane
    //    branch followed by the next lookup's wait would serialise them); views without the key-major directory
    //    search the dictId's containers afterwards
    uint32_t vw[R], id[R], live = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
      const uint32_t i = r0 + tid + NT * k;
      uint32_t l = 0, first = 0;
#pragma unroll
      for (uint32_t j = 1; j < kRoarMaxViews; j++) {
        l += vp[j] <= i ? 1u : 0u;
        first = vp[j] <= i ? vp[j] : first;
      }
      vw[k] = l;
      live |= (i < nids ? 1u : 0u) << k;
      id[k] = i < nids ? i - first : 0u;  // (the index into view l's dictIds, then the dictId below)
    }
#pragma unroll
    for (int k = 0; k < R; k++) id[k] = (uint32_t)ld_global(V[vw[k]].ids + id[k]);
    RoaringContainer c[R];
    bool search = false;
#pragma unroll
    for (int k = 0; k < R; k++) {
      const RoarView& v = V[vw[k]];
      const uint2* a = v.keydir ? v.keydir + ((uint64_t)key * v.card + id[k]) : (const uint2*)v.roaring;
      const uint2 e = (PG_IDX_SKIP & 16) ? make_uint2(~0u, ~0u) : ld_global(a);
      c[k] = RoaringContainer{key, e.y >> 30, e.y & 0x3FFFFFFFu, e.x};
      search |= !v.keydir && ((live >> k) & 1u);
    }
    if (search) {  // this dictId's containers, ascending keys: find `key`
#pragma unroll
      for (int k = 0; k < R; k++) {
        const RoarView& v = V[vw[k]];
        if (v.keydir || !((live >> k) & 1u)) continue;
        uint32_t lo = ld_global(v.dir + id[k]), hi = ld_global(v.dir + id[k] + 1);
        const uint32_t end = hi;
        while (lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (ld_global(&v.cs[m].key) < key) lo = m + 1; else hi = m;
        }
        const uint4 f = lo < end ? ld_global((const uint4*)(v.cs + lo)) : make_uint4(key + 1u, 3u, 0u, 0u);
        c[k] = f.x == key ? RoaringContainer{f.x, f.y, f.z, f.w} : RoaringContainer{key, 3u, 0u, 0u};
      }
    }
#pragma unroll
    for (int k = 0; k < R; k++)
      if (!((live >> k) & 1u)) c[k].type = 3u;  // (after every load: not a select at the load)
    ROAR_LAP(1);
    // 2. small arrays: both quads loaded now by their finder (unconditionally: a lane with none reads base0, so the
    //    loads stay in flight while the lists below are built); large arrays -> the block's list, bitmaps -> the
    //    block's list, runs expanded here
    uint2 sq[R][2];
    uint32_t sinfo[R];  // small array: card | its chunk's word offset << 4 (0: none)
#pragma unroll
    for (int k = 0; k < R; k++) {
      const bool sm = c[k].type == 0 && c[k].card <= kRoarSmall;
      sinfo[k] = sm ? c[k].card | V[vw[k]].chunk << 4 : 0u;
      const uint8_t* a = sm ? V[vw[k]].roaring + c[k].offset : base0;
      sq[k][0] = ld_global((const uint2*)a);
      sq[k][1] = ld_global((const uint2*)(a + (sm && c[k].card > 4u ? 8u : 0u)));
    }
#pragma unroll
    for (int k = 0; k < R; k++) {
      if (c[k].type == 0 && c[k].card > kRoarSmall) {
        const uint32_t g = atomicAdd(&S.ng[par], 1u);
        if (g < kBig) {
          S.goff[g] = c[k].offset;
          S.gcard[g] = (uint16_t)c[k].card;
          S.gview[g] = (uint8_t)vw[k];
        } else {
          roaring_array_or(V[vw[k]].roaring + c[k].offset, c[k].card, lds + V[vw[k]].chunk);
        }
      } else if (c[k].type == 1) {
        const uint32_t b = atomicAdd(&S.nbml[par], 1u);
        if (b < NT) {
          S.bml[b] = c[k].offset;
          S.bview[b] = (uint8_t)vw[k];
        } else {  // list full (more than NT bitmap containers in one round): this thread ORs it in word by word
          const uint32_t* src = (const uint32_t*)(V[vw[k]].roaring + c[k].offset);
          uint32_t* chunk = lds + V[vw[k]].chunk;
          for (uint32_t wd = 0; wd < 2048; wd++) {
            const uint32_t x = ld_global(src + wd);
            if (x) atomicOr(&chunk[wd], __builtin_bitreverse32(x));
          }
        }
      } else if (c[k].type == 2) {  // runs: uint16 nruns, then (start, length - 1)
        const uint16_t* rr = (const uint16_t*)(V[vw[k]].roaring + c[k].offset) + 1;
        uint32_t* chunk = lds + V[vw[k]].chunk;
        for (uint32_t q = 0; q < c[k].card; q++) {
          const uint32_t st = ld_global(rr + 2 * q), en = st + ld_global(rr + 2 * q + 1);
          for (uint32_t w = st >> 5; w <= (en >> 5); w++) {
            const uint32_t l = w * 32 > st ? 0 : st - w * 32, h = w * 32 + 31 < en ? 31 : en - w * 32;
            const uint32_t mask = (h == 31 ? 0xFFFFFFFFu : ((1u << (h + 1)) - 1u)) & ~((1u << l) - 1u);
            atomicOr(&chunk[w], __builtin_bitreverse32(mask));
          }
        }
      }
    }
    lds_barrier();
    // exclusive prefix of the listed containers' quads: entries 2 t, 2 t + 1 per thread (wave scan + wave sums); the
    // owner windows from the prefix in registers (entry g holds quads [gpre[g], gpre[g] + n), so the windows j with
    // 8 j in that range)
    const uint32_t ng = S.ng[par] < kBig ? S.ng[par] : kBig;
    const uint32_t nb = S.nbml[par] < NT ? S.nbml[par] : NT;
    if (tid == 0) { S.ng[par ^ 1u] = 0; S.nbml[par ^ 1u] = 0; }  // (the previous round's, read before its last barrier)
    const uint32_t q0 = 2 * tid < ng ? ((uint32_t)S.gcard[2 * tid] + 3u) >> 2 : 0u;
    const uint32_t q1 = 2 * tid + 1 < ng ? ((uint32_t)S.gcard[2 * tid + 1] + 3u) >> 2 : 0u;
    uint32_t x = q0 + q1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) S.wsum[wave] = x;
    lds_barrier();
    uint32_t wb = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; w++) {
      const uint32_t ws = S.wsum[w];
      wb += w < wave ? ws : 0u;
      total += ws;
    }
    const uint32_t p0 = wb + x - q0 - q1, p1 = wb + x - q1;
    if (2 * tid < kBig) S.gpre[2 * tid] = p0;
    if (2 * tid + 1 < kBig) S.gpre[2 * tid + 1] = p1;
    if (tid == 0) S.gpre[ng] = total;
    const bool own = total <= 8 * RoaringLds<NT>::kOwn;
    if (own) {
      for (uint32_t j = (p0 + 7) >> 3; j < (p0 + q0 + 7) >> 3; j++) S.gown[j] = (uint16_t)(2 * tid);
      for (uint32_t j = (p1 + 7) >> 3; j < (p1 + q1 + 7) >> 3; j++) S.gown[j] = (uint16_t)(2 * tid + 1);
    }
    lds_barrier();
    ROAR_LAP(2);
    // 3. the loads of the first bitmap container's words (this thread's 2048 / NT) and of the large arrays' first quads
    //    are issued, then the small arrays' entries (their loads were in flight over the lists and the scan) and the
    //    quads are OR-ed in.  Every LDS read this needs (list entries, view chunks) comes before the first OR: an LDS
    //    read after an OR would wait for it (lgkmcnt counts in order), one wait per container.
    constexpr uint32_t kWpt = 2048u / NT;
    uint32_t bw[kWpt];
#pragma unroll
    for (uint32_t j = 0; j < kWpt; j++) bw[j] = 0u;
    if (nb) {  // (block-uniform: a branch, not a select that would wait for the loads here)
      const uint32_t* src = (const uint32_t*)(V[S.bview[0]].roaring + S.bml[0]);
#pragma unroll
      for (uint32_t j = 0; j < kWpt; j++) bw[j] = ld_global(src + tid + j * NT);
    }
    const uint32_t bchunk0 = nb ? V[S.bview[0]].chunk : 0u;
    constexpr int kQ = kRoarQ;
    for (uint32_t e0 = tid;; e0 += kQ * NT) {
      uint2 w[kQ];
      uint32_t nq[kQ];  // entries of the quad (0..4) | its chunk's word offset << 4
#pragma unroll
      for (int u = 0; u < kQ; u++) {
        const uint32_t e = e0 + (uint32_t)u * NT;
        const uint8_t* a = base0;
        nq[u] = 0;
        if (e < total && !(PG_IDX_SKIP & 2)) {  // owner entry: the last prefix <= e
          uint32_t lo = 0;
          if (own) {  // from its window's owner, forward (entries hold >= 3 quads: at most 3 steps)
            lo = S.gown[e >> 3];
            while (lo + 1 < ng && S.gpre[lo + 1] <= e) lo++;
          } else {
            uint32_t hi = ng;
            while (hi - lo > 1) {
              const uint32_t m = (lo + hi) >> 1;
              if (S.gpre[m] <= e) lo = m; else hi = m;
            }
          }
          const uint32_t q = e - S.gpre[lo], left = (uint32_t)S.gcard[lo] - 4u * q;
          const RoarView& v = V[S.gview[lo]];
          nq[u] = (left < 4u ? left : 4u) | v.chunk << 4;
          a = v.roaring + S.goff[lo] + 8u * q;
        }
        w[u] = ld_global((const uint2*)a);
      }
      if (e0 == tid) {  // first step: the small arrays
#pragma unroll
        for (int k = 0; k < R; k++) {
          if (!sinfo[k] || (PG_IDX_SKIP & 1)) continue;
          uint32_t* chunk = lds + (sinfo[k] >> 4);
          const uint32_t card = sinfo[k] & 0xFu;
          const uint32_t v8[8] = {sq[k][0].x & 0xFFFFu, sq[k][0].x >> 16, sq[k][0].y & 0xFFFFu, sq[k][0].y >> 16,
                                  sq[k][1].x & 0xFFFFu, sq[k][1].x >> 16, sq[k][1].y & 0xFFFFu, sq[k][1].y >> 16};
#pragma unroll
          for (uint32_t h = 0; h < 8; h++)
            if (PG_IDX_SKIP & 32) sink ^= h < card ? v8[h] : 0u;
            else if (PG_ROAR_MASKED) atomicOr(&chunk[v8[h] >> 5], h < card ? 0x80000000u >> (v8[h] & 31u) : 0u);
            else if (h < card) atomicOr(&chunk[v8[h] >> 5], 0x80000000u >> (v8[h] & 31u));
          if (PG_ROAR_SB) __builtin_amdgcn_sched_barrier(0);  // (one container's addresses live at a time)
        }
      }
#pragma unroll
      for (int u = 0; u < kQ; u++) {
        uint32_t* chunk = lds + (nq[u] >> 4);
        const uint32_t n = nq[u] & 0xFu;
        const uint32_t v4[4] = {w[u].x & 0xFFFFu, w[u].x >> 16, w[u].y & 0xFFFFu, w[u].y >> 16};
#pragma unroll
        for (uint32_t h = 0; h < 4; h++)
          if (PG_IDX_SKIP & 64) sink ^= h < n ? v4[h] : 0u;
          else if (PG_ROAR_MASKED) atomicOr(&chunk[v4[h] >> 5], h < n ? 0x80000000u >> (v4[h] & 31u) : 0u);
          else if (h < n) atomicOr(&chunk[v4[h] >> 5], 0x80000000u >> (v4[h] & 31u));
        if (PG_ROAR_SB) __builtin_amdgcn_sched_barrier(0);
      }
      if (e0 + kQ * NT >= total) break;
    }
    ROAR_LAP(3);
    // 4. bitmap containers: 1 024 little-endian uint64 words each; a thread owns the same words of every chunk
    for (uint32_t k = 0; k < ((PG_IDX_SKIP & 4) ? 0u : nb); k++) {
      uint32_t* chunk = lds + (k ? V[S.bview[k]].chunk : bchunk0);
      if (k) {
        const uint32_t* src = (const uint32_t*)(V[S.bview[k]].roaring + S.bml[k]);
#pragma unroll
        for (uint32_t j = 0; j < kWpt; j++) bw[j] = ld_global(src + tid + j * NT);
      }
#pragma unroll
      for (uint32_t j = 0; j < kWpt; j++)
        if (bw[j]) atomicOr(&chunk[tid + j * NT], __builtin_bitreverse32(bw[j]));
    }
    lds_barrier();  // (the chunks complete; this round's lists free for the next)
    ROAR_LAP(4);
  }
  if ((PG_IDX_SKIP & 96) && sink == 0x9E3779B9u) lds[0] |= 1u;
}

}  // namespace pg
