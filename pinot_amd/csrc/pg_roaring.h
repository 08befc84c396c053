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

// dictIds per thread per round: a round issues its R container lookups per thread before any is consumed, and expands
// the round's array containers in one pass
#ifndef PG_ROAR_R
#define PG_ROAR_R 4
#endif
#ifndef PG_ROAR_Q
#define PG_ROAR_Q 4
#endif
constexpr int kRoarR = PG_ROAR_R;
constexpr int kRoarQ = PG_ROAR_Q;  // array-container quads per thread per expansion step (loads in flight together)
constexpr uint32_t kRoarMaxViews = 8;
static_assert(kRoarR >= 1 && kRoarR <= 16 && kRoarQ >= 1 && kRoarQ <= 16, "roaring decode knobs");

// One inverted leaf to decode: its column's containers, the selected dictIds, the LDS chunk it is OR-ed into.
struct RoarView {
  const uint8_t* roaring;
  const RoaringContainer* cs;
  const uint32_t* dir;
  const uint2* keydir;      // optional key-major directory: [key * card + dictId] = keydir_entry or ~0 ~0
  const int32_t* ids;
  uint32_t* chunk;          // LDS
  uint32_t nids, card;
};

// LDS scratch of one decode (besides the chunks and the views)
template <int NT>
struct RoaringLds {
  uint32_t bml[NT];            // bitmap containers of this round (payload offsets), OR-ed by the whole block
  uint8_t bview[NT];           //   and their views (more than NT in a round: the finder ORs it in by itself)
  uint32_t nbml;
  uint32_t tpre[NT + 1];       // exclusive prefix over the threads of their array containers' quads (4 entries each)
  uint32_t aoff[kRoarR][NT];   // thread t's j-th array container of the round: payload offset,
  uint16_t aq0[kRoarR][NT];    //   its first quad among t's quads (0xFFFF: no such container),
  uint16_t acard[kRoarR][NT];  //   its cardinality,
  uint8_t aview[kRoarR][NT];   //   its view
  uint32_t wsum[NT / 64];
  uint32_t vpre[kRoarMaxViews + 1];  // prefix of the views' dictId counts
};

// OR the containers of `key` of every view's selected dictIds into the view's chunk (zeroed by the caller).  The views'
// dictIds are taken as one list, so a round's lookups span the leaves (config 5: 4 leaves of 1 + 20 + 1 + 2 000 ids
// decode in 2 rounds, not 5).  `V` (nv <= kRoarMaxViews entries) is visible to the whole block; starts and ends with a
// block barrier.
template <int NT>
__device__ __forceinline__ void roaring_key_chunks(const RoarView* V, uint32_t nv, uint32_t key, RoaringLds<NT>& S) {
  constexpr int R = kRoarR;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  if (tid == 0) {
    S.nbml = 0;
    uint32_t a = 0;
    for (uint32_t l = 0; l < nv; l++) { S.vpre[l] = a; a += V[l].nids; }
    S.vpre[nv] = a;
  }
  __syncthreads();
  const uint32_t nids = S.vpre[nv];
  for (uint32_t r0 = 0; r0 < nids; r0 += NT * R) {
    // 1. the container of `key` of each of this thread's dictIds, all R lookups issued before any is consumed: with the
    //    key-major directory one 8-byte load each (the descriptor itself), else a search of the dictId's containers
    RoaringContainer c[R];
    uint32_t vw[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
      const uint32_t i = r0 + tid + NT * k;
      c[k] = RoaringContainer{key, 3u, 0u, 0u};
      vw[k] = 0;
      if (i >= nids) continue;
      uint32_t l = 0;
      while (l + 1 < nv && S.vpre[l + 1] <= i) l++;
      vw[k] = l;
      const RoarView& v = V[l];
      const uint32_t id = (uint32_t)v.ids[i - S.vpre[l]];
      if (v.keydir) {
        const uint2 e = v.keydir[(uint64_t)key * v.card + id];
        c[k] = RoaringContainer{key, e.y >> 30, e.y & 0x3FFFFFFFu, e.x};
      } else {  // this dictId's containers, ascending keys: find `key`
        uint32_t lo = v.dir[id], hi = v.dir[id + 1];
        const uint32_t end = hi;
        while (lo < hi) {
          const uint32_t m = (lo + hi) >> 1;
          if (v.cs[m].key < key) lo = m + 1; else hi = m;
        }
        if (lo < end && v.cs[lo].key == key) c[k] = v.cs[lo];
      }
    }
    // 2. classify: arrays -> this thread's quad list, bitmaps -> the block's list, runs expanded here
    uint32_t nq = 0;
    int na = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
      if (c[k].type == 0) {
        S.aoff[na][tid] = c[k].offset;
        S.aq0[na][tid] = (uint16_t)nq;
        S.acard[na][tid] = (uint16_t)c[k].card;
        S.aview[na][tid] = (uint8_t)vw[k];
        nq += (c[k].card + 3u) >> 2;
        na++;
      } else if (c[k].type == 1) {
        const uint32_t b = atomicAdd(&S.nbml, 1u);
        if (b < NT) {
          S.bml[b] = c[k].offset;
          S.bview[b] = (uint8_t)vw[k];
        } else {  // list full (more than NT bitmap containers in one round): this thread ORs it in word by word
          const uint32_t* src = (const uint32_t*)(V[vw[k]].roaring + c[k].offset);
          uint32_t* chunk = V[vw[k]].chunk;
          for (uint32_t wd = 0; wd < 2048; wd++)
            if (src[wd]) atomicOr(&chunk[wd], __builtin_bitreverse32(src[wd]));
        }
      } else if (c[k].type == 2) {  // runs: uint16 nruns, then (start, length - 1)
        const uint16_t* rr = (const uint16_t*)(V[vw[k]].roaring + c[k].offset) + 1;
        uint32_t* chunk = V[vw[k]].chunk;
        for (uint32_t q = 0; q < c[k].card; q++) {
          const uint32_t st = rr[2 * q], en = st + rr[2 * q + 1];
          for (uint32_t w = st >> 5; w <= (en >> 5); w++) {
            const uint32_t l = w * 32 > st ? 0 : st - w * 32, h = w * 32 + 31 < en ? 31 : en - w * 32;
            const uint32_t mask = (h == 31 ? 0xFFFFFFFFu : ((1u << (h + 1)) - 1u)) & ~((1u << l) - 1u);
            atomicOr(&chunk[w], __builtin_bitreverse32(mask));
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < R; k++)
      if (k >= na) S.aq0[k][tid] = 0xFFFFu;
    // exclusive prefix of the threads' quad counts (wave scan + wave sums)
    uint32_t x = nq;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) S.wsum[wave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (uint32_t w = 0; w < wave; w++) wb += S.wsum[w];
    S.tpre[tid] = wb + x - nq;
    if (tid == NT - 1) S.tpre[NT] = wb + x;
    __syncthreads();
    // 3. every quad of the round's array containers, kQ per thread per step (their loads in flight together): owner
    //    thread = the last prefix <= e, then its container; 4 entries per 8-byte load
    constexpr int kQ = kRoarQ;
    const uint32_t total = S.tpre[NT];
    for (uint32_t e0 = tid; e0 < total; e0 += kQ * NT) {
      uint2 w[kQ];
      uint32_t n[kQ];
      uint32_t* dst[kQ];
#pragma unroll
      for (int u = 0; u < kQ; u++) {
        const uint32_t e = e0 + (uint32_t)u * NT;
        n[u] = 0;
        w[u] = make_uint2(0u, 0u);
        dst[u] = nullptr;
        if (e < total) {
          uint32_t lo = 0, hi = NT;
          while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (S.tpre[m] <= e) lo = m; else hi = m;
          }
          const uint32_t local = e - S.tpre[lo];
          int j = 0;
#pragma unroll
          for (int k = 1; k < R; k++)
            if (S.aq0[k][lo] <= local) j = k;
          const uint32_t q = local - S.aq0[j][lo];
          const uint32_t left = (uint32_t)S.acard[j][lo] - 4u * q;
          const RoarView& v = V[S.aview[j][lo]];
          n[u] = left < 4u ? left : 4u;
          dst[u] = v.chunk;
          w[u] = *(const uint2*)(v.roaring + S.aoff[j][lo] + 8u * q);
        }
      }
#pragma unroll
      for (int u = 0; u < kQ; u++) {
        const uint32_t v4[4] = {w[u].x & 0xFFFFu, w[u].x >> 16, w[u].y & 0xFFFFu, w[u].y >> 16};
#pragma unroll
        for (int h = 0; h < 4; h++)
          if ((uint32_t)h < n[u]) atomicOr(&dst[u][v4[h] >> 5], 0x80000000u >> (v4[h] & 31u));
      }
    }
    __syncthreads();  // the bitmap containers below OR whole words without atomics
    // 4. bitmap containers: 1 024 little-endian uint64 words each; a thread owns the same words of every chunk
    const uint32_t nb = S.nbml < NT ? S.nbml : NT;
    for (uint32_t k = 0; k < nb; k++) {
      const uint32_t* src = (const uint32_t*)(V[S.bview[k]].roaring + S.bml[k]);
      uint32_t* chunk = V[S.bview[k]].chunk;
      constexpr uint32_t kWpt = 2048u / NT;  // this thread's words of the container, loaded together
      uint32_t bw[kWpt];
#pragma unroll
      for (uint32_t j = 0; j < kWpt; j++) bw[j] = src[tid + j * NT];
#pragma unroll
      for (uint32_t j = 0; j < kWpt; j++) chunk[tid + j * NT] |= __builtin_bitreverse32(bw[j]);
    }
    __syncthreads();
    if (tid == 0) S.nbml = 0;
    __syncthreads();
  }
}

}  // namespace pg
