// pg_roaring.h -- device-side decoding of one 64 K-doc key of an inverted-index leaf (BitmapBasedFilterOperator's OR of
// the selected dictIds' RoaringBitmaps, restricted to one high-16-bit key) into an LDS chunk of 2 048 words, shared by
// the index pre-pass (pg_kernels.hip roaring_keys_kernel) and the fused index count (pg_index.hip).
//
// Chunk word w, bit 31 - j <-> doc key * 65 536 + 32 w + j (the packed 1-bit column order).  Containers follow the
// RoaringBitmap portable format (RoaringBitmap 0.9.28): array (sorted uint16), bitmap (1 024 little-endian uint64) and
// run ((start, length - 1) uint16 pairs) containers, re-laid 8-byte aligned at upload (pg_runtime.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "pg_aux.h"

namespace pg {

// LDS scratch of one chunk build (besides the chunk itself)
template <int NT>
struct RoaringLds {
  uint32_t bml[NT];      // bitmap containers of this round, processed by the whole block
  uint32_t nbml;
  uint32_t apre[NT + 1];  // array containers of this round: exclusive prefix of their cardinalities
  uint32_t aoff[NT];      //   and their payload offsets (slot = the thread that found the container)
  uint32_t wsum[NT / 64];
};

// OR the containers of `key` of the nids selected dictIds into `chunk` (which the caller zeroed and synchronised).
// Ends with a block barrier.  keydir (optional): [key * card + dictId] = container index or ~0.
template <int NT>
__device__ __forceinline__ void roaring_key_chunk(const uint8_t* __restrict__ roaring, const RoaringContainer* __restrict__ cs,
                                                  const uint32_t* __restrict__ dir, const uint32_t* __restrict__ keydir,
                                                  uint32_t card, const int32_t* __restrict__ ids, uint32_t nids,
                                                  uint32_t key, uint32_t* chunk, RoaringLds<NT>& S) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  if (tid == 0) S.nbml = 0;
  __syncthreads();
  for (uint32_t r0 = 0; r0 < nids; r0 += NT) {
    const uint32_t i = r0 + tid;
    uint32_t alen = 0, aoffset = 0;  // this thread's array container (entries are spread over the block below)
    if (i < nids) {
      const uint32_t id = (uint32_t)ids[i];
      uint32_t a;
      bool hit;
      if (keydir) {  // one load: the key-major directory built at upload
        a = keydir[(uint64_t)key * card + id];
        hit = a != 0xFFFFFFFFu;
      } else {
        a = dir[id];
        uint32_t b = dir[id + 1];  // this dictId's containers, ascending keys: find `key`
        while (a < b) {
          const uint32_t m = (a + b) >> 1;
          if (cs[m].key < key) a = m + 1; else b = m;
        }
        hit = a < dir[id + 1] && cs[a].key == key;
      }
      if (hit) {
        const RoaringContainer c = cs[a];
        const uint8_t* p = roaring + c.offset;
        if (c.type == 0) {  // array of uint16: expanded by the whole block
          alen = c.card;
          aoffset = c.offset;
        } else if (c.type == 2) {  // runs: uint16 nruns, then (start, length - 1)
          const uint16_t* rr = (const uint16_t*)p + 1;
          for (uint32_t k = 0; k < c.card; k++) {
            const uint32_t st = rr[2 * k], en = st + rr[2 * k + 1];
            for (uint32_t w = st >> 5; w <= (en >> 5); w++) {
              const uint32_t l = w * 32 > st ? 0 : st - w * 32, h = w * 32 + 31 < en ? 31 : en - w * 32;
              const uint32_t mask = (h == 31 ? 0xFFFFFFFFu : ((1u << (h + 1)) - 1u)) & ~((1u << l) - 1u);
              atomicOr(&chunk[w], __builtin_bitreverse32(mask));
            }
          }
        } else {
          S.bml[atomicAdd(&S.nbml, 1u)] = c.offset;
        }
      }
    }
    // exclusive prefix of the array cardinalities over the block (wave scan + wave sums)
    uint32_t x = alen;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) S.wsum[wave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (uint32_t w = 0; w < wave; w++) wb += S.wsum[w];
    S.apre[tid] = wb + x - alen;
    S.aoff[tid] = aoffset;
    if (tid == NT - 1) S.apre[NT] = wb + x;
    __syncthreads();
    // every array entry of the round, one per thread per step: container k = the last prefix <= e
    const uint32_t total = S.apre[NT];
    for (uint32_t e = tid; e < total; e += NT) {
      uint32_t a = 0, b = NT;
      while (b - a > 1) {
        const uint32_t m = (a + b) >> 1;
        if (S.apre[m] <= e) a = m; else b = m;
      }
      const uint32_t v = ((const uint16_t*)(roaring + S.aoff[a]))[e - S.apre[a]];
      atomicOr(&chunk[v >> 5], 0x80000000u >> (v & 31u));
    }
    __syncthreads();  // the bitmap containers below OR whole words without atomics
    for (uint32_t k = 0; k < S.nbml; k++) {  // bitmap containers: 1 024 little-endian uint64 words each
      const uint32_t* w32 = (const uint32_t*)(roaring + S.bml[k]);
      for (uint32_t w = tid; w < 2048; w += NT) chunk[w] |= __builtin_bitreverse32(w32[w]);
      __syncthreads();
    }
    __syncthreads();
    if (tid == 0) S.nbml = 0;
    __syncthreads();
  }
}

}  // namespace pg
