// pg_kernels.hip -- gfx950 support kernels of the segment query hot path: upload-time re-layout (byte order,
// sorted -> packed, MV row offsets), the filter pre-pass for index-backed leaves (sorted ranges, roaring
// bitmaps, MV scans, IN-list LUTs) and state initialisation.  The fused scan itself is in pg_scan.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "pg_aux.h"
#include "pg_dict.h"
#include "pg_roaring.h"

namespace pg {

// FixedBitIntReader.readUnchecked on the native-word image: value `idx` of `b` bits (MV value streams).
__device__ __forceinline__ uint32_t unpack(const uint32_t* __restrict__ w, uint64_t idx, uint32_t b) {
  const uint64_t p = idx * b;
  const uint64_t wi = p >> 5;
  const uint32_t off = (uint32_t)p & 31u;
  const uint64_t win = ((uint64_t)w[wi] << 32) | (uint64_t)w[wi + 1];
  return (uint32_t)(win >> (64u - off - b)) & (0xFFFFFFFFu >> (32u - b));
}

// ------------------------------------------------------------------------------------------ state init

// SK_FX sums <-> 32-bit limbs (pg_partials_copy): out, each (lo, hi) pair as 4 int64 limbs of 32 bits (limb k = bits
// [32k, 32k + 32)), so that a plain SUM all-reduce of the limbs over up to 2^31 ranks is exact; in, the limbs'
// carries folded back into the 128-bit pair (mod 2^128, the pair's own wrap-around).
__global__ void fx_limbs_kernel(unsigned long long* pairs, long long* limbs, uint64_t n, int in) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (!in) {
      const uint64_t lo = pairs[2 * i], hi = pairs[2 * i + 1];
      limbs[4 * i] = (long long)(lo & 0xFFFFFFFFull);
      limbs[4 * i + 1] = (long long)(lo >> 32);
      limbs[4 * i + 2] = (long long)(hi & 0xFFFFFFFFull);
      limbs[4 * i + 3] = (long long)(hi >> 32);
    } else {
      uint64_t w[4], c = 0;
      for (int k = 0; k < 4; k++) {  // each limb is a sum of 32-bit values: < 2^63, carry its excess upward
        const uint64_t t = (uint64_t)limbs[4 * i + k] + c;
        w[k] = t & 0xFFFFFFFFull;
        c = t >> 32;
      }
      pairs[2 * i] = w[0] | (w[1] << 32);
      pairs[2 * i + 1] = w[2] | (w[3] << 32);
    }
  }
}

hipError_t launch_fx_limbs(unsigned long long* pairs, long long* limbs, uint64_t n, bool in, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(fx_limbs_kernel, dim3((uint32_t)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, pairs, limbs, n,
                     in ? 1 : 0);
  return hipGetLastError();
}

__global__ void init_minmax_kernel(long long* mn, uint64_t nmn, long long* mx, uint64_t nmx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = i; k < nmn; k += stride) mn[k] = order_key(__builtin_inf());
  for (uint64_t k = i; k < nmx; k += stride) mx[k] = order_key(-__builtin_inf());
}

// defer != null: the byte fills are appended there (applied by the query's arena-upload launch) while they fit
hipError_t launch_init_view(const StateView& v, hipStream_t s, FillSpans* defer) {
  hipError_t e;
  auto fill = [&](void* p, int b, uint64_t n) {
    if (defer && defer->add(p, (uint32_t)b, n)) return hipSuccess;
    return hipMemsetAsync(p, b, n, s);
  };
  if (v.n_i64 && (e = fill(v.i64, 0, v.num_slots * v.n_i64 * 8)) != hipSuccess) return e;
  if (v.n_fx && (e = fill(v.fx, 0, v.num_slots * v.n_fx * 16)) != hipSuccess) return e;
  if (v.bit_words && (e = fill(v.bits, 0, v.num_slots * v.bit_words * 4ull)) != hipSuccess) return e;
  if (v.keys && (e = fill(v.keys, 0xFF, v.num_slots * 8)) != hipSuccess) return e;
  if (v.first_doc && (e = fill(v.first_doc, 0xFF, v.num_slots * 8)) != hipSuccess) return e;
  if (v.fill && (e = fill(v.fill, 0, 8)) != hipSuccess) return e;  // fill + err
  const uint64_t n = v.num_slots * (v.n_min > v.n_max ? v.n_min : v.n_max);
  if (n) {
    const uint32_t blocks = (uint32_t)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(init_minmax_kernel, dim3(blocks), dim3(256), 0, s, v.mn, v.num_slots * v.n_min, v.mx,
                       v.num_slots * v.n_max);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ upload-time

// big-endian byte stream -> native uint32 words (word i = bytes 4i..4i+3, zero past nbytes)
__global__ void bswap_words_kernel(const uint8_t* __restrict__ src, uint32_t* __restrict__ dst, uint64_t nbytes,
                                   uint64_t nwords) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride) {
    const uint64_t b = i * 4;
    uint32_t w = 0;
    if (b + 4 <= nbytes) {
      w = ((uint32_t)src[b] << 24) | ((uint32_t)src[b + 1] << 16) | ((uint32_t)src[b + 2] << 8) | src[b + 3];
    } else {
      for (int k = 0; k < 4; k++) w = (w << 8) | (b + k < nbytes ? src[b + k] : 0u);
    }
    dst[i] = w;
  }
}

hipError_t launch_bswap_words(const uint8_t* src, uint32_t* dst, uint64_t nbytes, uint64_t nwords, hipStream_t s) {
  if (!nwords) return hipSuccess;
  const uint64_t blocks = (nwords + 255) / 256;
  hipLaunchKernelGGL(bswap_words_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, src,
                     dst, nbytes, nwords);
  return hipGetLastError();
}

__global__ void be_to_native_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t n,
                                    uint32_t width) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    for (uint32_t k = 0; k < width; k++) dst[i * width + k] = src[i * width + (width - 1 - k)];
}

hipError_t launch_be_to_native(const uint8_t* src, void* dst, uint64_t n, uint32_t width, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(be_to_native_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, src,
                     (uint8_t*)dst, n, width);
  return hipGetLastError();
}

// Sorted column (SortedIndexReaderImpl pairs) -> the same packed dictId stream an unsorted column has.
__global__ void sorted_to_packed_kernel(const int32_t* __restrict__ pairs, uint32_t card, uint32_t num_docs,
                                        uint32_t bits, uint32_t* __restrict__ words, uint64_t nwords) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    const uint64_t p0 = w * 32, p1 = p0 + 32;
    uint64_t d0 = p0 / bits, d1 = (p1 + bits - 1) / bits;
    if (d1 > num_docs) d1 = num_docs;
    uint32_t out = 0;
    for (uint64_t d = d0; d < d1; d++) {
      // dictId = last id with start <= d
      uint32_t lo = 0, hi = card;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)pairs[2 * mid] <= d) lo = mid; else hi = mid;
      }
      const uint64_t v = lo;
      const int64_t vs = (int64_t)(d * bits), ve = vs + bits;  // value bits [vs, ve)
      for (int64_t p = (vs > (int64_t)p0 ? vs : (int64_t)p0); p < (ve < (int64_t)p1 ? ve : (int64_t)p1); p++) {
        const uint32_t bit = (uint32_t)((v >> (ve - 1 - p)) & 1u);
        out |= bit << (31 - (uint32_t)(p - p0));
      }
    }
    words[w] = out;
  }
}

hipError_t launch_sorted_to_packed(const int32_t* pairs, uint32_t card, uint32_t num_docs, uint32_t bits,
                                   uint32_t* words, uint64_t nwords, hipStream_t s) {
  if (!nwords) return hipSuccess;
  const uint64_t blocks = (nwords + 255) / 256;
  hipLaunchKernelGGL(sorted_to_packed_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s,
                     pairs, card, num_docs, bits, words, nwords);
  return hipGetLastError();
}

// Decoded forward index of a large integer dictionary (upload-time, ColumnRes::vals): doc i's dictionary VALUE minus
// the dictionary minimum, bit-packed at `vbits` bits in the same MSB-first native-word layout as the dictId stream.
// A group key / aggregation input then reads one packed value per doc instead of a dictId + a random dictionary
// gather (a 5.4 M-entry userId dictionary is 21.6 MB per segment: one 64-byte line fetched per 4-byte read).
// One thread per output word: the values overlapping word w, each shifted so its last bit lands on its stream bit.
__global__ void decode_pack_kernel(const uint32_t* __restrict__ ids, uint32_t bits, const void* __restrict__ dict,
                                   uint32_t dtype, uint32_t card, int64_t vmin, uint32_t vbits, uint32_t num_docs,
                                   uint32_t* __restrict__ out, uint64_t nwords) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    const uint64_t p0 = w * 32;
    uint64_t d0 = p0 / vbits, d1 = (p0 + 32 + vbits - 1) / vbits;
    if (d1 > num_docs) d1 = num_docs;
    uint32_t word = 0;
    for (uint64_t d = d0; d < d1; d++) {
      uint32_t id = ids ? unpack(ids, d, bits) : (uint32_t)d;  // ids == nullptr: `dict` holds the doc values
      id = id < card ? id : card - 1u;
      const int64_t v = dtype == PG_INT ? (int64_t)((const int32_t*)dict)[id] : ((const int64_t*)dict)[id];
      const uint64_t x = (uint64_t)(v - vmin);
      const int64_t shift = (int64_t)(p0 + 31) - (int64_t)(d * vbits + vbits - 1);  // in [-31, 31]
      word |= (uint32_t)(shift >= 0 ? (x << shift) : (x >> -shift));
    }
    out[w] = word;
  }
}

hipError_t launch_decode_pack(const uint32_t* ids, uint32_t bits, const void* dict, uint32_t dtype, uint32_t card,
                              int64_t vmin, uint32_t vbits, uint32_t num_docs, uint32_t* out, uint64_t nwords,
                              hipStream_t s) {
  if (!nwords) return hipSuccess;
  const uint64_t blocks = (nwords + 255) / 256;
  hipLaunchKernelGGL(decode_pack_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, s, ids,
                     bits, dict, dtype, card, vmin, vbits, num_docs, out, nwords);
  return hipGetLastError();
}

// NonScanBasedAggregationOperator's DISTINCTCOUNT (operator/query/NonScanBasedAggregationOperator.java:124-127,
// getDistinctValueSet): every dictionary value of a segment whose filter matches all docs, as table-global value ids
// set in the aggregation's bitmap (VALUE_OFFSET: value - base; KEYMAP: keymap[dictId]).  O(cardinality).
__global__ void dict_bits_kernel(const void* __restrict__ dict, uint32_t dtype, uint32_t card, int64_t base,
                                 const int32_t* __restrict__ keymap, uint32_t key_card, uint32_t* __restrict__ bits,
                                 unsigned int* err) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < card; i += stride) {
    uint64_t key;
    if (keymap) key = (uint64_t)(uint32_t)keymap[i];
    else key = (uint64_t)((dtype == PG_INT ? (int64_t)((const int32_t*)dict)[i] : ((const int64_t*)dict)[i]) - base);
    if (key < key_card) atomicOr(&bits[key >> 5], 1u << (key & 31u));
    else atomicOr(err, 2u);
  }
}

hipError_t launch_dict_bits(const void* dict, uint32_t dtype, uint32_t card, int64_t base, const int32_t* keymap,
                            uint32_t key_card, uint32_t* bits, unsigned int* err, hipStream_t s) {
  if (!card) return hipSuccess;
  const uint64_t blocks = (card + 255) / 256;
  hipLaunchKernelGGL(dict_bits_kernel, dim3((uint32_t)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, dict, dtype,
                     card, base, keymap, key_card, bits, err);
  return hipGetLastError();
}

// MV row offsets: select the row-start bits of the start-of-row bitmap
// (FixedBitMVForwardIndexReader / PinotDataBitSet.getNextSetBitOffset, io/util/PinotDataBitSet.java:219-253).
__global__ void popc_words_kernel(const uint32_t* __restrict__ bm, uint64_t nwords, uint64_t nbits,
                                  uint32_t* __restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    uint32_t x = bm[w];
    const uint64_t end = (w + 1) * 32;
    if (end > nbits) x &= ~((1u << (uint32_t)(end - nbits)) - 1u);  // bit order: MSB = first
    cnt[w] = __popc(x);
  }
}
__global__ void select_rows_kernel(const uint32_t* __restrict__ bm, uint64_t nwords, uint64_t nbits,
                                   const uint32_t* __restrict__ prefix, uint32_t num_docs,
                                   uint32_t* __restrict__ offsets) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    uint32_t x = bm[w];
    const uint64_t end = (w + 1) * 32;
    if (end > nbits) x &= ~((1u << (uint32_t)(end - nbits)) - 1u);
    uint32_t r = prefix[w];
    while (x) {
      const uint32_t k = __clz(x);  // first (MSB) set bit
      if (r < num_docs) offsets[r] = (uint32_t)(w * 32 + k);
      r++;
      x &= ~(0x80000000u >> k);
    }
  }
}
__global__ void set_last_offset_kernel(uint32_t* offsets, uint32_t num_docs, uint32_t num_values) {
  offsets[num_docs] = num_values;
}

size_t mv_offsets_scratch_bytes(uint64_t num_values) {
  const uint64_t nwords = (num_values + 31) / 32;
  size_t temp = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)nwords);
  return temp + 2 * nwords * sizeof(uint32_t) + 256;
}

hipError_t launch_mv_offsets(const uint32_t* bm, uint64_t num_values, uint32_t num_docs, uint32_t* offsets,
                             void* scratch, size_t scratch_bytes, hipStream_t s) {
  const uint64_t nwords = (num_values + 31) / 32;
  uint32_t* cnt = (uint32_t*)scratch;
  uint32_t* prefix = cnt + nwords;
  void* temp = (void*)(((uintptr_t)(prefix + nwords) + 255) & ~(uintptr_t)255);
  size_t temp_bytes = scratch_bytes - ((uint8_t*)temp - (uint8_t*)scratch);
  if (nwords) {
    const uint64_t blocks = (nwords + 255) / 256;
    const uint32_t g = (uint32_t)(blocks < 65536 ? blocks : 65536);
    hipLaunchKernelGGL(popc_words_kernel, dim3(g), dim3(256), 0, s, bm, nwords, num_values, cnt);
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, cnt, prefix, (int)nwords, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(select_rows_kernel, dim3(g), dim3(256), 0, s, bm, nwords, num_values, prefix, num_docs,
                       offsets);
  }
  hipLaunchKernelGGL(set_last_offset_kernel, dim3(1), dim3(1), 0, s, offsets, num_docs, (uint32_t)num_values);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ filter pre-pass

// Doc bitmaps produced by the pre-pass use the packed-column bit order (doc d = bit 31-(d&31) of word d>>5), so
// the scan reads them as 1-bit packed columns (staged or gathered like any other column).
// Doc ranges (inclusive, sorted, disjoint) -> doc bitmap: SortedIndexBasedFilterOperator's range list
// (filter/SortedIndexBasedFilterOperator.java:51-138).  One thread per bitmap word.
__global__ void fill_ranges_kernel(const int32_t* __restrict__ r, uint32_t n, uint32_t num_docs,
                                   uint32_t* __restrict__ bm) {
  const uint32_t nwords = (num_docs + 31) / 32;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    const int64_t d0 = (int64_t)w * 32, d1 = d0 + 31;
    uint32_t lo = 0, hi = n;  // first range with end >= d0
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (r[2 * mid + 1] < d0) lo = mid + 1; else hi = mid;
    }
    uint32_t out = 0;
    for (uint32_t i = lo; i < n && r[2 * i] <= d1; i++) {
      const int64_t s = r[2 * i] > d0 ? r[2 * i] : d0;
      const int64_t e = r[2 * i + 1] < d1 ? r[2 * i + 1] : d1;
      for (int64_t d = s; d <= e; d++) out |= 0x80000000u >> (uint32_t)(d - d0);
    }
    bm[w] = out;
  }
}

hipError_t launch_fill_ranges(const int32_t* ranges, uint32_t n, uint32_t num_docs, uint32_t* bitmap,
                              hipStream_t s) {
  const uint32_t nwords = (num_docs + 31) / 32;
  if (!nwords) return hipSuccess;
  const uint32_t blocks = (nwords + 255) / 256;
  hipLaunchKernelGGL(fill_ranges_kernel, dim3(blocks < 65536 ? blocks : 65536), dim3(256), 0, s, ranges, n,
                     num_docs, bitmap);
  return hipGetLastError();
}

// Roaring containers (portable format, payloads re-laid 8-byte aligned at upload) OR-ed into a doc bitmap:
// BitmapBasedFilterOperator's ImmutableRoaringBitmap.or of the matching dictIds (filter/BitmapBasedFilterOperator.java:66-115).
// One workgroup per selected container.
__global__ void roaring_or_kernel(const uint8_t* __restrict__ roaring, const RoaringContainer* __restrict__ cs,
                                  const uint32_t* __restrict__ sel, uint32_t num_docs, uint32_t* __restrict__ bm) {
  const RoaringContainer c = cs[sel[blockIdx.x]];
  const uint32_t nwords = (num_docs + 31) / 32;
  const uint32_t base = c.key << 16;
  const uint8_t* p = roaring + c.offset;
  if (c.type == 0) {  // array of uint16
    const uint16_t* a = (const uint16_t*)p;
    for (uint32_t i = threadIdx.x; i < c.card; i += blockDim.x) {
      const uint32_t x = base + a[i];
      if (x < num_docs) atomicOr(&bm[x >> 5], 0x80000000u >> (x & 31u));
    }
  } else if (c.type == 1) {  // 1024 little-endian uint64 words
    const uint32_t* w32 = (const uint32_t*)p;
    for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x) {
      const uint32_t wi = (base >> 5) + i;
      const uint32_t v = w32[i];
      if (v && wi < nwords) atomicOr(&bm[wi], __builtin_bitreverse32(v));
    }
  } else {  // runs: uint16 nruns, then (start, length-1) pairs
    const uint16_t* r = (const uint16_t*)p + 1;
    for (uint32_t i = threadIdx.x; i < c.card; i += blockDim.x) {
      const uint32_t s = base + r[2 * i];
      uint32_t e = s + r[2 * i + 1];  // inclusive
      if (e >= num_docs) e = num_docs - 1;
      for (uint32_t w = s >> 5; s <= e && w <= (e >> 5); w++) {
        const uint32_t lo = w * 32 > s ? 0 : s - w * 32;
        const uint32_t hi = w * 32 + 31 < e ? 31 : e - w * 32;
        const uint32_t mask = (hi == 31 ? 0xFFFFFFFFu : ((1u << (hi + 1)) - 1u)) & ~((1u << lo) - 1u);
        atomicOr(&bm[w], __builtin_bitreverse32(mask));
      }
    }
  }
}

hipError_t launch_roaring_or(const uint8_t* roaring, const RoaringContainer* containers, const uint32_t* sel,
                             uint32_t nsel, uint32_t num_docs, uint32_t* bitmap, hipStream_t s) {
  if (!nsel) return hipSuccess;
  hipLaunchKernelGGL(roaring_or_kernel, dim3(nsel), dim3(256), 0, s, roaring, containers, sel, num_docs, bitmap);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void roaring_keys_kernel(const RoaringJob* __restrict__ jobs, uint32_t njobs) {
  __shared__ uint32_t chunk[2048];     // the key's 65 536 docs
  __shared__ RoaringLds<256> S;
  __shared__ RoarView V;
  uint32_t lo = 0, hi = njobs;         // the job whose block range holds this block
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (jobs[mid].first_block <= blockIdx.x) lo = mid; else hi = mid;
  }
  const RoaringJob J = jobs[lo];
  const uint32_t key = J.key0 + (blockIdx.x - J.first_block), tid = threadIdx.x;
  for (uint32_t w = tid; w < 2048; w += 256) chunk[w] = 0;
  if (tid == 0) V = RoarView{J.roaring, J.cs, J.dir, J.keydir, J.ids, 0u, J.nids, J.card};
  roaring_key_chunks<256>(&V, 1, key, S, chunk);  // (its first barrier publishes V and the zeroed chunk)
  const uint32_t nwords = (J.num_docs + 31) / 32, tail = J.num_docs & 31u;
  for (uint32_t w = tid; w < 2048; w += 256) {
    const uint32_t gw = key * 2048 + w;
    if (gw >= nwords) break;
    uint32_t v = chunk[w];
    if (J.negate) {
      v = ~v;
      if (gw == nwords - 1 && tail) v &= ~(0xFFFFFFFFu >> tail);
    }
    J.bm[gw] = v;
  }
}

hipError_t launch_roaring_keys(const RoaringJob* jobs, uint32_t njobs, uint32_t blocks, hipStream_t s) {
  if (!njobs || !blocks) return hipSuccess;
  hipLaunchKernelGGL(roaring_keys_kernel, dim3(blocks), dim3(256), 0, s, jobs, njobs);
  return hipGetLastError();
}

__global__ void bitmap_not_kernel(uint32_t* bm, uint32_t num_docs) {
  const uint32_t nwords = (num_docs + 31) / 32;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    uint32_t v = ~bm[w];
    if (w == nwords - 1 && (num_docs & 31u)) v &= ~(0xFFFFFFFFu >> (num_docs & 31u));
    bm[w] = v;
  }
}

hipError_t launch_bitmap_not(uint32_t* bitmap, uint32_t num_docs, hipStream_t s) {
  const uint32_t nwords = (num_docs + 31) / 32;
  if (!nwords) return hipSuccess;
  const uint32_t blocks = (nwords + 255) / 256;
  hipLaunchKernelGGL(bitmap_not_kernel, dim3(blocks < 65536 ? blocks : 65536), dim3(256), 0, s, bitmap, num_docs);
  return hipGetLastError();
}

// MV scan leaf (MVScanDocIdIterator + BaseDictionaryBasedPredicateEvaluator.applyMV): any value in S, or
// for exclusive predicates all values not in S (== NOT any).  One thread per doc, ballot per wave.
__global__ void mv_scan_kernel(const uint32_t* __restrict__ words, uint32_t bits, const uint32_t* __restrict__ off,
                               uint32_t num_docs, int32_t lo, int32_t hi, const uint32_t* __restrict__ lut,
                               uint32_t excl, uint32_t* __restrict__ bm) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t d0 = blockIdx.x * blockDim.x; d0 < num_docs; d0 += stride) {
    const uint32_t d = d0 + threadIdx.x;
    bool any = false;
    if (d < num_docs) {
      for (uint32_t v = off[d]; v < off[d + 1] && !any; v++) {
        const uint32_t id = unpack(words, v, bits);
        any = lut ? ((lut[id >> 5] >> (id & 31u)) & 1u) : ((int32_t)id >= lo && (int32_t)id < hi);
      }
    }
    const bool match = (d < num_docs) && (any != (excl != 0));
    const uint64_t b = __ballot(match);
    if ((threadIdx.x & 63) == 0) {
      const uint32_t w = d >> 5;  // d is a multiple of 64 here
      if (w < (num_docs + 31) / 32) bm[w] = __builtin_bitreverse32((uint32_t)b);
      if (w + 1 < (num_docs + 31) / 32) bm[w + 1] = __builtin_bitreverse32((uint32_t)(b >> 32));
    }
  }
}

hipError_t launch_mv_scan(const uint32_t* words, uint32_t bits, const uint32_t* offsets, uint32_t num_docs,
                          int32_t lo, int32_t hi, const uint32_t* lut, uint32_t excl, uint32_t* bitmap,
                          hipStream_t s) {
  if (!num_docs) return hipSuccess;
  const uint32_t blocks = (num_docs + 255) / 256;
  hipLaunchKernelGGL(mv_scan_kernel, dim3(blocks < 65536 ? blocks : 65536), dim3(256), 0, s, words, bits, offsets,
                     num_docs, lo, hi, lut, excl, bitmap);
  return hipGetLastError();
}

// IN / NOT_IN dictId sets -> global bitmaps over dictIds and the LDS filter bitmaps over dictId >> shift (both in
// zeroed scratch); one launch for all (segment, leaf) sets of a query: block b handles job b.

__global__ void set_lut_bits_kernel(const LutJob* __restrict__ jobs) {
  const LutJob J = jobs[blockIdx.x];
  // blockIdx.y: this block's 256-element chunk (one element per thread: a values-mode lookup is a chain of dependent
  // loads, so the chains run side by side rather than one after another per thread)
  for (uint32_t i = blockIdx.y * blockDim.x + threadIdx.x; i < J.n; i += gridDim.y * blockDim.x) {
    const int32_t sid = J.ids ? J.ids[i] : dict_find_typed(J.dict, J.card, J.dtype, J.values, i);
    if (sid < 0) continue;  // values mode: a literal this segment's dictionary does not hold
    const uint32_t id = (uint32_t)sid;
    if (J.lut) atomicOr(&J.lut[id >> 5], 1u << (id & 31u));
    if (J.region) atomicOr(&J.region[(id >> J.shift) >> 5], 1u << ((id >> J.shift) & 31u));
  }
}

hipError_t launch_set_lut_bits(const LutJob* jobs, uint32_t njobs, uint32_t max_n, hipStream_t s) {
  if (!njobs) return hipSuccess;
  const uint32_t chunks = std::max(1u, std::min(64u, (max_n + 255u) / 256u));
  hipLaunchKernelGGL(set_lut_bits_kernel, dim3(njobs, chunks), dim3(256), 0, s, jobs);
  return hipGetLastError();
}

__global__ void dict_lookup_kernel(const DictLookupJob* __restrict__ jobs, const void* __restrict__ values, uint32_t n,
                                   uint32_t dtype, int32_t* __restrict__ out) {
  const uint32_t s = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DictLookupJob j = jobs[s];
  out[(uint64_t)s * n + i] = dict_find_typed(j.dict, j.card, dtype, values, i);
}

hipError_t launch_dict_lookup(const DictLookupJob* jobs, uint32_t num_segments, const void* values, uint32_t n,
                              uint32_t dtype, int32_t* out, hipStream_t s) {
  if (!n || !num_segments) return hipSuccess;
  hipLaunchKernelGGL(dict_lookup_kernel, dim3((n + 255) / 256, num_segments), dim3(256), 0, s, jobs, values, n, dtype,
                     out);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ parameter arena upload

// one byte value over [z, z + n) (z 16-byte aligned: pooled blocks), the grid's x dimension striding it
__device__ __forceinline__ void fill_span(uint8_t* __restrict__ z, uint64_t n, uint32_t b, uint64_t t,
                                          uint64_t stride) {
  const uint32_t w = b * 0x01010101u;
  const uint64_t n16 = n / 16;
  for (uint64_t i = t; i < n16; i += stride) ((uint4*)z)[i] = make_uint4(w, w, w, w);
  for (uint64_t i = n16 * 16 + t; i < n; i += stride) z[i] = (uint8_t)b;
}

// blockIdx.y == 0: the arena copy + the scratch zeroing; blockIdx.y == k + 1: deferred fill k
__global__ void __launch_bounds__(256) arena_upload_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          uint64_t n16, uint8_t* __restrict__ z, uint64_t zbytes,
                                                          FillSpans fills) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y) {
    const uint32_t k = blockIdx.y - 1;
    fill_span((uint8_t*)fills.p[k], fills.n[k], fills.byte[k], t, stride);
    return;
  }
  for (uint64_t i = t; i < n16; i += stride) dst[i] = src[i];
  fill_span(z, zbytes, 0u, t, stride);
}

hipError_t launch_arena_upload(const void* host_src, void* dst, uint64_t bytes, void* zero, uint64_t zero_bytes,
                               const FillSpans& fills, hipStream_t s) {
  // the source is read in whole 16-byte units: the pinned image's capacity is a multiple of 16 covering them
  const uint64_t n16 = (bytes + 15) / 16;
  uint64_t units = std::max<uint64_t>(n16, (zero_bytes + 15) / 16);
  for (uint32_t k = 0; k < fills.count; k++) units = std::max<uint64_t>(units, (fills.n[k] + 15) / 16);
  if (!units) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((units + 255) / 256, 1024);
  hipLaunchKernelGGL(arena_upload_kernel, dim3((uint32_t)blocks, 1 + fills.count), dim3(256), 0, s,
                     (const uint4*)host_src, (uint4*)dst, n16, (uint8_t*)zero, zero_bytes, fills);
  return hipGetLastError();
}

// blockIdx.y == k: span k, 8-byte words, the grid's x dimension striding it (the destinations are mapped host memory:
// the end-of-query readback in one dispatch instead of one blit per span)
__global__ void __launch_bounds__(256) copy_spans_kernel(CopySpans c) {
  const uint32_t k = blockIdx.y;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const unsigned long long* __restrict__ src = (const unsigned long long*)c.src[k];
  unsigned long long* __restrict__ dst = (unsigned long long*)c.dst[k];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.words[k]; i += stride) dst[i] = src[i];
}

hipError_t launch_copy_spans(const CopySpans& c, hipStream_t s) {
  uint64_t w = 0;
  for (uint32_t k = 0; k < c.count; k++) w = std::max<uint64_t>(w, c.words[k]);
  if (!w) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((w + 255) / 256, 256);
  hipLaunchKernelGGL(copy_spans_kernel, dim3((uint32_t)blocks, c.count), dim3(256), 0, s, c);
  return hipGetLastError();
}

}  // namespace pg
