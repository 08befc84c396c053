// pg_dict.h -- sorted-dictionary lookups on the device (gfx950): a literal's dictId in one segment's dictionary
// (PredicateUtils.getDictIdSet / Dictionary.indexOf), shared by the IN-list LUT jobs (pg_kernels.hip), the dictionary
// lookups of pg_dict_id_sets, and the exact-mode stream's in-LDS LUT (pg_filter.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pinot_gpu.h"

namespace pg {

// PredicateUtils.getDictIdSet over many segments at once: thread (segment s, literal i) binary-searches literal i
// (already in the dictionary's stored type) in segment s's sorted dictionary -> its dictId, or -1 when absent.
// A few interpolation probes first (dictionaries of dense value ranges -- ids, days, dense keys -- resolve in 2-3
// dependent loads instead of log2(card) ~ 20), then a binary search of what is left: exact either way.
template <class T>
__device__ __forceinline__ int32_t dict_find(const T* __restrict__ d, uint32_t card, T x) {
  if (!card) return -1;
  uint32_t lo = 0, hi = card;  // x, if present, is in [lo, hi)
  T vlo = d[0], vhi = d[card - 1];
  if (x < vlo || vhi < x) return -1;
  for (int it = 0; it < 6 && hi - lo > 8; it++) {
    // vlo = d[lo] <= x <= vhi = d[hi - 1]
    const double span = (double)vhi - (double)vlo;
    uint32_t pos = lo;
    if (span > 0 && span <= __DBL_MAX__) {  // finite: an infinite bound or a NaN literal takes the binary search
      const double f = ((double)x - (double)vlo) / span;
      if (f >= 0.0 && f <= 1.0) {  // (false for NaN) so the conversion below is defined
        pos = lo + (uint32_t)(f * (double)(hi - 1 - lo));
        pos = pos < lo ? lo : (pos > hi - 1 ? hi - 1 : pos);
      }
    }
    const T v = d[pos];
    if (v == x) return (int32_t)pos;
    if (v < x) { lo = pos + 1; if (lo < hi) vlo = d[lo]; }
    else { hi = pos; if (hi > lo) vhi = d[hi - 1]; }
    if (lo >= hi || x < vlo || vhi < x) return -1;
  }
  uint32_t n = hi - lo;
  while (n > 0) {  // lower bound in [lo, hi)
    const uint32_t h = n >> 1;
    if (d[lo + h] < x) { lo += h + 1; n -= h + 1; } else n = h;
  }
  return lo < hi && d[lo] == x ? (int32_t)lo : -1;
}

__device__ __forceinline__ int32_t dict_find_typed(const void* dict, uint32_t card, uint32_t dtype, const void* vals,
                                                   uint32_t i) {
  switch (dtype) {
    case PG_INT: return dict_find((const int32_t*)dict, card, ((const int32_t*)vals)[i]);
    case PG_LONG: return dict_find((const int64_t*)dict, card, ((const int64_t*)vals)[i]);
    case PG_FLOAT: return dict_find((const float*)dict, card, ((const float*)vals)[i]);
    default: return dict_find((const double*)dict, card, ((const double*)vals)[i]);
  }
}


}  // namespace pg
