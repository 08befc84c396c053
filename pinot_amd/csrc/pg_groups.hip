// pg_groups.hip -- group-state kernels of libpinot_gpu (gfx950): the device side of what the reference does after
// the per-segment aggregation loop.
//
//   * numGroupsLimit truncation per segment (DictionaryBasedGroupKeyGenerator.IntGroupIdMap.getGroupId,
//     query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:991-1016: ids in first-seen doc order,
//     INVALID_ID once the limit is reached): from a GM_HASH_SEG table every segment keeps the `limit` keys whose
//     first matching doc comes first, then the kept (segment, key) entries are merged by key.
//   * merge by VALUE key (GroupByOrderByCombineOperator.processSegments -> IndexedTable.upsert,
//     operator/combine/GroupByOrderByCombineOperator.java:127-214, data/table/IndexedTable.java:103-118) as
//     exchange rows inserted into an open-addressing table with each function's merge (SUM / MIN / MAX / OR).
//   * finalisation: final values per group (extractFinalResult of each function; DISTINCTCOUNT = set size,
//     DistinctCountAggregationFunction.java:252-310), the ORDER BY trim (TableResizer.getTopRecords,
//     data/table/TableResizer.java:248) as a radix sort on the first ORDER BY item, and value-set extraction.
// Everything here is HBM / atomic bound, O(groups); no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "pg_aux.h"

namespace pg {

__host__ __device__ inline uint32_t key_owner(uint64_t key, uint32_t parts) {
  // high bits of a second mix: independent of the table position bits (mix64(key) & mask) of the receiver
  return (uint32_t)((mix64(key ^ 0x9E3779B97F4A7C15ull) >> 32) % parts);
}

__device__ __forceinline__ bool present(const StateView& v, uint64_t s) {
  if (v.keys && v.keys[s] == kEmptyKey) return false;
  return v.i64[s * v.n_i64] > 0;
}

// ------------------------------------------------------------------------------------------ slot selection

struct SlotPred {
  StateView v;
  uint32_t kind, part, parts;
  __device__ bool operator()(const uint32_t& s) const {
    switch (kind) {
      case SEL_OCCUPIED: return v.keys[s] != kEmptyKey;
      case SEL_PRESENT_PART: return present(v, s) && key_owner(v.keys ? v.keys[s] : (uint64_t)s, parts) == part;
      default: return present(v, s);
    }
  }
};

size_t select_temp_bytes(uint64_t n) {
  size_t a = 0, b = 0, c = 0;
  hipcub::CountingInputIterator<uint32_t> it(0);
  hipcub::DeviceSelect::If(nullptr, a, it, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, SlotPred{});
  hipcub::DeviceSelect::Flagged(nullptr, b, (uint32_t*)nullptr, (uint8_t*)nullptr, (uint32_t*)nullptr,
                                (uint32_t*)nullptr, (int)n);
  hipcub::DeviceScan::ExclusiveSum(nullptr, c, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)n + 1);
  return std::max(a, std::max(b, c)) + 256;
}

hipError_t launch_select_slots(const StateView& v, uint32_t kind, uint32_t part, uint32_t parts, uint32_t* out,
                               uint32_t* d_num, void* temp, size_t temp_bytes, hipStream_t s) {
  hipcub::CountingInputIterator<uint32_t> it(0);
  return hipcub::DeviceSelect::If(temp, temp_bytes, it, out, d_num, (int)v.num_slots, SlotPred{v, kind, part, parts},
                                  s);
}

// Present slots of a large state in block-chunk order (order inside the output is irrelevant to the trim that
// consumes it). Each block owns one contiguous chunk: it counts its present slots, reserves its output range with ONE
// global atomic, then writes the chunk again in slot order. (A per-wave atomic on the single counter serialised 156K
// atomics at L2 for 10M slots: 1.8 ms; hipcub's ordered select is 0.17 ms.)
// MODE 0: every present slot; 1 / 2: present slots whose DISTINCTCOUNT set size (dc_pop) is >= / <= t
template <int MODE>
__device__ __forceinline__ bool take_slot(const StateView& v, uint64_t s, uint32_t t, uint32_t maxv) {
  if (!present(v, s)) return false;
  if (MODE == 1) return min(v.dc_pop[s], maxv) >= t;  // (clamped as pop_hist_kernel bins it: the counts agree)
  if (MODE == 2) return min(v.dc_pop[s], maxv) <= t;
  return true;
}

template <int MODE>
__global__ void __launch_bounds__(256) select_present_unordered_kernel(StateView v, uint32_t* __restrict__ out,
                                                                       unsigned int* __restrict__ count,
                                                                       uint32_t chunk, uint32_t thr, uint32_t maxv) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t base_s;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t lo = (uint64_t)blockIdx.x * chunk;
  const uint64_t hi = std::min<uint64_t>(lo + chunk, v.num_slots);
  uint32_t mine = 0;
  for (uint64_t s = lo + threadIdx.x; s < hi; s += 256) mine += take_slot<MODE>(v, s, thr, maxv) ? 1u : 0u;
  for (int o = 32; o; o >>= 1) mine += __shfl_xor(mine, o);
  if (lane == 0) wsum[w] = mine;
  __syncthreads();
  if (threadIdx.x == 0) base_s = atomicAdd(count, wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  __syncthreads();
  uint32_t run = base_s;
  for (uint64_t t = lo; t < hi; t += 256) {
    const uint64_t s = t + threadIdx.x;
    const bool take = s < hi && take_slot<MODE>(v, s, thr, maxv);
    const uint64_t m = __ballot(take);
    __syncthreads();  // wsum of the previous tile fully read
    if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < 4; ++i) {
      pre += i < w ? wsum[i] : 0u;
      tot += wsum[i];
    }
    if (take) out[run + pre + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)s;
    run += tot;
  }
}

hipError_t launch_select_present_unordered(const StateView& v, uint32_t* out, unsigned int* count, hipStream_t s) {
  const uint64_t tiles = (v.num_slots + 255) / 256;
  const uint64_t per = std::max<uint64_t>((tiles + 2047) / 2048, 1);  // ≤2048 blocks: ≤2048 atomics on the counter
  const uint64_t blocks = std::max<uint64_t>((tiles + per - 1) / per, 1);
  hipLaunchKernelGGL(select_present_unordered_kernel<0>, dim3((uint32_t)blocks), dim3(256), 0, s, v, out, count,
                     (uint32_t)(per * 256), 0u, 0u);
  return hipGetLastError();
}

// The trim of a DISTINCTCOUNT-ordered state whose set sizes the bucket pass kept (dc_pop): a histogram of the present
// groups' set sizes (<= maxv + 1 bins) in one pass, then the groups at or beyond the limit-th size in a second --
// instead of present slots + order images + a radix select over every group.
__global__ void __launch_bounds__(256) pop_hist_kernel(StateView v, uint32_t maxv, unsigned int* __restrict__ hist) {
  extern __shared__ unsigned int lh[];
  for (uint32_t i = threadIdx.x; i <= maxv; i += 256) lh[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < v.num_slots; s += stride)
    if (present(v, s)) atomicAdd(&lh[min(v.dc_pop[s], maxv)], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i <= maxv; i += 256)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

hipError_t launch_pop_hist(const StateView& v, uint32_t maxv, unsigned int* hist, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>((v.num_slots + 255) / 256, 2048);
  hipLaunchKernelGGL(pop_hist_kernel, dim3((uint32_t)(blocks ? blocks : 1)), dim3(256), 4ull * (maxv + 1), s, v, maxv, hist);
  return hipGetLastError();
}

hipError_t launch_select_pop(const StateView& v, uint32_t t, uint32_t maxv, bool at_least, uint32_t* out,
                             unsigned int* count, hipStream_t s) {
  const uint64_t per = 16;  // 4 096 slots per block
  const uint64_t blocks = (v.num_slots + per * 256 - 1) / (per * 256);
  if (!blocks) return hipSuccess;
  if (at_least)
    hipLaunchKernelGGL(select_present_unordered_kernel<1>, dim3((uint32_t)blocks), dim3(256), 0, s, v, out, count,
                       (uint32_t)(per * 256), t, maxv);
  else
    hipLaunchKernelGGL(select_present_unordered_kernel<2>, dim3((uint32_t)blocks), dim3(256), 0, s, v, out, count,
                       (uint32_t)(per * 256), t, maxv);
  return hipGetLastError();
}

hipError_t launch_select_flagged(const uint32_t* in, const uint8_t* flags, uint64_t n, uint32_t* out, uint32_t* d_num,
                                 void* temp, size_t temp_bytes, hipStream_t s) {
  return hipcub::DeviceSelect::Flagged(temp, temp_bytes, in, flags, out, d_num, (int)n, s);
}

hipError_t launch_exclusive_sum(const uint64_t* in, uint64_t* out, uint64_t n, void* temp, size_t temp_bytes,
                                hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}

size_t sort_temp_bytes(uint64_t n, uint32_t begin_bit, uint32_t end_bit) {
  size_t t = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, (int)begin_bit, (int)end_bit);
  return t + 256;
}

// Stable LSD radix sort of (key, pos) pairs on key bits [begin_bit, end_bit): when the other bits are equal in every
// key (order_keys_kernel's span) the order is the full-width sort's, in fewer passes.
hipError_t launch_sort_pairs(const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout, uint64_t n,
                             void* temp, size_t temp_bytes, hipStream_t s, uint32_t begin_bit, uint32_t end_bit) {
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, kin, kout, vin, vout, (int)n, (int)begin_bit,
                                            (int)end_bit, s);
}

// ------------------------------------------------------------------------------------------ finalisation

__host__ __device__ __forceinline__ uint32_t bits_words(uint32_t card) { return (card + 31u) / 32u; }

// The final SUM of SK_FX aggregation A in slot s (fx_final: the exact fixed-point sum, or IEEE's sum of the
// non-finite inputs seen)
__device__ __forceinline__ double fx_value(const StateView& v, const AggSpec& A, uint64_t s) {
  const unsigned long long* p = v.fx + (s * v.n_fx + A.slot) * 2;
  const int64_t smn = A.sp_min != kNoSp ? (int64_t)v.mn[s * v.n_min + A.sp_min] : 0;
  const int64_t smx = A.sp_max != kNoSp ? (int64_t)v.mx[s * v.n_max + A.sp_max] : 0;
  return fx_final(A, (const uint64_t*)p, smn, smx);
}

// Final value of every aggregation of the groups at `slots` (AggregationFunction.extractFinalResult; AVG keeps
// its (sum, count) pair in vals / cnts, DISTINCTCOUNT its set size).  One thread per group.
__global__ void final_values_kernel(StateView v, FinalSpec f, const uint32_t* __restrict__ slots, uint64_t n,
                                    uint64_t* __restrict__ keys, double* __restrict__ vals,
                                    int64_t* __restrict__ cnts) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t s = slots ? slots[i] : 0;
    keys[i] = v.keys ? v.keys[s] : s;
    const int64_t count = (int64_t)v.i64[s * v.n_i64];
    for (uint32_t a = 0; a < f.num_aggs; a++) {
      const AggSpec& A = f.aggs[a];
      double x = 0;
      int64_t c = 0;
      switch (A.fn) {
        case PG_AGG_COUNT: x = (double)count; break;
        case PG_AGG_COUNTMV: x = (double)(int64_t)v.i64[s * v.n_i64 + A.slot]; break;
        case PG_AGG_SUM:
        case PG_AGG_AVG:
          x = A.integer ? (double)(int64_t)v.i64[s * v.n_i64 + A.slot] : fx_value(v, A, s);
          if (A.fn == PG_AGG_AVG) c = A.cnt_slot ? (int64_t)v.i64[s * v.n_i64 + A.cnt_slot] : count;
          break;
        case PG_AGG_MIN: x = order_key_decode(v.mn[s * v.n_min + A.slot]); break;
        case PG_AGG_MAX: x = order_key_decode(v.mx[s * v.n_max + A.slot]); break;
        case PG_AGG_DISTINCTCOUNT: continue;  // set sizes: dc_sizes_kernel (coalesced bitmap rows)
      }
      vals[i * f.num_aggs + a] = x;
      cnts[i * f.num_aggs + a] = c;
    }
  }
}

// DISTINCTCOUNT a of the groups at `slots`: the popcount of each group's bitmap row (extractFinalResult = set size),
// read coalesced: `lpg` lanes (a power of two covering the row's words, <= 64) share a row, 64 / lpg rows per wave.
// One thread per row would read each 128-byte row alone (config 4: 10 M rows took 5.5 ms that way).
__global__ void dc_sizes_kernel(StateView v, uint32_t dc_word, uint32_t words, uint32_t lpg, uint32_t vec4,
                                const uint32_t* __restrict__ slots,
                                uint64_t n, uint32_t A, uint32_t a, double* __restrict__ vals, int64_t* __restrict__ cnts) {
  const uint32_t lane = threadIdx.x & 63u, sub = lane & (lpg - 1u);
  const uint64_t per_wave = 64u / lpg;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t i0 = wave * per_wave; i0 < n; i0 += nwaves * per_wave) {
    const uint64_t i = i0 + lane / lpg;
    uint32_t pc = 0;
    if (i < n) {
      const uint32_t* w = v.bits + (uint64_t)slots[i] * v.bit_words + dc_word;
      if (vec4) {  // 16-byte aligned rows: 4 words per lane per load
        for (uint32_t k = 4 * sub; k < words; k += 4 * lpg) {
          const uint4 x = *(const uint4*)(w + k);
          pc += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        }
      } else {
        for (uint32_t k = sub; k < words; k += lpg) pc += __popc(w[k]);
      }
    }
    for (uint32_t o = 1; o < lpg; o <<= 1) pc += __shfl_xor(pc, o);
    if (i < n && sub == 0) {
      vals[i * A + a] = (double)pc;
      cnts[i * A + a] = 0;
    }
  }
}

// DISTINCTCOUNT a from the set sizes the bucket pass recorded (StateView::dc_pop): 4 bytes per group read
__global__ void dc_pop_kernel(const uint32_t* __restrict__ pop, const uint32_t* __restrict__ slots, uint64_t n,
                              uint32_t A, uint32_t a, double* __restrict__ vals, int64_t* __restrict__ cnts) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    vals[i * A + a] = (double)pop[slots ? slots[i] : 0];
    cnts[i * A + a] = 0;
  }
}

hipError_t launch_final_values(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                               uint64_t* keys, double* vals, int64_t* cnts, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(final_values_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v, f,
                     slots, n, keys, vals, cnts);
  for (uint32_t a = 0; a < f.num_aggs; a++) {
    if (f.aggs[a].fn != PG_AGG_DISTINCTCOUNT) continue;
    if (v.dc_pop && v.dc_pop_agg == a) {
      hipLaunchKernelGGL(dc_pop_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v.dc_pop,
                         slots, n, f.num_aggs, a, vals, cnts);
      continue;
    }
    const uint32_t words = bits_words(f.aggs[a].key_card);
    // whole uint4 loads when every row and this aggregation's words start 16-byte aligned and fill whole uint4s
    const uint32_t vec4 = (v.bit_words % 4 == 0 && f.aggs[a].dc_word % 4 == 0 && words % 4 == 0) ? 1u : 0u;
    const uint32_t per_lane = vec4 ? 4u : 1u;
    uint32_t lpg = 1;
    while (lpg * per_lane < words && lpg < 64) lpg <<= 1;
    const uint64_t waves = (n * lpg + 63) / 64, b2 = (waves + 3) / 4;
    hipLaunchKernelGGL(dc_sizes_kernel, dim3((uint32_t)(b2 < 16384 ? b2 : 16384)), dim3(256), 0, s, v,
                       f.aggs[a].dc_word, words, lpg, vec4, slots, n, f.num_aggs, a, vals, cnts);
  }
  return hipGetLastError();
}

// Ascending u64 image of the first ORDER BY item (DESC = bit complement), for the radix-sort trim.
__global__ void order_keys_kernel(FinalSpec f, const uint64_t* __restrict__ keys, const double* __restrict__ vals,
                                  const int64_t* __restrict__ cnts, uint64_t n, uint64_t* __restrict__ out,
                                  uint32_t* __restrict__ pos, unsigned long long* __restrict__ span) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t any = 0, anyz = 0;  // OR of the keys, OR of their complements
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t o;
    if (f.order_kind == PG_ORDER_KEY) {
      o = (keys[i] / f.key_stride[f.order_index]) % f.key_card[f.order_index];
    } else {
      const uint32_t a = f.order_index;
      double x = vals[i * f.num_aggs + a];
      if (f.aggs[a].fn == PG_AGG_AVG) {
        const int64_t c = cnts[i * f.num_aggs + a];
        x = c ? x / (double)c : -__builtin_inf();
      }
      int64_t b;
      __builtin_memcpy(&b, &x, 8);
      o = b >= 0 ? ((uint64_t)b | 0x8000000000000000ull) : ~(uint64_t)b;
    }
    o = f.order_desc ? ~o : o;
    out[i] = o;
    pos[i] = (uint32_t)i;
    any |= o;
    anyz |= ~o;
  }
  if (!span) return;
  // block ORs -> one global atomic pair per block (the grid is capped, so a few thousand per launch)
  for (int d = 1; d < 64; d <<= 1) {
    any |= __shfl_xor(any, d);
    anyz |= __shfl_xor(anyz, d);
  }
  __shared__ unsigned long long wa[4], wb[4];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (lane == 0) { wa[w] = any; wb[w] = anyz; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < (blockDim.x >> 6); k++) { any |= wa[k]; anyz |= wb[k]; }
    atomicOr(&span[0], (unsigned long long)any);
    atomicOr(&span[1], (unsigned long long)anyz);
  }
}

hipError_t launch_order_keys(const FinalSpec& f, const uint64_t* keys, const double* vals, const int64_t* cnts,
                             uint64_t n, uint64_t* out, uint32_t* pos, hipStream_t s, uint64_t* span) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256, cap = span ? 2048 : 16384;
  if (span) {
    const hipError_t e = hipMemsetAsync(span, 0, 16, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(order_keys_kernel, dim3((uint32_t)(blocks < cap ? blocks : cap)), dim3(256), 0, s, f, keys,
                     vals, cnts, n, out, pos, (unsigned long long*)span);
  return hipGetLastError();
}

// The same order image straight from the state (no final values of every group first): the ORDER BY aggregation of
// the group at slots[i] -- for a trim, whose final values are then computed for its candidates only (config 4: 10 M
// groups, 240 MB of key / value / count arrays not written and not re-read).  Callers check order_keys_from_state_ok.
__global__ void order_keys_state_kernel(StateView v, FinalSpec f, const uint32_t* __restrict__ slots, uint64_t n,
                                        uint64_t* __restrict__ out, uint32_t* __restrict__ pos,
                                        unsigned long long* __restrict__ span) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t any = 0, anyz = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t s = slots ? slots[i] : 0;
    uint64_t o;
    if (f.order_kind == PG_ORDER_KEY) {
      const uint64_t key = v.keys ? v.keys[s] : s;
      o = (key / f.key_stride[f.order_index]) % f.key_card[f.order_index];
    } else {
      const AggSpec& A = f.aggs[f.order_index];
      const int64_t count = (int64_t)v.i64[s * v.n_i64];
      double x = 0;
      switch (A.fn) {
        case PG_AGG_COUNT: x = (double)count; break;
        case PG_AGG_COUNTMV: x = (double)(int64_t)v.i64[s * v.n_i64 + A.slot]; break;
        case PG_AGG_SUM:
        case PG_AGG_AVG:
          x = A.integer ? (double)(int64_t)v.i64[s * v.n_i64 + A.slot] : fx_value(v, A, s);
          if (A.fn == PG_AGG_AVG) {
            const int64_t c = A.cnt_slot ? (int64_t)v.i64[s * v.n_i64 + A.cnt_slot] : count;
            x = c ? x / (double)c : -__builtin_inf();
          }
          break;
        case PG_AGG_MIN: x = order_key_decode(v.mn[s * v.n_min + A.slot]); break;
        case PG_AGG_MAX: x = order_key_decode(v.mx[s * v.n_max + A.slot]); break;
        case PG_AGG_DISTINCTCOUNT: x = (double)v.dc_pop[s]; break;
      }
      int64_t b;
      __builtin_memcpy(&b, &x, 8);
      o = b >= 0 ? ((uint64_t)b | 0x8000000000000000ull) : ~(uint64_t)b;
    }
    o = f.order_desc ? ~o : o;
    out[i] = o;
    pos[i] = (uint32_t)i;
    any |= o;
    anyz |= ~o;
  }
  for (int d = 1; d < 64; d <<= 1) {
    any |= __shfl_xor(any, d);
    anyz |= __shfl_xor(anyz, d);
  }
  __shared__ unsigned long long wa[4], wb[4];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (lane == 0) { wa[w] = any; wb[w] = anyz; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < (blockDim.x >> 6); k++) { any |= wa[k]; anyz |= wb[k]; }
    atomicOr(&span[0], (unsigned long long)any);
    atomicOr(&span[1], (unsigned long long)anyz);
  }
}

bool order_keys_from_state_ok(const StateView& v, const FinalSpec& f) {
  if (f.order_kind == PG_ORDER_KEY) return true;
  if (f.order_index >= f.num_aggs) return false;
  const AggSpec& A = f.aggs[f.order_index];
  return A.fn != PG_AGG_DISTINCTCOUNT || (v.dc_pop && v.dc_pop_agg == f.order_index);
}

hipError_t launch_order_keys_state(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                                   uint64_t* out, uint32_t* pos, uint64_t* span, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(span, 0, 16, s);
  if (e != hipSuccess || !n) return e;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(order_keys_state_kernel, dim3((uint32_t)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, s, v, f,
                     slots, n, out, pos, (unsigned long long*)span);
  return hipGetLastError();
}

__global__ void gather_slots_kernel(const uint32_t* __restrict__ slots, const uint32_t* __restrict__ pos, uint64_t n,
                                    uint32_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = slots[pos[i]];
}

hipError_t launch_gather_slots(const uint32_t* slots, const uint32_t* pos, uint64_t n, uint32_t* out, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(gather_slots_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, slots,
                     pos, n, out);
  return hipGetLastError();
}

// Number of sorted entries that rank within the first `limit`, ties with the limit-th included.
__global__ void cutoff_kernel(const uint64_t* __restrict__ sorted, uint64_t n, uint64_t limit, uint64_t* out) {
  const uint64_t t = sorted[limit - 1];
  uint64_t lo = limit, hi = n;  // first index with sorted > t
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (sorted[mid] <= t) lo = mid + 1;
    else hi = mid;
  }
  *out = lo;
}

hipError_t launch_cutoff(const uint64_t* sorted, uint64_t n, uint64_t limit, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(cutoff_kernel, dim3(1), dim3(1), 0, s, sorted, n, limit, out);
  return hipGetLastError();
}

// ---- ORDER BY trim by radix select (instead of sorting every group): in the key space k' = (okey >> b0) & (2^W - 1)
// (the only bits in which the order keys differ, order_keys_kernel's span), the limit-th smallest k' is found digit by
// digit from the top: per pass a histogram of one <= kOkeyDigitBits-bit digit over the keys whose higher digits equal the prefix
// chosen so far.  The candidates are then every key <= that value (the sorted cutoff's set: ties at the boundary
// kept), compacted into a position list.
__device__ __forceinline__ uint64_t kprime(uint64_t k, uint32_t b0, uint32_t W) {
  const uint64_t x = k >> b0;
  return W >= 64 ? x : (x & ((1ull << W) - 1ull));
}

__global__ void okey_hist_kernel(const uint64_t* __restrict__ keys, uint64_t n, uint32_t b0, uint32_t W, uint32_t lo,
                                 uint32_t hi, uint64_t prefix, unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[1u << kOkeyDigitBits];
  const uint32_t tid = threadIdx.x, nd = 1u << (hi - lo);
  for (uint32_t d = tid; d < nd; d += blockDim.x) h[d] = 0;
  __syncthreads();
  const uint64_t dmask = (1ull << (hi - lo)) - 1ull;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + tid; i < n; i += stride) {
    const uint64_t k = kprime(keys[i], b0, W);
    if (hi >= 64 || (k >> hi) == prefix) atomicAdd(&h[(k >> lo) & dmask], 1u);
  }
  __syncthreads();
  for (uint32_t d = tid; d < nd; d += blockDim.x)
    if (h[d]) atomicAdd(&hist[d], h[d]);
}

__global__ void okey_select_kernel(const uint64_t* __restrict__ keys, uint64_t n, uint32_t b0, uint32_t W,
                                   uint64_t tstar, uint32_t* __restrict__ pos, unsigned long long* __restrict__ count) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    const bool take = i < n && kprime(keys[i], b0, W) <= tstar;
    const uint64_t m = __ballot(take);
    if (!m) continue;
    unsigned long long base = 0;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(m));
    base = __shfl(base, (int)leader);
    if (take) pos[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
  }
}

hipError_t launch_okey_hist(const uint64_t* keys, uint64_t n, uint32_t b0, uint32_t W, uint32_t lo, uint32_t hi,
                            uint64_t prefix, unsigned int* hist, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(okey_hist_kernel, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256), 0, s, keys, n, b0, W,
                     lo, hi, prefix, hist);
  return hipGetLastError();
}

hipError_t launch_okey_select(const uint64_t* keys, uint64_t n, uint32_t b0, uint32_t W, uint64_t tstar, uint32_t* pos,
                              unsigned long long* count, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(okey_select_kernel, dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256), 0, s, keys, n, b0,
                     W, tstar, pos, count);
  return hipGetLastError();
}

// out[i] = in[pos[i]] for the candidates (keys, per-agg values / counts, slots).
__global__ void gather_final_kernel(uint32_t A, const uint32_t* __restrict__ pos, uint64_t n,
                                    const uint64_t* __restrict__ keys, const double* __restrict__ vals,
                                    const int64_t* __restrict__ cnts, const uint32_t* __restrict__ slots,
                                    uint64_t* __restrict__ okeys, double* __restrict__ ovals,
                                    int64_t* __restrict__ ocnts, uint32_t* __restrict__ oslots) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t p = pos[i];
    okeys[i] = keys[p];
    oslots[i] = slots ? slots[p] : 0u;
    for (uint32_t a = 0; a < A; a++) {
      ovals[i * A + a] = vals[(uint64_t)p * A + a];
      ocnts[i * A + a] = cnts[(uint64_t)p * A + a];
    }
  }
}

hipError_t launch_gather_final(uint32_t A, const uint32_t* pos, uint64_t n, const uint64_t* keys, const double* vals,
                               const int64_t* cnts, const uint32_t* slots, uint64_t* okeys, double* ovals,
                               int64_t* ocnts, uint32_t* oslots, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(gather_final_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, A, pos,
                     n, keys, vals, cnts, slots, okeys, ovals, ocnts, oslots);
  return hipGetLastError();
}

// Value sets: sizes[i*A + a] = |set| of DISTINCTCOUNT aggregation a of group slots[i] (0 for other functions).
__global__ void set_sizes_kernel(StateView v, FinalSpec f, const uint32_t* __restrict__ slots, uint64_t n,
                                 uint64_t* __restrict__ sizes) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t s = slots[i];
    for (uint32_t a = 0; a < f.num_aggs; a++) {
      uint64_t pc = 0;
      if (f.aggs[a].fn == PG_AGG_DISTINCTCOUNT) {
        const uint32_t* w = v.bits + s * v.bit_words + f.aggs[a].dc_word;
        for (uint32_t k = 0; k < bits_words(f.aggs[a].key_card); k++) pc += __popc(w[k]);
      }
      sizes[i * f.num_aggs + a] = pc;
    }
  }
}

hipError_t launch_set_sizes(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                            uint64_t* sizes, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(set_sizes_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v, f,
                     slots, n, sizes);
  return hipGetLastError();
}

// One wave per (group, DISTINCTCOUNT aggregation): the set bits of its bitmap, ascending, at offsets[i*A + a]
// (an exclusive scan of set_sizes).  A lane takes one word per round; a wave prefix sum of the word popcounts
// places its ids.
__global__ void set_extract_kernel(StateView v, FinalSpec f, const uint32_t* __restrict__ slots, uint64_t n,
                                   const uint64_t* __restrict__ offsets, uint32_t* __restrict__ ids) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t job = wave; job < n * f.num_aggs; job += nwaves) {
    const uint64_t i = job / f.num_aggs;
    const uint32_t a = (uint32_t)(job % f.num_aggs);
    if (f.aggs[a].fn != PG_AGG_DISTINCTCOUNT) continue;
    const uint32_t* w = v.bits + (uint64_t)slots[i] * v.bit_words + f.aggs[a].dc_word;
    const uint32_t nw = bits_words(f.aggs[a].key_card);
    uint64_t out = offsets[job];
    for (uint32_t k0 = 0; k0 < nw; k0 += 64) {
      const uint32_t k = k0 + lane;
      uint32_t x = k < nw ? w[k] : 0u;
      const uint32_t c = __popc(x);
      uint32_t incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
      }
      uint64_t at = out + incl - c;
      while (x) {
        const uint32_t b = (uint32_t)__ffs(x) - 1u;
        ids[at++] = k * 32u + b;
        x &= x - 1u;
      }
      out += __shfl(incl, 63);
    }
  }
}

hipError_t launch_set_extract(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                              const uint64_t* offsets, uint32_t* ids, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t waves = n * f.num_aggs;
  const uint64_t blocks = (waves + 3) / 4;
  hipLaunchKernelGGL(set_extract_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v, f,
                     slots, n, offsets, ids);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ exchange rows

uint64_t row_bytes(const StateView& v) {
  const uint64_t b = 8ull * (1 + v.n_i64 + 2ull * v.n_fx + v.n_min + v.n_max) + 4ull * v.bit_words;
  return (b + 7) & ~7ull;
}

// rows[i] = { key / key_div | state of slots[i] } (GroupByOrderByCombineOperator's per-group record).
__global__ void gather_rows_kernel(StateView v, const uint32_t* __restrict__ slots, uint64_t n, uint64_t key_div,
                                   uint8_t* __restrict__ dst, uint64_t rb) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t s = slots[i];
    uint64_t* r = (uint64_t*)(dst + i * rb);
    r[0] = (v.keys ? v.keys[s] : s) / key_div;
    uint64_t o = 1;
    for (uint32_t k = 0; k < v.n_i64; k++) r[o++] = v.i64[s * v.n_i64 + k];
    for (uint32_t k = 0; k < 2 * v.n_fx; k++) r[o++] = v.fx[s * v.n_fx * 2 + k];
    for (uint32_t k = 0; k < v.n_min; k++) r[o++] = (uint64_t)v.mn[s * v.n_min + k];
    for (uint32_t k = 0; k < v.n_max; k++) r[o++] = (uint64_t)v.mx[s * v.n_max + k];
    uint32_t* b = (uint32_t*)(r + o);
    for (uint32_t k = 0; k < v.bit_words; k++) b[k] = v.bits[s * v.bit_words + k];
  }
}

hipError_t launch_gather_rows(const StateView& v, const uint32_t* slots, uint64_t n, uint64_t key_div, uint8_t* dst,
                              hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v,
                     slots, n, key_div, dst, row_bytes(v));
  return hipGetLastError();
}

// Insert-merge rows into a GM_HASH table: AggregationFunction.merge per state kind.
__global__ void merge_rows_kernel(StateView v, const uint8_t* __restrict__ src, uint64_t n, uint64_t rb) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t* r = (const uint64_t*)(src + i * rb);
    const uint64_t key = r[0];
    uint64_t h = mix64(key) & v.hmask, s = ~0ull;
    for (uint64_t probe = 0; probe <= v.hmask; probe++) {
      const unsigned long long cur = v.keys[h];
      if (cur == key) { s = h; break; }
      if (cur == kEmptyKey) {
        if (__hip_atomic_load(v.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v.max_fill) break;
        const unsigned long long prev = atomicCAS(&v.keys[h], kEmptyKey, (unsigned long long)key);
        if (prev == kEmptyKey) { atomicAdd(v.fill, 1u); s = h; break; }
        if (prev == key) { s = h; break; }
      }
      h = (h + 1) & v.hmask;
    }
    if (s == ~0ull) {
      atomicOr(v.err, 4u);
      continue;
    }
    uint64_t o = 1;
    for (uint32_t k = 0; k < v.n_i64; k++) atomicAdd(&v.i64[s * v.n_i64 + k], (unsigned long long)r[o++]);
    for (uint32_t k = 0; k < v.n_fx; k++, o += 2) {  // 128-bit add: the low word's carry-out goes to the high word
      unsigned long long* p = v.fx + (s * v.n_fx + k) * 2;
      const uint64_t lo = r[o], old = atomicAdd(p, (unsigned long long)lo);
      const uint64_t hi = r[o + 1] + (old + lo < old ? 1ull : 0ull);
      if (hi) atomicAdd(p + 1, (unsigned long long)hi);
    }
    for (uint32_t k = 0; k < v.n_min; k++) atomicMin(&v.mn[s * v.n_min + k], (long long)r[o++]);
    for (uint32_t k = 0; k < v.n_max; k++) atomicMax(&v.mx[s * v.n_max + k], (long long)r[o++]);
    const uint32_t* b = (const uint32_t*)(r + o);
    for (uint32_t k = 0; k < v.bit_words; k++)
      if (b[k]) atomicOr(&v.bits[s * v.bit_words + k], b[k]);
  }
}

hipError_t launch_merge_rows(const StateView& v, const uint8_t* rows, uint64_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(merge_rows_kernel, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, s, v, rows,
                     n, row_bytes(v));
  return hipGetLastError();
}

// Dense merge: every array element-wise, one thread per (slot, word) of each array -- no atomics (each element has
// one owner), coalesced reads of both states.  fx pairs: one thread per pair, carry from the low word to the high word.
__global__ void merge_dense_kernel(StateView d, StateView s) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x, t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t G = d.num_slots;
  for (uint64_t i = t0; i < G * d.n_i64; i += stride) d.i64[i] += s.i64[i];
  for (uint64_t i = t0; i < G * d.n_fx; i += stride) {
    const uint64_t lo = d.fx[2 * i] + s.fx[2 * i];
    d.fx[2 * i + 1] += s.fx[2 * i + 1] + (lo < (uint64_t)s.fx[2 * i] ? 1ull : 0ull);
    d.fx[2 * i] = lo;
  }
  for (uint64_t i = t0; i < G * d.n_min; i += stride) d.mn[i] = s.mn[i] < d.mn[i] ? s.mn[i] : d.mn[i];
  for (uint64_t i = t0; i < G * d.n_max; i += stride) d.mx[i] = s.mx[i] > d.mx[i] ? s.mx[i] : d.mx[i];
  const uint64_t nb = G * d.bit_words;
  const uint64_t nb4 = (d.bits && s.bits && ((uintptr_t)d.bits % 16 == 0) && ((uintptr_t)s.bits % 16 == 0)) ? nb / 4 : 0;
  for (uint64_t i = t0; i < nb4; i += stride) {  // 16-byte words for the bitmaps (config 4: 1.28 GB of them)
    uint4 a = ((uint4*)d.bits)[i];
    const uint4 b = ((const uint4*)s.bits)[i];
    a.x |= b.x; a.y |= b.y; a.z |= b.z; a.w |= b.w;
    ((uint4*)d.bits)[i] = a;
  }
  for (uint64_t i = 4 * nb4 + t0; i < nb; i += stride) d.bits[i] |= s.bits[i];
}

hipError_t launch_merge_dense(const StateView& dst, const StateView& src, hipStream_t s) {
  hipLaunchKernelGGL(merge_dense_kernel, dim3(4096), dim3(256), 0, s, dst, src);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ numGroupsLimit

// Sort key of an occupied GM_HASH_SEG entry -> the segment's first-seen order: (segment, first matching doc) in 32 + 32
// bits, or with multi-value keys (segment, doc, tuple position) in 16 + 32 + 16 bits (first_doc = doc << 16 | position).
__global__ void seg_order_kernel(StateView v, const uint32_t* __restrict__ slots, uint64_t n, uint32_t num_segments,
                                 uint32_t shift, uint64_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t s = slots[i];
    const uint64_t seg = v.keys[s] % num_segments;
    const uint64_t first = v.first_doc[s];
    out[i] = (seg << shift) | (shift == 32 ? first >> 16 : first);
  }
}

// keep[i] = rank of sorted entry i within its segment < limit (seg_first: first sorted index of each segment).
__global__ void seg_first_kernel(const uint64_t* __restrict__ sorted, uint64_t n, uint32_t shift,
                                 uint32_t* __restrict__ seg_first) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    if (i == 0 || (sorted[i] >> shift) != (sorted[i - 1] >> shift)) seg_first[sorted[i] >> shift] = (uint32_t)i;
}
// reached: set when some segment holds >= limit keys (its rank limit - 1 exists: numGroupsLimitReached)
__global__ void seg_keep_kernel(const uint64_t* __restrict__ sorted, uint64_t n, uint32_t shift,
                                const uint32_t* __restrict__ seg_first, uint64_t limit, uint8_t* __restrict__ keep,
                                unsigned int* __restrict__ reached) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t rank = i - seg_first[sorted[i] >> shift];
    keep[i] = rank < limit;
    if (rank + 1 == limit) atomicOr(reached, 1u);
  }
}

hipError_t launch_seg_truncate(const StateView& v, const uint32_t* slots, uint64_t n, uint32_t num_segments,
                               uint64_t limit, bool mv, uint64_t* tmp_keys, uint64_t* sorted_keys, uint32_t* sorted_slots,
                               uint32_t* seg_first, uint8_t* keep, unsigned int* reached, void* temp, size_t temp_bytes,
                               hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  const dim3 g((uint32_t)(blocks < 16384 ? blocks : 16384));
  const uint32_t shift = mv ? 48u : 32u;
  hipLaunchKernelGGL(seg_order_kernel, g, dim3(256), 0, s, v, slots, n, num_segments, shift, tmp_keys);
  hipError_t e = launch_sort_pairs(tmp_keys, sorted_keys, slots, sorted_slots, n, temp, temp_bytes, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(seg_first_kernel, g, dim3(256), 0, s, sorted_keys, n, shift, seg_first);
  hipLaunchKernelGGL(seg_keep_kernel, g, dim3(256), 0, s, sorted_keys, n, shift, seg_first, limit, keep, reached);
  return hipGetLastError();
}

}  // namespace pg

extern "C" uint32_t pg_key_owner(uint64_t key, uint32_t num_parts) {
  return num_parts ? pg::key_owner(key, num_parts) : 0u;
}
