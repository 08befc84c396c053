// pg_kernels.hip -- gfx950 kernels of the segment query hot path.
//
// scan_kernel is the fused hot loop that replaces, per tile of 4096 docs, Pinot's chain
//   DocIdSetOperator (10 000-doc blocks, operator/DocIdSetOperator.java:58-83)
//   -> SVScanDocIdIterator + PredicateEvaluator.applySV (dociditerators/SVScanDocIdIterator.java:67-125)
//   -> FixedBitSVForwardIndexReaderV2.readDictIds / FixedBitIntReader (readers/forward/...V2.java:62-97)
//   -> AND/OR/NOT doc-id algebra (docidsets/AndDocIdSet.java:60-150, OrDocIdSet.java:58-114)
//   -> DataFetcher.readDoubleValues + Dictionary.readDoubleValues (common/DataFetcher.java:511-521)
//   -> Sum/Count/Min/Max/Avg/DistinctCount/CountMV aggregate / aggregateGroupBySV
//   -> DictionaryBasedGroupKeyGenerator mixed-radix keys (groupby/DictionaryBasedGroupKeyGenerator.java:280-322)
// with no intermediate doc-id lists: each thread owns docs base + j*256 + tid (j < 16), so the 64 lanes
// of a wave read 64 consecutive packed values (one contiguous run of 8*b bytes) per load instruction.
// Nothing here is a dense contraction: there is no MFMA; the roofline is HBM bandwidth.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "pg_internal.h"

namespace pg {

// ------------------------------------------------------------------------------------------ helpers

// FixedBitIntReader.readUnchecked equivalent on the native-word image: value `idx` of `b` bits.
__device__ __forceinline__ uint32_t unpack(const uint32_t* __restrict__ w, uint64_t idx, uint32_t b) {
  const uint64_t p = idx * b;
  const uint64_t wi = p >> 5;
  const uint32_t off = (uint32_t)p & 31u;
  const uint64_t win = ((uint64_t)w[wi] << 32) | (uint64_t)w[wi + 1];
  const uint32_t mask = b >= 32 ? 0xFFFFFFFFu : ((1u << b) - 1u);
  return (uint32_t)(win >> (64u - off - b)) & mask;
}

__device__ __forceinline__ double dict_double(const DevCol& c, uint32_t id) {
  switch (c.dtype) {
    case PG_INT: return (double)((const int32_t*)c.dict)[id];
    case PG_LONG: return (double)((const int64_t*)c.dict)[id];
    case PG_FLOAT: return (double)((const float*)c.dict)[id];
    default: return ((const double*)c.dict)[id];
  }
}

__device__ __forceinline__ int64_t dict_i64(const DevCol& c, uint32_t id) {
  return c.dtype == PG_INT ? (int64_t)((const int32_t*)c.dict)[id] : ((const int64_t*)c.dict)[id];
}

// TransformFunction value of an aggregation input (double path).
// MultiplicationTransformFunction.transformToDoubleValuesSV (transform/function/MultiplicationTransformFunction.java:91-111):
// start from the literal product 1.0, multiply arguments in order; compiled with -ffp-contract=off.
__device__ __forceinline__ double agg_value_f64(const AggSpec& a, const DevCol* c, uint32_t d) {
  const double va = dict_double(c[0], unpack(c[0].words, d, c[0].bits));
  if (a.op == PG_EXPR_COL) return va;
  const double vb = dict_double(c[1], unpack(c[1].words, d, c[1].bits));
  switch (a.op) {
    case PG_EXPR_MUL: return (1.0 * va) * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// integer-exact path (host proved |result| bounds): identical value to the double path when < 2^53
__device__ __forceinline__ int64_t agg_value_i64(const AggSpec& a, const DevCol* c, uint32_t d) {
  const int64_t va = dict_i64(c[0], unpack(c[0].words, d, c[0].bits));
  if (a.op == PG_EXPR_COL) return va;
  const int64_t vb = dict_i64(c[1], unpack(c[1].words, d, c[1].bits));
  switch (a.op) {
    case PG_EXPR_MUL: return va * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

__device__ __forceinline__ uint64_t col_key(uint32_t kind, int64_t base, const DevCol& c, uint32_t d) {
  const uint32_t id = unpack(c.words, d, c.bits);
  return kind == PG_KEY_KEYMAP ? (uint64_t)(uint32_t)c.keymap[id] : (uint64_t)(dict_i64(c, id) - base);
}

// One leaf over the thread's 16 docs -> 16-bit mask (bit j <-> doc base + j*256 + tid).
__device__ __forceinline__ uint32_t eval_leaf(const DevLeaf& L, uint32_t base, uint32_t last_doc, int tid) {
  uint32_t m = 0;
  switch (L.kind) {
    case DL_ALL: m = 0xFFFFu; break;
    case DL_NONE: m = 0u; break;
    case DL_RANGE: {
      const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll
      for (int j = 0; j < kDocsPerThread; j++) {
        const uint32_t d = min(base + (uint32_t)(j * kBlock + tid), last_doc);
        const uint32_t v = unpack(L.words, d, L.bits);
        m |= (uint32_t)((v - lo) < span) << j;
      }
      break;
    }
    case DL_LUT: {
#pragma unroll
      for (int j = 0; j < kDocsPerThread; j++) {
        const uint32_t d = min(base + (uint32_t)(j * kBlock + tid), last_doc);
        const uint32_t v = unpack(L.words, d, L.bits);
        m |= ((L.lut[v >> 5] >> (v & 31u)) & 1u) << j;
      }
      break;
    }
    case DL_DOCBITMAP: {
#pragma unroll
      for (int j = 0; j < kDocsPerThread; j++) {
        const uint32_t d = min(base + (uint32_t)(j * kBlock + tid), last_doc);
        m |= ((L.words[d >> 5] >> (d & 31u)) & 1u) << j;
      }
      break;
    }
    default: {  // DL_DOCRANGE
#pragma unroll
      for (int j = 0; j < kDocsPerThread; j++) {
        const uint32_t d = base + (uint32_t)(j * kBlock + tid);
        m |= (uint32_t)(d >= (uint32_t)L.lo && d < (uint32_t)L.hi) << j;
      }
      break;
    }
  }
  return L.excl ? (~m & 0xFFFFu) : m;
}

// Postfix filter program over 16-bit masks; the stack (<= 8 entries) lives in two 64-bit registers.
__device__ __forceinline__ uint32_t eval_program(const QuerySpec& q, const DevLeaf* __restrict__ leaves,
                                                 uint32_t base, uint32_t last_doc, int tid) {
  uint64_t lo = 0, hi = 0;
  for (uint32_t i = 0; i < q.num_ops; i++) {
    const int32_t op = q.ops[i];
    if (op >= 0) {
      const uint32_t m = eval_leaf(leaves[op], base, last_doc, tid);
      hi = (hi << 16) | (lo >> 48);
      lo = (lo << 16) | m;
    } else if (op == PG_OP_NOT) {
      lo ^= 0xFFFFull;
    } else {
      const int n = (-op) & 0xFF;
      const bool is_and = ((-op) & 0x100) != 0;
      uint32_t acc = (uint32_t)(lo & 0xFFFFu);
      lo = (lo >> 16) | (hi << 48);
      hi >>= 16;
      for (int k = 1; k < n; k++) {
        const uint32_t m = (uint32_t)(lo & 0xFFFFu);
        lo = (lo >> 16) | (hi << 48);
        hi >>= 16;
        acc = is_and ? (acc & m) : (acc | m);
      }
      hi = (hi << 16) | (lo >> 48);
      lo = (lo << 16) | acc;
    }
  }
  return q.num_ops ? (uint32_t)(lo & 0xFFFFu) : 0xFFFFu;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t x = __shfl_xor(v, o); v = x < v ? x : v; }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { int64_t x = __shfl_xor(v, o); v = x > v ? x : v; }
  return v;
}

// ------------------------------------------------------------------------------------------ scan

__global__ __launch_bounds__(kBlock) void scan_kernel(QuerySpec q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const uint64_t T = q.total_tiles;
  const uint64_t t0 = (uint64_t)blockIdx.x * T / gridDim.x;
  const uint64_t t1 = ((uint64_t)blockIdx.x + 1) * T / gridDim.x;
  const bool grouped = q.num_keys > 0;

  // LDS-privatised group table: [G][n_i64] u64 | [G][n_f64] f64 | [G][n_min] i64 | [G][n_max] i64
  unsigned long long* l_i64 = (unsigned long long*)smem;
  double* l_f64 = (double*)(l_i64 + q.num_slots * q.n_i64);
  long long* l_mn = (long long*)(l_f64 + q.num_slots * q.n_f64);
  long long* l_mx = l_mn + q.num_slots * q.n_min;
  if (grouped && q.use_lds) {
    for (uint64_t i = tid; i < q.num_slots * q.n_i64; i += kBlock) l_i64[i] = 0;
    for (uint64_t i = tid; i < q.num_slots * q.n_f64; i += kBlock) l_f64[i] = 0.0;
    for (uint64_t i = tid; i < q.num_slots * q.n_min; i += kBlock) l_mn[i] = order_key(__builtin_inf());
    for (uint64_t i = tid; i < q.num_slots * q.n_max; i += kBlock) l_mx[i] = order_key(-__builtin_inf());
    __syncthreads();
  }

  // aggregation-only accumulators (registers; indices compile-time via unrolled agg loops)
  uint64_t acc[kMaxAggs];
#pragma unroll
  for (int a = 0; a < kMaxAggs; a++) {
    acc[a] = 0;
    if (a < (int)q.num_aggs) {
      if (q.aggs[a].kind == SK_MIN) acc[a] = (uint64_t)order_key(__builtin_inf());
      if (q.aggs[a].kind == SK_MAX) acc[a] = (uint64_t)order_key(-__builtin_inf());
    }
  }
  uint64_t doc_count = 0;  // matched docs of this thread (aggregation-only slot 0)

  // segment of the first tile
  uint32_t seg = 0;
  if (t0 < t1) {
    uint32_t lo = 0, hi = q.num_segments;  // last seg with tile_prefix[seg] <= t0
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (q.tile_prefix[mid] <= t0) lo = mid; else hi = mid;
    }
    seg = lo;
  }
  uint64_t seg_count = 0;

  for (uint64_t t = t0; t < t1; t++) {
    while (t >= q.tile_prefix[seg + 1]) {
      const uint64_t c = wave_sum_u64(seg_count);
      if ((tid & 63) == 0 && c) atomicAdd(&q.seg_matched[seg], (unsigned long long)c);
      seg_count = 0;
      seg++;
    }
    const uint32_t nd = q.num_docs[seg];
    const uint32_t base = (uint32_t)(t - q.tile_prefix[seg]) * (uint32_t)kTileDocs;
    const uint32_t last_doc = nd - 1;
    uint32_t valid = 0;
#pragma unroll
    for (int j = 0; j < kDocsPerThread; j++) valid |= (uint32_t)(base + (uint32_t)(j * kBlock + tid) < nd) << j;

    const DevLeaf* leaves = q.leaves + (uint64_t)seg * q.num_leaves;
    uint32_t m = eval_program(q, leaves, base, last_doc, tid) & valid;
    const uint32_t nm = __popc(m);
    seg_count += nm;
    if (m == 0) continue;

    const DevCol* aggcols = q.aggcols + (uint64_t)seg * q.num_aggs * 2;
    if (!grouped) {
      doc_count += nm;
      while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1;
        const uint32_t d = base + (uint32_t)(j * kBlock + tid);
#pragma unroll
        for (int a = 0; a < kMaxAggs; a++) {
          if (a >= (int)q.num_aggs) break;
          const AggSpec& A = q.aggs[a];
          const DevCol* c = aggcols + 2 * a;
          switch (A.fn) {
            case PG_AGG_COUNT: acc[a] += 1; break;
            case PG_AGG_COUNTMV: acc[a] += c[0].mv_offsets[d + 1] - c[0].mv_offsets[d]; break;
            case PG_AGG_SUM:
            case PG_AGG_AVG:
              if (A.integer) acc[a] += (uint64_t)agg_value_i64(A, c, d);
              else acc[a] = __double_as_longlong(__longlong_as_double(acc[a]) + agg_value_f64(A, c, d));
              break;  // AVG count == the group's doc count (slot 0)
            case PG_AGG_MIN: {
              const int64_t k = order_key(agg_value_f64(A, c, d));
              if (k < (int64_t)acc[a]) acc[a] = (uint64_t)k;
              break;
            }
            case PG_AGG_MAX: {
              const int64_t k = order_key(agg_value_f64(A, c, d));
              if (k > (int64_t)acc[a]) acc[a] = (uint64_t)k;
              break;
            }
            case PG_AGG_DISTINCTCOUNT: {
              const uint64_t key = col_key(A.key_kind, A.key_base, c[0], d);
              q.flags[A.flag_off + key] = 1;
              break;
            }
          }
        }
      }
    } else {
      const DevCol* keycols = q.keycols + (uint64_t)seg * q.num_keys;
      while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1;
        const uint32_t d = base + (uint32_t)(j * kBlock + tid);
        uint64_t g = 0;
#pragma unroll
        for (int k = 0; k < kMaxKeys; k++) {
          if (k >= (int)q.num_keys) break;
          g += col_key(q.key_kind[k], q.key_base[k], keycols[k], d) * q.key_stride[k];
        }
        unsigned long long* gi = q.use_lds ? l_i64 : q.i64;
        double* gf = q.use_lds ? l_f64 : q.f64;
        long long* gmn = q.use_lds ? l_mn : q.mn;
        long long* gmx = q.use_lds ? l_mx : q.mx;
        atomicAdd(&gi[g * q.n_i64], 1ull);  // slot 0: doc count / presence
#pragma unroll
        for (int a = 0; a < kMaxAggs; a++) {
          if (a >= (int)q.num_aggs) break;
          const AggSpec& A = q.aggs[a];
          const DevCol* c = aggcols + 2 * a;
          switch (A.fn) {
            case PG_AGG_COUNT: break;  // = slot 0
            case PG_AGG_COUNTMV:
              atomicAdd(&gi[g * q.n_i64 + A.slot],
                        (unsigned long long)(c[0].mv_offsets[d + 1] - c[0].mv_offsets[d]));
              break;
            case PG_AGG_SUM:
            case PG_AGG_AVG:
              if (A.integer) atomicAdd(&gi[g * q.n_i64 + A.slot], (unsigned long long)agg_value_i64(A, c, d));
              else atomicAdd(&gf[g * q.n_f64 + A.slot], agg_value_f64(A, c, d));
              break;  // AVG count == slot 0
            case PG_AGG_MIN:
              atomicMin(&gmn[g * q.n_min + A.slot], (long long)order_key(agg_value_f64(A, c, d)));
              break;
            case PG_AGG_MAX:
              atomicMax(&gmx[g * q.n_max + A.slot], (long long)order_key(agg_value_f64(A, c, d)));
              break;
            case PG_AGG_DISTINCTCOUNT: {
              const uint64_t key = col_key(A.key_kind, A.key_base, c[0], d);
              q.flags[g * q.flag_bytes_per_slot + A.flag_off + key] = 1;
              break;
            }
          }
        }
      }
    }
  }
  {
    const uint64_t c = wave_sum_u64(seg_count);
    if ((tid & 63) == 0 && c) atomicAdd(&q.seg_matched[seg], (unsigned long long)c);
  }

  if (!grouped) {
    // wave-reduce then one global atomic per wave per slot
    const uint64_t dc = wave_sum_u64(doc_count);
    const bool lead = (tid & 63) == 0;
    if (lead && dc) atomicAdd(&q.i64[0], (unsigned long long)dc);
#pragma unroll
    for (int a = 0; a < kMaxAggs; a++) {
      if (a >= (int)q.num_aggs) break;
      const AggSpec& A = q.aggs[a];
      switch (A.kind) {
        case SK_I64: {
          const uint64_t v = wave_sum_u64(acc[a]);
          if (lead && v) atomicAdd(&q.i64[A.slot], (unsigned long long)v);
          break;
        }
        case SK_F64: {
          const double v = wave_sum_f64(__longlong_as_double(acc[a]));
          if (lead && v != 0.0) atomicAdd(&q.f64[A.slot], v);
          break;
        }
        case SK_MIN: {
          const int64_t v = wave_min_i64((int64_t)acc[a]);
          if (lead) atomicMin(&q.mn[A.slot], (long long)v);
          break;
        }
        case SK_MAX: {
          const int64_t v = wave_max_i64((int64_t)acc[a]);
          if (lead) atomicMax(&q.mx[A.slot], (long long)v);
          break;
        }
        default: break;
      }
    }
  } else if (q.use_lds) {
    __syncthreads();
    for (uint64_t g = tid; g < q.num_slots; g += kBlock) {
      if (l_i64[g * q.n_i64] == 0) continue;
      for (uint32_t s = 0; s < q.n_i64; s++) {
        const unsigned long long v = l_i64[g * q.n_i64 + s];
        if (v) atomicAdd(&q.i64[g * q.n_i64 + s], v);
      }
      for (uint32_t s = 0; s < q.n_f64; s++) atomicAdd(&q.f64[g * q.n_f64 + s], l_f64[g * q.n_f64 + s]);
      for (uint32_t s = 0; s < q.n_min; s++) atomicMin(&q.mn[g * q.n_min + s], l_mn[g * q.n_min + s]);
      for (uint32_t s = 0; s < q.n_max; s++) atomicMax(&q.mx[g * q.n_max + s], l_mx[g * q.n_max + s]);
    }
  }
}

hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s) {
  size_t lds = 0;
  if (q.num_keys && q.use_lds) lds = q.num_slots * 8ull * (q.n_i64 + q.n_f64 + q.n_min + q.n_max);
  hipLaunchKernelGGL(scan_kernel, dim3(blocks), dim3(kBlock), lds, s, q);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ state init

__global__ void init_minmax_kernel(long long* mn, uint64_t nmn, long long* mx, uint64_t nmx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = i; k < nmn; k += stride) mn[k] = order_key(__builtin_inf());
  for (uint64_t k = i; k < nmx; k += stride) mx[k] = order_key(-__builtin_inf());
}

hipError_t launch_init_state(const QuerySpec& q, hipStream_t s) {
  hipError_t e;
  if (q.n_i64 && (e = hipMemsetAsync(q.i64, 0, q.num_slots * q.n_i64 * 8, s)) != hipSuccess) return e;
  if (q.n_f64 && (e = hipMemsetAsync(q.f64, 0, q.num_slots * q.n_f64 * 8, s)) != hipSuccess) return e;
  if (q.flag_bytes_per_slot && (e = hipMemsetAsync(q.flags, 0, q.num_slots * q.flag_bytes_per_slot, s)) != hipSuccess)
    return e;
  if ((e = hipMemsetAsync(q.seg_matched, 0, q.num_segments * 8ull, s)) != hipSuccess) return e;
  const uint64_t n = q.num_slots * (q.n_min > q.n_max ? q.n_min : q.n_max);
  if (n) {
    const uint32_t blocks = (uint32_t)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(init_minmax_kernel, dim3(blocks), dim3(256), 0, s, q.mn, q.num_slots * q.n_min, q.mx,
                       q.num_slots * q.n_max);
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
      for (int64_t d = s; d <= e; d++) out |= 1u << (uint32_t)(d - d0);
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
      if (x < num_docs) atomicOr(&bm[x >> 5], 1u << (x & 31u));
    }
  } else if (c.type == 1) {  // 1024 little-endian uint64 words
    const uint32_t* w32 = (const uint32_t*)p;
    for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x) {
      const uint32_t wi = (base >> 5) + i;
      const uint32_t v = w32[i];
      if (v && wi < nwords) atomicOr(&bm[wi], v);
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
        atomicOr(&bm[w], mask);
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

__global__ void bitmap_not_kernel(uint32_t* bm, uint32_t num_docs) {
  const uint32_t nwords = (num_docs + 31) / 32;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
    uint32_t v = ~bm[w];
    if (w == nwords - 1 && (num_docs & 31u)) v &= (1u << (num_docs & 31u)) - 1u;
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
      if (w < (num_docs + 31) / 32) bm[w] = (uint32_t)b;
      if (w + 1 < (num_docs + 31) / 32) bm[w + 1] = (uint32_t)(b >> 32);
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

__global__ void set_lut_bits_kernel(const int32_t* __restrict__ ids, uint32_t n, uint32_t* __restrict__ lut) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicOr(&lut[(uint32_t)ids[i] >> 5], 1u << ((uint32_t)ids[i] & 31u));
}

hipError_t launch_set_lut_bits(const int32_t* ids, uint32_t n, uint32_t* lut, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(set_lut_bits_kernel, dim3(blocks < 4096 ? blocks : 4096), dim3(256), 0, s, ids, n, lut);
  return hipGetLastError();
}

}  // namespace pg
