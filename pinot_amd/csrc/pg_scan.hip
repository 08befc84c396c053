// pg_scan.hip -- the fused hot loop of the segment query path (gfx950).
//
// scan_kernel replaces, per tile of 4096 docs, Pinot's per-segment operator chain
//   DocIdSetOperator (10 000-doc blocks, operator/DocIdSetOperator.java:58-83)
//   -> AndDocIdSet / OrDocIdSet / NotDocIdIterator (docidsets/AndDocIdSet.java:60-150, OrDocIdSet.java:58-114)
//      whose scan children only look at docs that survived the previous children
//      (SVScanDocIdIterator.applyAnd, dociditerators/SVScanDocIdIterator.java:106-125)
//   -> PredicateEvaluator.applySV on FixedBitSVForwardIndexReaderV2.readDictIds / FixedBitIntReader
//      (readers/forward/FixedBitSVForwardIndexReaderV2.java:62-97, io/reader/impl/FixedBitIntReader.java:52-118)
//   -> DataFetcher.readDoubleValues + Dictionary.readDoubleValues (common/DataFetcher.java:511-521) of the
//      matching docs only (projection)
//   -> Sum/Count/Min/Max/Avg/DistinctCount/CountMV aggregate / aggregateGroupBySV
//   -> DictionaryBasedGroupKeyGenerator mixed-radix keys (groupby/DictionaryBasedGroupKeyGenerator.java:280-322)
// with no intermediate doc-id lists.  Thread t of a block owns docs base + j*256 + t (j < 16), so for each j the
// 64 lanes of a wave read 64 consecutive packed values (one contiguous run of 8*b bytes).  Every leaf and every
// aggregation input is read only for the docs still needed (exec-masked loads), so a selective first leaf turns
// the remaining columns into cache-line gathers: the HBM bytes actually moved are those of the most selective
// leaf's column plus the lines that hold surviving docs.  Nothing here is a dense contraction: no MFMA; the
// roofline is HBM bandwidth.
#include <hip/hip_runtime.h>

#include "pg_internal.h"

namespace pg {

// FixedBitIntReader.readUnchecked on the native-word image: value `idx` of `b` (1..32) bits.
__device__ __forceinline__ uint32_t unpack(const uint32_t* __restrict__ w, uint32_t idx, uint32_t b) {
  const uint64_t p = (uint64_t)idx * b;
  const uint64_t wi = p >> 5;
  const uint32_t off = (uint32_t)p & 31u;
  const uint64_t win = ((uint64_t)w[wi] << 32) | (uint64_t)w[wi + 1];
  return (uint32_t)(win >> (64u - off - b)) & (0xFFFFFFFFu >> (32u - b));
}

// Dictionary reads clamp the dictId to the dictionary: valid data never needs it, and a corrupt forward index
// then yields wrong values (caught by parity checks) instead of an out-of-bounds access.
__device__ __forceinline__ double dict_double(const ColDesc& c, uint32_t id) {
  id = min(id, c.card - 1u);
  switch (c.dtype) {
    case PG_INT: return (double)((const int32_t*)c.dict)[id];
    case PG_LONG: return (double)((const int64_t*)c.dict)[id];
    case PG_FLOAT: return (double)((const float*)c.dict)[id];
    default: return ((const double*)c.dict)[id];
  }
}

__device__ __forceinline__ int64_t dict_i64(const ColDesc& c, uint32_t id) {
  id = min(id, c.card - 1u);
  return c.dtype == PG_INT ? (int64_t)((const int32_t*)c.dict)[id] : ((const int64_t*)c.dict)[id];
}

// TransformFunction value of an aggregation input (double path).
// MultiplicationTransformFunction.transformToDoubleValuesSV (transform/function/MultiplicationTransformFunction.java:91-111):
// start from the literal product 1.0, multiply arguments in order; compiled with -ffp-contract=off.
__device__ __forceinline__ double agg_value_f64(const AggSpec& a, const ColDesc* c, uint32_t d) {
  const double va = dict_double(c[0], unpack(c[0].words, d, c[0].bits));
  if (a.op == PG_EXPR_COL) return va;
  const double vb = dict_double(c[1], unpack(c[1].words, d, c[1].bits));
  switch (a.op) {
    case PG_EXPR_MUL: return (1.0 * va) * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// integer-exact path (host proved |partial sums| < 2^62): identical to the double path while < 2^53
__device__ __forceinline__ int64_t agg_value_i64(const AggSpec& a, const ColDesc* c, uint32_t d) {
  const int64_t va = dict_i64(c[0], unpack(c[0].words, d, c[0].bits));
  if (a.op == PG_EXPR_COL) return va;
  const int64_t vb = dict_i64(c[1], unpack(c[1].words, d, c[1].bits));
  switch (a.op) {
    case PG_EXPR_MUL: return va * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

__device__ __forceinline__ uint64_t col_key(uint32_t kind, int64_t base, const ColDesc& c, uint32_t d) {
  const uint32_t id = unpack(c.words, d, c.bits);
  if (id >= c.card) return ~0ull;  // corrupt input: rejected by the caller's range check
  return kind == PG_KEY_KEYMAP ? (uint64_t)(uint32_t)c.keymap[id] : (uint64_t)(dict_i64(c, id) - base);
}

// IN-list membership in an LDS open-addressing table (<= 50 % full, empty = -1).
__device__ __forceinline__ bool set_contains(const int32_t* tab, uint32_t log2, uint32_t id) {
  const uint32_t mask = (1u << log2) - 1u;
  uint32_t h = set_hash(id, log2);
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const int32_t v = tab[h];
    if (v == (int32_t)id) return true;
    if (v < 0) return false;
    h = (h + 1) & mask;
  }
  return false;
}

// One leaf over the thread's 16 docs, evaluated only for the docs in `need` -> 16-bit mask
// (bit j <-> doc base + j*256 + tid).  Bits outside `need` are don't-care.
__device__ __forceinline__ uint32_t eval_leaf(const LeafDesc& L, const int32_t* lds_sets, uint32_t need,
                                              uint32_t base, int tid) {
  uint32_t m = 0;
  switch (L.kind) {
    case LK_ALL: m = 0xFFFFu; break;
    case LK_NONE: break;
    case LK_RANGE: {
      const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        if ((need >> j) & 1u) {
          const uint32_t v = unpack(L.words, base + (uint32_t)(j * kBlock + tid), L.bits);
          m |= (uint32_t)((v - lo) < span) << j;
        }
      }
      break;
    }
    case LK_SET_LDS: {
      const int32_t* tab = lds_sets + L.lds_off;
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        if ((need >> j) & 1u) {
          const uint32_t v = unpack(L.words, base + (uint32_t)(j * kBlock + tid), L.bits);
          m |= (uint32_t)set_contains(tab, L.set_log2, v) << j;
        }
      }
      break;
    }
    case LK_SET_LUT: {
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        if ((need >> j) & 1u) {
          const uint32_t v = unpack(L.words, base + (uint32_t)(j * kBlock + tid), L.bits);
          m |= ((L.aux[v >> 5] >> (v & 31u)) & 1u) << j;
        }
      }
      break;
    }
    case LK_DOCBITMAP: {
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        if ((need >> j) & 1u) {
          const uint32_t d = base + (uint32_t)(j * kBlock + tid);
          m |= ((L.aux[d >> 5] >> (d & 31u)) & 1u) << j;
        }
      }
      break;
    }
    default: {  // LK_DOCRANGE
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        const uint32_t d = base + (uint32_t)(j * kBlock + tid);
        m |= (uint32_t)(d >= (uint32_t)L.lo && d < (uint32_t)L.hi) << j;
      }
      break;
    }
  }
  return L.excl ? (~m & 0xFFFFu) : m;
}

// Filter tree (prefix form) over 16-bit masks with short-circuit needs: an AND child only sees docs every
// earlier child accepted, an OR child only docs no earlier child accepted.  The group stack (<= 8 open groups)
// lives in registers: 16-bit acc / need fields packed into 64-bit words, 2-bit types in one word.
enum GroupType : uint32_t { GT_ROOT = 0, GT_AND = 1, GT_OR = 2, GT_NOT = 3 };

__device__ __forceinline__ uint32_t eval_filter(const QuerySpec& q, const LeafDesc* __restrict__ leaves,
                                                const int32_t* lds_sets, uint32_t valid, uint32_t base, int tid) {
  if (q.num_ops == 0) return valid;
  uint32_t gtype = GT_ROOT, gacc = 0, gneed = valid, need = valid;
  uint64_t sacc0 = 0, sacc1 = 0, sneed0 = 0, sneed1 = 0;
  uint32_t stype = 0;
  for (uint32_t i = 0; i < q.num_ops; i++) {
    const int32_t op = q.ops[i];
    if (op >= 0 || op == kOpEnd) {
      uint32_t r;
      if (op >= 0) {
        r = __ballot(need != 0) ? eval_leaf(leaves[op], lds_sets, need, base, tid) : 0u;
      } else {
        r = gtype == GT_NOT ? (~gacc & gneed) : gacc;
        gtype = stype & 3u;
        stype >>= 2;
        gacc = (uint32_t)(sacc0 & 0xFFFFu);
        sacc0 = (sacc0 >> 16) | (sacc1 << 48);
        sacc1 >>= 16;
        gneed = (uint32_t)(sneed0 & 0xFFFFu);
        sneed0 = (sneed0 >> 16) | (sneed1 << 48);
        sneed1 >>= 16;
      }
      switch (gtype) {
        case GT_AND: gacc &= r; need = gneed & gacc; break;
        case GT_OR: gacc |= r; need = gneed & ~gacc; break;
        case GT_NOT: gacc = r; need = 0; break;
        default: gacc = r; need = 0; break;
      }
    } else {  // open a group: its children see the docs currently needed
      stype = (stype << 2) | gtype;
      sacc1 = (sacc1 << 16) | (sacc0 >> 48);
      sacc0 = (sacc0 << 16) | gacc;
      sneed1 = (sneed1 << 16) | (sneed0 >> 48);
      sneed0 = (sneed0 << 16) | gneed;
      gneed = need;
      gtype = op == kOpAnd ? GT_AND : (op == kOpOr ? GT_OR : GT_NOT);
      gacc = gtype == GT_AND ? 0xFFFFu : 0u;
    }
  }
  return gacc & valid;
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

__global__ __launch_bounds__(kBlock) void scan_kernel(QuerySpec q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* lds_sets = (int32_t*)smem;
  unsigned char* lds_groups = smem + (uint64_t)q.set_lds_ints * 4;
  const int tid = threadIdx.x;
  const bool grouped = q.num_keys > 0;

  // LDS-privatised group table: [G][n_i64] u64 | [G][n_f64] f64 | [G][n_min] i64 | [G][n_max] i64
  unsigned long long* l_i64 = (unsigned long long*)lds_groups;
  double* l_f64 = (double*)(l_i64 + q.num_slots * q.n_i64);
  long long* l_mn = (long long*)(l_f64 + q.num_slots * q.n_f64);
  long long* l_mx = l_mn + q.num_slots * q.n_min;
  if (grouped && q.use_lds) {
    for (uint64_t i = tid; i < q.num_slots * q.n_i64; i += kBlock) l_i64[i] = 0;
    for (uint64_t i = tid; i < q.num_slots * q.n_f64; i += kBlock) l_f64[i] = 0.0;
    for (uint64_t i = tid; i < q.num_slots * q.n_min; i += kBlock) l_mn[i] = order_key(__builtin_inf());
    for (uint64_t i = tid; i < q.num_slots * q.n_max; i += kBlock) l_mx[i] = order_key(-__builtin_inf());
  }
  unsigned long long* gi = q.use_lds ? l_i64 : q.i64;
  double* gf = q.use_lds ? l_f64 : q.f64;
  long long* gmn = q.use_lds ? l_mn : q.mn;
  long long* gmx = q.use_lds ? l_mx : q.mx;

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

  // contiguous item range of this block (consecutive items share a segment -> few LDS set reloads)
  const uint32_t i0 = (uint32_t)((uint64_t)blockIdx.x * q.num_items / gridDim.x);
  const uint32_t i1 = (uint32_t)(((uint64_t)blockIdx.x + 1) * q.num_items / gridDim.x);
  uint32_t cur_seg = 0xFFFFFFFFu;
  for (uint32_t item = i0; item < i1; item++) {
    const WorkItem it = q.items[item];
    const SegDesc sd = q.segs[it.seg];
    if (it.seg != cur_seg) {
      if (q.set_lds_ints) {  // stage this segment's IN-list hash sets
        __syncthreads();
        for (uint32_t l = 0; l < q.num_leaves; l++) {
          const LeafDesc L = sd.leaves[l];
          if (L.kind != LK_SET_LDS) continue;
          const uint32_t n = 1u << L.set_log2;
          for (uint32_t k = tid; k < n; k += kBlock) lds_sets[L.lds_off + k] = ((const int32_t*)L.aux)[k];
        }
      }
      __syncthreads();
      cur_seg = it.seg;
    }
    const uint32_t nd = sd.num_docs;
    uint64_t seg_count = 0;
    for (uint32_t tile = it.tile_begin; tile < it.tile_end; tile++) {
      const uint32_t base = tile * (uint32_t)kTileDocs;
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < kRows; j++) valid |= (uint32_t)(base + (uint32_t)(j * kBlock + tid) < nd) << j;
      uint32_t m = eval_filter(q, sd.leaves, lds_sets, valid, base, tid);
      const uint32_t nm = __popc(m);
      seg_count += nm;
      if (__ballot(m != 0) == 0) continue;

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
            const ColDesc* c = sd.aggcols + 2 * a;
            switch (A.fn) {
              case PG_AGG_COUNT: break;  // = doc_count
              case PG_AGG_COUNTMV: acc[a] += c[0].mv_offsets[d + 1] - c[0].mv_offsets[d]; break;
              case PG_AGG_SUM:
              case PG_AGG_AVG:
                if (A.integer) acc[a] += (uint64_t)agg_value_i64(A, c, d);
                else acc[a] = __double_as_longlong(__longlong_as_double(acc[a]) + agg_value_f64(A, c, d));
                break;  // AVG count == doc_count
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
                if (key < A.key_card) q.flags[A.flag_off + key] = 1;
                else atomicOr(q.err, 2u);
                break;
              }
            }
          }
        }
      } else {
        while (m) {
          const int j = __ffs(m) - 1;
          m &= m - 1;
          const uint32_t d = base + (uint32_t)(j * kBlock + tid);
          uint64_t g = 0;
          bool in_range = true;
#pragma unroll
          for (int k = 0; k < kMaxKeys; k++) {
            if (k >= (int)q.num_keys) break;
            const uint64_t kid = col_key(q.key_kind[k], q.key_base[k], sd.keycols[k], d);
            in_range &= kid < q.key_card[k];
            g += kid * q.key_stride[k];
          }
          if (!in_range) {  // never expected (host proved the key ranges): refuse rather than write out of bounds
            atomicOr(q.err, 1u);
            continue;
          }
          atomicAdd(&gi[g * q.n_i64], 1ull);  // slot 0: doc count / presence
#pragma unroll
          for (int a = 0; a < kMaxAggs; a++) {
            if (a >= (int)q.num_aggs) break;
            const AggSpec& A = q.aggs[a];
            const ColDesc* c = sd.aggcols + 2 * a;
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
                if (key < A.key_card) q.flags[g * q.flag_bytes_per_slot + A.flag_off + key] = 1;
                else atomicOr(q.err, 2u);
                break;
              }
            }
          }
        }
      }
    }
    const uint64_t c = wave_sum_u64(seg_count);
    if ((tid & 63) == 0 && c) atomicAdd(&q.seg_matched[it.seg], (unsigned long long)c);
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
  size_t lds = (size_t)q.set_lds_ints * 4;
  if (q.num_keys && q.use_lds) lds += q.num_slots * 8ull * (q.n_i64 + q.n_f64 + q.n_min + q.n_max);
  hipLaunchKernelGGL(scan_kernel, dim3(blocks), dim3(kBlock), lds, s, q);
  return hipGetLastError();
}

}  // namespace pg
