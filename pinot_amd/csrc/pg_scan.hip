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
// with no intermediate doc-id lists.  Thread t of a block owns docs base + j*256 + t (j < 8), so for each j the
// 64 lanes of a wave read 64 consecutive packed values (one contiguous run of 8*b bytes).
//
// Memory-level parallelism: every gather of packed values is straight-line code -- docs a phase does not need
// read the tile's first doc instead (one cache line for the whole wave) -- so all 2 x 8 window loads of a leaf
// are in flight before the first is consumed.  Leaves after the first of an AND only need the docs that
// survived, so after a selective first leaf the other columns move as a few cache lines, not as streams.
// Packed columns are read through buffer descriptors: 32-bit offsets, and the hardware range check turns any
// read past the column into 0 instead of a fault.  Nothing here is a dense contraction: no MFMA; the roofline
// is HBM bandwidth.
#include <hip/hip_runtime.h>

#include "pg_internal.h"

namespace pg {
constexpr uint32_t kRowMask = (1u << kRows) - 1u;

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// Buffer descriptor of a packed column; built from readfirstlane'd (wave-uniform) values so it lives in SGPRs.
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// FixedBitIntReader.readUnchecked on the native-word image: value `idx` of `b` (1..32) bits.
__device__ __forceinline__ uint32_t unpack(rsrc_t r, uint32_t idx, uint32_t b) {
  const uint64_t p = (uint64_t)idx * b;
  const uint32_t off = (uint32_t)(p >> 5) << 2;
  const uint32_t sh = (uint32_t)p & 31u;
  const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0);
  const uint64_t win = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)(win >> (64u - sh - b)) & (0xFFFFFFFFu >> (32u - b));
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

// TransformFunction value of an aggregation input from its (already unpacked) dictIds.
// MultiplicationTransformFunction.transformToDoubleValuesSV (transform/function/MultiplicationTransformFunction.java:91-111):
// start from the literal product 1.0, multiply arguments in order; compiled with -ffp-contract=off.
__device__ __forceinline__ double value_f64(const AggSpec& a, const ColDesc* c, uint32_t ia, uint32_t ib) {
  const double va = dict_double(c[0], ia);
  if (a.op == PG_EXPR_COL) return va;
  const double vb = dict_double(c[1], ib);
  switch (a.op) {
    case PG_EXPR_MUL: return (1.0 * va) * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// integer-exact path (host proved |partial sums| < 2^62): identical to the double path while < 2^53
__device__ __forceinline__ int64_t value_i64(const AggSpec& a, const ColDesc* c, uint32_t ia, uint32_t ib) {
  const int64_t va = dict_i64(c[0], ia);
  if (a.op == PG_EXPR_COL) return va;
  const int64_t vb = dict_i64(c[1], ib);
  switch (a.op) {
    case PG_EXPR_MUL: return va * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// table-global key id of dictId `id` (~0 when the id is outside the dictionary: rejected by the caller)
__device__ __forceinline__ uint64_t key_of(uint32_t kind, int64_t base, const ColDesc& c, uint32_t id) {
  if (id >= c.card) return ~0ull;
  return kind == PG_KEY_KEYMAP ? (uint64_t)(uint32_t)c.keymap[id] : (uint64_t)(dict_i64(c, id) - base);
}

__device__ __forceinline__ uint32_t agg_ncols(const AggSpec& A) {
  if (A.fn == PG_AGG_COUNT || A.fn == PG_AGG_COUNTMV) return 0;
  if (A.fn == PG_AGG_DISTINCTCOUNT) return 1;
  return A.op == PG_EXPR_COL ? 1u : 2u;
}

// IN-list membership in an LDS open-addressing table (<= 50 % full, empty = -1), given the home-slot entry `t0`
// already read (the batched first probe).
__device__ __forceinline__ bool set_resolve(const int32_t* tab, uint32_t log2, uint32_t id, int32_t t0) {
  if (t0 == (int32_t)id) return true;
  if (t0 < 0) return false;
  const uint32_t mask = (1u << log2) - 1u;
  uint32_t h = (set_hash(id, log2) + 1) & mask;
  for (uint32_t probe = 1; probe <= mask; probe++) {
    const int32_t v = tab[h];
    if (v == (int32_t)id) return true;
    if (v < 0) return false;
    h = (h + 1) & mask;
  }
  return false;
}

// Gather the dictIds of rows [0, N) of `need` starting at `base` (row r = doc base + r*256 + tid); rows outside
// `need` read the doc `base` instead, keeping the loads straight-line.
template <int N>
__device__ __forceinline__ void gather_ids(rsrc_t r, uint32_t bits, uint32_t need, uint32_t base, int tid,
                                           uint32_t (&v)[N]) {
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint32_t d = ((need >> j) & 1u) ? base + (uint32_t)(j * kBlock + tid) : base;
    v[j] = unpack(r, d, bits);
  }
}

// One leaf over the thread's 8 docs, evaluated only for the docs in `need` -> 16-bit mask
// (bit j <-> doc base + j*256 + tid).  Bits outside `need` are don't-care.
__device__ __forceinline__ uint32_t eval_leaf(const LeafDesc& L, const int32_t* lds_sets, uint32_t need,
                                              uint32_t base, int tid) {
  uint32_t m = 0;
  switch (L.kind) {
    case LK_ALL: m = kRowMask; break;
    case LK_NONE: break;
    case LK_RANGE: {
      const rsrc_t r = make_rsrc(L.words, L.wbytes);
      uint32_t v[kRows];
      gather_ids<kRows>(r, L.bits, need, base, tid, v);
      const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll
      for (int j = 0; j < kRows; j++) m |= (uint32_t)((v[j] - lo) < span) << j;
      break;
    }
    case LK_SET_LDS: {
      const rsrc_t r = make_rsrc(L.words, L.wbytes);
      uint32_t v[kRows];
      gather_ids<kRows>(r, L.bits, need, base, tid, v);
      const int32_t* tab = lds_sets + L.lds_off;
      int32_t t0[kRows];
#pragma unroll
      for (int j = 0; j < kRows; j++) t0[j] = tab[set_hash(v[j], L.set_log2)];
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        const bool hit = t0[j] == (int32_t)v[j];
        const bool decided = hit || t0[j] < 0;
        m |= (uint32_t)(decided ? hit : set_resolve(tab, L.set_log2, v[j], t0[j])) << j;
      }
      break;
    }
    case LK_SET_LUT: {
      const rsrc_t r = make_rsrc(L.words, L.wbytes);
      uint32_t v[kRows];
      gather_ids<kRows>(r, L.bits, need, base, tid, v);
      uint32_t lw[kRows];
#pragma unroll
      for (int j = 0; j < kRows; j++) lw[j] = L.aux[v[j] >> 5];
#pragma unroll
      for (int j = 0; j < kRows; j++) m |= ((lw[j] >> (v[j] & 31u)) & 1u) << j;
      break;
    }
    case LK_DOCBITMAP: {
      uint32_t bw[kRows];
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        const uint32_t d = ((need >> j) & 1u) ? base + (uint32_t)(j * kBlock + tid) : base;
        bw[j] = L.aux[d >> 5] >> (d & 31u);
      }
#pragma unroll
      for (int j = 0; j < kRows; j++) m |= (bw[j] & 1u) << j;
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
  return L.excl ? (~m & kRowMask) : m;
}

// Filter tree (prefix form) over 8-bit masks with short-circuit needs: an AND child only sees docs every
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
        gacc = (uint32_t)(sacc0 & kRowMask);
        sacc0 = (sacc0 >> 16) | (sacc1 << 48);
        sacc1 >>= 16;
        gneed = (uint32_t)(sneed0 & kRowMask);
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
      gacc = gtype == GT_AND ? kRowMask : 0u;
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

// Group-state pointers: the block's LDS copy when the table is privatised, else the global arrays.
struct GroupState {
  unsigned long long* i64;
  double* f64;
  long long* mn;
  long long* mx;
};

// Per-doc update of one aggregation in group slot g (aggregateGroupBySV of each function).
__device__ __forceinline__ void group_update(const QuerySpec& q, const GroupState& S, const AggSpec& A,
                                             const ColDesc* c, uint64_t g, uint32_t d, uint32_t ia, uint32_t ib) {
  switch (A.fn) {
    case PG_AGG_COUNT: break;  // = slot 0
    case PG_AGG_COUNTMV:
      atomicAdd(&S.i64[g * q.n_i64 + A.slot], (unsigned long long)(c[0].mv_offsets[d + 1] - c[0].mv_offsets[d]));
      break;
    case PG_AGG_SUM:
    case PG_AGG_AVG:  // AVG count == slot 0
      if (A.integer) atomicAdd(&S.i64[g * q.n_i64 + A.slot], (unsigned long long)value_i64(A, c, ia, ib));
      else atomicAdd(&S.f64[g * q.n_f64 + A.slot], value_f64(A, c, ia, ib));
      break;
    case PG_AGG_MIN: atomicMin(&S.mn[g * q.n_min + A.slot], (long long)order_key(value_f64(A, c, ia, ib))); break;
    case PG_AGG_MAX: atomicMax(&S.mx[g * q.n_max + A.slot], (long long)order_key(value_f64(A, c, ia, ib))); break;
    case PG_AGG_DISTINCTCOUNT: {
      const uint64_t key = key_of(A.key_kind, A.key_base, c[0], ia);
      if (key < A.key_card) q.flags[g * q.flag_bytes_per_slot + A.flag_off + key] = 1;
      else atomicOr(q.err, 2u);
      break;
    }
  }
}

// Per-doc update of one aggregation-only accumulator (aggregate() of each function; COUNT = doc count).
__device__ __forceinline__ void acc_update(const QuerySpec& q, const AggSpec& A, const ColDesc* c, uint64_t& acc,
                                           uint32_t d, uint32_t ia, uint32_t ib) {
  switch (A.fn) {
    case PG_AGG_COUNT: break;
    case PG_AGG_COUNTMV: acc += c[0].mv_offsets[d + 1] - c[0].mv_offsets[d]; break;
    case PG_AGG_SUM:
    case PG_AGG_AVG:
      if (A.integer) acc += (uint64_t)value_i64(A, c, ia, ib);
      else acc = __double_as_longlong(__longlong_as_double(acc) + value_f64(A, c, ia, ib));
      break;
    case PG_AGG_MIN: {
      const int64_t k = order_key(value_f64(A, c, ia, ib));
      if (k < (int64_t)acc) acc = (uint64_t)k;
      break;
    }
    case PG_AGG_MAX: {
      const int64_t k = order_key(value_f64(A, c, ia, ib));
      if (k > (int64_t)acc) acc = (uint64_t)k;
      break;
    }
    case PG_AGG_DISTINCTCOUNT: {
      const uint64_t key = key_of(A.key_kind, A.key_base, c[0], ia);
      if (key < A.key_card) q.flags[A.flag_off + key] = 1;
      else atomicOr(q.err, 2u);
      break;
    }
  }
}

constexpr int kHalf = kRows / 2;  // rows per batch of the dense aggregation path (bounds live registers)

// Dense tiles (many matches): half a tile of rows at a time, every gather straight-line.
template <bool GROUPED, int MAXA>
__device__ __forceinline__ void aggregate_dense(const QuerySpec& q, const SegDesc& sd, const GroupState& S,
                                                uint64_t (&acc)[MAXA], uint32_t m, uint32_t base, int tid) {
#pragma unroll
  for (int h = 0; h < kRows / kHalf; h++) {
    const uint32_t mh = (m >> (h * kHalf)) & ((1u << kHalf) - 1u);
    if (__ballot(mh != 0) == 0) continue;
    const uint32_t hb = base + (uint32_t)(h * kHalf * kBlock);
    uint32_t g[kHalf];  // slot index (< num_slots <= 2^31)
    uint32_t live = mh;
#pragma unroll
    for (int r = 0; r < kHalf; r++) g[r] = 0;
    if constexpr (GROUPED) {
      for (uint32_t k = 0; k < q.num_keys; k++) {
        const ColDesc& kc = sd.keycols[k];
        uint32_t ids[kHalf];
        gather_ids<kHalf>(make_rsrc(kc.words, kc.wbytes), kc.bits, mh, hb, tid, ids);
        uint64_t kid[kHalf];
#pragma unroll
        for (int r = 0; r < kHalf; r++) kid[r] = key_of(q.key_kind[k], q.key_base[k], kc, ids[r]);
#pragma unroll
        for (int r = 0; r < kHalf; r++) {
          if (kid[r] >= q.key_card[k]) live &= ~(1u << r);
          else g[r] += (uint32_t)kid[r] * (uint32_t)q.key_stride[k];
        }
      }
      if (live != mh) atomicOr(q.err, 1u);  // never expected: the host proved the key ranges
#pragma unroll
      for (int r = 0; r < kHalf; r++)
        if ((live >> r) & 1u) atomicAdd(&S.i64[(uint64_t)g[r] * q.n_i64], 1ull);  // slot 0: doc count / presence
    }
    for (uint32_t a = 0; a < q.num_aggs; a++) {
      const AggSpec& A = q.aggs[a];
      if (A.fn == PG_AGG_COUNT) continue;
      const ColDesc* c = sd.aggcols + 2 * a;
      const uint32_t nc = agg_ncols(A);
      uint32_t ia[kHalf], ib[kHalf];
#pragma unroll
      for (int r = 0; r < kHalf; r++) ia[r] = ib[r] = 0;
      if (nc >= 1) gather_ids<kHalf>(make_rsrc(c[0].words, c[0].wbytes), c[0].bits, mh, hb, tid, ia);
      if (nc >= 2) gather_ids<kHalf>(make_rsrc(c[1].words, c[1].wbytes), c[1].bits, mh, hb, tid, ib);
#pragma unroll
      for (int r = 0; r < kHalf; r++) {
        if (!((live >> r) & 1u)) continue;
        const uint32_t d = hb + (uint32_t)(r * kBlock + tid);
        if constexpr (GROUPED) {
          group_update(q, S, A, c, g[r], d, ia[r], ib[r]);
        } else {
#pragma unroll
          for (int x = 0; x < MAXA; x++)
            if ((uint32_t)x == a) acc_update(q, A, c, acc[x], d, ia[r], ib[r]);
        }
      }
    }
  }
}

// Sparse tiles (few matches): one matched doc per lane per round; the round's dictId loads for every key and
// aggregation input are issued before any is consumed.
template <bool GROUPED, int MAXA, int MAXK>
__device__ __forceinline__ void aggregate_sparse(const QuerySpec& q, const SegDesc& sd, const GroupState& S,
                                                 uint64_t (&acc)[MAXA], uint32_t m, uint32_t base, int tid) {
  while (__ballot(m != 0)) {
    const bool act = m != 0;
    const int j = act ? __ffs(m) - 1 : 0;
    m &= m - 1;
    const uint32_t d = act ? base + (uint32_t)(j * kBlock + tid) : base;
    uint32_t kidx[MAXK > 0 ? MAXK : 1], ia[MAXA], ib[MAXA];
#pragma unroll
    for (int k = 0; k < MAXK; k++) {
      kidx[k] = 0;
      if (GROUPED && k < (int)q.num_keys)
        kidx[k] = unpack(make_rsrc(sd.keycols[k].words, sd.keycols[k].wbytes), d, sd.keycols[k].bits);
    }
#pragma unroll
    for (int a = 0; a < MAXA; a++) {
      ia[a] = ib[a] = 0;
      if (a >= (int)q.num_aggs) continue;
      const uint32_t nc = agg_ncols(q.aggs[a]);
      const ColDesc* c = sd.aggcols + 2 * a;
      if (nc >= 1) ia[a] = unpack(make_rsrc(c[0].words, c[0].wbytes), d, c[0].bits);
      if (nc >= 2) ib[a] = unpack(make_rsrc(c[1].words, c[1].wbytes), d, c[1].bits);
    }
    if (!act) continue;
    if constexpr (GROUPED) {
      uint64_t g = 0;
      bool in_range = true;
#pragma unroll
      for (int k = 0; k < MAXK; k++) {
        if (k >= (int)q.num_keys) break;
        const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], sd.keycols[k], kidx[k]);
        in_range &= kid < q.key_card[k];
        g += kid * q.key_stride[k];
      }
      if (!in_range) {  // never expected: the host proved the key ranges; refuse rather than write out of bounds
        atomicOr(q.err, 1u);
        continue;
      }
      atomicAdd(&S.i64[g * q.n_i64], 1ull);
#pragma unroll
      for (int a = 0; a < MAXA; a++) {
        if (a >= (int)q.num_aggs) break;
        group_update(q, S, q.aggs[a], sd.aggcols + 2 * a, g, d, ia[a], ib[a]);
      }
    } else {
#pragma unroll
      for (int a = 0; a < MAXA; a++) {
        if (a >= (int)q.num_aggs) break;
        acc_update(q, q.aggs[a], sd.aggcols + 2 * a, acc[a], d, ia[a], ib[a]);
      }
    }
  }
}

// MAXA / MAXK: compile-time bounds on the aggregations / group keys of the query (the smallest instantiation
// that fits is launched), so registers are sized for the query shape, not for the ABI maximum.
template <bool GROUPED, int MAXA, int MAXK>
__global__ __launch_bounds__(kBlock) void scan_kernel(QuerySpec q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int32_t* lds_sets = (int32_t*)smem;
  unsigned char* lds_groups = smem + (uint64_t)q.set_lds_ints * 4;
  const int tid = threadIdx.x;

  // LDS-privatised group table: [G][n_i64] u64 | [G][n_f64] f64 | [G][n_min] i64 | [G][n_max] i64
  unsigned long long* l_i64 = (unsigned long long*)lds_groups;
  double* l_f64 = (double*)(l_i64 + q.num_slots * q.n_i64);
  long long* l_mn = (long long*)(l_f64 + q.num_slots * q.n_f64);
  long long* l_mx = l_mn + q.num_slots * q.n_min;
  if (GROUPED && q.use_lds) {
    for (uint64_t i = tid; i < q.num_slots * q.n_i64; i += kBlock) l_i64[i] = 0;
    for (uint64_t i = tid; i < q.num_slots * q.n_f64; i += kBlock) l_f64[i] = 0.0;
    for (uint64_t i = tid; i < q.num_slots * q.n_min; i += kBlock) l_mn[i] = order_key(__builtin_inf());
    for (uint64_t i = tid; i < q.num_slots * q.n_max; i += kBlock) l_mx[i] = order_key(-__builtin_inf());
  }
  const GroupState S = q.use_lds ? GroupState{l_i64, l_f64, l_mn, l_mx} : GroupState{q.i64, q.f64, q.mn, q.mx};

  // aggregation-only accumulators (registers; indices compile-time via unrolled agg loops)
  uint64_t acc[MAXA];
#pragma unroll
  for (int a = 0; a < MAXA; a++) {
    acc[a] = 0;
    if (!GROUPED && a < (int)q.num_aggs) {
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
      const uint32_t m = eval_filter(q, sd.leaves, lds_sets, valid, base, tid);
      const uint32_t nm = __popc(m);
      seg_count += nm;
      if (!GROUPED) doc_count += nm;
      const uint64_t lanes = __ballot(m != 0);
      if (lanes == 0) continue;
      if (!GROUPED && q.num_aggs == 0) continue;
      // dense when more than a quarter of the wave's lanes hold matches
      if (__popcll(lanes) > 16) aggregate_dense<GROUPED, MAXA>(q, sd, S, acc, m, base, tid);
      else aggregate_sparse<GROUPED, MAXA, MAXK>(q, sd, S, acc, m, base, tid);
    }
    const uint64_t c = wave_sum_u64(seg_count);
    if ((tid & 63) == 0 && c) atomicAdd(&q.seg_matched[it.seg], (unsigned long long)c);
  }

  if (!GROUPED) {
    // wave-reduce then one global atomic per wave per slot
    const uint64_t dc = wave_sum_u64(doc_count);
    const bool lead = (tid & 63) == 0;
    if (lead && dc) atomicAdd(&q.i64[0], (unsigned long long)dc);
#pragma unroll
    for (int a = 0; a < MAXA; a++) {
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

template <bool G, int A, int K>
static void launch_one(const QuerySpec& q, uint32_t blocks, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((scan_kernel<G, A, K>), dim3(blocks), dim3(kBlock), lds, s, q);
}

hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s) {
  size_t lds = (size_t)q.set_lds_ints * 4;
  if (q.num_keys && q.use_lds) lds += q.num_slots * 8ull * (q.n_i64 + q.n_f64 + q.n_min + q.n_max);
  const uint32_t na = q.num_aggs;
  if (q.num_keys == 0) {
    if (na <= 2) launch_one<false, 2, 0>(q, blocks, lds, s);
    else if (na <= 4) launch_one<false, 4, 0>(q, blocks, lds, s);
    else launch_one<false, kMaxAggs, 0>(q, blocks, lds, s);
  } else if (q.num_keys == 1) {
    if (na <= 2) launch_one<true, 2, 1>(q, blocks, lds, s);
    else if (na <= 4) launch_one<true, 4, 1>(q, blocks, lds, s);
    else launch_one<true, kMaxAggs, 1>(q, blocks, lds, s);
  } else {
    if (na <= 2) launch_one<true, 2, kMaxKeys>(q, blocks, lds, s);
    else if (na <= 4) launch_one<true, 4, kMaxKeys>(q, blocks, lds, s);
    else launch_one<true, kMaxAggs, kMaxKeys>(q, blocks, lds, s);
  }
  return hipGetLastError();
}

}  // namespace pg
