// pg_scan.hip -- the fused hot loop of the segment query path (gfx950).
//
// scan_kernel replaces, per tile of 8192 docs, Pinot's per-segment operator chain
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
// with no intermediate doc-id lists.  Thread t of a block owns docs base + j*256 + t (j < 32): per-thread doc sets
// are 32-bit masks.
//
// Two ways to read a packed column, chosen per column by the host from the expected fraction of docs the query
// needs from it:
//   * staged  -- the tile's whole word range (8192*b bits) moves HBM -> registers -> LDS with coalesced 16-byte
//                loads (every byte fetched is used), then each doc's value is unpacked from LDS.  Used for the
//                driving filter leaf and any column most of whose cache lines are needed anyway.
//   * gathered -- per needed doc, a 2-word window read through a buffer descriptor (32-bit offsets; the hardware
//                range check turns a read past the column into 0, never a fault), issued in straight-line rounds
//                of up to 4 docs per lane so the loads of a round are in flight together.  Used for leaves after
//                a selective one, and for aggregation inputs of few matching docs.
// Doc bitmaps (sorted ranges, roaring, MV pre-pass) are 1-bit packed columns and go through the same two paths.
// Nothing here is a dense contraction: no MFMA; the roofline is HBM bandwidth.
#include <hip/hip_runtime.h>

#include "pg_internal.h"

namespace pg {

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kRowMask = 0xFFFFFFFFu;                     // kRows == 32
constexpr int kStageJobs = kLdsStageBytes / (16 * kBlock);      // 16-byte staging loads per thread per tile
static_assert(kRows == 32, "masks are 32-bit");

// Buffer descriptor of a packed column; built from readfirstlane'd (wave-uniform) values so it lives in SGPRs.
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ uint32_t bits_mask(uint32_t b) { return 0xFFFFFFFFu >> (32u - b); }

// FixedBitIntReader.readUnchecked on the native-word image: value `idx` of `b` (1..32) bits.
__device__ __forceinline__ uint32_t unpack(rsrc_t r, uint32_t idx, uint32_t b) {
  const uint64_t p = (uint64_t)idx * b;
  const uint32_t off = (uint32_t)(p >> 5) << 2;
  const uint32_t sh = (uint32_t)p & 31u;
  const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0);
  const uint64_t win = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)(win >> (64u - sh - b)) & bits_mask(b);
}

// The same from a staged tile in LDS: `rel` = doc - tile base.
__device__ __forceinline__ uint32_t unpack_lds(const uint32_t* st, uint32_t rel, uint32_t b) {
  const uint32_t p = rel * b;
  const uint32_t w = p >> 5, sh = p & 31u;
  const uint64_t win = ((uint64_t)st[w] << 32) | (uint64_t)st[w + 1];
  return (uint32_t)(win >> (64u - sh - b)) & bits_mask(b);
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

// IN-list membership in the exact LDS open-addressing table (<= 50 % full, empty = -1).
__device__ __forceinline__ bool set_contains(const int32_t* tab, uint32_t log2, uint32_t id) {
  const uint32_t mask = (1u << log2) - 1u;
  uint32_t h = set_hash(id, log2);
  int32_t v = tab[h];
  for (uint32_t probe = 0; probe <= mask; probe++) {
    if (v == (int32_t)id) return true;
    if (v < 0) return false;
    h = (h + 1) & mask;
    v = tab[h];
  }
  return false;
}

// IN-set filter bitmap test (exact when shift == 0, else a candidate test resolved by set_contains).
__device__ __forceinline__ uint32_t set_bit(const uint32_t* bm, uint32_t shift, uint32_t v) {
  const uint32_t x = v >> shift;
  return (bm[x >> 5] >> (x & 31u)) & 1u;
}

// Leaf predicate on a dictId (doc bitmaps: RANGE [1,2) on a 1-bit column).
__device__ __forceinline__ bool leaf_pred(const LeafDesc& L, const int32_t* lds_sets, uint32_t v) {
  switch (L.kind) {
    case LK_RANGE: return (v - (uint32_t)L.lo) < (uint32_t)(L.hi - L.lo);
    case LK_SET_LDS: {
      const uint32_t* bm = (const uint32_t*)(lds_sets + L.lds_off);
      if (!set_bit(bm, L.shift, v)) return false;
      return L.shift == 0 || set_contains((const int32_t*)bm + L.nbw, L.set_log2, v);
    }
    default: return (L.aux[v >> 5] >> (v & 31u)) & 1u;  // LK_SET_LUT
  }
}

// Per-tile staging of the packed columns the host chose (QuerySpec::staged): coalesced 16-byte loads of each
// column's word range for the tile into registers, then into LDS.  Slot geometry of the current segment.
struct StageSrc {
  const uint32_t* words[kMaxStaged];
  uint32_t nwords[kMaxStaged];     // words in the column (loads past it read zeros)
  uint32_t bits[kMaxStaged];
};

__device__ __forceinline__ void stage_tile(const QuerySpec& q, const StageSrc& src, uint32_t tile, uint32_t* lds,
                                           int tid) {  // `src` lives in LDS (keeps SGPRs free)
  uint4 buf[kStageJobs];
  uint32_t dst[kStageJobs];  // LDS word offset of each 16-byte job (~0: none)
#pragma unroll
  for (int k = 0; k < kStageJobs; k++) {
    buf[k] = make_uint4(0, 0, 0, 0);
    dst[k] = 0xFFFFFFFFu;
    const uint32_t qi = (uint32_t)(tid + k * kBlock);  // quad index within the concatenated slot tiles
    uint32_t q0 = 0;
#pragma unroll
    for (int s = 0; s < kMaxStaged; s++) {
      if (s < (int)q.num_staged) {
        const uint32_t nq = (uint32_t)(kTileDocs / 128) * src.bits[s] + 1;  // 16-byte quads of this slot's tile
        if (qi >= q0 && qi < q0 + nq) {
          const uint32_t local = qi - q0;
          dst[k] = q.staged[s].lds_word_off + local * 4;
          const uint32_t w = tile * (uint32_t)(kTileDocs / 32) * src.bits[s] + local * 4;
          if (src.words[s] && w < src.nwords[s]) {
            if (w + 4 <= src.nwords[s]) {
              buf[k] = *(const uint4*)(src.words[s] + w);
            } else {
              uint32_t t[4] = {0, 0, 0, 0};
              for (uint32_t x = 0; x < 4 && w + x < src.nwords[s]; x++) t[x] = src.words[s][w + x];
              buf[k] = make_uint4(t[0], t[1], t[2], t[3]);
            }
          }
        }
        q0 += nq;
      }
    }
  }
  __syncthreads();  // every wave is done reading the previous tile's staged words
#pragma unroll
  for (int k = 0; k < kStageJobs; k++)
    if (dst[k] != 0xFFFFFFFFu) *(uint4*)(lds + dst[k]) = buf[k];
  __syncthreads();
}

// One leaf over the thread's 32 docs, evaluated for the docs in `need` -> 32-bit mask (bit j <-> doc
// base + j*256 + tid).  Bits outside `need` are don't-care.
__device__ __forceinline__ uint32_t eval_leaf(const QuerySpec& q, uint32_t li, const LeafDesc& L,
                                              const int32_t* lds_sets, const uint32_t* stage, uint32_t need,
                                              uint32_t base, int tid) {
  uint32_t m = 0;
  switch (L.kind) {
    case LK_ALL: m = kRowMask; break;
    case LK_NONE: break;
    case LK_DOCRANGE: {
#pragma unroll
      for (int j = 0; j < kRows; j++) {
        const uint32_t d = base + (uint32_t)(j * kBlock + tid);
        m |= (uint32_t)(d >= (uint32_t)L.lo && d < (uint32_t)L.hi) << j;
      }
      break;
    }
    default: {  // packed column: RANGE / SET_LDS / SET_LUT
      const uint32_t slot = q.leaf_slot[li];
      if (slot != kNoSlot) {
        const uint32_t* st = stage + q.staged[slot].lds_word_off;
        const uint32_t b = L.bits;
        if (L.kind == LK_RANGE) {
          const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll 8
          for (int j = 0; j < kRows; j++)
            m |= (uint32_t)((unpack_lds(st, (uint32_t)(j * kBlock + tid), b) - lo) < span) << j;
        } else if (L.kind == LK_SET_LDS) {
          const uint32_t* bm = (const uint32_t*)(lds_sets + L.lds_off);
          const uint32_t shift = L.shift;
#pragma unroll 8
          for (int j = 0; j < kRows; j++) m |= set_bit(bm, shift, unpack_lds(st, (uint32_t)(j * kBlock + tid), b)) << j;
          if (shift) {  // resolve the (few) bitmap candidates exactly
            uint32_t cand = m & need;
            m = 0;
            while (cand) {
              const uint32_t j = (uint32_t)__ffs(cand) - 1u;
              cand &= cand - 1u;
              if (set_contains((const int32_t*)bm + L.nbw, L.set_log2, unpack_lds(st, j * kBlock + (uint32_t)tid, b)))
                m |= 1u << j;
            }
          }
        } else {
#pragma unroll 8
          for (int j = 0; j < kRows; j++) {
            const uint32_t v = unpack_lds(st, (uint32_t)(j * kBlock + tid), b);
            m |= ((L.aux[v >> 5] >> (v & 31u)) & 1u) << j;
          }
        }
      } else {
        const rsrc_t r = make_rsrc(L.words, L.wbytes);
        uint32_t rem = need;
        while (__ballot(rem != 0)) {  // rounds of up to 4 needed docs per lane, loads in flight together
          uint32_t jj[4], v[4];
#pragma unroll
          for (int x = 0; x < 4; x++) {
            jj[x] = rem ? (uint32_t)__ffs(rem) - 1u : 32u;
            rem &= rem - 1u;
            const uint32_t d = jj[x] < 32u ? base + jj[x] * (uint32_t)kBlock + (uint32_t)tid : base;
            v[x] = unpack(r, d, L.bits);
          }
#pragma unroll
          for (int x = 0; x < 4; x++)
            if (jj[x] < 32u && leaf_pred(L, lds_sets, v[x])) m |= 1u << jj[x];
        }
      }
      break;
    }
  }
  return L.excl ? ~m : m;
}

// Filter tree (prefix form) over 32-bit masks with short-circuit needs: an AND child only sees docs every
// earlier child accepted, an OR child only docs no earlier child accepted.  Open groups (<= 4) are kept in
// registers: 32-bit acc / need fields packed into 64-bit words, 2-bit types in one word.
enum GroupType : uint32_t { GT_ROOT = 0, GT_AND = 1, GT_OR = 2, GT_NOT = 3 };

__device__ __forceinline__ uint32_t eval_filter(const QuerySpec& q, const LeafDesc* __restrict__ leaves,
                                                const int32_t* lds_sets, const uint32_t* stage, uint32_t valid,
                                                uint32_t base, int tid) {
  if (q.num_ops == 0) return valid;
  uint32_t gtype = GT_ROOT, gacc = 0, gneed = valid, need = valid;
  uint64_t sacc0 = 0, sacc1 = 0, sneed0 = 0, sneed1 = 0;
  uint32_t stype = 0;
  for (uint32_t i = 0; i < q.num_ops; i++) {
    const int32_t op = q.ops[i];
    if (op >= 0 || op == kOpEnd) {
      uint32_t r;
      if (op >= 0) {
        r = __ballot(need != 0) ? eval_leaf(q, (uint32_t)op, leaves[op], lds_sets, stage, need, base, tid) : 0u;
      } else {
        r = gtype == GT_NOT ? (~gacc & gneed) : gacc;
        gtype = stype & 3u;
        stype >>= 2;
        gacc = (uint32_t)sacc0;
        sacc0 = (sacc0 >> 32) | (sacc1 << 32);
        sacc1 >>= 32;
        gneed = (uint32_t)sneed0;
        sneed0 = (sneed0 >> 32) | (sneed1 << 32);
        sneed1 >>= 32;
      }
      switch (gtype) {
        case GT_AND: gacc &= r; need = gneed & gacc; break;
        case GT_OR: gacc |= r; need = gneed & ~gacc; break;
        case GT_NOT: gacc = r; need = 0; break;
        default: gacc = r; need = 0; break;
      }
    } else {  // open a group: its children see the docs currently needed
      stype = (stype << 2) | gtype;
      sacc1 = (sacc1 << 32) | (sacc0 >> 32);
      sacc0 = (sacc0 << 32) | gacc;
      sneed1 = (sneed1 << 32) | (sneed0 >> 32);
      sneed0 = (sneed0 << 32) | gneed;
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

// dictId of doc `d` (row offset `rel` in the tile) of a column read by an aggregation / key: from the staged
// tile when the column is staged, else a gathered window.
__device__ __forceinline__ uint32_t col_id(const QuerySpec& q, uint32_t slot, const ColDesc& c,
                                          const uint32_t* stage, uint32_t d, uint32_t rel) {
  if (slot != kNoSlot) return unpack_lds(stage + q.staged[slot].lds_word_off, rel, c.bits);
  return unpack(make_rsrc(c.words, c.wbytes), d, c.bits);
}

// Dense tiles: the aggregation of 8 rows at a time with every dictionary / keymap read of the batch in flight
// together (the switch on the function is outside the row loop so the 8 reads are straight-line).
template <bool GROUPED>
__device__ __forceinline__ void agg_rows8(const QuerySpec& q, const GroupState& S, const AggSpec& A, const ColDesc* c,
                                          const uint32_t (&ia)[8], const uint32_t (&ib)[8], const uint32_t (&g)[8],
                                          const uint32_t (&d)[8], uint32_t live, uint64_t& acc) {
  switch (A.fn) {
    case PG_AGG_COUNT: break;
    case PG_AGG_SUM:
    case PG_AGG_AVG:
      if (A.integer) {
        int64_t v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = value_i64(A, c, ia[r], ib[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          if (!((live >> r) & 1u)) continue;
          if constexpr (GROUPED) atomicAdd(&S.i64[(uint64_t)g[r] * q.n_i64 + A.slot], (unsigned long long)v[r]);
          else acc += (uint64_t)v[r];
        }
      } else {
        double v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = value_f64(A, c, ia[r], ib[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          if (!((live >> r) & 1u)) continue;
          if constexpr (GROUPED) atomicAdd(&S.f64[(uint64_t)g[r] * q.n_f64 + A.slot], v[r]);
          else acc = __double_as_longlong(__longlong_as_double(acc) + v[r]);
        }
      }
      break;
    case PG_AGG_MIN:
    case PG_AGG_MAX: {
      int64_t k[8];
#pragma unroll
      for (int r = 0; r < 8; r++) k[r] = order_key(value_f64(A, c, ia[r], ib[r]));
      const bool is_min = A.fn == PG_AGG_MIN;
#pragma unroll
      for (int r = 0; r < 8; r++) {
        if (!((live >> r) & 1u)) continue;
        if constexpr (GROUPED) {
          if (is_min) atomicMin(&S.mn[(uint64_t)g[r] * q.n_min + A.slot], (long long)k[r]);
          else atomicMax(&S.mx[(uint64_t)g[r] * q.n_max + A.slot], (long long)k[r]);
        } else {
          if (is_min ? k[r] < (int64_t)acc : k[r] > (int64_t)acc) acc = (uint64_t)k[r];
        }
      }
      break;
    }
    default:  // COUNTMV / DISTINCTCOUNT: per row
#pragma unroll
      for (int r = 0; r < 8; r++) {
        if (!((live >> r) & 1u)) continue;
        if constexpr (GROUPED) group_update(q, S, A, c, g[r], d[r], ia[r], ib[r]);
        else acc_update(q, A, c, acc, d[r], ia[r], ib[r]);
      }
      break;
  }
}

template <bool GROUPED, int MAXA, int MAXK>
__device__ __forceinline__ void aggregate_dense(const QuerySpec& q, const SegDesc& sd, const GroupState& S,
                                                const uint32_t* stage, uint64_t (&acc)[MAXA], uint32_t m,
                                                uint32_t base, int tid) {
  constexpr int NK = MAXK > 0 ? MAXK : 1;
  for (int ch = 0; ch < kRows / 8; ch++) {
    const uint32_t mc = (m >> (8 * ch)) & 0xFFu;
    if (__ballot(mc != 0) == 0) continue;
    uint32_t d[8], rel[8], g[8];
    uint32_t live = mc;
#pragma unroll
    for (int r = 0; r < 8; r++) {
      rel[r] = ((mc >> r) & 1u) ? (uint32_t)((8 * ch + r) * kBlock + tid) : 0u;
      d[r] = base + rel[r];
      g[r] = 0;
    }
    if constexpr (GROUPED) {
#pragma unroll
      for (int k = 0; k < NK; k++) {
        if (k >= (int)q.num_keys) break;
        const ColDesc& kc = sd.keycols[k];
        uint32_t ids[8];
        uint64_t kid[8];
#pragma unroll
        for (int r = 0; r < 8; r++) ids[r] = col_id(q, q.key_slot[k], kc, stage, d[r], rel[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) kid[r] = key_of(q.key_kind[k], q.key_base[k], kc, ids[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          if (kid[r] >= q.key_card[k]) live &= ~(1u << r);
          else g[r] += (uint32_t)kid[r] * (uint32_t)q.key_stride[k];
        }
      }
      if (live != mc) atomicOr(q.err, 1u);  // never expected: the host proved the key ranges
#pragma unroll
      for (int r = 0; r < 8; r++)
        if ((live >> r) & 1u) atomicAdd(&S.i64[(uint64_t)g[r] * q.n_i64], 1ull);  // slot 0: doc count / presence
    }
#pragma unroll
    for (int a = 0; a < MAXA; a++) {
      if (a >= (int)q.num_aggs) break;
      const AggSpec& A = q.aggs[a];
      if (A.fn == PG_AGG_COUNT) continue;
      const ColDesc* c = sd.aggcols + 2 * a;
      const uint32_t nc = agg_ncols(A);
      uint32_t ia[8], ib[8];
#pragma unroll
      for (int r = 0; r < 8; r++) {
        ia[r] = nc >= 1 ? col_id(q, q.agg_slot[a][0], c[0], stage, d[r], rel[r]) : 0u;
        ib[r] = nc >= 2 ? col_id(q, q.agg_slot[a][1], c[1], stage, d[r], rel[r]) : 0u;
      }
      agg_rows8<GROUPED>(q, S, A, c, ia, ib, g, d, live, acc[a]);
    }
  }
}

// Aggregation over the matched docs `m` of a tile, in rounds of up to 2 docs per lane; a round's dictId reads for
// every key and aggregation operand are issued before any is consumed.
template <bool GROUPED, int MAXA, int MAXK>
__device__ __forceinline__ void aggregate_tile(const QuerySpec& q, const SegDesc& sd, const GroupState& S,
                                               const uint32_t* stage, uint64_t (&acc)[MAXA], uint32_t m,
                                               uint32_t base, int tid) {
  constexpr int R = 2;
  constexpr int NK = MAXK > 0 ? MAXK : 1;
  while (__ballot(m != 0)) {
    uint32_t jj[R], d[R];
#pragma unroll
    for (int x = 0; x < R; x++) {
      jj[x] = m ? (uint32_t)__ffs(m) - 1u : 32u;
      m &= m - 1u;
      d[x] = jj[x] < 32u ? base + jj[x] * (uint32_t)kBlock + (uint32_t)tid : base;
    }
    uint32_t kidx[R][NK], ia[R][MAXA], ib[R][MAXA];
#pragma unroll
    for (int x = 0; x < R; x++) {
      const uint32_t rel = d[x] - base;
#pragma unroll
      for (int k = 0; k < NK; k++) {
        kidx[x][k] = 0;
        if (GROUPED && k < (int)q.num_keys) kidx[x][k] = col_id(q, q.key_slot[k], sd.keycols[k], stage, d[x], rel);
      }
#pragma unroll
      for (int a = 0; a < MAXA; a++) {
        ia[x][a] = ib[x][a] = 0;
        if (a >= (int)q.num_aggs) continue;
        const uint32_t nc = agg_ncols(q.aggs[a]);
        const ColDesc* c = sd.aggcols + 2 * a;
        if (nc >= 1) ia[x][a] = col_id(q, q.agg_slot[a][0], c[0], stage, d[x], rel);
        if (nc >= 2) ib[x][a] = col_id(q, q.agg_slot[a][1], c[1], stage, d[x], rel);
      }
    }
#pragma unroll
    for (int x = 0; x < R; x++) {
      if (jj[x] >= 32u) continue;
      if constexpr (GROUPED) {
        uint64_t g = 0;
        bool in_range = true;
#pragma unroll
        for (int k = 0; k < NK; k++) {
          if (k >= (int)q.num_keys) break;
          const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], sd.keycols[k], kidx[x][k]);
          in_range &= kid < q.key_card[k];
          g += kid * q.key_stride[k];
        }
        if (!in_range) {  // never expected: the host proved the key ranges; refuse rather than write out of bounds
          atomicOr(q.err, 1u);
          continue;
        }
        atomicAdd(&S.i64[g * q.n_i64], 1ull);  // slot 0: doc count / presence
#pragma unroll
        for (int a = 0; a < MAXA; a++) {
          if (a >= (int)q.num_aggs) break;
          group_update(q, S, q.aggs[a], sd.aggcols + 2 * a, g, d[x], ia[x][a], ib[x][a]);
        }
      } else {
#pragma unroll
        for (int a = 0; a < MAXA; a++) {
          if (a >= (int)q.num_aggs) break;
          acc_update(q, q.aggs[a], sd.aggcols + 2 * a, acc[a], d[x], ia[x][a], ib[x][a]);
        }
      }
    }
  }
}

// MAXA / MAXK: compile-time bounds on the aggregations / group keys of the query (the smallest instantiation
// that fits is launched), so registers are sized for the query shape, not for the ABI maximum.
#ifndef PG_SCAN_MIN_WAVES
#define PG_SCAN_MIN_WAVES 3  // waves per SIMD the register budget must allow (3 blocks of 256 threads per CU)
#endif

template <bool GROUPED, int MAXA, int MAXK>
__global__ __launch_bounds__(kBlock, PG_SCAN_MIN_WAVES) void scan_kernel(QuerySpec q) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* stage = (uint32_t*)smem;                                   // staged tiles (16-byte aligned)
  int32_t* lds_sets = (int32_t*)(stage + q.stage_lds_words);          // IN-list hash sets
  unsigned char* lds_groups = (unsigned char*)(lds_sets + q.set_lds_ints);
  const int tid = threadIdx.x;
  const uint64_t group_bytes = (GROUPED && q.use_lds) ? q.num_slots * 8ull * (q.n_i64 + q.n_f64 + q.n_min + q.n_max) : 0;
  StageSrc& src = *(StageSrc*)(lds_groups + ((group_bytes + 15) & ~15ull));  // per-segment staging sources

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

  // contiguous item range of this block (consecutive items share a segment -> few per-segment reloads)
  const uint32_t i0 = (uint32_t)((uint64_t)blockIdx.x * q.num_items / gridDim.x);
  const uint32_t i1 = (uint32_t)(((uint64_t)blockIdx.x + 1) * q.num_items / gridDim.x);
  uint32_t cur_seg = 0xFFFFFFFFu;
  for (uint32_t item = i0; item < i1; item++) {
    const WorkItem it = q.items[item];
    const SegDesc sd = q.segs[it.seg];
    if (it.seg != cur_seg) {
      __syncthreads();  // every wave is done with the previous segment's LDS sets
      if (q.set_lds_ints) {  // stage this segment's IN-list hash sets
        for (uint32_t l = 0; l < q.num_leaves; l++) {
          const LeafDesc L = sd.leaves[l];
          if (L.kind != LK_SET_LDS) continue;
          for (uint32_t k = tid; k < L.set_ints; k += kBlock) lds_sets[L.lds_off + k] = ((const int32_t*)L.aux)[k];
        }
      }
      if (tid < kMaxStaged) {
        const int s = tid;
        src.words[s] = nullptr;
        src.nwords[s] = 0;
        src.bits[s] = 1;
        if (s >= (int)q.num_staged) goto staged_done;
        const StagedCol& sc = q.staged[s];
        const uint32_t* w = nullptr;
        uint32_t bytes = 0, bits = 1;
        if (sc.role == 0) {
          const LeafDesc& L = sd.leaves[sc.idx];
          if (L.kind == LK_RANGE || L.kind == LK_SET_LDS || L.kind == LK_SET_LUT) { w = L.words; bytes = L.wbytes; bits = L.bits; }
        } else {
          const ColDesc& c = sc.role == 1 ? sd.aggcols[2 * sc.idx + sc.operand] : sd.keycols[sc.idx];
          w = c.words; bytes = c.wbytes; bits = c.bits;
        }
        src.words[s] = w;
        src.nwords[s] = bytes / 4;
        src.bits[s] = bits;
      }
    staged_done:
      __syncthreads();
      cur_seg = it.seg;
    }
    const uint32_t nd = sd.num_docs;
    uint64_t seg_count = 0;
    for (uint32_t tile = it.tile_begin; tile < it.tile_end; tile++) {
      const uint32_t base = tile * (uint32_t)kTileDocs;
      if (q.num_staged) stage_tile(q, src, tile, stage, tid);
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < kRows; j++) valid |= (uint32_t)(base + (uint32_t)(j * kBlock + tid) < nd) << j;
      const uint32_t m = eval_filter(q, sd.leaves, lds_sets, stage, valid, base, tid);
      const uint32_t nm = __popc(m);
      seg_count += nm;
      if (!GROUPED) doc_count += nm;
      if (!GROUPED && !q.agg_reads) continue;  // COUNT(*) only: the matched-doc count is the answer
      // dense when at least a quarter of the lanes hold >= 8 matches: batched rows; else per-doc rounds
      if (__popcll(__ballot(__popc(m) >= 8)) >= 16) aggregate_dense<GROUPED, MAXA, MAXK>(q, sd, S, stage, acc, m, base, tid);
      else aggregate_tile<GROUPED, MAXA, MAXK>(q, sd, S, stage, acc, m, base, tid);
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

size_t scan_lds_bytes(const QuerySpec& q) {
  size_t lds = (size_t)q.stage_lds_words * 4 + (size_t)q.set_lds_ints * 4;
  if (q.num_keys && q.use_lds) lds += q.num_slots * 8ull * (q.n_i64 + q.n_f64 + q.n_min + q.n_max);
  return ((lds + 15) & ~(size_t)15) + sizeof(StageSrc);
}

hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s) {
  const size_t lds = scan_lds_bytes(q);
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
