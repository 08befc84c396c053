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

#include <type_traits>

#include "pg_internal.h"

namespace pg {

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// The per-query descriptors (arena) are read-only for the whole launch: reading them through the constant address
// space lets the compiler use scalar loads (the kernel's own atomics would otherwise force vector loads and full
// vmcnt drains).  Per-doc data (dictionaries, LUTs, keymaps, MV offsets) is read through the global address space.
#define PG_CONST __attribute__((address_space(4)))
#define PG_GLOBAL __attribute__((address_space(1)))
// p[i] of a read-only descriptor array, loaded word by word through the constant address space
template <class T> __device__ __forceinline__ T ldc(const T* p, uint64_t i) {
  static_assert(sizeof(T) % 4 == 0, "descriptor size");
  const PG_CONST uint32_t* src = (const PG_CONST uint32_t*)(p + i);
  T v;
  uint32_t* dst = (uint32_t*)&v;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = src[k];
  return v;
}
template <class T> __device__ __forceinline__ const PG_GLOBAL T* glb(const T* p) { return (const PG_GLOBAL T*)p; }
#define PG_LDS __attribute__((address_space(3)))

// Atomics through address-space-typed pointers: a generic pointer makes every atomic a FLAT atomic, which counts on
// both the vector-memory and the LDS counters, so each LDS-privatised update waited for the wave's outstanding HBM
// stores (config 4's entry append ran 4x slower that way).  g_*: global (agent scope), l_*: LDS (workgroup scope).
template <class T> __device__ __forceinline__ T g_add(T* p, T v) {
  return __hip_atomic_fetch_add((PG_GLOBAL T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> __device__ __forceinline__ T l_add(T* p, T v) {
  return __hip_atomic_fetch_add((PG_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class T> __device__ __forceinline__ void g_min(T* p, T v) {
  __hip_atomic_fetch_min((PG_GLOBAL T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> __device__ __forceinline__ void l_min(T* p, T v) {
  __hip_atomic_fetch_min((PG_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <class T> __device__ __forceinline__ void g_max(T* p, T v) {
  __hip_atomic_fetch_max((PG_GLOBAL T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T> __device__ __forceinline__ void l_max(T* p, T v) {
  __hip_atomic_fetch_max((PG_LDS T*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void g_or(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_or((PG_GLOBAL uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint32_t kRowMask = 0xFFFFFFFFu;                     // kRows == 32
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

// The same from a staged tile in LDS, addressed by the value's LAST bit e = rel*b + b - 1: the 64-bit window
// (st[k-1], st[k]) with k = e >> 5 holds the value in its low 32 + (e & 31) + 1 bits, so one v_alignbit by
// 31 - (e & 31) (= ~e mod 32) right-aligns it.  st[-1] is readable (the ring starts 16 bytes into LDS) and
// only ever contributes bits that the mask drops.
__device__ __forceinline__ uint32_t unpack_end(const uint32_t* st, uint32_t e, uint32_t mask) {
  const uint32_t k = e >> 5;
  return __builtin_amdgcn_alignbit(st[k - 1], st[k], ~e) & mask;
}
__device__ __forceinline__ uint32_t unpack_lds(const uint32_t* st, uint32_t rel, uint32_t b) {
  return unpack_end(st, rel * b + b - 1u, bits_mask(b));
}

// Dictionary reads clamp the dictId to the dictionary: valid data never needs it, and a corrupt forward index
// then yields wrong values (caught by parity checks) instead of an out-of-bounds access.
__device__ __forceinline__ double dict_double(const ColDesc c, uint32_t id) {
  if (c.decoded) return (double)(c.vbase + (int64_t)id);
  id = min(id, c.card - 1u);
  switch (c.dtype) {
    case PG_INT: return (double)glb((const int32_t*)c.dict)[id];
    case PG_LONG: return (double)glb((const int64_t*)c.dict)[id];
    case PG_FLOAT: return (double)glb((const float*)c.dict)[id];
    default: return glb((const double*)c.dict)[id];
  }
}

__device__ __forceinline__ int64_t dict_i64(const ColDesc c, uint32_t id) {
  if (c.decoded) return c.vbase + (int64_t)id;
  id = min(id, c.card - 1u);
  return c.dtype == PG_INT ? (int64_t)glb((const int32_t*)c.dict)[id] : glb((const int64_t*)c.dict)[id];
}

// TransformFunction value of an aggregation input from its (already unpacked) dictIds.
// MultiplicationTransformFunction.transformToDoubleValuesSV (transform/function/MultiplicationTransformFunction.java:91-111):
// start from the literal product 1.0, multiply arguments in order; compiled with -ffp-contract=off.
__device__ __forceinline__ double value_f64(const AggSpec& a, const ColDesc* c, uint32_t ia, uint32_t ib) {
  const double va = dict_double(ldc(c, 0), ia);
  if (a.op == PG_EXPR_COL) return va;
  const double vb = dict_double(ldc(c, 1), ib);
  switch (a.op) {
    case PG_EXPR_MUL: return (1.0 * va) * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// integer-exact path (host proved |partial sums| < 2^62): identical to the double path while < 2^53
__device__ __forceinline__ int64_t value_i64(const AggSpec& a, const ColDesc* c, uint32_t ia, uint32_t ib) {
  const int64_t va = dict_i64(ldc(c, 0), ia);
  if (a.op == PG_EXPR_COL) return va;
  const int64_t vb = dict_i64(ldc(c, 1), ib);
  switch (a.op) {
    case PG_EXPR_MUL: return va * vb;
    case PG_EXPR_ADD: return va + vb;
    default: return va - vb;
  }
}

// table-global key id of dictId `id` (~0 when the id is outside the dictionary: rejected by the caller)
__device__ __forceinline__ uint64_t key_of(uint32_t kind, int64_t base, const ColDesc c, uint32_t id) {
  if (id >= c.card) return ~0ull;
  return kind == PG_KEY_KEYMAP ? (uint64_t)(uint32_t)glb(c.keymap)[id] : (uint64_t)(dict_i64(c, id) - base);
}

__device__ __forceinline__ uint32_t agg_ncols(const AggSpec& A) {
  if (A.fn == PG_AGG_COUNT || A.fn == PG_AGG_COUNTMV || A.mv) return 0;  // (MV values: read through the row offsets)
  if (A.fn == PG_AGG_DISTINCTCOUNT) return 1;
  return A.op == PG_EXPR_COL ? 1u : 2u;
}

// Raw-value predicate of doc d (RawValueBasedPredicateEvaluator.applySV): the value in its stored type against the
// leaf's closed integer range / floating range with inclusivity / sorted value set.
__device__ __forceinline__ bool raw_pred(const LeafDesc& L, uint32_t d) {
  if (L.rtype <= PG_LONG) {
    const int64_t v = L.rtype == PG_INT ? (int64_t)glb((const int32_t*)L.words)[d] : glb((const int64_t*)L.words)[d];
    if (!L.nvals) return v >= L.ilo && v <= L.ihi;
    const PG_GLOBAL int64_t* set = glb((const int64_t*)L.rvals);
    uint32_t lo = 0, hi = L.nvals;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (set[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo < L.nvals && set[lo] == v;
  }
  const double v = L.rtype == PG_FLOAT ? (double)glb((const float*)L.words)[d] : glb((const double*)L.words)[d];
  if (!L.nvals)
    return ((L.rflags & 1u) ? v >= L.dlo : v > L.dlo) && ((L.rflags & 2u) ? v <= L.dhi : v < L.dhi);
  const PG_GLOBAL double* set = glb((const double*)L.rvals);
  uint32_t lo = 0, hi = L.nvals;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (set[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo < L.nvals && set[lo] == v;
}

// IN-set filter bitmap test (exact when shift == 0, else a candidate test resolved by the global LUT).
__device__ __forceinline__ uint32_t set_bit(const uint32_t* bm, uint32_t shift, uint32_t v) {
  const uint32_t x = v >> shift;
  return (bm[x >> 5] >> (x & 31u)) & 1u;
}

// Leaf predicate on a dictId (doc bitmaps: RANGE [1,2) on a 1-bit column).
__device__ __forceinline__ bool leaf_pred(const LeafDesc L, const int32_t* lds_sets, uint32_t v) {
  switch (L.kind) {
    case LK_RANGE: return (v - (uint32_t)L.lo) < (uint32_t)(L.hi - L.lo);
    case LK_SET_LDS: {
      const uint32_t* bm = (const uint32_t*)(lds_sets + L.lds_off);
      if (!set_bit(bm, L.shift, v)) return false;
      return L.shift == 0 || ((glb(L.lut)[v >> 5] >> (v & 31u)) & 1u);
    }
    default: return (glb(L.aux)[v >> 5] >> (v & 31u)) & 1u;  // LK_SET_LUT
  }
}

// LDS-DMA of 16 bytes per lane (buffer_load_dwordx4 ... lds): the wave's 64 lanes fill 1 KiB of LDS at `dst`
// (wave-uniform) from byte offsets `voff` of the column; reads past the descriptor's range return zeros.
__device__ __forceinline__ void dma16(rsrc_t r, uint32_t* dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0, 0);
}

// Words / bits of staged slot `s` in segment `sd` (nullptr: the segment's form of the leaf reads no column).
__device__ __forceinline__ const uint32_t* staged_src(const QuerySpec& q, const SegDesc& sd, uint32_t s,
                                                      uint32_t& bytes, uint32_t& bits) {
  const StagedCol& sc = q.staged[s];
  if (sc.role == 0) {
    const LeafDesc L = ldc(sd.leaves, sc.idx);
    bytes = L.wbytes;
    bits = L.bits;
    return (L.kind == LK_RANGE || L.kind == LK_SET_LDS || L.kind == LK_SET_LUT) ? L.words : nullptr;
  }
  const ColDesc c = sc.role == 1 ? ldc(sd.aggcols, 2 * sc.idx + sc.operand) : ldc(sd.keycols, sc.idx);
  bytes = c.wbytes;
  bits = c.bits;
  return c.words;
}

// Issue the asynchronous copy of tile `tile` of every staged column into the LDS buffer `buf`: the tile's
// 256*b words as b pieces of 1 KiB, pieces dealt round-robin to the 4 waves.  Control
// flow is wave-uniform; nothing waits here (the consumer's barrier drains vmcnt).
__device__ __forceinline__ void stage_issue(const QuerySpec& q, const SegDesc& sd, uint32_t tile, uint32_t* buf,
                                            uint32_t wave, uint32_t lane) {
  for (uint32_t s = 0; s < q.num_staged; s++) {
    uint32_t bytes, bits;
    const uint32_t* w = staged_src(q, sd, s, bytes, bits);
    if (!w) continue;
    const rsrc_t r = make_rsrc(w, bytes);
    const uint32_t pieces = bits;  // the tile's 256*b words = b pieces of 1 KiB
    const uint32_t tb = tile * (uint32_t)(kTileDocs / 8) * bits;  // byte offset of the tile's first word
    uint32_t* dst = buf + q.staged[s].lds_word_off;
    for (uint32_t c = wave; c < pieces; c += kBlock / 64) {
      dma16(r, dst + c * 256, tb + (c * 64 + lane) * 16);
    }
  }
}

// One leaf over the thread's 32 docs, evaluated for the docs in `need` -> 32-bit mask (bit j <-> doc
// base + j*256 + tid).  Bits outside `need` are don't-care.
// The docs a thread evaluates, as rows j of its 32-bit masks:
//   TileRows  -- the tile's docs base + j*256 + tid (j < 32); staged columns are readable at rel = j*256 + tid.
//   QueueRows -- docs compacted into the block's LDS queue: entry j*256 + tid (j < 4), gathers only.
struct TileRows {
  static constexpr bool kTile = true;
  uint32_t base, tid;
  __device__ __forceinline__ uint32_t doc(uint32_t j) const { return base + j * (uint32_t)kBlock + tid; }
  __device__ __forceinline__ uint32_t rel(uint32_t d) const { return d - base; }
};
struct QueueRows {
  static constexpr bool kTile = false;
  const uint32_t* qd;
  uint32_t n, tid;
  __device__ __forceinline__ uint32_t doc(uint32_t j) const {
    const uint32_t i = j * (uint32_t)kBlock + tid;
    return i < n ? qd[i] : 0u;
  }
  __device__ __forceinline__ uint32_t rel(uint32_t) const { return 0u; }
};

template <class Rows>
__device__ __forceinline__ uint32_t eval_leaf(const QuerySpec& q, uint32_t li, const LeafDesc L,
                                              const int32_t* lds_sets, const uint32_t* stage, uint32_t need,
                                              const Rows& rows, int tid) {
  uint32_t m = 0;
  switch (L.kind) {
    case LK_ALL: m = kRowMask; break;
    case LK_NONE: break;
    case LK_RAW: {  // per needed doc, rounds of up to 4 docs per lane with their loads in flight together
      uint32_t rem = need;
      while (__ballot(rem != 0)) {
        uint32_t jj[4];
        bool ok[4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
          jj[x] = rem ? (uint32_t)__ffs(rem) - 1u : 32u;
          rem &= rem - 1u;
          ok[x] = jj[x] < 32u && raw_pred(L, rows.doc(jj[x]));
        }
#pragma unroll
        for (int x = 0; x < 4; x++)
          if (ok[x]) m |= 1u << jj[x];
      }
      break;
    }
    case LK_DOCRANGE: {
      if constexpr (Rows::kTile) {
#pragma unroll
        for (int j = 0; j < kRows; j++) {
          const uint32_t d = rows.doc((uint32_t)j);
          m |= (uint32_t)(d >= (uint32_t)L.lo && d < (uint32_t)L.hi) << j;
        }
      } else {
        uint32_t rem = need;
        while (rem) {
          const uint32_t j = (uint32_t)__ffs(rem) - 1u;
          rem &= rem - 1u;
          const uint32_t d = rows.doc(j);
          m |= (uint32_t)(d >= (uint32_t)L.lo && d < (uint32_t)L.hi) << j;
        }
      }
      break;
    }
    default: {  // packed column: RANGE / SET_LDS / SET_LUT
      const uint32_t slot = Rows::kTile ? q.leaf_slot[li] : (uint32_t)kNoSlot;
      if (slot != kNoSlot) {
        // staged: all 32 rows from LDS, 8 rows per batch with the batch's LDS reads issued together
        const uint32_t* st = stage + q.staged[slot].lds_word_off;
        const uint32_t b = L.bits, mask = bits_mask(b);
        const uint32_t e0 = (uint32_t)tid * b + b - 1u, estep = (uint32_t)kBlock * b;
        if (L.kind == LK_RANGE) {
          const uint32_t lo = (uint32_t)L.lo, span = (uint32_t)(L.hi - L.lo);
#pragma unroll
          for (int j0 = 0; j0 < kRows; j0 += 8) {
            uint32_t v[8];
#pragma unroll
            for (int r = 0; r < 8; r++) v[r] = unpack_end(st, e0 + (uint32_t)(j0 + r) * estep, mask);
#pragma unroll
            for (int r = 0; r < 8; r++) m |= (uint32_t)((v[r] - lo) < span) << (j0 + r);
          }
        } else if (L.kind == LK_SET_LDS) {
          const uint32_t* bm = (const uint32_t*)(lds_sets + L.lds_off);
          const uint32_t shift = L.shift;
#pragma unroll
          for (int j0 = 0; j0 < kRows; j0 += 8) {
            uint32_t x[8], w[8];
#pragma unroll
            for (int r = 0; r < 8; r++) x[r] = unpack_end(st, e0 + (uint32_t)(j0 + r) * estep, mask) >> shift;
#pragma unroll
            for (int r = 0; r < 8; r++) w[r] = bm[x[r] >> 5];
#pragma unroll
            for (int r = 0; r < 8; r++) m |= __builtin_amdgcn_ubfe(w[r], x[r] & 31u, 1u) << (j0 + r);
          }
          if (shift) {  // resolve the (few) bitmap candidates exactly: LUT reads in rounds of 4 per lane
            const PG_GLOBAL uint32_t* lut = glb(L.lut);
            uint32_t cand = m & need;
            m = 0;
            while (__ballot(cand != 0)) {
              uint32_t jj[4], v[4], w[4];
#pragma unroll
              for (int x = 0; x < 4; x++) {
                jj[x] = cand ? (uint32_t)__ffs(cand) - 1u : 0u;
                v[x] = cand ? unpack_end(st, e0 + jj[x] * estep, mask) : 0u;
                jj[x] = cand ? jj[x] : 32u;
                cand &= cand - 1u;
              }
#pragma unroll
              for (int x = 0; x < 4; x++) w[x] = lut[v[x] >> 5];
#pragma unroll
              for (int x = 0; x < 4; x++)
                if (jj[x] < 32u) m |= __builtin_amdgcn_ubfe(w[x], v[x] & 31u, 1u) << jj[x];
            }
          }
        } else {
          const PG_GLOBAL uint32_t* lut = glb(L.aux);
#pragma unroll
          for (int j0 = 0; j0 < kRows; j0 += 8) {
            uint32_t v[8], w[8];
#pragma unroll
            for (int r = 0; r < 8; r++) v[r] = unpack_end(st, e0 + (uint32_t)(j0 + r) * estep, mask);
#pragma unroll
            for (int r = 0; r < 8; r++) w[r] = lut[v[r] >> 5];
#pragma unroll
            for (int r = 0; r < 8; r++) m |= __builtin_amdgcn_ubfe(w[r], v[r] & 31u, 1u) << (j0 + r);
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
            v[x] = unpack(r, rows.doc(jj[x] < 32u ? jj[x] : 0u), L.bits);
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

// Ops [o0, o1) of the program as the children of a group of type `gtype0` (GT_ROOT: the whole program).
template <class Rows>
__device__ __forceinline__ uint32_t eval_filter(const QuerySpec& q, const LeafDesc* leaves, uint32_t o0, uint32_t o1,
                                                uint32_t gtype0, const int32_t* lds_sets, const uint32_t* stage,
                                                uint32_t valid, const Rows& rows, int tid) {
  if (o0 >= o1) return valid;  // no program / no remaining children: every valid doc
  uint32_t gtype = gtype0, gacc = gtype0 == GT_AND ? kRowMask : 0u, gneed = valid, need = valid;
  uint64_t sacc0 = 0, sacc1 = 0, sneed0 = 0, sneed1 = 0;
  uint32_t stype = 0;
  for (uint32_t i = o0; i < o1; i++) {
    const int32_t op = q.ops[i];
    if (op >= 0 || op == kOpEnd) {
      uint32_t r;
      if (op >= 0) {
        r = __ballot(need != 0) ? eval_leaf(q, (uint32_t)op, ldc(leaves, (uint32_t)op), lds_sets, stage, need, rows, tid) : 0u;
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
// exact 128-bit wave sum of (lo, hi) fixed-point partials (SK_FX): integer adds, so the butterfly's order is irrelevant
__device__ __forceinline__ void wave_sum_fx(uint64_t& lo, uint64_t& hi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t xl = __shfl_xor(lo, o), xh = __shfl_xor(hi, o);
    fx_add(lo, hi, xl, xh);
  }
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

// Hash-mode slot of packed key `key`: its table position, claimed with one 64-bit CAS on first sight (linear
// probing; keys only ever change PG_EMPTY_KEY -> key, so a stale read of an empty entry just costs a failed CAS).
// ~0 when the table is over its fill budget: err bit 4, and the runtime reruns the scan with a larger table.
__device__ __forceinline__ uint64_t hash_slot(const QuerySpec& q, uint64_t key) {
  uint64_t h = mix64(key) & q.hmask;
  for (uint64_t n = 0; n <= q.hmask; n++) {
    const unsigned long long cur = q.hkeys[h];
    if (cur == key) return h;
    if (cur == kEmptyKey) {
      if (__hip_atomic_load(q.hfill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= q.hmax_fill) break;
      const unsigned long long prev = atomicCAS(&q.hkeys[h], kEmptyKey, (unsigned long long)key);
      if (prev == kEmptyKey) {
        atomicAdd(q.hfill, 1u);
        return h;
      }
      if (prev == key) return h;
    }
    h = (h + 1) & q.hmask;
  }
  atomicOr(q.err, 4u);
  return ~0ull;
}

// State slot of a doc's group from its packed key (dense: the key itself).  GM_HASH_SEG keys carry the segment and
// record the segment's first sighting of the key (IntGroupIdMap assigns ids in first-seen order): doc << 16 | pos, pos
// = the key's position among the doc's multi-value key tuples (0 for single-value keys).
__device__ __forceinline__ uint64_t group_slot(const QuerySpec& q, uint64_t packed, uint32_t seg, uint32_t doc,
                                               uint32_t pos = 0) {
  if (q.group_mode == GM_DENSE) return packed;
  if (q.group_mode == GM_HASH) return hash_slot(q, packed);
  const uint64_t h = hash_slot(q, packed * q.num_segments + seg);
  if (h != ~0ull) atomicMin(&q.first_doc[h], ((unsigned long long)doc << 16) | pos);
  return h;
}

// GM_PART: the doc's entry instead of a state update.  The lanes with `on` append (key << part_vbits | value id)
// to the block's region of the entry array in lane order -- one LDS atomic per wave per call, and the wave's stores
// are consecutive 8-byte words -- and count it in the block's histogram of level-1 partitions (key >> part_shift).
// Called by every lane of the wave (it ballots).  lds[0] = the block's entry count, lds[1 + p] = its histogram.
__device__ __forceinline__ void part_append(const QuerySpec& q, uint32_t* lds, unsigned long long* out, bool on,
                                            uint64_t g, uint32_t vid) {
  const uint64_t bal = __ballot(on);
  if (!bal) return;
  const uint32_t leader = (uint32_t)__builtin_ctzll(bal);
  uint32_t base = 0;
  if ((threadIdx.x & 63u) == leader) base = l_add(&lds[0], (uint32_t)__popcll(bal));
  base = __builtin_amdgcn_readlane(base, leader);
  if (on) {
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    out[base + rank] = (g << q.part_vbits) | vid;
    l_add(&lds[1 + (uint32_t)(g >> q.part_shift)], 1u);
  }
}

// part_append for the 8 rows of a dense chunk at once: one LDS cursor atomic per wave for all of them (the cursor's
// return latency is paid once per chunk, not once per row).
template <class GK>
__device__ __forceinline__ void part_append8(const QuerySpec& q, uint32_t* lds, unsigned long long* out, uint32_t live,
                                             const GK (&g)[8], const uint32_t (&vid)[8]) {
  uint64_t bal[8];
  uint32_t pre[8], total = 0;
#pragma unroll
  for (int r = 0; r < 8; r++) {
    bal[r] = __ballot((live >> r) & 1u);
    pre[r] = total;
    total += (uint32_t)__popcll(bal[r]);
  }
  if (!total) return;
  uint32_t base = 0;
  if ((threadIdx.x & 63u) == 0) base = l_add(&lds[0], total);
  base = __builtin_amdgcn_readlane(base, 0);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    if (!((live >> r) & 1u)) continue;
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
    out[base + pre[r] + rank] = ((uint64_t)g[r] << q.part_vbits) | vid[r];
    l_add(&lds[1 + (uint32_t)((uint64_t)g[r] >> q.part_shift)], 1u);
  }
}

// Packed group key / state slot of a doc: a single key's global id and every slot (dense <= 2^26, hash tables <=
// 2^30) fit 32 bits; only a mixed-radix key of several columns needs 64 (and 32-bit keys keep the single-key shapes
// free of scratch spills).
template <int MAXK> using GKey = typename std::conditional<(MAXK > 1), uint64_t, uint32_t>::type;

// Group-state pointers: the block's LDS copy when the table is privatised, else the global arrays.
struct GroupState {
  unsigned long long* i64;   // GM_PART: the block's LDS entry count + level-1 histogram (uint32 words)
  unsigned long long* fx;    // SK_FX pairs (lo, hi)
  long long* mn;
  long long* mx;
  unsigned long long* out;   // GM_PART: the block's region of the entry array
  bool lds;                  // the arrays are the block's LDS copy (block-uniform)
};
__device__ __forceinline__ void s_add(const GroupState& S, unsigned long long* p, unsigned long long v) {
  if (S.lds) l_add(p, v); else g_add(p, v);
}
__device__ __forceinline__ void s_min(const GroupState& S, long long* p, long long v) {
  if (S.lds) l_min(p, v); else g_min(p, v);
}
__device__ __forceinline__ void s_max(const GroupState& S, long long* p, long long v) {
  if (S.lds) l_max(p, v); else g_max(p, v);
}
// 128-bit atomic add of (lo, hi) at p[0], p[1]: the low word's carry-out (seen in its old value) goes to the high word,
// which makes the pair's final value the exact sum in any interleaving of the atomics
__device__ __forceinline__ void g_addfx(unsigned long long* p, uint64_t lo, uint64_t hi) {
  const uint64_t old = g_add(p, (unsigned long long)lo);
  const uint64_t h = hi + (old + lo < old ? 1ull : 0ull);
  if (h) g_add(p + 1, (unsigned long long)h);
}
__device__ __forceinline__ void s_addfx(const GroupState& S, unsigned long long* p, uint64_t lo, uint64_t hi) {
  if (S.lds) {
    const uint64_t old = l_add(p, (unsigned long long)lo);
    const uint64_t h = hi + (old + lo < old ? 1ull : 0ull);
    if (h) l_add(p + 1, (unsigned long long)h);
  } else {
    g_addfx(p, lo, hi);
  }
}
// One SK_FX input: its exact fixed-point value into its exponent window's pair, or (+-inf / NaN) its order image into
// the special slots
__device__ __forceinline__ void fx_update(const QuerySpec& q, const GroupState& S, const AggSpec& A, uint64_t g,
                                          double v) {
  if (__builtin_isfinite(v)) {
    if (v == 0.0) return;
    uint64_t lo, hi;
    const uint32_t w = fx_split(v, A.fx_shift, A.fx_nwin, lo, hi);
    s_addfx(S, &S.fx[(g * q.n_fx + A.slot + w) * 2], lo, hi);
  } else if (A.sp_min != kNoSp) {
    const long long k = (long long)order_key(v);
    s_min(S, &S.mn[g * q.n_min + A.sp_min], k);
    s_max(S, &S.mx[g * q.n_max + A.sp_max], k);
  }
}
// SUMMV / MINMV / MAXMV / AVGMV / DISTINCTCOUNTMV (PG_AGG_MV_VALUES): every value of doc d's list in the aggregation's
// multi-value column, in stored order (*MVAggregationFunction: `for (value : valuesArray[i])`); AVGMV also counts the
// values into its count slot.  noinline: one copy per kernel, not one per unrolled aggregation slot of every shape.
__device__ __attribute__((noinline)) uint64_t mv_update(const QuerySpec* qp, GroupState S, const AggSpec* Ap,
                                                        const ColDesc* c, uint64_t g, uint32_t d, uint64_t acc,
                                                        bool grouped) {
  const QuerySpec& q = *qp;
  const AggSpec& A = *Ap;
  const ColDesc c0 = ldc(c, 0);
  const PG_GLOBAL uint32_t* off = glb(c0.mv_offsets);
  const uint32_t v0 = off[d], v1 = off[d + 1];
  const rsrc_t rs = make_rsrc(c0.words, c0.wbytes);
  for (uint32_t v = v0; v < v1; v++) {
    const uint32_t id = unpack(rs, v, c0.bits);
    switch (A.fn) {
      case PG_AGG_SUM:
      case PG_AGG_AVG:
        if (!A.integer) fx_update(q, S, A, grouped ? g : 0ull, value_f64(A, c, id, 0));
        else if (grouped) s_add(S, &S.i64[g * q.n_i64 + A.slot], (unsigned long long)value_i64(A, c, id, 0));
        else acc += (uint64_t)value_i64(A, c, id, 0);
        break;
      case PG_AGG_MIN:
      case PG_AGG_MAX: {
        const int64_t k = order_key(value_f64(A, c, id, 0));
        if (grouped && A.fn == PG_AGG_MIN) s_min(S, &S.mn[g * q.n_min + A.slot], (long long)k);
        else if (grouped) s_max(S, &S.mx[g * q.n_max + A.slot], (long long)k);
        else if (A.fn == PG_AGG_MIN ? k < (int64_t)acc : k > (int64_t)acc) acc = (uint64_t)k;
        break;
      }
      default: {  // DISTINCTCOUNT
        const uint64_t key = key_of(A.key_kind, A.key_base, c0, id);
        if (key < A.key_card) g_or(&q.dbits[(grouped ? g * q.dc_row_words : 0ull) + A.dc_word + (key >> 5)], 1u << (key & 31u));
        else atomicOr(q.err, 2u);
      }
    }
  }
  if (A.fn == PG_AGG_AVG) s_add(S, &S.i64[(grouped ? g * q.n_i64 : 0ull) + A.cnt_slot], (unsigned long long)(v1 - v0));
  return acc;
}

// Per-doc update of one aggregation in group slot g (aggregateGroupBySV of each function).
__device__ __forceinline__ void group_update(const QuerySpec& q, const GroupState& S, const AggSpec& A,
                                             const ColDesc* c, uint64_t g, uint32_t d, uint32_t ia, uint32_t ib) {
  switch (A.fn) {
    case PG_AGG_COUNT: break;  // = slot 0
    case PG_AGG_COUNTMV:
      s_add(S, &S.i64[g * q.n_i64 + A.slot], (unsigned long long)(glb(ldc(c, 0).mv_offsets)[d + 1] - glb(ldc(c, 0).mv_offsets)[d]));
      break;
    case PG_AGG_SUM:
    case PG_AGG_AVG:  // AVG count == slot 0
      if (A.integer) s_add(S, &S.i64[g * q.n_i64 + A.slot], (unsigned long long)value_i64(A, c, ia, ib));
      else fx_update(q, S, A, g, value_f64(A, c, ia, ib));
      break;
    case PG_AGG_MIN: s_min(S, &S.mn[g * q.n_min + A.slot], (long long)order_key(value_f64(A, c, ia, ib))); break;
    case PG_AGG_MAX: s_max(S, &S.mx[g * q.n_max + A.slot], (long long)order_key(value_f64(A, c, ia, ib))); break;
    case PG_AGG_DISTINCTCOUNT: {
      const uint64_t key = key_of(A.key_kind, A.key_base, ldc(c, 0), ia);
      if (key < A.key_card) g_or(&q.dbits[g * q.dc_row_words + A.dc_word + (key >> 5)], 1u << (key & 31u));
      else atomicOr(q.err, 2u);
      break;
    }
  }
}

// Per-doc update of one aggregation-only accumulator (aggregate() of each function; COUNT = doc count).
// SK_FX sums go to the block's one-slot LDS table S (use_lds): a 128-bit accumulator per thread would cost the
// aggregation-only shapes registers they do not have.
__device__ __forceinline__ void acc_update(const QuerySpec& q, const GroupState& S, const AggSpec& A, const ColDesc* c,
                                           uint64_t& acc, uint32_t d, uint32_t ia, uint32_t ib) {
  switch (A.fn) {
    case PG_AGG_COUNT: break;
    case PG_AGG_COUNTMV: acc += glb(ldc(c, 0).mv_offsets)[d + 1] - glb(ldc(c, 0).mv_offsets)[d]; break;
    case PG_AGG_SUM:
    case PG_AGG_AVG:
      if (A.integer) acc += (uint64_t)value_i64(A, c, ia, ib);
      else fx_update(q, S, A, 0, value_f64(A, c, ia, ib));
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
      const uint64_t key = key_of(A.key_kind, A.key_base, ldc(c, 0), ia);
      if (key < A.key_card) g_or(&q.dbits[A.dc_word + (key >> 5)], 1u << (key & 31u));
      else atomicOr(q.err, 2u);
      break;
    }
  }
}

// dictId of doc `d` (row offset `rel` in the tile) of a column read by an aggregation / key: from the staged
// tile when the column is staged, else a gathered window.
__device__ __forceinline__ uint32_t col_id(const QuerySpec& q, uint32_t slot, const ColDesc c,
                                          const uint32_t* stage, uint32_t d, uint32_t rel) {
  if (!c.bits) return d;  // raw forward index: the value array is indexed by doc id
  if (slot != kNoSlot) return unpack_lds(stage + q.staged[slot].lds_word_off, rel, c.bits);
  return unpack(make_rsrc(c.words, c.wbytes), d, c.bits);
}

// GROUP BY multi-value columns: doc d joins the group of each tuple of the cartesian product of its MV keys' lists, in
// stored order, duplicates included (DictionaryBasedGroupKeyGenerator.generateKeysForBlock(.., int[][]) :188-200,
// getIntRawKeys :472-540: the lowest MV key outermost), each with the doc's own aggregation inputs
// (aggregateGroupByMV); g0 = the packed key of the SV keys.  noinline, the aggregations in a runtime loop: one copy
// per kernel, not one per unrolled aggregation slot of every shape.
__device__ __attribute__((noinline)) void mv_key_update(const QuerySpec* qp, GroupState S, SegDesc sd, uint32_t d,
                                                        uint64_t g0) {
  const QuerySpec& q = *qp;
  uint32_t mk_k[kMaxKeys], cur[kMaxKeys], beg[kMaxKeys], end[kMaxKeys];
  uint32_t nmv = 0;
  for (uint32_t k = 0; k < q.num_keys; k++) {
    if (!((q.mv_keys >> k) & 1u)) continue;
    const ColDesc mk = ldc(sd.keycols, k);
    const PG_GLOBAL uint32_t* off = glb(mk.mv_offsets);
    mk_k[nmv] = k;
    beg[nmv] = cur[nmv] = off[d];
    end[nmv] = off[d + 1];
    if (beg[nmv] == end[nmv]) return;  // an empty list: no tuple
    nmv++;
  }
  if (!nmv) return;
  for (uint32_t pos = 0;; pos++) {  // odometer over the lists, the last MV key fastest; pos = the tuple's position
    uint64_t gk = g0;
    bool in_range = true;
    for (uint32_t m = 0; m < nmv; m++) {
      const uint32_t k = mk_k[m];
      const ColDesc mk = ldc(sd.keycols, k);
      const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], mk, unpack(make_rsrc(mk.words, mk.wbytes), cur[m], mk.bits));
      in_range &= kid < q.key_card[k];
      gk += kid * q.key_stride[k];
    }
    int m = (int)nmv - 1;
    while (m >= 0 && ++cur[m] == end[m]) { cur[m] = beg[m]; m--; }
    if (!in_range) {  // never expected: the host proved the key ranges
      atomicOr(q.err, 1u);
      if (m < 0) break;
      continue;
    }
    if (pos > 0xFFFFu && q.group_mode == GM_HASH_SEG) {  // beyond the first-seen order's 16 bits: fail loudly
      atomicOr(q.err, 128u);
      break;
    }
    const uint64_t g = group_slot(q, gk, sd.index, d, pos);
    if (g == ~0ull) { if (m < 0) break; continue; }
    s_add(S, &S.i64[g * q.n_i64], 1ull);  // slot 0: (doc, value) count / presence
#pragma unroll 1
    for (uint32_t a = 0; a < q.num_aggs; a++) {
      const AggSpec& A = q.aggs[a];
      const ColDesc* c = sd.aggcols + 2 * a;
      const uint32_t nc = agg_ncols(A);
      const uint32_t ia = nc >= 1 ? col_id(q, kNoSlot, ldc(c, 0), nullptr, d, 0) : 0u;
      const uint32_t ib = nc >= 2 ? col_id(q, kNoSlot, ldc(c, 1), nullptr, d, 0) : 0u;
      if (A.mv) mv_update(&q, S, &A, c, g, d, 0ull, true);
      else group_update(q, S, A, c, g, d, ia, ib);
    }
    if (m < 0) break;
  }
}

// Dense tiles: the aggregation of 8 rows at a time with every dictionary / keymap read of the batch in flight
// together (the switch on the function is outside the row loop so the 8 reads are straight-line).
template <bool GROUPED, class GK>
__device__ __forceinline__ void agg_rows8(const QuerySpec& q, const GroupState& S, const AggSpec& A, const ColDesc* c,
                                          const uint32_t (&ia)[8], const uint32_t (&ib)[8], const GK (&g)[8],
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
          if constexpr (GROUPED) s_add(S, &S.i64[(uint64_t)g[r] * q.n_i64 + A.slot], (unsigned long long)v[r]);
          else acc += (uint64_t)v[r];
        }
      } else {
        double v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = value_f64(A, c, ia[r], ib[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          if (!((live >> r) & 1u)) continue;
          fx_update(q, S, A, GROUPED ? (uint64_t)g[r] : 0ull, v[r]);
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
          if (is_min) s_min(S, &S.mn[(uint64_t)g[r] * q.n_min + A.slot], (long long)k[r]);
          else s_max(S, &S.mx[(uint64_t)g[r] * q.n_max + A.slot], (long long)k[r]);
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
        else acc_update(q, S, A, c, acc, d[r], ia[r], ib[r]);
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
    uint32_t d[8], rel[8];
    GKey<MAXK> g[8];
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
        const ColDesc kc = ldc(sd.keycols, k);
        uint32_t ids[8];
        uint64_t kid[8];
#pragma unroll
        for (int r = 0; r < 8; r++) ids[r] = col_id(q, q.key_slot[k], kc, stage, d[r], rel[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) kid[r] = key_of(q.key_kind[k], q.key_base[k], kc, ids[r]);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          if (kid[r] >= q.key_card[k]) live &= ~(1u << r);
          else g[r] += (GKey<MAXK>)(kid[r] * q.key_stride[k]);
        }
      }
      if (live != mc) atomicOr(q.err, 1u);  // never expected: the host proved the key ranges
      if (q.group_mode == GM_PART) {
        uint32_t vid[8];
#pragma unroll
        for (int r = 0; r < 8; r++) vid[r] = 0;
        if (q.part_dc != (uint32_t)kNoSlot) {
          const uint32_t a = q.part_dc;
          const AggSpec& A = q.aggs[a];
          const ColDesc c0 = ldc(sd.aggcols + 2 * a, 0);
          uint32_t ids[8];
#pragma unroll
          for (int r = 0; r < 8; r++) ids[r] = col_id(q, q.agg_slot[a][0], c0, stage, d[r], rel[r]);
#pragma unroll
          for (int r = 0; r < 8; r++) {
            const uint64_t k = key_of(A.key_kind, A.key_base, c0, ids[r]);
            if (k < A.key_card) vid[r] = (uint32_t)k;
            else if ((live >> r) & 1u) { atomicOr(q.err, 2u); live &= ~(1u << r); }
          }
        }
        part_append8(q, (uint32_t*)S.i64, S.out, live, g, vid);
        continue;
      }
      if (q.group_mode != GM_DENSE) {
        for (int r = 0; r < 8; r++) {
          if (!((live >> r) & 1u)) continue;
          const uint64_t slot = group_slot(q, (uint64_t)g[r], sd.index, d[r]);
          if (slot == ~0ull) live &= ~(1u << r);
          else g[r] = (GKey<MAXK>)slot;
        }
      }
#pragma unroll
      for (int r = 0; r < 8; r++)
        if ((live >> r) & 1u) s_add(S, &S.i64[(uint64_t)g[r] * q.n_i64], 1ull);  // slot 0: doc count / presence
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
        ia[r] = nc >= 1 ? col_id(q, q.agg_slot[a][0], ldc(c, 0), stage, d[r], rel[r]) : 0u;
        ib[r] = nc >= 2 ? col_id(q, q.agg_slot[a][1], ldc(c, 1), stage, d[r], rel[r]) : 0u;
      }
      agg_rows8<GROUPED, GKey<MAXK>>(q, S, A, c, ia, ib, g, d, live, acc[a]);
    }
  }
}

// Aggregation over the matched docs `m` of a tile, in rounds of up to 2 docs per lane; a round's dictId reads for
// every key and aggregation operand are issued before any is consumed.
template <bool GROUPED, int MAXA, int MAXK, class Rows>
__device__ __forceinline__ void aggregate_tile(const QuerySpec& q, const SegDesc& sd, const GroupState& S,
                                               const uint32_t* stage, uint64_t (&acc)[MAXA], uint32_t m,
                                               const Rows& rows) {
  constexpr int R = 2;
  constexpr int NK = MAXK > 0 ? MAXK : 1;
  while (__ballot(m != 0)) {
    uint32_t jj[R], d[R];
#pragma unroll
    for (int x = 0; x < R; x++) {
      jj[x] = m ? (uint32_t)__ffs(m) - 1u : 32u;
      m &= m - 1u;
      d[x] = rows.doc(jj[x] < 32u ? jj[x] : 0u);
    }
    uint32_t kidx[R][NK], ia[R][MAXA], ib[R][MAXA];
#pragma unroll
    for (int x = 0; x < R; x++) {
      const uint32_t rel = rows.rel(d[x]);
#pragma unroll
      for (int k = 0; k < NK; k++) {
        kidx[x][k] = 0;
        if (GROUPED && k < (int)q.num_keys && !((q.mv_keys >> k) & 1u))
          kidx[x][k] = col_id(q, Rows::kTile ? q.key_slot[k] : (uint32_t)kNoSlot, ldc(sd.keycols, k), stage, d[x], rel);
      }
#pragma unroll
      for (int a = 0; a < MAXA; a++) {
        ia[x][a] = ib[x][a] = 0;
        if (a >= (int)q.num_aggs) continue;
        const uint32_t nc = agg_ncols(q.aggs[a]);
        const ColDesc* c = sd.aggcols + 2 * a;
        const uint32_t s0 = Rows::kTile ? q.agg_slot[a][0] : (uint32_t)kNoSlot;
        const uint32_t s1 = Rows::kTile ? q.agg_slot[a][1] : (uint32_t)kNoSlot;
        if (nc >= 1) ia[x][a] = col_id(q, s0, ldc(c, 0), stage, d[x], rel);
        if (nc >= 2) ib[x][a] = col_id(q, s1, ldc(c, 1), stage, d[x], rel);
      }
    }
#pragma unroll
    for (int x = 0; x < R; x++) {
      if constexpr (GROUPED) {
        if (q.group_mode == GM_PART) {  // block-uniform: every lane takes part in the append
          uint64_t g = 0;
          bool on = jj[x] < 32u;
#pragma unroll
          for (int k = 0; k < NK; k++) {
            if (k >= (int)q.num_keys) break;
            const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], ldc(sd.keycols, k), kidx[x][k]);
            if (on && kid >= q.key_card[k]) { atomicOr(q.err, 1u); on = false; }
            g += kid * q.key_stride[k];
          }
          uint32_t vid = 0;
#pragma unroll
          for (int a = 0; a < MAXA; a++) {
            if ((uint32_t)a != q.part_dc) continue;
            const AggSpec& A = q.aggs[a];
            const uint64_t k = key_of(A.key_kind, A.key_base, ldc(sd.aggcols + 2 * a, 0), ia[x][a]);
            if (k < A.key_card) vid = (uint32_t)k;
            else if (on) { atomicOr(q.err, 2u); on = false; }
          }
          part_append(q, (uint32_t*)S.i64, S.out, on, g, vid);
          continue;
        }
      }
      if (jj[x] >= 32u) continue;
      if constexpr (GROUPED && MAXA == kMaxAggs) {  // (the multi-value paths live in the widest shapes only)
        if (q.mv_keys) {
          // multi-value keys: the doc joins the group of each tuple of their lists' product (mv_key_update)
          uint64_t g0 = 0;
          bool in_range = true;
#pragma unroll
          for (int k = 0; k < NK; k++) {
            if (k >= (int)q.num_keys) break;
            if ((q.mv_keys >> k) & 1u) continue;
            const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], ldc(sd.keycols, k), kidx[x][k]);
            in_range &= kid < q.key_card[k];
            g0 += kid * q.key_stride[k];
          }
          if (!in_range) {  // never expected: the host proved the key ranges
            atomicOr(q.err, 1u);
            continue;
          }
          mv_key_update(&q, S, sd, d[x], g0);
          continue;
        }
      }
      if constexpr (GROUPED) {
        uint64_t g = 0;
        bool in_range = true;
#pragma unroll
        for (int k = 0; k < NK; k++) {
          if (k >= (int)q.num_keys) break;
          const uint64_t kid = key_of(q.key_kind[k], q.key_base[k], ldc(sd.keycols, k), kidx[x][k]);
          in_range &= kid < q.key_card[k];
          g += kid * q.key_stride[k];
        }
        if (!in_range) {  // never expected: the host proved the key ranges; refuse rather than write out of bounds
          atomicOr(q.err, 1u);
          continue;
        }
        g = group_slot(q, g, sd.index, d[x]);
        if (g == ~0ull) continue;
        s_add(S, &S.i64[g * q.n_i64], 1ull);  // slot 0: doc count / presence
#pragma unroll
        for (int a = 0; a < MAXA; a++) {
          if (a >= (int)q.num_aggs) break;
          if (MAXA == kMaxAggs && q.aggs[a].mv) mv_update(&q, S, &q.aggs[a], sd.aggcols + 2 * a, g, d[x], 0ull, true);
          else group_update(q, S, q.aggs[a], sd.aggcols + 2 * a, g, d[x], ia[x][a], ib[x][a]);
        }
      } else {
#pragma unroll
        for (int a = 0; a < MAXA; a++) {
          if (a >= (int)q.num_aggs) break;
          if (MAXA == kMaxAggs && q.aggs[a].mv) acc[a] = mv_update(&q, S, &q.aggs[a], sd.aggcols + 2 * a, 0ull, d[x], acc[a], false);
          else acc_update(q, S, q.aggs[a], sd.aggcols + 2 * a, acc[a], d[x], ia[x][a], ib[x][a]);
        }
      }
    }
  }
}

// MAXA / MAXK: compile-time bounds on the aggregations / group keys of the query (the smallest instantiation
// that fits is launched), so registers are sized for the query shape, not for the ABI maximum.
// Waves per SIMD the register budget must allow (= resident 256-thread blocks per CU).  Grouped shapes keep 3;
// aggregation-only shapes hold fewer live registers and run 4 (measured: config 3 scan 1.73 -> 1.44 ms at 4, while
// config 2, grouped, goes 0.93 -> 0.99 ms at 4).
#ifndef PG_SCAN_MIN_WAVES
#define PG_SCAN_MIN_WAVES 3
#endif
#ifndef PG_SCAN_MIN_WAVES_AGG
#define PG_SCAN_MIN_WAVES_AGG 4
#endif

// LDS layout of a launch: [16 B][staging ring][IN sets][group table at a 16-byte boundary][queue]
__host__ __device__ inline size_t scan_groups_off(const QuerySpec& q) {
  size_t off = 16 + (size_t)q.stage_ring * q.stage_lds_words * 4 + (size_t)q.set_lds_ints * 4;
  // aggregation-only with a one-slot table (SK_FX sums): past the block reduction's words, which reuse the ring
  const size_t red = 16 + (size_t)(kBlock / 64) * (1 + kMaxAggs) * 8;
  if (!q.num_keys && q.use_lds && off < red) off = red;
  return (off + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t scan_queue_off(const QuerySpec& q) {
  const size_t g = (q.num_keys && q.group_mode == GM_PART) ? (1 + q.part_nparts) * 4ull
                   : q.use_lds ? q.num_slots * 8ull * (q.n_i64 + 2 * q.n_fx + q.n_min + q.n_max) : 0;
  return scan_groups_off(q) + ((g + 15) & ~(size_t)15);
}

template <bool GROUPED, int MAXA, int MAXK>
__device__ __forceinline__ void scan_body() {
  // the spec is read where the launch put it (the kernel-argument segment, offset 0): bound by reference to the
  // by-value parameter, a lane-varying index into it made the compiler copy all of it to scratch (1.4 KB per lane)
  const QuerySpec& q = *(const QuerySpec*)__builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* stage = (uint32_t*)(smem + 16);                                   // staging ring (16 bytes in: st[-1])
  int32_t* lds_sets = (int32_t*)(stage + q.stage_ring * q.stage_lds_words);  // IN-list filter bitmaps / hash sets
  unsigned char* lds_groups = smem + scan_groups_off(q);                       // 16-byte aligned
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);

  // LDS-privatised group table: [G][n_i64] u64 | [G][n_fx][2] u64 | [G][n_min] i64 | [G][n_max] i64
  unsigned long long* l_i64 = (unsigned long long*)lds_groups;
  unsigned long long* l_fx = l_i64 + q.num_slots * q.n_i64;
  long long* l_mn = (long long*)(l_fx + q.num_slots * q.n_fx * 2);
  long long* l_mx = l_mn + q.num_slots * q.n_min;
  if (q.use_lds) {  // (aggregation-only: one slot for SK_FX sums and their special slots)
    for (uint64_t i = tid; i < q.num_slots * q.n_i64; i += kBlock) l_i64[i] = 0;
    for (uint64_t i = tid; i < q.num_slots * q.n_fx * 2; i += kBlock) l_fx[i] = 0;
    for (uint64_t i = tid; i < q.num_slots * q.n_min; i += kBlock) l_mn[i] = order_key(__builtin_inf());
    for (uint64_t i = tid; i < q.num_slots * q.n_max; i += kBlock) l_mx[i] = order_key(-__builtin_inf());
  }
  // GM_PART: the block's entry count and level-1 histogram (LDS), its region of the entry array
  const bool part = GROUPED && q.group_mode == GM_PART;
  if (part) {
    uint32_t* h = (uint32_t*)lds_groups;
    for (uint32_t p = tid; p <= q.part_nparts; p += kBlock) h[p] = 0u;
    __syncthreads();
  }
  const GroupState S = (q.use_lds || part)
                           ? GroupState{l_i64, l_fx, l_mn, l_mx, part ? q.part_out + q.part_base[blockIdx.x] : nullptr, true}
                           : GroupState{q.i64, q.fx, q.mn, q.mx, nullptr, false};

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

  // The block walks the tiles of a contiguous item range (consecutive items share a segment) as one sequence;
  // the staged columns of the next tile are copied HBM -> LDS while the current tile is evaluated (ring of 2
  // buffers), or right after it (ring of 1, overlap across the CU's blocks only).
  const uint32_t i0 = (uint32_t)((uint64_t)blockIdx.x * q.num_items / gridDim.x);
  const uint32_t i1 = (uint32_t)(((uint64_t)blockIdx.x + 1) * q.num_items / gridDim.x);
  // queue (queue_mode): [kQueueCap] doc ids + [4] wave totals of the compaction scan
  uint32_t* queue = (uint32_t*)(smem + scan_queue_off(q));
  uint32_t* scan_tmp = queue + kQueueCap;
  uint32_t qn = 0;  // queued docs (block-uniform)
  // cooperative cancellation (pg_cancel / deadline): thread 0 loads the query's host-visible flag during a tile and
  // publishes it in LDS before the next tile's barrier; every wave reads the word of that tile's parity after the
  // barrier, so the whole block leaves the loop at the same tile (the words live in the pad before the ring, whose
  // st[-1] bits are always masked off)
  // Polled every kPollTiles tiles into alternating words; a raised flag ends the loop through has_next (a separate
  // exit path out of the tile loop spilled 48 bytes per lane to scratch at 4 waves per SIMD: config 3 1.7x slower).
  volatile unsigned int* stop = (volatile unsigned int*)smem;
  if (tid == 0) stop[0] = stop[1] = 0u;
  uint32_t iter = 0;     // block-uniform tile counter
  uint32_t pending = 0;  // thread 0: the flag loaded at the previous poll (arrived long before it is stored)

  if (i0 < i1) {
    const bool ring2 = q.stage_ring > 1;
    uint32_t item = i0;
    WorkItem it = ldc(q.items, item);
    uint32_t tile = it.tile_begin;
    uint32_t buf = 0;
    uint32_t cur_seg = 0xFFFFFFFFu;
    SegDesc cur_sd = ldc(q.segs, it.seg);
    uint64_t seg_count = 0;

    // phase B over the queued docs of segment `cur_sd`: the root AND's remaining children, then aggregation
    auto flush = [&]() __attribute__((always_inline)) {
      __syncthreads();  // queue entries visible
      const QueueRows rows{queue, qn, (uint32_t)tid};
      uint32_t valid = 0;
#pragma unroll
      for (int j = 0; j < kQueueRows; j++) valid |= (uint32_t)((uint32_t)(j * kBlock + tid) < qn) << j;
      const uint32_t m = eval_filter(q, cur_sd.leaves, q.opB_begin, q.opB_end, GT_AND, lds_sets, stage, valid, rows, tid);
      const uint32_t nm = __popc(m);
      seg_count += nm;
      if (!GROUPED) doc_count += nm;
      if (GROUPED || q.agg_reads) aggregate_tile<GROUPED, MAXA, MAXK>(q, cur_sd, S, stage, acc, m, rows);
      __syncthreads();  // every lane is done reading the queue
      qn = 0;
    };
    // a new segment: the previous one's queued docs and match count, then this one's IN-list sets in LDS
    auto enter_segment = [&](uint32_t seg) __attribute__((always_inline)) {
      if (cur_seg != 0xFFFFFFFFu) {
        if (qn) flush();  // the queue holds docs of the previous segment
        const uint64_t c = wave_sum_u64(seg_count);
        if (lane == 0 && c) g_add(&q.seg_matched[cur_seg], (unsigned long long)c);
        seg_count = 0;
      }
      cur_sd = ldc(q.segs, seg);
      if (q.set_lds_ints) {  // this segment's IN-list filter bitmaps + hash tables
        for (uint32_t l = 0; l < q.num_leaves; l++) {
          const LeafDesc L = ldc(cur_sd.leaves, l);
          if (L.kind != LK_SET_LDS) continue;
          const PG_GLOBAL int32_t* src = glb((const int32_t*)L.aux);
          int32_t* dst = lds_sets + L.lds_off;
          for (uint32_t k = tid; k < L.set_ints; k += kBlock) dst[k] = src[k];
        }
        __syncthreads();
      }
      cur_seg = seg;
    };

    if (q.list_mode) {
      // the stream kernel's survivors: item by item into the queue, phase B + aggregation per flush
      for (;;) {
        if (it.seg != cur_seg) enter_segment(it.seg);
        const uint32_t n = __builtin_amdgcn_readfirstlane(min(glb(q.list_counts)[item], q.list_cap));
        const PG_GLOBAL uint32_t* src = glb(q.list_docs + (uint64_t)item * q.list_cap);
        for (uint32_t c0 = 0; c0 < n;) {
          const uint32_t take = min(n - c0, (uint32_t)kQueueCap - qn);
          for (uint32_t k = tid; k < take; k += kBlock) queue[qn + k] = src[c0 + k];
          qn += take;
          c0 += take;
          if (qn >= (uint32_t)kQueueFlush) flush();
        }
        if (++item >= i1) break;
        it = ldc(q.items, item);
      }
      if (qn) flush();
      const uint64_t c = wave_sum_u64(seg_count);
      if (lane == 0 && c) g_add(&q.seg_matched[cur_seg], (unsigned long long)c);
    } else {
    if (q.num_staged) stage_issue(q, cur_sd, tile, stage, wave, lane);
    for (;;) {
      // successor of (item, tile) in the block's sequence
      uint32_t n_item = item, n_tile = tile + 1, n_seg = it.seg;
      bool has_next = true;
      WorkItem n_it = it;
      if (n_tile >= it.tile_end) {
        n_item = item + 1;
        has_next = n_item < i1;
        if (has_next) { n_it = ldc(q.items, n_item); n_tile = n_it.tile_begin; n_seg = n_it.seg; }
      }
      __builtin_amdgcn_s_waitcnt(0);  // this wave's copies of the current tile have landed
      const bool poll = q.cancel && (iter & (kPollTiles - 1u)) == 0;
      const uint32_t k = iter / kPollTiles;
      if (poll && tid == 0) stop[k & 1u] = pending;  // loaded at poll k - 1: no wait on the PCIe round trip here
      __syncthreads();                // ... and every wave's; every wave is done with the other buffer
      if (poll) {
        // word (k & 1) is read by every wave after this barrier and rewritten only at poll k + 2
        if (__builtin_amdgcn_readfirstlane(stop[k & 1u])) has_next = false;  // finish this tile, then leave
        if (tid == 0) pending = __hip_atomic_load(q.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      iter++;
      if (it.seg != cur_seg) enter_segment(it.seg);
      const SegDesc& sd = cur_sd;
      if (ring2 && has_next && q.num_staged) stage_issue(q, ldc(q.segs, n_seg), n_tile, stage + (buf ^ 1u) * q.stage_lds_words, wave, lane);

      const uint32_t* st = stage + buf * q.stage_lds_words;
      const uint32_t base = tile * (uint32_t)kTileDocs;
      const uint32_t nd = sd.num_docs;
      uint32_t valid = kRowMask;
      if (base + (uint32_t)kTileDocs > nd) {
        valid = 0;
#pragma unroll
        for (int j = 0; j < kRows; j++) valid |= (uint32_t)(base + (uint32_t)(j * kBlock + tid) < nd) << j;
      }
      const TileRows rows{base, (uint32_t)tid};
      uint32_t m = eval_filter(q, sd.leaves, q.opA_begin, q.opA_end, q.opA_type, lds_sets, st, valid, rows, tid);
      bool direct = !q.queue_mode;
      if (q.queue_mode) {
        // compact the phase-A survivors into the queue (block-wide exclusive scan of per-thread counts)
        const uint32_t cnt = __popc(m);
        uint32_t x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(x, o);
          if (lane >= (uint32_t)o) x += y;
        }
        if (lane == 63) scan_tmp[wave] = x;
        __syncthreads();
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; w++) {
          const uint32_t t = scan_tmp[w];
          wbase += (uint32_t)w < wave ? t : 0u;
          tot += t;
        }
        if (tot > (uint32_t)kQueueCap) {
          direct = true;  // a dense tile: finish it in place
          m = eval_filter(q, sd.leaves, q.opB_begin, q.opB_end, GT_AND, lds_sets, st, m, rows, tid);
        } else if (tot) {
          if (qn + tot > (uint32_t)kQueueCap) flush();
          uint32_t pos = qn + wbase + x - cnt;
          for (uint32_t r = m; r; r &= r - 1u) queue[pos++] = rows.doc((uint32_t)__ffs(r) - 1u);
          qn += tot;
          if (qn >= (uint32_t)kQueueFlush) flush();
        }
      }
      if (direct) {
        const uint32_t nm = __popc(m);
        seg_count += nm;
        if (!GROUPED) doc_count += nm;
        if (GROUPED || q.agg_reads) {
          // dense when at least a quarter of the lanes hold >= 8 matches: batched rows; else per-doc rounds
          if (__popcll(__ballot(nm >= 8)) >= 16 && (!GROUPED || !q.mv_keys) && !q.mv_aggs)
            aggregate_dense<GROUPED, MAXA, MAXK>(q, sd, S, st, acc, m, base, tid);
          else aggregate_tile<GROUPED, MAXA, MAXK>(q, sd, S, st, acc, m, rows);
        }
      }
      if (!has_next) break;
      if (!ring2 && q.num_staged) {
        __syncthreads();  // every wave is done with the single buffer
        stage_issue(q, ldc(q.segs, n_seg), n_tile, stage, wave, lane);
      }
      item = n_item;
      it = n_it;
      tile = n_tile;
      if (ring2) buf ^= 1u;
    }
    if (qn && !(q.cancel && (stop[0] | stop[1]))) flush();
    const uint64_t c = wave_sum_u64(seg_count);
    if (lane == 0 && c) g_add(&q.seg_matched[cur_seg], (unsigned long long)c);
    }  // tile loop
  }

  if (!GROUPED) {
    // wave-reduce, then the block's waves combine through LDS: one global atomic per block per slot
    __syncthreads();  // the staging ring is free
    uint64_t* red = (uint64_t*)stage;  // [wave][1 + MAXA]
    constexpr int RW = 1 + MAXA;
    const uint64_t dc = wave_sum_u64(doc_count);
    if (lane == 0) red[wave * RW] = dc;
#pragma unroll
    for (int a = 0; a < MAXA; a++) {
      if (a >= (int)q.num_aggs) break;
      uint64_t v = 0;
      switch (q.aggs[a].kind) {
        case SK_I64: v = wave_sum_u64(acc[a]); break;
        case SK_MIN: v = (uint64_t)wave_min_i64((int64_t)acc[a]); break;
        case SK_MAX: v = (uint64_t)wave_max_i64((int64_t)acc[a]); break;
        default: break;  // SK_FX: the LDS slot below
      }
      if (lane == 0) red[wave * RW + 1 + a] = v;
    }
    __syncthreads();
    constexpr int NW = kBlock / 64;
    if (tid == 0) {
      uint64_t t = 0;
      for (int w = 0; w < NW; w++) t += red[w * RW];
      if (t) atomicAdd(&q.i64[0], (unsigned long long)t);
    } else if (tid <= MAXA && tid <= (int)q.num_aggs) {
      const int a = tid - 1;
      const AggSpec& A = q.aggs[a];
      switch (A.kind) {
        case SK_I64: {
          uint64_t t = 0;
          for (int w = 0; w < NW; w++) t += red[w * RW + 1 + a];
          if (t) atomicAdd(&q.i64[A.slot], (unsigned long long)t);
          break;
        }
        case SK_MIN: {
          int64_t t = (int64_t)red[1 + a];
          for (int w = 1; w < NW; w++) t = min(t, (int64_t)red[w * RW + 1 + a]);
          atomicMin(&q.mn[A.slot], (long long)t);
          break;
        }
        case SK_MAX: {
          int64_t t = (int64_t)red[1 + a];
          for (int w = 1; w < NW; w++) t = max(t, (int64_t)red[w * RW + 1 + a]);
          atomicMax(&q.mx[A.slot], (long long)t);
          break;
        }
        default: break;
      }
    }
    if (q.use_lds && tid == 0) {  // the one-slot LDS table: SK_FX sums and their special slots, AVGMV value counts
      for (uint32_t s = 1; s < q.n_i64; s++)
        if (l_i64[s]) atomicAdd(&q.i64[s], l_i64[s]);
      for (uint32_t s = 0; s < q.n_fx; s++)
        if (l_fx[2 * s] | l_fx[2 * s + 1]) g_addfx(&q.fx[2 * s], l_fx[2 * s], l_fx[2 * s + 1]);
      for (uint32_t s = 0; s < q.n_min; s++) atomicMin(&q.mn[s], l_mn[s]);
      for (uint32_t s = 0; s < q.n_max; s++) atomicMax(&q.mx[s], l_mx[s]);
    }
  } else if (part) {
    __syncthreads();
    const uint32_t* h = (const uint32_t*)lds_groups;
    for (uint32_t p = tid; p < q.part_nparts; p += kBlock) q.part_hist[(uint64_t)p * gridDim.x + blockIdx.x] = h[1 + p];
    if (tid == 0) q.part_count[blockIdx.x] = h[0];
  } else if (q.use_lds) {
    __syncthreads();
#ifdef PG_LIST_FLUSH_SKIP  // dev ablation only (wrong results): the block's table is not added to the global state
    if (q.list_mode) return;
#endif
    for (uint64_t g = tid; g < q.num_slots; g += kBlock) {
      if (l_i64[g * q.n_i64] == 0) continue;
      for (uint32_t s = 0; s < q.n_i64; s++) {
        const unsigned long long v = l_i64[g * q.n_i64 + s];
        if (v) atomicAdd(&q.i64[g * q.n_i64 + s], v);
      }
      for (uint32_t s = 0; s < q.n_fx; s++) {
        const uint64_t lo = l_fx[(g * q.n_fx + s) * 2], hi = l_fx[(g * q.n_fx + s) * 2 + 1];
        if (lo | hi) g_addfx(&q.fx[(g * q.n_fx + s) * 2], lo, hi);
      }
      for (uint32_t s = 0; s < q.n_min; s++) atomicMin(&q.mn[g * q.n_min + s], l_mn[g * q.n_min + s]);
      for (uint32_t s = 0; s < q.n_max; s++) atomicMax(&q.mx[g * q.n_max + s], l_mx[g * q.n_max + s]);
    }
  }
}

template <bool GROUPED, int MAXA, int MAXK>
__global__ __launch_bounds__(kBlock, GROUPED ? PG_SCAN_MIN_WAVES : PG_SCAN_MIN_WAVES_AGG) void scan_kernel(QuerySpec qarg) {
  (void)qarg;
  scan_body<GROUPED, MAXA, MAXK>();
}
// The same body under a 128-VGPR budget (4 waves / SIMD): a list-mode launch that runs beside the exact-mode stream
// kernel (4 waves x 96 VGPRs per SIMD) fits the SIMD's remaining 128 registers, so the two overlap on every CU.
template <bool GROUPED, int MAXA, int MAXK>
__global__ __launch_bounds__(kBlock, 4) void scan_kernel_co(QuerySpec qarg) {
  (void)qarg;
  scan_body<GROUPED, MAXA, MAXK>();
}

template <bool G, int A, int K>
void launch_one(const QuerySpec& q, uint32_t blocks, size_t lds, hipStream_t s, bool co) {
  if constexpr (G && A == 2 && K == 1) {  // the one grouped shape with a co-resident variant (config 2's list scan)
    if (co) {
      hipLaunchKernelGGL((scan_kernel_co<G, A, K>), dim3(blocks), dim3(kBlock), lds, s, q);
      return;
    }
  }
  hipLaunchKernelGGL((scan_kernel<G, A, K>), dim3(blocks), dim3(kBlock), lds, s, q);
}

// Each (grouped, aggs, keys) shape is compiled in its own translation unit (the Makefile builds this file once per
// PG_SCAN_SHARD = 0..8 plus once without it for the dispatcher), so the nine kernel bodies build in parallel.
#define PG_SCAN_SHAPES(X)                                                                                           \
  X(0, false, 2, 0) X(1, false, 4, 0) X(2, false, kMaxAggs, 0) X(3, true, 2, 1) X(4, true, 4, 1)                    \
  X(5, true, kMaxAggs, 1) X(6, true, 2, kMaxKeys) X(7, true, 4, kMaxKeys) X(8, true, kMaxAggs, kMaxKeys)

#ifdef PG_SCAN_SHARD
#if PG_SCAN_SHARD == 0
template void launch_one<false, 2, 0>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 1
template void launch_one<false, 4, 0>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 2
template void launch_one<false, kMaxAggs, 0>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 3
template void launch_one<true, 2, 1>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 4
template void launch_one<true, 4, 1>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 5
template void launch_one<true, kMaxAggs, 1>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 6
template void launch_one<true, 2, kMaxKeys>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 7
template void launch_one<true, 4, kMaxKeys>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#elif PG_SCAN_SHARD == 8
template void launch_one<true, kMaxAggs, kMaxKeys>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
#endif
#else
#define PG_SCAN_EXTERN(i, G, A, K) \
  extern template void launch_one<G, A, K>(const QuerySpec&, uint32_t, size_t, hipStream_t, bool);
PG_SCAN_SHAPES(PG_SCAN_EXTERN)

bool scan_co_resident(const QuerySpec& q) {  // shapes whose launch fits beside the exact-mode stream kernel
  static_assert(PG_SCAN_MIN_WAVES_AGG >= 4, "the aggregation-only 2-aggregation shape runs within 128 VGPRs as is");
  return q.num_aggs <= 2 && q.num_keys <= 1;
}

// LDS of a launch: staging ring | IN sets | group table; at least the aggregation-only block reduction's
// [4][1 + kMaxAggs] words, which reuses the ring.
size_t scan_lds_bytes(const QuerySpec& q) {
  size_t lds = scan_queue_off(q) + (q.queue_mode ? (kQueueCap + 4) * 4 : 0);
  const size_t red = 16 + (size_t)(kBlock / 64) * (1 + kMaxAggs) * 8;  // the IN sets are dead by then: may overlap
  if (lds < red) lds = red;
  return (lds + 15) & ~(size_t)15;
}

uint32_t scan_min_blocks_per_cu(bool grouped) {  // 256-thread blocks: waves/SIMD == blocks/CU
  return grouped ? PG_SCAN_MIN_WAVES : PG_SCAN_MIN_WAVES_AGG;
}

hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s, bool co) {
  const size_t lds = scan_lds_bytes(q);
  // multi-value keys / aggregations: the widest shapes, the only ones compiled with those paths
  const uint32_t na = (q.mv_keys || q.mv_aggs) ? (uint32_t)kMaxAggs : q.num_aggs;
  if (q.num_keys == 0) {
    if (na <= 2) launch_one<false, 2, 0>(q, blocks, lds, s, co);
    else if (na <= 4) launch_one<false, 4, 0>(q, blocks, lds, s, co);
    else launch_one<false, kMaxAggs, 0>(q, blocks, lds, s, co);
  } else if (q.num_keys == 1) {
    if (na <= 2) launch_one<true, 2, 1>(q, blocks, lds, s, co);
    else if (na <= 4) launch_one<true, 4, 1>(q, blocks, lds, s, co);
    else launch_one<true, kMaxAggs, 1>(q, blocks, lds, s, co);
  } else {
    if (na <= 2) launch_one<true, 2, kMaxKeys>(q, blocks, lds, s, co);
    else if (na <= 4) launch_one<true, 4, kMaxKeys>(q, blocks, lds, s, co);
    else launch_one<true, kMaxAggs, kMaxKeys>(q, blocks, lds, s, co);
  }
  return hipGetLastError();
}
#endif  // PG_SCAN_SHARD

}  // namespace pg
