// pg_internal.h -- device-side data layout and kernel interface of libpinot_gpu (gfx950 only).
//
// HBM layout of a resident segment column (built once by pg_column_upload):
//   * bit-packed forward index   : the reference's big-endian stream re-laid as native uint32 words
//                                  (byte-swapped per 32-bit word), so bit p of the stream is bit
//                                  31-(p&31) of word p>>5.  +4 zero words of tail padding so the 64-bit
//                                  window read of the last value never leaves the allocation.
//                                  Sorted columns get the same packed stream synthesised from their
//                                  (start,end) pairs, so every column is readable per doc.
//   * dictionary                 : native typed array (int32 / int64 / float / double).
//   * MV forward index           : packed values as above + uint32 row offsets[num_docs+1]
//                                  (selected once from the start-of-row bitmap).
//   * inverted index             : roaring bytes kept as-is (compressed in HBM) + a container
//                                  directory (per dictId CSR of {key, type, card, offset}).
// Per query, ONE parameter arena (one pinned H2D copy) holds the per-segment tables the scan kernel
// reads: SegDesc[seg], LeafDesc[seg][leaf], ColDesc[seg][agg*2 | key], WorkItem[item], the hash sets of
// IN / NOT_IN leaves (staged into LDS by the kernel) and sorted-index doc ranges.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pinot_gpu.h"

namespace pg {

constexpr int kBlock = 256;                          // 4 waves of 64
constexpr int kRows = 32;                            // docs of a thread in a tile: base + j*256 + tid (32-bit masks)
constexpr int kChunk = 8;                            // rows gathered per straight-line batch
constexpr int kTileDocs = kBlock * kRows;            // 8192 docs per tile
constexpr int kItemTiles = 4;                        // tiles per work item (32 768 docs), within one segment
constexpr int kMaxAggs = 8;
constexpr int kMaxKeys = 8;
constexpr int kMaxLeaves = 24;
constexpr int kMaxOps = 64;
constexpr int kMaxDepth = 4;                         // filter tree nesting (open groups)
constexpr int kLdsGroupBytes = 32 * 1024;            // LDS-privatised group table budget
constexpr int kLdsSetBytes = 16 * 1024;              // LDS filter bitmaps of IN / NOT_IN leaves
constexpr int kLdsStageBytes = 40 * 1024;            // LDS tiles of densely read packed columns (per ring buffer; config 4 stages 23 + 10 bits: 19.2 -> 16.3 ms)
constexpr int kMaxStaged = 6;                        // packed columns staged per tile
constexpr int kNoSlot = 255;
constexpr uint32_t kPollTiles = 2;                   // scan tiles between polls of the cancel / deadline flag

// Filter program as the kernel runs it: a tree in prefix form (host-compiled from the ABI's postfix program,
// AND children ordered most-selective first so later children are evaluated only on surviving docs).
constexpr int32_t kOpAnd = -1, kOpOr = -2, kOpNot = -3, kOpEnd = -4;  // >= 0: leaf index
enum GroupType : uint32_t { GT_ROOT = 0, GT_AND = 1, GT_OR = 2, GT_NOT = 3 };

// Compaction queue (QuerySpec::queue_mode): docs that pass the staged (phase A) children of a root AND are appended
// to a per-block LDS queue; the remaining children and the aggregation run over the queue once it holds at least
// kQueueFlush docs (every lane busy) instead of over a few docs per tile.
constexpr int kQueueRows = 4;
constexpr int kQueueCap = kBlock * kQueueRows;       // 1024 docs
constexpr int kQueueFlush = kBlock * 2;              // flush at >= 512 queued docs

enum LeafKind : uint32_t {
  LK_ALL = 0,        // match all
  LK_NONE = 1,       // match none
  LK_RANGE = 2,      // dictId in [lo,hi), dictIds unpacked from a packed SV forward index
  LK_SET_LDS = 3,    // dictId in set: LDS filter bitmap staged per segment (+ exact global LUT when coarse)
  LK_SET_LUT = 4,    // dictId in set: bit dictId of `aux` (global LSB-first words)
  LK_DOCRANGE = 6,   // doc id in [lo,hi)
  LK_RAW = 7         // raw value of the doc (`words` = typed values, rtype) in [ilo, ihi] / (dlo, dhi) / rvals set
};

struct LeafDesc {
  uint32_t kind;
  uint32_t excl;      // invert the leaf (NOT_EQ / NOT_IN on a scan)
  int32_t lo, hi;
  const uint32_t* words;  // packed forward words (RANGE / SET_*); doc bitmaps are 1-bit columns
  const uint32_t* aux;    // SET_LUT bitmap / SET_LDS source region (global)
  uint32_t bits;
  uint32_t wbytes;        // bytes of `words` (buffer-descriptor range)
  // SET_LDS: an LDS region of `set_ints` words at `lds_off`: a filter bitmap of `nbw` words over dictId >> shift
  // (LSB-first).  shift == 0: the bitmap is exact; else its candidates are resolved by bit dictId of `lut`
  // (global, LSB-first words, built per query by set_lut_bits).
  uint32_t lds_off;
  uint32_t set_ints;
  uint32_t shift;
  uint32_t nbw;
  const uint32_t* lut;
  // LK_RAW: INT / LONG in [ilo, ihi]; FLOAT / DOUBLE in (dlo, dhi) with rflags bit 0 / 1 = inclusive lo / hi; with
  // nvals > 0, membership in rvals (nvals sorted int64 for INT / LONG, double for FLOAT / DOUBLE)
  int64_t ilo, ihi;
  double dlo, dhi;
  uint32_t rtype, rflags, nvals, pad;
  const uint32_t* rvals;
};

// A column as read by aggregation inputs and group keys.  `decoded`: `words` is the column's decoded forward index
// (value - vbase per doc, launch_decode_pack) instead of dictIds, and the "dictionary" is v -> vbase + v.
struct ColDesc {
  const uint32_t* words;      // packed SV forward words
  const void* dict;           // typed dictionary values
  const int32_t* keymap;      // dictId -> global key (PG_KEY_KEYMAP)
  const uint32_t* mv_offsets; // MV: row offsets [num_docs+1]
  uint32_t bits;
  uint32_t dtype;             // pg_data_type
  uint32_t card;
  uint32_t wbytes;            // bytes of `words` (buffer-descriptor range)
  int64_t vbase;
  uint32_t decoded;
  uint32_t identity;          // decoded from an identity dictionary: `words` are the column's dictIds (host-side flag)
};

struct SegDesc {
  uint32_t num_docs;
  uint32_t index;           // segment index within the plan (GM_HASH_SEG keys)
  const LeafDesc* leaves;   // [num_leaves]
  const ColDesc* aggcols;   // [num_aggs][2]
  const ColDesc* keycols;   // [num_keys]
};

struct WorkItem {
  uint32_t seg;
  uint32_t tile_begin, tile_end;  // tiles of kTileDocs docs within the segment
  uint32_t pad;
};

// SK_FX: a SUM / AVG whose inputs are not provably integer accumulates EXACTLY, as a 128-bit two's-complement
// fixed-point number (lo, hi words of the `fx` state array) in units of 2^fx_shift (see fx_from_double): integer adds
// are associative, so the sum has the same bits whatever the order of the atomics, the grid, the number of GPUs or the
// merge order -- the reference's double sum depends on its thread scheduling.
enum SlotKind : uint32_t { SK_NONE = 0, SK_I64 = 1, SK_FX = 2, SK_MIN = 3, SK_MAX = 4, SK_BITS = 5 };

// Group state addressing (QuerySpec::group_mode):
//   GM_NONE     aggregation-only: one slot (0).
//   GM_DENSE    slot = packed key (mixed radix of table-global key ids, first key least significant);
//               LDS-privatised per block when the whole table fits (use_lds).
//   GM_HASH     open-addressing table of 2^k packed keys (linear probing, PG_EMPTY_KEY = free), slot = the
//               key's table position; keys are claimed with one 64-bit CAS (IntGroupIdMap on the device).
//   GM_HASH_SEG as GM_HASH over (packed key * num_segments + segment), with the first matching doc of every
//               (segment, key) in first_doc: the per-segment table when numGroupsLimit can truncate a segment
//               (the runtime then keeps, per segment, the limit keys seen first and merges them by key).
//   GM_PART     radix-partitioned dense group-by (pg_part.hip) for key spaces whose state is far larger than any
//               cache: the scan only appends one 64-bit entry (packed key << part_vbits | value id) per matching doc to
//               its block's region of an entry array (coalesced, LDS-atomic cursor) and counts it in the block's
//               histogram of level-1 partitions; pg_part.hip partitions the entries twice (LDS counting sorts,
//               coalesced runs) and aggregates each bucket in LDS into GM_DENSE's state layout.
enum GroupMode : uint32_t { GM_NONE = 0, GM_DENSE = 1, GM_HASH = 2, GM_HASH_SEG = 3, GM_PART = 4 };
constexpr unsigned long long kEmptyKey = 0xFFFFFFFFFFFFFFFFull;

#ifdef __HIPCC__  // (hipcc only: a plain C++ build of this header, as the fixed-point test does, skips it)
// A load through a generic pointer that points to global memory, issued as a global load.  A pointer the compiler
// cannot trace to a kernel argument (one read back from LDS, or from a table in memory) is generic, and its loads
// compile to flat loads -- which also count in lgkmcnt, so every later LDS wait (a barrier, a ds_read's use) waits
// for them too: prefetches issued through such pointers would land before the LDS work they were meant to overlap.
template <typename T>
__device__ __forceinline__ T ld_global(const T* p) {
#ifdef __HIP_DEVICE_COMPILE__
  return *(const __attribute__((address_space(1))) T*)p;
#else
  return *p;  // (the host pass only parses device code)
#endif
}
// (HIP's uint2 / uint4 copy through a constructor taking a generic reference, which would turn the load flat again:
// load them as plain vectors)
__device__ __forceinline__ uint2 ld_global(const uint2* p) {
  typedef unsigned int v2u __attribute__((ext_vector_type(2)));
  const v2u v = *(const __attribute__((address_space(1))) v2u*)p;
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint4 ld_global(const uint4* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = *(const __attribute__((address_space(1))) v4u*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
#endif

__host__ __device__ inline uint64_t mix64(uint64_t x) {  // murmur3 fmix64 (the HashCommon.mix role)
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct AggSpec {
  uint32_t fn;        // pg_agg_fn
  uint32_t op;        // pg_expr_op
  uint32_t kind;      // SlotKind of the primary slot
  uint32_t slot;      // primary slot index within its array
  uint32_t cnt_slot;  // AVG count slot (i64)
  uint32_t integer;   // SUM/AVG inputs integer-exact -> i64 accumulate
  uint32_t key_kind;  // DISTINCTCOUNT: pg_key_kind of its value ids
  uint32_t key_card;  // DISTINCTCOUNT: size of the table-global value id space (bits of its bitmap)
  int64_t key_base;
  uint32_t dc_word;   // DISTINCTCOUNT: first uint32 word of this aggregation's bitmap within a slot's row
  int32_t fx_shift;   // SK_FX: the unit of window 0 is 2^fx_shift (fx_split)
  // SK_FX over a column that may hold +-inf / NaN: mn / mx slots that receive the order images of the non-finite
  // inputs (the fixed-point sum skips them), so that finalisation gives IEEE's sum of them (fx_final); else kNoSp
  uint32_t sp_min, sp_max;
  uint32_t fx_nwin;   // SK_FX: exponent windows = consecutive fx slots slot .. slot + fx_nwin - 1 (fx_split)
  uint32_t mv;        // PG_AGG_MV_VALUES: fn over every value of the doc's list in the MV column (AVG: cnt_slot counts
                      // the values; 0 = the doc count in slot 0)
};
constexpr uint32_t kNoSp = 0xFFFFFFFFu;

// A packed column staged per tile into LDS (LDS-DMA of the tile's whole word range in 1 KiB pieces) because
// most of its cache lines are needed anyway; every other read of a packed column is a per-doc gather.
// Source = the words of a leaf (role 0), an aggregation operand (role 1) or a group key (role 2) of the current
// segment.  Slots are uniform across segments; `lds_words` is sized for the widest bitsPerElement.
struct StagedCol {
  uint32_t role, idx, operand;
  uint32_t lds_word_off;     // offset of this slot in a staging buffer (uint32 words, multiple of 256)
};

struct QuerySpec {
  uint32_t num_segments, num_leaves, num_ops, num_aggs, num_keys, num_items;
  uint32_t agg_reads;        // some aggregation reads a column (else COUNT(*) only: matched-doc counts suffice)
  uint32_t use_lds;          // group table privatised in LDS
  uint32_t set_lds_ints;     // int32 slots of LDS hash sets per block
  uint32_t num_staged;
  uint32_t stage_lds_words;  // uint32 words of one staging buffer (a multiple of 256: 1 KiB DMA pieces)
  uint32_t stage_ring;       // staging buffers (2: the next tile is copied while the current one is evaluated)
  uint32_t queue_mode;       // phase A per tile -> LDS queue -> phase B per flush (see kQueueCap)
  uint32_t opA_begin, opA_end, opA_type;  // phase A ops (the whole program as GT_ROOT when queue_mode == 0)
  uint32_t opB_begin, opB_end;            // phase B ops: the root AND's remaining children
  StagedCol staged[kMaxStaged];
  uint8_t leaf_slot[kMaxLeaves];     // staged slot of each leaf's column or kNoSlot
  uint8_t agg_slot[kMaxAggs][2];     // staged slot of each aggregation operand or kNoSlot
  uint8_t key_slot[kMaxKeys];        // staged slot of each group key column or kNoSlot
  int32_t ops[kMaxOps];
  AggSpec aggs[kMaxAggs];
  uint32_t key_kind[kMaxKeys];
  uint32_t key_card[kMaxKeys];
  int64_t key_base[kMaxKeys];
  uint64_t key_stride[kMaxKeys];
  uint32_t group_mode;       // GroupMode
  uint32_t hmax_fill;        // GM_HASH*: keys claimed before the table reports overflow (err bit 4)
  uint64_t num_slots;        // dense: key space size; hash: table capacity (a power of two)
  uint64_t hmask;            // hash: num_slots - 1
  uint32_t n_i64, n_fx, n_min, n_max;  // n_fx: SK_FX slots, 2 words each
  uint32_t dc_row_words;     // uint32 words of DISTINCTCOUNT bitmaps per slot
  uint32_t mv_keys;          // bit k: group key k is multi-value (a doc joins the group of each tuple of the
                             // cartesian product of its MV keys' lists); 0: no multi-value group key
  uint32_t mv_aggs;          // bit a: aggregation a reads every value of an MV column (AggSpec.mv)
  unsigned long long* i64;
  unsigned long long* fx;    // [num_slots][n_fx][2] (lo, hi)
  long long* mn;
  long long* mx;
  uint32_t* dbits;           // [num_slots][dc_row_words]
  unsigned long long* hkeys; // GM_HASH*: [num_slots] packed keys
  unsigned int* hfill;       // GM_HASH*: claimed keys
  unsigned long long* first_doc;  // GM_HASH_SEG: [num_slots] first-seen order of the (segment, key): first matching
                                  // doc << 16 | the key's position among that doc's multi-value key tuples (0: SV keys)
  const SegDesc* segs;       // [seg]
  const WorkItem* items;     // [item]
  unsigned long long* seg_matched;  // [seg]
  unsigned int* err;                // device-side violations: bit 0 group key, bit 1 DISTINCTCOUNT key, bit 2 hash table full
  const unsigned int* cancel;       // host-mapped flag polled once per tile (nonzero: stop); null = not cancellable
  // GM_PART: level-1 partition of packed key g = g >> part_shift (< part_nparts); entry = g << part_vbits | value id
  // of aggregation part_dc (0 when part_dc == kNoSlot: COUNTs only)
  uint32_t part_shift, part_vbits, part_nparts, part_dc;
  unsigned long long* part_hist;    // [part_nparts][gridDim.x] entries per (level-1 partition, block)
  unsigned int* part_count;         // [gridDim.x] entries of each block
  const unsigned long long* part_base;  // [gridDim.x] first entry of each block's region (its docs: an upper bound)
  unsigned long long* part_out;     // the entry array
  // list mode (stream_kernel ran first): `items` are the stream's items and item i's survivors of the driving leaf
  // are list_docs[i * list_cap, + list_counts[i]); the kernel feeds them to the LDS queue (phase B = the rest of the
  // root AND, then aggregation) instead of walking tiles
  uint32_t list_mode, list_cap;
  const uint32_t* list_docs;
  const uint32_t* list_counts;
};

// order-preserving int64 image of a double (for MIN/MAX slots)
__host__ __device__ inline int64_t order_key(double v) {
  int64_t b;
  __builtin_memcpy(&b, &v, 8);
  return b >= 0 ? b : (b ^ 0x7FFFFFFFFFFFFFFFLL);
}
__host__ __device__ inline double order_key_decode(int64_t k) {
  int64_t b = k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFLL);
  double v;
  __builtin_memcpy(&v, &b, 8);
  return v;
}

// ---- exact fixed-point sums (SK_FX)
// Every finite input is converted EXACTLY: a double is m * 2^q (m < 2^53 an integer, q = its last mantissa bit's
// exponent), and the host bounds every nonzero finite input of the plan by 2^klo <= |x| <= 2^khi (the columns'
// smallest nonzero and largest |value|, combined through the expression), so q lies in [u0, qmax] with
// u0 = max(klo - 52, -1074) and qmax = khi - 52.  That exponent range is cut into windows of kFxWinBits exponents:
// window w holds the inputs with q - u0 in [32w, 32w + 32), as the 128-bit two's-complement integer x / 2^(u0 + 32w) =
// m * 2^(q - u0 - 32w) < 2^85, so 2^40 inputs sum within 126 bits (no overflow for any table this library can hold).
// Each window is one fx slot (consecutive slots of the aggregation); integer adds are associative, and the final value
// is the windows' exact total rounded once to the nearest double (fx_windows_to_double): the correctly rounded sum of
// the inputs, for any range of magnitudes (64 windows cover every finite double) and in every order.
constexpr int kFxWinBits = 32;
constexpr int kFxMaxWin = 64;
__host__ __device__ inline int32_t fx_u0(int32_t klo) { return klo - 52 < -1074 ? -1074 : klo - 52; }
__host__ __device__ inline uint32_t fx_num_windows(int32_t klo, int32_t khi) {
  const int32_t u0 = fx_u0(klo), qmax = khi - 52;
  return qmax <= u0 ? 1u : (uint32_t)((qmax - u0) / kFxWinBits + 1);
}

// x / 2^shift rounded to nearest (ties to even) as a 128-bit two's-complement integer; 0 for +-inf / NaN (those are
// tracked apart, AggSpec::sp_min / sp_max).  Exact whenever x's last mantissa bit is at or above 2^shift.
__host__ __device__ inline void fx_from_double(double x, int32_t shift, uint64_t& lo, uint64_t& hi) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  int e = (int)((b >> 52) & 0x7FF);
  uint64_t m = b & ((1ull << 52) - 1);
  lo = hi = 0;
  if (e == 0x7FF) return;
  if (e == 0) e = 1; else m |= 1ull << 52;
  if (!m) return;
  const int sh = e - 1075 - shift;  // x = m * 2^(e - 1075) = m * 2^sh units
  if (sh >= 0) {
    if (sh >= 128) return;  // outside the range the host's bound allows (never for valid plans)
    if (sh >= 64) { hi = m << (sh - 64); }
    else if (sh == 0) { lo = m; }
    else { lo = m << sh; hi = m >> (64 - sh); }
  } else {
    const int r = -sh;
    if (r > 54) return;  // below half a unit: m < 2^53 <= 2^(r - 1)
    uint64_t q = m >> r;
    const uint64_t rem = m & ((1ull << r) - 1), half = 1ull << (r - 1);
    if (rem > half || (rem == half && (q & 1))) q++;
    lo = q;
  }
  if (b >> 63) {  // negate
    lo = ~lo + 1;
    hi = ~hi + (lo == 0 ? 1 : 0);
  }
}

// The window of a finite input x (see above) and its exact value in that window's unit 2^(u0 + 32 w).  Zero, +-inf and
// NaN give (0, 0) in window 0.  An input outside the host's bounds (never for a validated plan) lands in the nearest
// window, rounded below it or shifted further above it.
__host__ __device__ inline uint32_t fx_split(double x, int32_t u0, uint32_t nwin, uint64_t& lo, uint64_t& hi) {
  uint64_t b;
  __builtin_memcpy(&b, &x, 8);
  const int e = (int)((b >> 52) & 0x7FF);
  const int d = (e ? e : 1) - 1075 - u0;  // q - u0
  if (e == 0x7FF || d < 0) {
    fx_from_double(x, u0, lo, hi);
    return 0;
  }
  uint32_t w = (uint32_t)d / kFxWinBits;
  if (w >= nwin) w = nwin - 1;
  fx_from_double(x, u0 + kFxWinBits * (int32_t)w, lo, hi);  // exact: x's last bit is at or above the window's unit
  return w;
}

// (lo, hi) * 2^shift as the nearest double (ties to even; exact integer rounding of the 128-bit value, then one exact
// scaling -- the same bits on the host and on the device)
__host__ __device__ inline double fx_to_double(uint64_t lo, uint64_t hi, int32_t shift) {
  const bool neg = (int64_t)hi < 0;
  if (neg) {
    lo = ~lo + 1;
    hi = ~hi + (lo == 0 ? 1 : 0);
  }
  if (!hi && !lo) return 0.0;
  const int nb = hi ? 128 - __builtin_clzll(hi) : 64 - __builtin_clzll(lo);  // significant bits
  uint64_t mant;
  int exp2 = 0;
  if (nb <= 53) {
    mant = lo;
  } else {
    const int r = nb - 53;  // 1..75 bits dropped
    mant = r >= 64 ? hi >> (r - 64) : ((lo >> r) | (hi << (64 - r)));
    const int rb = r - 1;   // the rounding bit; sticky = any bit below it
    const uint64_t round = rb >= 64 ? (hi >> (rb - 64)) & 1 : (lo >> rb) & 1;
    bool sticky;
    if (rb >= 64) sticky = lo != 0 || (rb > 64 && (hi & ((1ull << (rb - 64)) - 1)) != 0);
    else sticky = rb > 0 && (lo & ((1ull << rb) - 1)) != 0;
    if (round && (sticky || (mant & 1))) mant++;  // may carry to 2^53: still exact as a double
    exp2 = r;
  }
  const double d = __builtin_ldexp((double)mant, exp2 + shift);
  return neg ? -d : d;
}

// 128-bit add of (blo, bhi) into (lo, hi)
__host__ __device__ inline void fx_add(uint64_t& lo, uint64_t& hi, uint64_t blo, uint64_t bhi) {
  const uint64_t t = lo + blo;
  hi += bhi + (t < lo ? 1 : 0);
  lo = t;
}

// The exact total of nwin windows (p[2w], p[2w + 1] = window w's 128-bit sum in units of 2^(u0 + 32 w)) rounded once
// to the nearest double (ties to even): the windows are added into one two's-complement integer of up to 35 64-bit
// limbs in units of 2^u0, whose top 53 significant bits (rounded with the bits below) are the result.
constexpr int kFxLimbs = (kFxWinBits * (kFxMaxWin - 1) + 128) / 64 + 2;
__host__ __device__ inline double fx_windows_to_double(const uint64_t* p, uint32_t nwin, int32_t u0) {
  if (nwin <= 1) return fx_to_double(p[0], p[1], u0);
  if (nwin > (uint32_t)kFxMaxWin) nwin = kFxMaxWin;
  uint64_t L[kFxLimbs];
  const int n = (kFxWinBits * ((int)nwin - 1) + 128) / 64 + 2;
  for (int i = 0; i < n; i++) L[i] = 0;
  for (uint32_t w = 0; w < nwin; w++) {
    const uint64_t lo = p[2 * w], hi = p[2 * w + 1];
    if (!lo && !hi) continue;
    const uint64_t sgn = (int64_t)hi < 0 ? ~0ull : 0ull;
    const int bit = kFxWinBits * (int)w, k = bit / 64, s = bit % 64;  // s is 0 or 32
    uint64_t x[3];
    if (s) {
      x[0] = lo << s;
      x[1] = (hi << s) | (lo >> (64 - s));
      x[2] = (uint64_t)((int64_t)hi >> (64 - s));
    } else {
      x[0] = lo; x[1] = hi; x[2] = sgn;
    }
    uint64_t c = 0;
    for (int i = k; i < n; i++) {
      const uint64_t a = i - k < 3 ? x[i - k] : sgn;
      const uint64_t t = L[i] + a, c1 = t < a, t2 = t + c, c2 = t2 < c;
      L[i] = t2;
      c = c1 | c2;
    }
  }
  const bool neg = (int64_t)L[n - 1] < 0;
  if (neg) {
    uint64_t c = 1;
    for (int i = 0; i < n; i++) { const uint64_t t = ~L[i] + c; c = (c && t == 0) ? 1 : 0; L[i] = t; }
  }
  int top = n - 1;
  while (top >= 0 && !L[top]) top--;
  if (top < 0) return 0.0;
  const int nb = 64 * top + 64 - __builtin_clzll(L[top]);  // significant bits
  auto bit_at = [&](int i) -> uint64_t { return (L[i / 64] >> (i % 64)) & 1ull; };
  uint64_t mant = 0;
  int exp2 = 0;
  if (nb <= 53) {
    mant = L[0];
  } else {
    const int r = nb - 53;
    for (int i = 0; i < 53; i++) mant |= bit_at(r + i) << i;
    const uint64_t round = bit_at(r - 1);
    bool sticky = false;
    for (int i = 0; i < (r - 1) / 64 && !sticky; i++) sticky = L[i] != 0;
    if (!sticky && (r - 1) % 64) sticky = (L[(r - 1) / 64] & ((1ull << ((r - 1) % 64)) - 1)) != 0;
    if (round && (sticky || (mant & 1))) mant++;
    exp2 = r;
  }
  const double d = __builtin_ldexp((double)mant, exp2 + u0);
  return neg ? -d : d;
}

// The final SUM of an SK_FX aggregation from its windows p (fx slots A.slot ..): the exact sum of the finite inputs,
// unless non-finite inputs were seen (their order images in the sp_min / sp_max slots): IEEE 754 addition gives NaN
// for any NaN or for +inf with -inf, else the infinity -- whatever the order, so the special cases stay exact too.
__host__ __device__ inline double fx_final(const AggSpec& A, const uint64_t* p, int64_t sp_mn, int64_t sp_mx) {
  if (A.sp_min != kNoSp) {
    const int64_t kpinf = order_key(__builtin_inf()), kninf = order_key(-__builtin_inf());
    const bool nan = sp_mx > kpinf || sp_mn < kninf, pinf = sp_mx == kpinf, ninf = sp_mn == kninf;
    if (nan || (pinf && ninf)) return __builtin_nan("");
    if (pinf) return __builtin_inf();
    if (ninf) return -__builtin_inf();
  }
  return fx_windows_to_double(p, A.fx_nwin, A.fx_shift);
}


// ---- the fused scan (pg_scan.hip).  Everything else the runtime launches is declared in pg_aux.h, so that the scan's
// nine shapes (a ~15 minute build) recompile only when this header changes.
hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s, bool co = false);  // pg_scan.hip
// co: the 128-VGPR variant that runs beside the exact-mode stream kernel (scan_co_resident shapes)
bool scan_co_resident(const QuerySpec& q);
size_t scan_lds_bytes(const QuerySpec& q);
uint32_t scan_min_blocks_per_cu(bool grouped);

}  // namespace pg
