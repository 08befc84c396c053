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

enum SlotKind : uint32_t { SK_NONE = 0, SK_I64 = 1, SK_F64 = 2, SK_MIN = 3, SK_MAX = 4, SK_BITS = 5 };

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
  uint32_t pad;
};

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
  uint32_t n_i64, n_f64, n_min, n_max;
  uint32_t dc_row_words;     // uint32 words of DISTINCTCOUNT bitmaps per slot
  uint32_t pad2;
  unsigned long long* i64;
  double* f64;
  long long* mn;
  long long* mx;
  uint32_t* dbits;           // [num_slots][dc_row_words]
  unsigned long long* hkeys; // GM_HASH*: [num_slots] packed keys
  unsigned int* hfill;       // GM_HASH*: claimed keys
  unsigned int* first_doc;   // GM_HASH_SEG: [num_slots] first matching doc of the (segment, key)
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


// ---- kernel launchers
hipError_t launch_scan(const QuerySpec& q, uint32_t blocks, hipStream_t s);                  // pg_scan.hip
size_t scan_lds_bytes(const QuerySpec& q);
uint32_t scan_min_blocks_per_cu(bool grouped);
hipError_t launch_bswap_words(const uint8_t* src, uint32_t* dst, uint64_t nbytes, uint64_t nwords_out, hipStream_t s);
hipError_t launch_be_to_native(const uint8_t* src, void* dst, uint64_t n, uint32_t width, hipStream_t s);
hipError_t launch_sorted_to_packed(const int32_t* pairs, uint32_t card, uint32_t num_docs, uint32_t bits,
                                   uint32_t* words, uint64_t nwords, hipStream_t s);
hipError_t launch_decode_pack(const uint32_t* ids, uint32_t bits, const void* dict, uint32_t dtype, uint32_t card,
                              int64_t vmin, uint32_t vbits, uint32_t num_docs, uint32_t* out, uint64_t nwords,
                              hipStream_t s);
hipError_t launch_dict_bits(const void* dict, uint32_t dtype, uint32_t card, int64_t base, const int32_t* keymap,
                            uint32_t key_card, uint32_t* bits, unsigned int* err, hipStream_t s);
hipError_t launch_mv_offsets(const uint32_t* bitmap_words, uint64_t num_values, uint32_t num_docs,
                             uint32_t* offsets, void* scratch, size_t scratch_bytes, hipStream_t s);
size_t mv_offsets_scratch_bytes(uint64_t num_values);
hipError_t launch_fill_ranges(const int32_t* ranges /*[n][2] inclusive, sorted, disjoint*/, uint32_t n,
                              uint32_t num_docs, uint32_t* bitmap, hipStream_t s);
struct RoaringContainer {
  uint32_t key;      // high 16 bits of the doc ids
  uint32_t type;     // 0 array, 1 bitmap, 2 run
  uint32_t card;     // array: cardinality; run: number of runs
  uint32_t offset;   // byte offset of the payload within the column's roaring region
};
hipError_t launch_roaring_or(const uint8_t* roaring, const RoaringContainer* containers, const uint32_t* sel,
                             uint32_t nsel, uint32_t num_docs, uint32_t* bitmap, hipStream_t s);
hipError_t launch_bitmap_not(uint32_t* bitmap, uint32_t num_docs, hipStream_t s);
hipError_t launch_mv_scan(const uint32_t* words, uint32_t bits, const uint32_t* offsets, uint32_t num_docs,
                          int32_t lo, int32_t hi, const uint32_t* lut, uint32_t excl, uint32_t* bitmap,
                          hipStream_t s);
struct LutJob {            // set bits ids[0..n) in lut and ids >> shift in region (one batched launch per query)
  const int32_t* ids;
  uint32_t* lut;             // exact bitmap over dictIds, or null
  uint32_t* region;          // LDS-set filter bitmap over dictId >> shift, or null
  uint32_t n;
  uint32_t shift;
};
hipError_t launch_set_lut_bits(const LutJob* jobs, uint32_t njobs, hipStream_t s);

// ---- streaming pre-filter (pg_filter.hip): one leaf of the root AND over the segments whose form of it reads
// `bits`-bit values, into (first) or AND-ed into (later) one doc bitmap per segment
constexpr uint32_t kPreItemGroups = 8192;   // 32-doc groups per pre-filter work item (262 144 docs)
struct PreSpec {
  uint32_t num_items, leaf, first, set_lds_ints;
  const SegDesc* segs;
  const WorkItem* items;          // tile_begin / tile_end in 32-doc groups
  uint32_t* const* out;           // [seg] bitmap words, packed 1-bit column order
};
hipError_t launch_prefilter(const PreSpec& p, uint32_t bits, uint32_t blocks, hipStream_t s);

// ---- selective stream (pg_filter.hip): the driving leaf of the root AND (a packed scan leaf passing few docs) over
// every segment, bit width a template parameter, values loaded straight into registers; the survivors' doc ids are
// compacted into one region per item, which the scan kernel then consumes in list mode
constexpr int kMaxStreamExtra = 3;
struct StreamSpec {
  uint32_t num_items, leaf, cap, set_lds_ints;
  uint32_t num_extra;                 // further leaves of the root AND tested in the stream, on the survivors only
  uint32_t interleave;                // block b streams items first + b + k * gridDim.x (first = block_first[0], end =
                                      // block_first[gridDim.x]); else the range [block_first[b], block_first[b + 1])
  uint32_t extra[kMaxStreamExtra];    // (runtime bit width: per-doc windows, like the scan's gathered leaves)
  const SegDesc* segs;
  const WorkItem* items;          // tile_begin / tile_end in 32-doc groups
  const uint32_t* block_first;    // [gridDim.x + 1]: block b streams items [block_first[b], block_first[b + 1])
  uint32_t* docs;                 // [num_items][cap]
  uint32_t* counts;               // [num_items] survivors written (<= cap)
  unsigned int* err;              // bit 3: some item had more than `cap` survivors
  // exact mode (1 024-thread blocks, one per CU): a coarse IN bitmap's exact LUT (exact_nwords[seg] words, <= 128 KiB)
  // is staged whole in LDS, so no value is a candidate to resolve
  const uint32_t* exact_nwords;
};
hipError_t launch_stream(const StreamSpec& p, uint32_t bits, uint32_t blocks, hipStream_t s);

// ---- radix-partitioned group-by (pg_part.hip): level 2 + per-bucket aggregation, after the two scan passes
constexpr uint32_t kPartL1 = 256;        // level-1 partitions (scan passes)
constexpr uint32_t kPartNB = 32;         // level-2 blocks per level-1 partition
constexpr uint32_t kPartLdsBytes = 72 * 1024;  // LDS state of one bucket (count + value bitmap per group)
struct PartSpec {
  uint32_t nparts1, nparts2;       // level-1 partitions, level-2 sub-partitions per level-1 partition
  uint32_t vbits, shift1, shift2;  // value-id bits; key bits below the level-1 / level-2 digit (2^shift2 = bucket)
  uint32_t dc_words;               // uint32 words of the value bitmap (0: COUNT only)
  uint32_t row_words, dc_word;     // state bitmap row width / this aggregation's first word (StateView layout)
  uint32_t n_i64;
  uint32_t blocks1;                // scan blocks (regions of the 64-bit entry array)
  uint64_t num_groups;             // G (packed key space)
  const unsigned long long* in0;   // scan entries (64-bit), block b's at [base0[b], base0[b] + count0[b])
  const unsigned long long* base0;
  const unsigned int* count0;
  const unsigned long long* off1;  // [nparts1 * blocks1 + 1] exclusive scan of the scan's (partition, block) counts
  uint32_t* in1;                   // level-1 entries (32-bit: key below the level-1 digit << vbits | value id)
  unsigned long long* hist2;       // [nparts1 * nparts2 * kPartNB + 1] level-2 counts (last = 0)
  const unsigned long long* off2;  // their exclusive scan: bucket b's entries start at off2[b * kPartNB]
  uint32_t* out2;                  // level-2 entries, bucket-major
  unsigned long long* i64;         // dense state written by the bucket pass
  uint32_t* bits;
};
hipError_t launch_part_split1(const PartSpec& p, hipStream_t s);
hipError_t launch_part_count2(const PartSpec& p, hipStream_t s);
hipError_t launch_part_split2(const PartSpec& p, hipStream_t s);
hipError_t launch_part_aggregate(const PartSpec& p, hipStream_t s);

// ---- group keys wider than a packed 62-bit key (pg_wide.hip): ArrayMapBasedHolder as a device tuple table
constexpr uint32_t kMaxWideKeys = 64;
struct WideSpec {
  uint32_t K, num_segments, max_fill, pad;
  uint64_t mask;                    // table slots - 1 (a power of two)
  unsigned long long* tags;         // [slots]: 0 free, 1 being written, else the tuple's hash | 2
  uint32_t* tuples;                 // [slots][K] table-global key ids
  unsigned int* fill;               // claimed slots
  unsigned int* err;                // bit 0: key id outside its key space; bit 2: table over its fill budget
  const ColDesc* keycols;           // [seg][K] (the scan's key column descriptors)
  const uint32_t* num_docs;         // [seg]
  uint32_t* const* out;             // [seg] -> uint32[num_docs]: tuple slot of each doc
  const uint32_t* key_kind;         // [K]
  const int64_t* key_base;          // [K]
  const uint32_t* key_card;         // [K]
};
hipError_t launch_intern_tuples(const WideSpec& w, uint32_t max_docs, hipStream_t s);
hipError_t launch_gather_tuples(const uint32_t* tuples, uint32_t K, const uint64_t* slots, uint64_t n, uint32_t* out,
                                hipStream_t s);

// ---- group state (pg_groups.hip)
struct StateView {            // the device arrays of one partial state
  uint64_t num_slots, hmask;
  unsigned long long* keys;   // hash tables: [num_slots] packed keys (kEmptyKey = free); dense: null
  unsigned long long* i64;
  double* f64;
  long long* mn;
  long long* mx;
  uint32_t* bits;
  unsigned int* first_doc;    // GM_HASH_SEG tables
  unsigned int* fill;         // hash tables: claimed keys
  unsigned int* err;          // bit 2: table full
  uint32_t n_i64, n_f64, n_min, n_max, bit_words, max_fill;
};
struct FinalSpec {            // what finalisation needs of the plan
  uint32_t num_aggs, num_keys;
  uint32_t order_kind, order_index, order_desc, pad;  // first ORDER BY item (pg_order)
  AggSpec aggs[kMaxAggs];
  uint32_t key_card[kMaxKeys];
  uint64_t key_stride[kMaxKeys];
};
enum SelectKind : uint32_t { SEL_PRESENT = 0, SEL_OCCUPIED = 1, SEL_PRESENT_PART = 2 };
size_t select_temp_bytes(uint64_t n);
size_t sort_temp_bytes(uint64_t n, uint32_t begin_bit = 0, uint32_t end_bit = 64);
uint64_t row_bytes(const StateView& v);
hipError_t launch_select_slots(const StateView& v, uint32_t kind, uint32_t part, uint32_t parts, uint32_t* out,
                               uint32_t* d_num, void* temp, size_t temp_bytes, hipStream_t s);
hipError_t launch_select_flagged(const uint32_t* in, const uint8_t* flags, uint64_t n, uint32_t* out, uint32_t* d_num,
                                 void* temp, size_t temp_bytes, hipStream_t s);
hipError_t launch_exclusive_sum(const uint64_t* in, uint64_t* out, uint64_t n, void* temp, size_t temp_bytes,
                                hipStream_t s);
hipError_t launch_sort_pairs(const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout, uint64_t n,
                             void* temp, size_t temp_bytes, hipStream_t s, uint32_t begin_bit = 0, uint32_t end_bit = 64);
hipError_t launch_final_values(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                               uint64_t* keys, double* vals, int64_t* cnts, hipStream_t s);
// span (optional, 2 words, set here): the OR of every order key and the OR of their complements; the bits set in
// both differ between keys, the others are equal in all of them and the sort can skip them
hipError_t launch_order_keys(const FinalSpec& f, const uint64_t* keys, const double* vals, const int64_t* cnts,
                             uint64_t n, uint64_t* out, uint32_t* pos, hipStream_t s, uint64_t* span = nullptr);
hipError_t launch_cutoff(const uint64_t* sorted, uint64_t n, uint64_t limit, uint64_t* out, hipStream_t s);
hipError_t launch_gather_final(uint32_t A, const uint32_t* pos, uint64_t n, const uint64_t* keys, const double* vals,
                               const int64_t* cnts, const uint32_t* slots, uint64_t* okeys, double* ovals,
                               int64_t* ocnts, uint32_t* oslots, hipStream_t s);
hipError_t launch_set_sizes(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                            uint64_t* sizes, hipStream_t s);
hipError_t launch_set_extract(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                              const uint64_t* offsets, uint32_t* ids, hipStream_t s);
hipError_t launch_gather_rows(const StateView& v, const uint32_t* slots, uint64_t n, uint64_t key_div, uint8_t* dst,
                              hipStream_t s);
hipError_t launch_merge_rows(const StateView& v, const uint8_t* rows, uint64_t n, hipStream_t s);
hipError_t launch_init_view(const StateView& v, hipStream_t s);  // pg_kernels.hip: zero / empty / +-inf state
hipError_t launch_seg_truncate(const StateView& v, const uint32_t* slots, uint64_t n, uint32_t num_segments,
                               uint64_t limit, uint64_t* tmp_keys, uint64_t* sorted_keys, uint32_t* sorted_slots,
                               uint32_t* seg_first, uint8_t* keep, void* temp, size_t temp_bytes, hipStream_t s);

}  // namespace pg
