// pg_aux.h -- kernel interfaces of libpinot_gpu other than the fused scan (gfx950): upload re-layout, index pre-pass,
// selective stream, radix-partitioned group-by, wide group keys, group-state finalisation.
#pragma once
#include "pg_internal.h"

namespace pg {

// ---- host-side chunk decoders of raw forward indexes (pg_codec.hip): ChunkCompressionType codes (pinot_codec.h);
// *why = the reason of a failure
int decompress_chunk(uint32_t kind, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out,
                     const char** why);

// ---- kernel launchers
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
// The per-query parameter arena read by the device straight from its pinned (fine-grained, mapped) host image, and
// the query's scratch zeroed, in ONE launch on the query stream (instead of an SDMA copy, whose completion the compute
// queue waits on, plus a fill).
struct FillSpans {  // byte fills deferred into the arena-upload launch (a state's zero / empty initialisation)
  static constexpr uint32_t kMax = 8;
  void* p[kMax];
  uint64_t n[kMax];
  uint32_t byte[kMax];
  uint32_t count;
  bool add(void* ptr, uint32_t b, uint64_t bytes) {
    if (count >= kMax) return false;
    p[count] = ptr;
    n[count] = bytes;
    byte[count] = b;
    count++;
    return true;
  }
};
hipError_t launch_arena_upload(const void* host_src, void* dst, uint64_t bytes, void* zero, uint64_t zero_bytes,
                               const FillSpans& fills, hipStream_t s);
struct CopySpans {  // device -> mapped host spans of 8-byte words copied by one launch (the end-of-query readback)
  static constexpr uint32_t kMax = 5;
  const void* src[kMax];
  void* dst[kMax];
  uint64_t words[kMax];
  uint32_t count;
  void add(const void* from, void* to, uint64_t bytes) {  // bytes: a multiple of 8
    src[count] = from;
    dst[count] = to;
    words[count] = bytes / 8;
    count++;
  }
};
hipError_t launch_copy_spans(const CopySpans& c, hipStream_t s);
hipError_t launch_fill_ranges(const int32_t* ranges /*[n][2] inclusive, sorted, disjoint*/, uint32_t n,
                              uint32_t num_docs, uint32_t* bitmap, hipStream_t s);
struct RoaringContainer {
  uint32_t key;      // high 16 bits of the doc ids
  uint32_t type;     // 0 array, 1 bitmap, 2 run
  uint32_t card;     // array: cardinality; run: number of runs
  uint32_t offset;   // byte offset of the payload within the column's roaring region
};
// Key-major directory entry (x = payload offset, y = type << 30 | card; ~0 ~0: the dictId has no container under the
// key): the container's descriptor itself, so a key's lookup is one 8-byte load, not a directory load and then a
// dependent descriptor load.
__host__ __device__ inline uint2 keydir_entry(const RoaringContainer& c) {
  return make_uint2(c.offset, (c.type << 30) | c.card);
}
constexpr uint32_t kKeyDirNone = 0xFFFFFFFFu;
hipError_t launch_roaring_or(const uint8_t* roaring, const RoaringContainer* containers, const uint32_t* sel,
                             uint32_t nsel, uint32_t num_docs, uint32_t* bitmap, hipStream_t s);
hipError_t launch_bitmap_not(uint32_t* bitmap, uint32_t num_docs, hipStream_t s);
// Inverted-index leaves of a query, all segments in one launch (BitmapBasedFilterOperator: the OR of the selected
// dictIds' roaring bitmaps, flipped when exclusive).  One workgroup per (job, 64 K-doc key): it ORs every selected
// dictId's container of that key into an LDS chunk, then writes the chunk's words of the doc bitmap once (negated for
// NOT_EQ / NOT_IN).  Keys [key0, key0 + nkeys) only: a root-AND doc range (sorted leaf) bounds the docs ever read.
struct RoaringJob {
  const uint8_t* roaring;          // container payloads (8-byte aligned)
  const RoaringContainer* cs;      // container directory, per dictId sorted by key
  const uint32_t* dir;             // [card + 1] first container of each dictId
  const int32_t* ids;              // selected dictIds (sorted)
  uint32_t nids, num_docs;
  uint32_t* bm;                    // doc bitmap (packed 1-bit column order)
  uint32_t negate, key0, nkeys, first_block;  // first_block: prefix of nkeys over the jobs
  const uint2* keydir;             // optional key-major directory: [key * card + dictId] = the container (KeyDirEntry)
  uint32_t card, pad;
};
hipError_t launch_roaring_keys(const RoaringJob* jobs, uint32_t njobs, uint32_t blocks, hipStream_t s);

// ---- fused index count (pg_index.hip): an aggregation-only COUNT / COUNTMV query whose filter is index leaves only
// (sorted doc ranges, inverted dictId sets, constants) in at most two levels of AND / OR / NOT.  One workgroup per
// (segment, 64 K-doc key) of the segment's doc range decodes each inverted leaf's containers of that key into LDS,
// evaluates the filter on the words and counts -- no doc bitmap goes through HBM.
enum IdxLeafKind : uint32_t { IL_ALL = 0, IL_NONE = 1, IL_DOCRANGE = 2, IL_ROARING = 3 };
struct IdxLeaf {                   // leaf l of segment s
  uint32_t kind, negate;           // negate: NOT_EQ / NOT_IN over an inverted index (flip of the OR)
  int32_t lo, hi;                  // IL_DOCRANGE: docs [lo, hi)
  const uint8_t* roaring;          // IL_ROARING: the column's containers and the selected dictIds
  const RoaringContainer* cs;
  const uint32_t* dir;
  const uint2* keydir;
  const int32_t* ids;
  uint32_t nids, card;
};
struct IdxSeg {
  uint32_t num_docs, key0, first_block, pad;  // keys [key0, key0 + blocks) of the doc range; blocks prefix
  const IdxLeaf* leaves;                      // [num_leaves]
  const uint32_t* mv_cnt;                     // COUNTMV: 4-bit value counts per doc (packed, bit 31-4j.. <- doc 8w+j) or
  const uint32_t* mv_offsets;                 //   the row offsets [num_docs + 1] when no count column exists
};
constexpr uint32_t kIdxMaxLeaves = 8, kIdxMaxItems = 16;
struct IdxSpec {
  uint32_t num_segs, num_leaves;
  uint32_t root_or;                 // root combines its items by OR (else AND)
  uint32_t num_items;
  uint32_t item[kIdxMaxItems];      // bit 31 NOT, bit 30 group, else leaf index (low 8 bits)
  uint32_t group_or[kIdxMaxItems];  // group g: OR (else AND) over gleaf[gfirst[g], gfirst[g] + gn[g])
  uint32_t gfirst[kIdxMaxItems], gn[kIdxMaxItems];
  uint32_t gleaf[kIdxMaxItems];     // bit 31 NOT, else leaf index
  uint32_t chunk_of[kIdxMaxLeaves]; // LDS chunk slot of leaf l (~0: not an inverted leaf anywhere)
  uint32_t num_chunks;
  uint32_t cntmv_slot;              // i64 slot of COUNTMV (~0: none)
  const IdxSeg* segs;
  const IdxLeaf* leaves;            // [num_segs][num_leaves]
  const uint32_t* blk_seg;          // block -> its segment
  unsigned long long* i64;          // slot 0: doc count
  unsigned long long* seg_matched;  // [num_segs]
};
hipError_t launch_index_count(const IdxSpec& p, uint32_t blocks, hipStream_t s);
// COUNTMV's count column of an MV forward index: 4 bits per doc (min(count, 15)); *over set when a count exceeds 15
hipError_t launch_mv_counts(const uint32_t* offsets, uint32_t num_docs, uint32_t* out, unsigned int* over, hipStream_t s);
hipError_t launch_mv_scan(const uint32_t* words, uint32_t bits, const uint32_t* offsets, uint32_t num_docs,
                          int32_t lo, int32_t hi, const uint32_t* lut, uint32_t excl, uint32_t* bitmap,
                          hipStream_t s);
struct LutJob {            // set bits ids[0..n) in lut and ids >> shift in region (one batched launch per query)
  const int32_t* ids;        // or null: the dictIds of the n literals `values` found in `dict` (values mode)
  uint32_t* lut;             // exact bitmap over dictIds, or null
  uint32_t* region;          // LDS-set filter bitmap over dictId >> shift, or null
  uint32_t n;
  uint32_t shift;
  const void* values;        // values mode: n sorted literals of the dictionary's type (dtype)
  const void* dict;          //   the segment's typed dictionary of `card` values
  uint32_t card, dtype;
};
hipError_t launch_set_lut_bits(const LutJob* jobs, uint32_t njobs, uint32_t max_n, hipStream_t s);

// IN / NOT_IN literal lowering for many segments in one launch (PredicateUtils.getDictIdSet): out[s * n + i] = the
// dictId of values[i] in segment s's dictionary, or -1
struct DictLookupJob {
  const void* dict;  // typed sorted dictionary values (dtype)
  uint32_t card, pad;
};
hipError_t launch_dict_lookup(const DictLookupJob* jobs, uint32_t num_segments, const void* values, uint32_t n,
                              uint32_t dtype, int32_t* out, hipStream_t s);

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
struct ExactSet {       // one segment's IN list of the exact-mode stream leaf, resolved in the stream block's LDS
  const int32_t* ids;    // its dictIds, or null: values mode ...
  const void* vals;      // ... its literals in the dictionary's stored type, looked up in `dict` (card entries); both
  const void* dict;      //     null: stage the leaf's global LUT instead
  uint32_t n, nwords;    // ids / literals; LUT words (ceil(cardinality / 32))
  uint32_t card, dtype;
};
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
  // exact mode (1 024-thread blocks, one per CU): a coarse IN bitmap's exact LUT (exact[seg].nwords words, <= 128 KiB)
  // is whole in LDS, so no value is a candidate to resolve: built there from the segment's dictIds (exact[seg].ids), or
  // staged from the global LUT (ids == null)
  const ExactSet* exact;
  // further leaves over packed columns of at most kStreamStageBits bits: a wave stages its 64 groups' words of the
  // column into its LDS slice (16-byte coalesced loads) and tests its survivors from there instead of per-doc window
  // reads.  stage_words: words per wave slice (0: off), placed after the IN-set words (set_lds_ints, a multiple of 4).
  // stage_pre: every further leaf has its own slice per wave, DMA'd into LDS at the start of each group round with the
  // driving leaf's loads (one load latency per round instead of two; set when the driving leaf passes >= 1/16, where
  // nearly every wave's groups have survivors and the slices would be read anyway)
  uint32_t stage_words, stage_pre;
  // optional [2] wall-clock stamps of the launch (the phase timing without an event record between dependent kernels):
  // [0] max of ~(block start), i.e. ~(earliest start); [1] the latest block end; both zeroed before the launch
  unsigned long long* stamp;
};
constexpr uint32_t kStreamStageBits = 16;
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
  // speculative layout (fill1 != null; part_direct + part_split2s): level-1 partition p's entries at
  // [p * cap1, p * cap1 + min(fill1[p], cap1)), bucket b's at [b * cap2, b * cap2 + min(fill2[b], cap2)); no histograms
  const unsigned int* fill1;
  unsigned int* fill2;
  uint64_t cap1, cap2;
  unsigned int* err;               // bit 4: a region over its capacity (the runtime reruns with exact offsets)
  uint32_t* dc_pop;                // optional [num_groups]: each group's distinct-value count (its bitmap's popcount)
  uint32_t count_docs;             // 1: i64 slot 0 = doc count (a COUNT reads it); 0: the value set's size (presence)
  uint32_t pad2;
};
// Level 1 straight from the columns, speculative (filter matching every doc, one group key, at most one DISTINCTCOUNT
// value column): 256-thread blocks take rounds of one 8 192-doc tile; the tile's packed words of the key / value column
// are read coalesced (16-byte loads of the whole word range) into LDS, each thread unpacks 32 docs from there, and the
// round's 32-bit entries are counting-sorted by level-1 digit in LDS and written as runs reserved in fixed-capacity
// partition regions (split_round RES).  One read of each column, one write of the entries, no histogram pass.
struct PartDirectSpec {
  uint32_t blocks, num_items, nparts1, shift1;
  uint32_t vbits, has_val, key_kind, val_kind;
  uint64_t key_card, val_card;
  int64_t key_base, val_base;
  uint64_t cap1;                   // entries per level-1 partition region
  uint32_t val_agg, stage_words;   // stage_words: set by launch_part_direct (LDS words of the widest tile stage)
  const SegDesc* segs;
  const WorkItem* items;           // tile ranges (kTileDocs docs)
  unsigned int* fill1;             // [nparts1] entries reserved so far (zeroed before the launch)
  uint32_t* out1;                  // level-1 regions
  unsigned int* err;               // bit 0: key outside its space, bit 1: value outside, bit 4: a region overflowed
};
// Id modes (uniform over the segments, else the exact path): 0 decoded image (vbase + raw), 1 int32 gather (int32
// dictionary or keymap); value mode -1 = no value column.  part_id_mode() gives a column's mode (2 = not direct).
int part_id_mode(uint32_t key_kind, const ColDesc& c);
hipError_t launch_part_direct(const PartDirectSpec& p, uint32_t key_bits, uint32_t val_bits, int key_mode, int val_mode,
                              hipStream_t s);
hipError_t launch_part_split2s(const PartSpec& p, hipStream_t s);
// Level 1 straight from the columns when the filter matches every doc (no 64-bit scan entries, no split1): block b
// walks the work items [b * num_items / blocks, (b + 1) * num_items / blocks) twice -- part_hist counts its docs'
// level-1 digits, part_scatter counting-sorts them (LDS rounds of kSplitChunk) into its runs of the level-1
// partitions at off1[p * blocks + b] as 32-bit entries (key bits below the digit << vbits | value id).
struct PartScanSpec {
  uint32_t num_keys, blocks, num_items, nparts1;
  uint32_t shift1, vbits, val_agg, pad;  // val_agg: the DISTINCTCOUNT aggregation (kNoSlot: COUNTs only)
  const SegDesc* segs;
  const WorkItem* items;                 // tile ranges (kTileDocs docs) of the scan's split
  uint32_t key_kind[kMaxKeys];
  uint32_t key_card[kMaxKeys];
  int64_t key_base[kMaxKeys];
  uint64_t key_stride[kMaxKeys];
  AggSpec val;
  unsigned long long* hist1;             // [nparts1][blocks]
  const unsigned long long* off1;        // its exclusive scan
  uint32_t* out1;                        // level-1 entries
  unsigned int* err;                     // bit 0: key outside its space, bit 1: value outside its space
};
hipError_t launch_part_hist(const PartScanSpec& p, hipStream_t s);
hipError_t launch_part_scatter(const PartScanSpec& p, hipStream_t s);
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
// cross-state merge of wide keys (rows gathered with key_div 1: the key word is the tuple slot): owner part of each
// row's tuple; rows widened with their tuples (rbw = rb + K uint32
// padded to 8 bytes); exchanged rows' tuples interned into `w` (err bit 2: table full), out = rows keyed by the slot
hipError_t launch_wide_owner(const uint32_t* tuples, uint32_t K, const uint8_t* rows, uint64_t rb, uint64_t n,
                             uint32_t parts, uint32_t* owner, hipStream_t s);
hipError_t launch_widen_rows(const uint8_t* rows, uint64_t rb, const uint32_t* tuples, uint32_t K, uint64_t n,
                             uint8_t* dst, uint64_t rbw, hipStream_t s);
hipError_t launch_intern_rows(const WideSpec& w, const uint8_t* rows, uint64_t n, uint64_t rb, uint64_t rbw,
                              uint8_t* out, hipStream_t s);

// ---- group state (pg_groups.hip)
struct StateView {            // the device arrays of one partial state
  uint64_t num_slots, hmask;
  unsigned long long* keys;   // hash tables: [num_slots] packed keys (kEmptyKey = free); dense: null
  unsigned long long* i64;
  unsigned long long* fx;     // [num_slots][n_fx][2]: SK_FX (lo, hi) pairs
  long long* mn;
  long long* mx;
  uint32_t* bits;
  unsigned long long* first_doc;  // GM_HASH_SEG tables: doc << 16 | tuple position (QuerySpec.first_doc)
  unsigned int* fill;         // hash tables: claimed keys
  unsigned int* err;          // bit 2: table full
  uint32_t n_i64, n_fx, n_min, n_max, bit_words, max_fill;
  const uint32_t* dc_pop;     // optional: DISTINCTCOUNT dc_pop_agg's set size per slot (GM_PART's bucket pass)
  uint32_t dc_pop_agg, pad;
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
// The present slots of a state in no particular order (one pass, one atomic per wave): count must be zeroed
hipError_t launch_select_present_unordered(const StateView& v, uint32_t* out, unsigned int* count, hipStream_t s);
// DISTINCTCOUNT-ordered trim from the bucket pass's set sizes (StateView::dc_pop): a histogram of the present groups'
// sizes (maxv + 1 bins, hist zeroed), then the present groups with size >= t (at_least) or <= t, unordered (count
// zeroed)
hipError_t launch_pop_hist(const StateView& v, uint32_t maxv, unsigned int* hist, hipStream_t s);
hipError_t launch_select_pop(const StateView& v, uint32_t t, uint32_t maxv, bool at_least, uint32_t* out,
                             unsigned int* count, hipStream_t s);
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
// The order image straight from the state for the trim's candidate selection (no final values of every group);
// order_keys_from_state_ok: the first ORDER BY item is a key or an aggregation whose final value is one state read
bool order_keys_from_state_ok(const StateView& v, const FinalSpec& f);
hipError_t launch_order_keys_state(const StateView& v, const FinalSpec& f, const uint32_t* slots, uint64_t n,
                                   uint64_t* out, uint32_t* pos, uint64_t* span, hipStream_t s);
hipError_t launch_gather_slots(const uint32_t* slots, const uint32_t* pos, uint64_t n, uint32_t* out, hipStream_t s);
// ORDER BY trim by radix select (pg_groups.hip): histogram of key bits [lo, hi) of k' = (key >> b0) & (2^W - 1) over the
// keys whose k' >> hi equals prefix (hist: 256 counters, zeroed by the caller); then the positions of every key with
// k' <= tstar (count: zeroed by the caller)
constexpr uint32_t kOkeyDigitBits = 11;  // radix-select digit width: config 4's 21 differing bits in 2 passes, not 3
hipError_t launch_okey_hist(const uint64_t* keys, uint64_t n, uint32_t b0, uint32_t W, uint32_t lo, uint32_t hi,
                            uint64_t prefix, unsigned int* hist, hipStream_t s);
hipError_t launch_okey_select(const uint64_t* keys, uint64_t n, uint32_t b0, uint32_t W, uint64_t tstar, uint32_t* pos,
                              unsigned long long* count, hipStream_t s);
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
// Element-wise merge of two dense states of one layout (in-library multi-device combine, pg_init_devices): i64 += ,
// fx 128-bit += , mn min, mx max, bits |= (AggregationFunction.merge of each function; src arrays on this device)
hipError_t launch_merge_dense(const StateView& dst, const StateView& src, hipStream_t s);
// SK_FX pairs <-> 4 x 32-bit limbs per pair (in: fold the limbs' carries back into the pairs)
hipError_t launch_fx_limbs(unsigned long long* pairs, long long* limbs, uint64_t n, bool in, hipStream_t s);
hipError_t launch_init_view(const StateView& v, hipStream_t s, FillSpans* defer = nullptr);  // pg_kernels.hip: zero / empty / +-inf state
hipError_t launch_seg_truncate(const StateView& v, const uint32_t* slots, uint64_t n, uint32_t num_segments,
                               uint64_t limit, bool mv, uint64_t* tmp_keys, uint64_t* sorted_keys, uint32_t* sorted_slots,
                               uint32_t* seg_first, uint8_t* keep, unsigned int* reached, void* temp, size_t temp_bytes,
                               hipStream_t s);

}  // namespace pg
