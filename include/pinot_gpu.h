/*
 * pinot_gpu.h -- C ABI of libpinot_gpu.so, the MI355X (gfx950) segment query hot path.
 *
 * This is the drop-in boundary of SURVEY.md §8(b): the Java side keeps Pinot's PlanMaker /
 * Operator / AggregationFunction / ForwardIndexReader / Dictionary SPIs and calls these
 * entry points through JNI (binding stub in INTEGRATION.md).  Plain C types only; no HIP,
 * torch or C++ types cross this line.  All functions return 0 (PG_OK) or a negative
 * pg_status; the thread-local message is available from pg_last_error().  Nothing is ever
 * thrown or aborted across the ABI.
 *
 * Reference interfaces each entry point replaces (paths relative to navina/pinot):
 *   pg_column_upload  <- IndexingOverrides.registerProvider / DefaultIndexReaderProvider
 *                        (pinot-segment-spi/.../index/IndexingOverrides.java:82-92,
 *                         pinot-segment-local/.../readers/DefaultIndexReaderProvider.java:79-122):
 *                        the reader factories that wrap a segment's PinotDataBuffer at load time.
 *                        Here the same on-disk big-endian bytes are made device-resident.
 *   pg_segment_release<- IndexSegment.destroy (pinot-segment-spi/.../IndexSegment.java:122)
 *   pg_execute        <- PlanMaker.makeInstancePlan + Plan.execute for aggregation / group-by
 *                        queries (pinot-core/.../plan/maker/PlanMaker.java:42,
 *                        plan/GlobalPlanImplV0.java:48): per-segment FilterPlanNode ->
 *                        AggregationOperator / AggregationGroupByOrderByOperator, merged by
 *                        AggregationOnlyCombineOperator / GroupByOrderByCombineOperator
 *                        (operator/combine/).  Leaf predicates arrive already lowered to
 *                        dictId space exactly as PredicateEvaluatorProvider.getPredicateEvaluator
 *                        (operator/filter/predicate/PredicateEvaluatorProvider.java:38-90) does.
 *   pg_execute_partial / pg_partials_* <- the per-server partial results that
 *                        BaseCombineOperator.mergeResults (operator/combine/BaseCombineOperator.java:190-233)
 *                        merges; exposed as dense device arrays so that ranks (one process per
 *                        GPU) can merge them with an RCCL all-reduce over xGMI.
 *   pg_cancel         <- BaseOperator.nextBlock interrupt check (operator/BaseOperator.java:35-37)
 *   pg_last_error     <- ProcessingException text carried in the IntermediateResultsBlock
 *                        (operator/combine/BaseCombineOperator.java:104-108)
 */
#ifndef PINOT_GPU_H
#define PINOT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_ABI_VERSION 9

typedef enum pg_status {
  PG_OK = 0,
  PG_E_INVALID = -1,      /* malformed argument / plan */
  PG_E_HIP = -2,          /* HIP runtime error */
  PG_E_NOMEM = -3,        /* device allocation failed */
  PG_E_NOTFOUND = -4,     /* segment / column index not resident */
  PG_E_UNSUPPORTED = -5,  /* query shape not handled on the GPU: caller falls back to the CPU plan */
  PG_E_CANCELLED = -6,    /* pg_cancel() observed */
  PG_E_TIMEOUT = -7,      /* plan deadline passed */
  PG_E_STATE = -8         /* pg_init not called / wrong device */
} pg_status;

/* ---------------------------------------------------------------- device / library */

/* Bind the calling process to HIP device `device` (one process per GPU).  Idempotent.  = pg_init_devices(&device, 1). */
int pg_init(int device);
/* Bind the process to n logical devices: logical device i runs on HIP device devices[i] (a device may repeat -- two
 * logical devices sharing one GPU, e.g. to exercise the multi-device combine on a one-GPU host).  SURVEY §8(b)'s
 * pg_init(device_mask) as an explicit list.  With n > 1 every segment lives on one logical device (pg_segment_place,
 * else round-robin at its first upload), and pg_execute* runs a plan's segments on their devices concurrently and
 * merges the partial states inside the library -- over xGMI peer copies -- as one server's combine does
 * (BaseCombineOperator.mergeResults, operator/combine/BaseCombineOperator.java:190-233): a JNI caller gets one
 * merged result for all GPUs of the node from one call.  Idempotent for the same list; PG_E_STATE for another. */
int pg_init_devices(const int *devices, uint32_t n);
/* Number of logical devices (pg_init_devices' n). */
int pg_num_devices(uint32_t *out);
/* Place a segment on logical device `ldev` before its first pg_column_upload (the segment-to-GPU assignment a server
 * makes when it loads the segment).  PG_E_STATE if it is already resident elsewhere. */
int pg_segment_place(uint64_t seg_key, uint32_t ldev);
/* The logical device a resident segment lives on. */
int pg_segment_device(uint64_t seg_key, uint32_t *ldev);
/* Copy the calling thread's last error message (NUL-terminated, truncated to n). Returns its length. */
int pg_last_error(char *buf, size_t n);
/* Bytes of device memory held by resident segments. */
int pg_resident_bytes(uint64_t *out);
/* Cancel every pg_execute* carrying this query_id: one not yet launched fails before its launch, a running scan
 * stops at its next tile of 8 192 docs (a host-coherent flag the kernel polls), both with PG_E_CANCELLED.  A
 * plan's deadline_ms is enforced the same way (PG_E_TIMEOUT).  Callable from any thread. */
int pg_cancel(uint64_t query_id);
/* Library ABI version (PG_ABI_VERSION). */
int pg_abi_version(void);

/* ---------------------------------------------------------------- segment residency */

typedef enum pg_index_kind {
  PG_IDX_DICT = 1,            /* sorted dictionary, fixed-width big-endian values (V1 `.dict`)          */
  PG_IDX_FWD_SV_BITPACKED = 2,/* FixedBitSVForwardIndexWriter layout (`.sv.unsorted.fwd`)               */
  PG_IDX_FWD_SV_SORTED = 3,   /* sorted column: per dictId big-endian int32 [startDoc,endDoc] (`.sv.sorted.fwd`) */
  PG_IDX_FWD_MV_BITPACKED = 4,/* FixedBitMVForwardIndexWriter layout (`.mv.fwd`)                        */
  PG_IDX_INV_BITMAP = 5,      /* BitmapInvertedIndexWriter layout: (card+1) BE uint32 offsets + roaring */
  PG_IDX_KEYMAP = 6,          /* native int32[card]: dictId -> table-global key id (host-built, for
                                 group-by / DISTINCTCOUNT keys that are not integer value ranges)       */
  PG_IDX_FWD_SV_RAW = 7,      /* raw (no-dictionary) fixed-width chunked forward index (`.sv.raw.fwd`,
                                 BaseChunkSVForwardIndexWriter v1-v4, PASS_THROUGH or SNAPPY chunks;
                                 replaces FixedByteChunkSVForwardIndexReader /
                                 FixedBytePower2ChunkSVForwardIndexReader, DefaultIndexReaderProvider.java:92-101);
                                 data_type = stored type INT/LONG/FLOAT/DOUBLE                          */
  PG_IDX_RANGE = 8            /* range index file (`.bitmap.range`): BitSlicedRangeIndexCreator v2 (BE int 2,
                                 BE long min, RangeBitmap) or RangeIndexCreator v1 (BE int 1, value type, ranges,
                                 roaring bitmaps); replaces BitSlicedRangeIndexReader / RangeIndexReaderImpl
                                 (DefaultIndexReaderProvider.newRangeIndexReader).  Upload after the column's
                                 forward index: the header is validated and the device form is derived from the
                                 resident forward index (the index is a function of it) -- a dictionary column's
                                 packed dictIds serve as is; a raw INT / LONG column gets (value - min) packed at
                                 bits(max - min) bits per doc, which raw-column aggregations read too           */
} pg_index_kind;

typedef enum pg_data_type {
  PG_INT = 0, PG_LONG = 1, PG_FLOAT = 2, PG_DOUBLE = 3, PG_STRING = 4, PG_BYTES = 5
} pg_data_type;

#define PG_SRC_DEVICE 0x1u /* pg_col_desc.flags: `src` is a device pointer (same byte layout) */
/* col_id flag: a host-built dictionary encoding of the raw (no-dictionary) column col_id & ~PG_COL_DERIVED -- sorted
 * distinct values (Double.compare order) + bit-packed ids + a keymap to table-global ids -- uploaded for a GROUP BY key or
 * DISTINCTCOUNT value over a raw FLOAT / DOUBLE column or a raw INT / LONG column whose range spans 2^32 or more (the
 * reference's NoDictionarySingleColumnGroupKeyGenerator / NoDictionaryMultiColumnGroupKeyGenerator inputs,
 * DefaultGroupByExecutor.java:85-94).  It counts as that raw column in the statistics (numEntriesScannedPostFilter). */
#define PG_COL_DERIVED 0x40000000u

typedef struct pg_col_desc {
  uint32_t kind;             /* pg_index_kind */
  uint32_t data_type;        /* pg_data_type of the dictionary values (stored type) */
  uint32_t num_docs;         /* segment.total.docs */
  uint32_t cardinality;      /* column.<c>.cardinality */
  uint32_t bits_per_element; /* column.<c>.bitsPerElement */
  uint32_t num_values;       /* column.<c>.totalNumberOfEntries (MV: total values; SV: num_docs) */
  uint32_t entry_bytes;      /* dictionary bytes per entry (4/8 numeric, lengthOfEachEntry for strings) */
  uint32_t flags;            /* PG_SRC_DEVICE */
} pg_col_desc;

/* Make one index of one column of one segment device-resident.  `src` holds `nbytes` bytes in the
 * reference's on-disk (big-endian) layout and is borrowed only for the duration of the call.
 * Re-uploading the same (seg_key, col_id, kind) replaces it. */
int pg_column_upload(uint64_t seg_key, uint32_t col_id, const pg_col_desc *desc, const void *src,
                     uint64_t nbytes);
/* Free every device buffer of a segment. */
int pg_segment_release(uint64_t seg_key);

/* IN / NOT_IN literal lowering against the resident dictionaries of many segments at once -- the device form of
 * PredicateUtils.getDictIdSet (pinot-core/.../operator/filter/predicate/PredicateUtils.java:73-) as the
 * dictionary-based In / NotIn evaluators call it per segment (InPredicateEvaluatorFactory.java:153-199,
 * NotInPredicateEvaluatorFactory.java:153-).  `values`: num_values literals already converted to the column's stored
 * type `data_type` (PG_INT int32, PG_LONG int64, PG_FLOAT float, PG_DOUBLE double), sorted ascending, unique.
 * out_ids: [num_segments][num_values]; row s holds, in its first out_counts[s] entries, the dictIds (ascending) of the
 * literals present in segment s's dictionary of column col_id.  Every segment's dictionary must hold data_type. */
int pg_dict_id_sets(const uint64_t *seg_keys, uint32_t num_segments, uint32_t col_id, uint32_t data_type,
                    const void *values, uint32_t num_values, int32_t *out_ids, uint32_t *out_counts);

/* ---------------------------------------------------------------- query plan */

typedef enum pg_leaf_kind {
  PG_LEAF_MATCH_ALL = 0,  /* MatchAllFilterOperator / predicate evaluator isAlwaysTrue                  */
  PG_LEAF_EMPTY = 1,      /* EmptyFilterOperator / isAlwaysFalse                                        */
  PG_LEAF_SV_SCAN = 2,    /* ScanBasedFilterOperator over a bit-packed SV forward index                 */
  PG_LEAF_SORTED = 3,     /* SortedIndexBasedFilterOperator over PG_IDX_FWD_SV_SORTED                   */
  PG_LEAF_INVERTED = 4,   /* BitmapBasedFilterOperator over PG_IDX_INV_BITMAP                           */
  PG_LEAF_MV_SCAN = 5,    /* ScanBasedFilterOperator over a bit-packed MV forward index (any / all)     */
  PG_LEAF_RAW_SCAN = 6,   /* ScanBasedFilterOperator over a raw forward index with a raw-value predicate
                             evaluator (predicate/...PredicateEvaluatorFactory.newRawValueBasedEvaluator)    */
  PG_LEAF_RANGE_INDEX = 7 /* RangeIndexBasedFilterOperator (operator/filter/RangeIndexBasedFilterOperator.java
                             :62-100) over PG_IDX_RANGE, RANGE predicates only: a dictionary column matches
                             dictIds [lo, hi); a raw column takes the PG_LEAF_RAW_SCAN range fields (ilo / ihi,
                             dlo / dhi + inclusivity).  Exact; counts no entries scanned in the filter        */
} pg_leaf_kind;

/* A leaf matches dictIds in the set S, where S = [lo, hi) when num_ids == 0, else S = ids[0..num_ids).
 * exclusive = 0: SV doc matches iff dictId in S; MV doc matches iff ANY value in S.
 * exclusive = 1 (NOT_EQ / NOT_IN): SV doc matches iff dictId not in S; MV doc matches iff ALL values
 *   are not in S (BaseDictionaryBasedPredicateEvaluator.applyMV, :133-150); inverted: flip of the OR.
 * dictIds are per segment: each pg_segment_ref carries its own array of leaves. */
typedef struct pg_leaf {
  uint32_t kind;       /* pg_leaf_kind */
  uint32_t col_id;
  uint32_t exclusive;
  uint32_t num_ids;
  int32_t lo, hi;
  const int32_t *ids;  /* host pointer, sorted ascending, no duplicates */
  /* PG_LEAF_RAW_SCAN (values in the column's stored type): num_ids == 0 -> range; INT / LONG columns match
   * ilo <= v <= ihi (bounds folded to closed on the host), FLOAT / DOUBLE columns dlo <(=) v <(=) dhi per
   * lo_inclusive / hi_inclusive (+-inf = unbounded).  num_ids > 0 -> v in `values` (num_ids sorted unique values
   * of the stored type: EQ / IN).  `exclusive` inverts (NOT_EQ / NOT_IN / NOT BETWEEN by the caller's NOT). */
  int64_t ilo, ihi;
  double dlo, dhi;
  uint32_t lo_inclusive, hi_inclusive;
  const void *values;  /* host pointer */
  /* Dictionary SV / MV scan leaves may carry their IN / NOT_IN literals instead of dictIds: ids == NULL, `values` =
   * num_values sorted unique literals already converted to the column's stored type and widened (int64 for INT /
   * LONG, double for FLOAT / DOUBLE), num_ids = how many of them this segment's dictionary holds (pg_dict_id_sets'
   * count, > 0).  The device finds their dictIds in the resident dictionary itself (one launch for every such leaf of
   * the query), so the per-segment id lists never cross the boundary.  num_values is 0 for every other leaf. */
  uint32_t num_values;
  uint32_t pad;
} pg_leaf;

/* Filter program: postfix over leaves.  op >= 0 pushes leaf `op`; PG_OP_AND(n)/PG_OP_OR(n) pop n
 * operands; PG_OP_NOT pops one.  An empty program means match-all. */
#define PG_OP_NOT (-1)
#define PG_OP_AND(n) (-(int32_t)(0x100 | (n)))
#define PG_OP_OR(n) (-(int32_t)(0x200 | (n)))

typedef enum pg_agg_fn {
  PG_AGG_COUNT = 0,         /* CountAggregationFunction (COUNT(*))                 -> count          */
  PG_AGG_SUM = 1,           /* SumAggregationFunction                              -> double sum     */
  PG_AGG_MIN = 2,           /* MinAggregationFunction                              -> double         */
  PG_AGG_MAX = 3,           /* MaxAggregationFunction                              -> double         */
  PG_AGG_AVG = 4,           /* AvgAggregationFunction                              -> (sum, count)   */
  PG_AGG_DISTINCTCOUNT = 5, /* DistinctCountAggregationFunction (dictionary path) -> value set / size */
  PG_AGG_COUNTMV = 6        /* CountMVAggregationFunction                          -> sum numValues  */
} pg_agg_fn;

typedef enum pg_expr_op {   /* transform applied to the aggregation input (TransformFunction)      */
  PG_EXPR_COL = 0,          /* value(col_a)                                                          */
  PG_EXPR_MUL = 1,          /* MultiplicationTransformFunction: value(col_a) * value(col_b)          */
  PG_EXPR_ADD = 2,          /* AdditionTransformFunction                                             */
  PG_EXPR_SUB = 3           /* SubtractionTransformFunction                                          */
} pg_expr_op;

typedef struct pg_agg {
  uint32_t fn;      /* pg_agg_fn */
  uint32_t op;      /* pg_expr_op (SUM/MIN/MAX/AVG) */
  uint32_t col_a;   /* input column (unused for COUNT) */
  uint32_t col_b;   /* second operand for PG_EXPR_MUL/ADD/SUB */
  /* DISTINCTCOUNT only: how the value's table-global id is formed (see pg_key) */
  uint32_t key_kind;
  uint32_t key_cardinality;
  int64_t key_base;
  /* SUM / AVG accumulated exactly in fixed point (every input that is not provably an integer, or all of them with
   * PG_PLAN_F64_SUMS).  With PG_SUM_BOUNDS in sum_flags, 2^sum_exp_lo <= |x| <= 2^sum_exp bounds every nonzero finite
   * input value over the whole table (from the columns' metadata: largest and smallest nonzero |value|, combined
   * through the expression), so every GPU and server that merges this plan's partial states cuts the sum into the same
   * exponent windows (pg_partials.fx_sig); without it the library derives the bounds from the plan's resident
   * segments.  Ignored by the other functions. */
  int32_t sum_exp;
  uint32_t sum_flags;  /* SUM / AVG: PG_SUM_NONFINITE = some input of the table may be +-inf / NaN (a FLOAT / DOUBLE column
                          holding them, or a product / sum that overflows), so every GPU keeps the same slots for them;
                          PG_SUM_BOUNDS = sum_exp / sum_exp_lo are given */
  int32_t sum_exp_lo;
  uint32_t flags;   /* PG_AGG_MV_VALUES (ABI 9; zero before) */
} pg_agg;
#define PG_SUM_NONFINITE 0x1u
#define PG_SUM_BOUNDS 0x2u
/* pg_agg.flags: fn (SUM / MIN / MAX / AVG / DISTINCTCOUNT, op PG_EXPR_COL) over EVERY value of the multi-value column
 * col_a -- SumMVAggregationFunction, MinMVAggregationFunction, MaxMVAggregationFunction, AvgMVAggregationFunction,
 * DistinctCountMVAggregationFunction (query/aggregation/function/): the single-value function's intermediate and
 * final types, aggregate() over getDictionaryIdsMV / getDoubleValuesMV; AVG counts the values, not the docs */
#define PG_AGG_MV_VALUES 0x1u

typedef enum pg_key_kind {
  PG_KEY_VALUE_OFFSET = 0,  /* INT/LONG dictionary: global id = value - base                         */
  PG_KEY_KEYMAP = 1         /* global id = PG_IDX_KEYMAP[dictId] of (segment, col)                   */
} pg_key_kind;

typedef struct pg_key {
  uint32_t col_id;
  uint32_t kind;            /* pg_key_kind */
  uint32_t cardinality;     /* size of the table-global key space of this column */
  uint32_t pad;
  int64_t base;             /* PG_KEY_VALUE_OFFSET */
} pg_key;

typedef struct pg_segment_ref {
  uint64_t seg_key;
  uint32_t num_docs;
  uint32_t pad;
  const pg_leaf *leaves;    /* plan.num_leaves entries */
} pg_segment_ref;

/* ORDER BY item for the device-side trim of a group-by result (IndexedTable.finish ->
 * TableResizer.getTopRecords, data/table/IndexedTable.java:147-158, TableResizer.java:248).  AGG items order
 * by the aggregation's final value (AVG: sum / count, DISTINCTCOUNT: set size); KEY items by the key's
 * table-global id, which is value order for both key kinds. */
typedef enum pg_order_kind { PG_ORDER_AGG = 0, PG_ORDER_KEY = 1 } pg_order_kind;
typedef struct pg_order {
  uint32_t kind;            /* pg_order_kind */
  uint32_t index;           /* aggregation index (AGG) or group-key index (KEY) */
  uint32_t desc;            /* 1 = DESC */
  uint32_t pad;
} pg_order;

#define PG_PLAN_VALUE_SETS 0x1u  /* return DISTINCTCOUNT value sets (the reference's Set intermediate,
                                    DistinctCountAggregationFunction.java:252-310), not only their sizes */
#define PG_PLAN_HASH_GROUPS 0x2u /* group in a hash table even when the key space is small enough to address
                                    directly (same results; for tests and measurements) */
#define PG_PLAN_F64_SUMS 0x4u    /* accumulate every SUM / AVG as an exact 128-bit fixed-point sum (as the sums of
                                    non-integer inputs always are) instead of integer-exact int64 for integer
                                    inputs: the reference's double SUM, rounded once at the end; use when partial
                                    states of servers or GPUs whose columns differ in range must merge
                                    (pg_partials.layout) */
#define PG_PLAN_NO_STREAM 0x8u   /* never use the selective stream (a lean kernel over the root AND's first,
                                    selective scan leaf + the fused scan over its survivors); same results */
#define PG_PLAN_EXACT_LIMIT 0x10u /* keep exactly min(limit, #groups) groups: the first `limit` of the result order
                                    (ORDER BY items, then ascending key ids, first key first -- the tie-break that
                                    TableResizer.getTopRecords leaves arbitrary), or without ORDER BY the `limit`
                                    groups of smallest key ids (an IndexedTable without ORDER BY keeps the first
                                    `limit` keys it sees, IndexedTable.java:95-103).  The server-side result of
                                    GroupByOrderByCombineOperator (:79-93, limit = GroupByUtils.getTableCapacity)
                                    and the per-segment trim of AggregationGroupByOrderByOperator (:118-132). */

typedef struct pg_plan {
  uint32_t abi_version;     /* PG_ABI_VERSION */
  uint32_t num_segments;
  const pg_segment_ref *segments;
  uint32_t num_leaves;
  uint32_t num_ops;
  const int32_t *ops;       /* filter program (postfix) */
  uint32_t num_aggs;
  uint32_t num_keys;        /* 0 => aggregation-only query */
  const pg_agg *aggs;
  const pg_key *keys;       /* group-by expressions, in GROUP BY order */
  uint64_t num_groups_limit;/* InstancePlanMakerImplV2 num.groups.limit (per segment): as in the reference a
                               segment keeps the first num_groups_limit distinct keys in doc order
                               (IntGroupIdMap.getGroupId, DictionaryBasedGroupKeyGenerator.java:991-1016) and
                               drops the docs of later keys; 0 = the reference default 100 000 */
  uint64_t query_id;        /* for pg_cancel */
  int64_t deadline_ms;      /* CLOCK_MONOTONIC ms; 0 = none (QueryContext.getEndTimeMs)              */
  void *stream;             /* hipStream_t to launch on; NULL = the library's per-thread stream      */
  uint32_t flags;           /* PG_PLAN_* */
  uint32_t num_order;       /* ORDER BY items (group-by only); 0 = no device-side trim */
  const pg_order *order;
  uint64_t limit;           /* with num_order > 0: keep the groups that rank within the first `limit` under
                               the ORDER BY (every group tied with the limit-th is kept too, so any tie-break
                               the caller applies stays exact -- or exactly `limit` with PG_PLAN_EXACT_LIMIT,
                               which also applies without ORDER BY); 0 = keep all groups */
  uint64_t trim_threshold;  /* the server's IndexedTable trimThreshold (InstancePlanMakerImplV2 groupby.trim.threshold,
                               GroupByOrderByCombineOperator.java:79-93) for a group-by with ORDER BY and the server trim
                               on; 0 = none.  The reference's ConcurrentIndexedTable resizes to min(trimSize,
                               threshold / 2) records whenever it holds >= threshold of them during the merge
                               (ConcurrentIndexedTable.java:61-65, IndexedTable.java:77-80): a lossy, schedule-dependent
                               answer.  The device merges every group exactly and reports it:
                               PG_RESULT_TRIM_THRESHOLD_REACHED. */
} pg_plan;

/* ---------------------------------------------------------------- results */

typedef struct pg_stats {     /* ExecutionStatistics, summed over the plan's segments */
  uint64_t num_docs_scanned;
  uint64_t num_entries_scanned_in_filter;   /* device's own count; not a parity target */
  uint64_t num_entries_scanned_post_filter;
  uint64_t num_total_docs;
  uint64_t num_segments_processed;
  uint64_t num_segments_matched;
} pg_stats;

/* Host-side final result of one plan (library-owned until pg_result_free).
 * Aggregation-only: num_groups = 1.  Group-by: one row per group with at least one matching doc (after the
 * plan's ORDER BY trim, sorted by it with ascending key ids as the final tie-break; unsorted without one).
 * keys[g*num_keys + k] = table-global key id of group g's k-th key.
 * values[g*num_aggs + a]: COUNT / COUNTMV count, SUM sum, MIN/MAX value, AVG sum, DISTINCTCOUNT set size.
 * counts[g*num_aggs + a]: AVG count (0 for the others).
 * With PG_PLAN_VALUE_SETS, the value set of DISTINCTCOUNT aggregation a of group g is
 *   distinct_ids[distinct_offsets[g*num_aggs + a] .. distinct_offsets[g*num_aggs + a + 1]),
 * table-global value ids (the aggregation's key space) in ascending order; other aggregations have empty
 * ranges.  Without the flag both pointers are NULL. */
#define PG_RESULT_GROUPS_LIMIT_REACHED 0x1u  /* some segment reached num_groups_limit groups (its later keys dropped):
                                                IntermediateResultsBlock.isNumGroupsLimitReached, set as
                                                AggregationGroupByOrderByOperator.java:112-113 does */
#define PG_RESULT_TRIM_THRESHOLD_REACHED 0x2u /* the merged groups reached the plan's trim_threshold: the reference
                                                server would have resized its table mid-merge (numResizes > 0) */
typedef struct pg_result {
  pg_stats stats;
  uint64_t num_groups;
  uint32_t num_keys;
  uint32_t num_aggs;
  uint32_t *keys;
  double *values;
  int64_t *counts;
  uint64_t num_distinct;
  uint64_t *distinct_offsets;
  uint32_t *distinct_ids;
  uint64_t num_groups_merged; /* groups of the merged (combined) table before the ORDER BY / limit trim */
  uint32_t flags;             /* PG_RESULT_* */
  uint32_t pad;
} pg_result;

int pg_execute(const pg_plan *plan, pg_result **out);
int pg_result_free(pg_result *res);


/* ---------------------------------------------------------------- partial state (multi-GPU) */

/* Per-group partial state of one plan on this device (with several logical devices: the merged state of all of
 * them, on the first one that ran a segment of the plan; its pg_partials_* calls run there).  Groups are identified by their packed key: the
 * mixed-radix number of their table-global key ids, first key least significant (key k contributes
 * id_k * prod_{j<k} keys[j].cardinality), as DictionaryBasedGroupKeyGenerator forms raw keys (:280-322)
 * but over table-global ids so that segments, GPUs and servers merge by VALUE.
 *   mode PG_STATE_DENSE: slot = packed key, num_slots = prod of the key cardinalities; keys == NULL.
 *   mode PG_STATE_HASH : open-addressing table of num_slots entries; keys[slot] = packed key or
 *                        PG_EMPTY_KEY (IntGroupIdMap / Long2IntOpenHashMap on the device).
 * State arrays, per slot:
 *   i64 [num_slots][n_i64]      merged by SUM (slot 0: doc count; integer sums, AVG counts, COUNTMV)
 *   fx  [num_slots][n_fx][2]    merged by 128-bit SUM: the exact fixed-point sums of SUM / AVG inputs that are not
 *                               provably integers, one (lo, hi) two's-complement pair per exponent window of the
 *                               aggregation (a SUM spans one or more consecutive pairs; the low word's carry goes to the
 *                               high word: a word-wise SUM all-reduce is NOT a merge -- split the words into limbs)
 *   mn  [num_slots][n_min]      merged by MIN (order-preserving int64 image of double MIN)
 *   mx  [num_slots][n_max]      merged by MAX (order-preserving int64 image of double MAX)
 *   bitmaps [num_slots][bitmap_words] merged by OR: per DISTINCTCOUNT aggregation a bitmap over its
 *                               table-global value ids (the per-group RoaringBitmap of the reference)
 * All pointers are device pointers owned by the handle. */
#define PG_STATE_DENSE 0
#define PG_STATE_HASH 1
/* wide group keys (more than kMaxKeys keys, or a key-cardinality product of 2^62 and more: DictionaryBasedGroupKeyGenerator's
 * ArrayMapBasedHolder): the packed key is a slot of the state's own tuple table, local to it.  Such states merge only
 * through the row exchange, whose rows carry the tuple (pg_partials_export). */
#define PG_STATE_TUPLES 2
#define PG_EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

typedef struct pg_partials {
  pg_stats stats;
  uint64_t num_slots;
  uint32_t mode;            /* PG_STATE_* */
  uint32_t n_i64, n_fx, n_min, n_max;
  uint32_t bitmap_words;    /* uint32 words of DISTINCTCOUNT bitmaps per slot */
  uint32_t layout;          /* bit a: SUM / AVG aggregation a accumulates integer-exact in i64 (else in fx); partial
                               states merge only with equal layouts */
  uint32_t fx_sig;          /* signature of the fx sums' fixed-point units: partial states merge only when it agrees */
  uint64_t row_bytes;       /* bytes of one exchange row (pg_partials_export) */
  uint64_t *keys;
  int64_t *i64;
  int64_t *fx;
  int64_t *mn;
  int64_t *mx;
  uint32_t *bitmaps;
  void *impl;
  uint32_t flags;           /* PG_RESULT_* seen producing this state (the caller ORs the ranks' flags before finalize) */
  uint32_t pad;
} pg_partials;

int pg_execute_partial(const pg_plan *plan, pg_partials **out);
/* Decode (possibly merged) partial state into a host pg_result, applying the plan's ORDER BY trim and
 * PG_PLAN_VALUE_SETS.  `plan` must be the plan the partials were produced from (its aggs / keys / order are
 * read). */
int pg_partials_finalize(pg_partials *p, const pg_plan *plan, pg_result **out);
int pg_partials_free(pg_partials *p);
/* Dense merge: copy the state arrays out to (PG_COPY_OUT) or back in from (PG_COPY_IN) caller-owned DEVICE
 * buffers (e.g. torch tensors the ranks all-reduce over RCCL: SUM for i64, MIN for mn, MAX for mx).  i64 / mn / mx keep
 * their layout and size; fx travels as 4 int64 limbs per sum (num_slots * n_fx * 4 words: limb k = bits [32k, 32k+32)
 * of the 128-bit pair), so a plain SUM all-reduce over up to 2^31 ranks merges it exactly -- PG_COPY_IN folds the
 * limbs' carries back into the pairs.  Bitmaps are not all-reducible (OR): plans with DISTINCTCOUNT use the row exchange below.  A NULL
 * pointer skips that array.  `stream` NULL = the library's per-thread stream; synchronous. */
#define PG_COPY_OUT 0
#define PG_COPY_IN 1
int pg_partials_copy(pg_partials *p, int dir, void *i64, void *fx, void *mn, void *mx, void *stream);
/* Sparse merge (GroupByOrderByCombineOperator's value-keyed merge across GPUs): the groups of `p` as rows
 *   { u64 packed key | i64[n_i64] | i64 fx[n_fx][2] | i64 mn[n_min] | i64 mx[n_max] | u32 bitmaps[bitmap_words] }
 * (row_bytes each, 8-byte aligned), bucketed by owner part = pg_key_owner(key, num_parts), buckets in part order.
 * PG_STATE_TUPLES: each row is followed by its K table-global key ids (u32, padded to 8 bytes; row_bytes includes
 * them) and the owner part is a hash of those ids, so a group has one owner on every GPU; the merge target re-interns
 * them (IndexedTable.upsert of a Key(Object[]), IndexedTable.java:103-117).
 * part_counts[num_parts] (host) receives the rows per bucket.  dst (DEVICE, dst_rows rows) may be NULL to only
 * count.  Synchronous on `stream`. */
int pg_partials_export(pg_partials *p, uint32_t num_parts, void *dst, uint64_t dst_rows, uint64_t *part_counts,
                       void *stream);
/* A fresh, empty PG_STATE_HASH partial state with the layout of `like` (its plan's aggregations and keys) and room
 * for at least `capacity` groups; its stats are zero. */
int pg_partials_create(const pg_partials *like, uint64_t capacity, pg_partials **out);
/* Merge `n` exported rows (DEVICE buffer) into `p` (which must be PG_STATE_HASH): insert missing keys, then
 * SUM / MIN / MAX / OR the state (AggregationFunction.merge of each function). */
int pg_partials_merge(pg_partials *p, const void *rows, uint64_t n, void *stream);
/* Owner part of a packed key among num_parts (the bucketing of pg_partials_export). */
uint32_t pg_key_owner(uint64_t key, uint32_t num_parts);

/* ---------------------------------------------------------------- relocatable plan image (JNI / FFI callers)
 *
 * The same plan as ONE self-contained byte buffer whose sub-arrays are byte offsets from the buffer's start instead
 * of pointers, so a Java GpuPlanMaker (the PlanMaker.makeInstancePlan replacement, plan/maker/PlanMaker.java:42) fills
 * a direct ByteBuffer (native byte order, 8-byte aligned: ByteBuffer.allocateDirect(n + 8).alignedSlice(8)) with
 * putInt / putLong and hands its address and length over -- no Unsafe address arithmetic.
 * Layout (every offset a multiple of the element's alignment, every array inside [0, n); offset 0 = no array):
 *   pg_image_header at 0
 *   pg_image_segment[num_segments] at segments_off, each pointing at its pg_image_leaf[num_leaves] (leaves_off)
 *   int32 ops[num_ops], pg_agg[num_aggs], pg_key[num_keys], pg_order[num_order] at their offsets
 *   leaf arrays: int32 dictIds[num_ids] at ids_off; 8-byte values at values_off (num_values literals in values mode,
 *   else num_ids raw values) -- segments may share one array (the same offset).
 * The image is validated in full before anything runs (PG_E_INVALID names the first bad field); it is borrowed for
 * the call only.  The library's per-thread stream is used (a JNI caller has no HIP stream to pass). */
#define PG_IMAGE_MAGIC 0x49504750u /* "PGPI" */

typedef struct pg_image_header {
  uint32_t magic;           /* PG_IMAGE_MAGIC */
  uint32_t abi_version;     /* PG_ABI_VERSION */
  uint64_t image_bytes;     /* the buffer length n */
  uint32_t num_segments;
  uint32_t num_leaves;
  uint32_t num_ops;
  uint32_t num_aggs;
  uint32_t num_keys;
  uint32_t num_order;
  uint32_t flags;           /* PG_PLAN_* */
  uint32_t trim_threshold;  /* pg_plan.trim_threshold (an int on the reference's side) */
  uint64_t num_groups_limit;
  uint64_t query_id;
  int64_t deadline_ms;
  uint64_t limit;
  uint64_t segments_off;    /* pg_image_segment[num_segments] */
  uint64_t ops_off;         /* int32_t[num_ops] */
  uint64_t aggs_off;        /* pg_agg[num_aggs] */
  uint64_t keys_off;        /* pg_key[num_keys] */
  uint64_t order_off;       /* pg_order[num_order] */
} pg_image_header;          /* 120 bytes */

typedef struct pg_image_segment {
  uint64_t seg_key;
  uint32_t num_docs;
  uint32_t pad;
  uint64_t leaves_off;      /* pg_image_leaf[num_leaves] */
} pg_image_segment;         /* 24 bytes */

typedef struct pg_image_leaf { /* pg_leaf with its two host pointers replaced by offsets (same size, same fields) */
  uint32_t kind, col_id, exclusive, num_ids;
  int32_t lo, hi;
  uint64_t ids_off;
  int64_t ilo, ihi;
  double dlo, dhi;
  uint32_t lo_inclusive, hi_inclusive;
  uint64_t values_off;
  uint32_t num_values;
  uint32_t pad;
} pg_image_leaf;            /* 88 bytes */

int pg_execute_image(const void *image, uint64_t n, pg_result **out);
int pg_execute_partial_image(const void *image, uint64_t n, pg_partials **out);
int pg_partials_finalize_image(pg_partials *p, const void *image, uint64_t n, pg_result **out);

/* ---------------------------------------------------------------- measurement hooks */

/* Timing of the last pg_execute* / pg_partials_finalize on this thread.  Device time (ms, HIP events on the
 * execution stream): the index pre-pass (IN-set LUTs, sorted / inverted / MV leaf bitmaps), the streaming
 * pre-filter of the root AND's leaves, the fused scan/aggregate kernel, the finalize (group selection, ORDER BY
 * trim, read-back).  Host wall time (ms, steady clock): plan compile up to the scan launch, the whole execute call,
 * the finalize call. */
typedef struct pg_timing {
  float prepass_ms;
  float scan_ms;
  float finalize_ms;
  uint32_t scan_launches;  /* hot-path kernels: the fused scan (1) + the selective stream (1) when it ran */
  float host_compile_ms;
  float execute_wall_ms;
  float finalize_wall_ms;
  float prefilter_ms;
} pg_timing;
int pg_last_timing(pg_timing *out);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_GPU_H */
