/*
 * pinot_trace.h -- per-call trace recording of libpinot_gpu.so (C ABI).
 *
 * The reference wraps every operator in a trace scope (Tracing.getTracer().createScope, pinot-core/.../operator/
 * BaseOperator.java:38) and its filter operators record their kind and the docs they matched
 * (filter/BitmapBasedFilterOperator.java:102-107, SortedIndexBasedFilterOperator, ScanBasedFilterOperator).  A device
 * call replaces that whole operator tree, so its recording is one struct per call: which physical form each filter leaf
 * took in how many segments, which kernels ran, whether a speculative layout overflowed and the query re-ran, and the
 * docs / groups it produced.  The Java side attaches it to the query's trace (TraceContext) when tracing is on.
 */
#ifndef PINOT_TRACE_H
#define PINOT_TRACE_H

#include <stdint.h>

#include "pinot_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PG_TRACE_MAX_LEAVES 16

typedef enum pg_leaf_form {  /* the device form a filter leaf took in one segment */
  PG_FORM_MATCH_ALL = 0,     /* MatchAllFilterOperator (isAlwaysTrue, IS NOT NULL without a null vector)          */
  PG_FORM_EMPTY = 1,         /* EmptyFilterOperator (isAlwaysFalse, or a sorted range with no docs)               */
  PG_FORM_SCAN_RANGE = 2,    /* ScanBasedFilterOperator, dictId range test in registers                             */
  PG_FORM_SCAN_SET_LDS = 3,  /* ScanBasedFilterOperator, IN set as an LDS bitmap (+ exact LUT)                      */
  PG_FORM_SCAN_SET_LUT = 4,  /* ScanBasedFilterOperator, IN set as a global LUT over dictIds                        */
  PG_FORM_SORTED_RANGE = 5,  /* SortedIndexBasedFilterOperator, one doc range                                       */
  PG_FORM_SORTED_BITMAP = 6, /* SortedIndexBasedFilterOperator, several ranges -> doc bitmap (pre-pass)             */
  PG_FORM_INVERTED = 7,      /* BitmapBasedFilterOperator: roaring containers -> doc bitmap (pre-pass)              */
  PG_FORM_MV_SCAN = 8,       /* ScanBasedFilterOperator over an MV forward index -> doc bitmap (pre-pass)           */
  PG_FORM_RAW_SCAN = 9,      /* raw-value predicate over a raw forward index                                        */
  PG_FORM_RANGE_INDEX = 10,  /* RangeIndexBasedFilterOperator                                                       */
  PG_FORM_COUNT = 11
} pg_leaf_form;

#define PG_PATH_FUSED_SCAN 0x1u  /* the fused filter + aggregate scan kernel ran                                  */
#define PG_PATH_STREAM 0x2u      /* the selective stream drove the root AND's leaf `stream_leaf` (list-mode scan)   */
#define PG_PATH_PARTITIONED 0x4u /* the radix-partitioned group-by (pg_part.hip)                                    */
#define PG_PATH_WIDE_KEYS 0x8u   /* tuple-interned group keys (ArrayMapBasedHolder form)                            */
#define PG_PATH_NONSCAN 0x10u    /* some segments answered from metadata (NonScanBasedAggregationOperator)          */
#define PG_PATH_PREPASS 0x20u    /* index pre-pass kernels (IN-set LUTs, sorted / inverted / MV doc bitmaps)         */
#define PG_PATH_INDEX_COUNT 0x40u /* the fused index count: inverted leaves decoded per 64 K-doc key in LDS, COUNT /
                                     COUNTMV counted there (no doc bitmaps in HBM)                                    */

#define PG_RERUN_STREAM 0x1u     /* the stream's survivor regions overflowed: re-ran without the stream            */
#define PG_RERUN_PARTITION 0x2u  /* a speculative partition region overflowed: re-ran with exact offsets            */
#define PG_RERUN_HASH 0x4u       /* the group hash table filled up: re-ran with 8x the slots                        */

typedef struct pg_trace {
  uint64_t query_id;
  uint32_t path;             /* PG_PATH_* */
  uint32_t group_mode;       /* 0 aggregation only, 1 dense, 2 hash, 3 hash per segment (numGroupsLimit), 4 partitioned */
  uint32_t reruns;           /* re-runs of the call */
  uint32_t rerun_reasons;    /* PG_RERUN_* */
  uint32_t num_leaves;       /* filter leaves of the plan (forms recorded for the first PG_TRACE_MAX_LEAVES) */
  uint32_t stream_leaf;      /* leaf index the stream drove, 0xFFFFFFFF = none */
  uint32_t leaf_forms[PG_TRACE_MAX_LEAVES][PG_FORM_COUNT]; /* segments in which leaf l took form f */
  uint32_t pad;
  uint64_t num_segments;
  uint64_t num_segments_nonscan;
  uint64_t num_docs_matched; /* docs passing the filter (numDocsScanned) */
  uint64_t num_slots;        /* group state slots (dense key space or hash table size) */
  float device_ms;           /* pre-pass + stream + scan / partition passes (HIP events) */
  float wall_ms;             /* the whole call */
} pg_trace;

/* The recording of the calling thread's last pg_execute* call. */
int pg_last_trace(pg_trace *out);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_TRACE_H */
