/*
 * pinot_oracle.h — CPU restatement of the reference's segment-execution hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker for the HIP product path
 * (pinot_amd/csrc). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product never links or calls it.
 *
 * Every function is a scalar, line-by-line restatement of the Pinot Java code it
 * cites (paths relative to the reference checkout). Parity is pinned by
 * tests/test_oracle_golden.py against the expected values hard-coded in the
 * reference's own query tests (tests/golden/sv_queries_expected.json).
 */
#ifndef PINOT_ORACLE_H
#define PINOT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* stored types (FieldSpec.DataType stored types on the path) */
enum { OR_INT = 0, OR_LONG = 1, OR_FLOAT = 2, OR_DOUBLE = 3 };
/* forward-index encodings */
/* OR_ENC_IDS: a plain int32 group id per doc, the value -> id map a raw column's group key generator
 * builds (NoDictionarySingleColumnGroupKeyGenerator.java:98-143); fwd = int32[num_docs] */
enum { OR_ENC_FIXED_BIT = 0, OR_ENC_RAW = 1, OR_ENC_SORTED = 2, OR_ENC_IDS = 3 };
/* predicate leaf kinds */
enum {
  OR_PRED_DICT_RANGE = 0,   /* dictId in [lo, hi)            SortedDictionaryBasedRangePredicateEvaluator */
  OR_PRED_DICT_SET = 1,     /* dict_mask[dictId] != 0         DictionaryBasedIn/Eq/Unsorted-range evaluators */
  OR_PRED_RAW_RANGE = 2,    /* value in [lo, hi] inclusive   *RawValueBasedRangePredicateEvaluator */
  OR_PRED_RAW_IN = 3,       /* value in set                  *RawValueBasedInPredicateEvaluator */
  OR_PRED_DOC_BITSET = 4    /* precomputed docId bitset      BitmapBasedFilterOperator (inverted index) */
};
/* aggregation functions */
/* OR_AGG_RMIN / OR_AGG_RMAX: the two sides of MINMAXRANGE's MinMaxRangePair */
enum { OR_AGG_COUNT = 0, OR_AGG_SUM = 1, OR_AGG_MIN = 2, OR_AGG_MAX = 3, OR_AGG_SUMLONG = 4, OR_AGG_RMIN = 5,
       OR_AGG_RMAX = 6 };

typedef struct {
  int32_t encoding;      /* OR_ENC_* */
  int32_t stored_type;   /* value type (dictionary value type for dict columns) */
  int32_t bits;          /* fixed-bit width */
  int32_t cardinality;
  const uint8_t* fwd;    /* fixed-bit bytes | sorted (min,max) BE pairs | raw values (BE, at rawDataStart) */
  const void* dict;      /* dictionary values, little-endian native array, or NULL */
} oracle_column;

typedef struct {
  int32_t column;
  int32_t kind;
  int32_t negate;
  int32_t clause;        /* CNF clause index: filter = AND over clauses of (OR over leaves) */
  int64_t lo_i, hi_i;    /* integer bounds (dictIds or INT/LONG values) */
  double lo_d, hi_d;     /* FLOAT/DOUBLE bounds */
  const uint8_t* dict_mask;   /* OR_PRED_DICT_SET: one byte per dictId */
  const int64_t* set_i;       /* OR_PRED_RAW_IN (INT/LONG) */
  const double* set_d;        /* OR_PRED_RAW_IN (FLOAT/DOUBLE) */
  int32_t set_n;
  const uint64_t* doc_bitset; /* OR_PRED_DOC_BITSET */
} oracle_leaf;

/* aggregated expression: a column, or a binary arithmetic transform of two columns
 * (MultiplicationTransformFunction / SubtractionTransformFunction / AdditionTransformFunction:
 * DOUBLE results) */
enum { OR_EXPR_COL = 0, OR_EXPR_MUL = 1, OR_EXPR_SUB = 2, OR_EXPR_ADD = 3 };
typedef struct {
  int32_t func;
  int32_t column;        /* -1 for COUNT(*) */
  int32_t expr;          /* OR_EXPR_* */
  int32_t column2;       /* second operand of a binary expression */
} oracle_agg;

/* ---- forward index ---- */
int32_t oracle_fixedbit_read(const uint8_t* buf, int32_t bits, int64_t index);
void oracle_fixedbit_read_range(const uint8_t* buf, int32_t bits, int64_t start, int64_t n, int32_t* out);
void oracle_fixedbit_write(uint8_t* buf, int32_t bits, int64_t start, int64_t n, const int32_t* values);
int32_t oracle_sorted_dict_id(const uint8_t* pairs, int32_t cardinality, int64_t doc);
int64_t oracle_raw_read_i64(const uint8_t* raw, int32_t type, int64_t index);
double oracle_raw_read_f64(const uint8_t* raw, int32_t type, int64_t index);
void oracle_column_dict_ids(const oracle_column* col, int64_t start, int64_t n, int32_t* out);

int64_t oracle_lz4_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t oracle_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t oracle_delta_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t dd);

/* ---- inverted index (BitmapInvertedIndexReader + RoaringBitmap portable format) ---- */
int oracle_roaring_to_bitset(const uint8_t* buf, int64_t len, uint64_t* bitset, int64_t num_docs);
int oracle_inverted_to_bitset(const uint8_t* inv, int32_t cardinality, const int32_t* dict_ids, int32_t n,
                              uint64_t* bitset, int64_t num_docs);

/* ---- filter ---- */
int64_t oracle_filter(const oracle_column* cols, int64_t num_docs, const oracle_leaf* leaves, int32_t nleaves,
                      uint64_t* out_bitset);
int64_t oracle_bitset_to_doc_ids(const uint64_t* bitset, int64_t num_docs, int32_t* out);

/* ---- aggregation (AggregationOperator) ---- */
/* 1: integer SUMs accumulate in double in doc order as the reference does; 0 (default): exact 128-bit */
void oracle_set_literal_int_sum(int32_t on);
int32_t oracle_literal_int_sum(void);
/* out: per agg one double (COUNT as double too); out_i64 / out_hi64: COUNT / SUMLONG as int64, and an
 * integer SUM's exact 128-bit value as (low, high) words */
int oracle_aggregate(const oracle_column* cols, int64_t num_docs, const uint64_t* bitset, const oracle_agg* aggs,
                     int32_t naggs, double* out, int64_t* out_i64, int64_t* out_hi64);

/* ---- group-by (GroupByOperator + DefaultGroupByExecutor + DictionaryBasedGroupKeyGenerator) ---- */
/* Groups in group-id (first-seen) order, at most num_groups_limit of them (the map holders' trimming);
 * out_keys[g*ngroup + j] = dictId of group-by column j; out_vals[g*naggs + a]; out_i64 / out_hi64 as
 * in oracle_aggregate. *out_limit_reached = numGroupsLimitReached.
 * Returns number of groups or -1 if more than max_groups. */
int64_t oracle_group_by(const oracle_column* cols, int64_t num_docs, const uint64_t* bitset,
                        const int32_t* group_cols, int32_t ngroup, const oracle_agg* aggs, int32_t naggs,
                        int64_t num_groups_limit, int64_t max_groups, int32_t* out_keys, double* out_vals,
                        int64_t* out_i64, int64_t* out_hi64, int32_t* out_limit_reached);

#ifdef __cplusplus
}
#endif
#endif
