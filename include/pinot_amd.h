/*
 * pinot_amd.h — C ABI of the MI355X segment-execution library (libpinot_amd.so).
 *
 * This is the drop-in boundary for Pinot's server-side segment execution hot path:
 * forward-index scan, filter (scan + inverted index), aggregation and group-by over
 * immutable segments staged in HBM. Every entry point takes plain pointers and sizes
 * (no torch or Java types), so a JNI / Panama FFM binding in pinot-core can call it
 * directly; INTEGRATION.md shows the Java-side binding.
 *
 * Each entry point names the reference interface it replaces (paths relative to the
 * reference checkout root; "core" = pinot-core/src/main/java/org/apache/pinot/core,
 * "local" = pinot-segment-local/src/main/java/org/apache/pinot/segment/local).
 *
 * Conventions
 *   - Return value: 0 on success, a negative PINOT_AMD_E* code on failure; the message is
 *     available from pinot_amd_last_error() (thread-local). Invalid arguments fail loudly;
 *     nothing falls back to a CPU path.
 *   - "stream" is a hipStream_t passed as void* (NULL = the null stream). Calls that
 *     return results to host memory synchronise that stream.
 *   - Device pointers are marked d_. Host pointers are marked h_.
 */
#ifndef PINOT_AMD_H
#define PINOT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PINOT_AMD_ABI_VERSION 1

/* error codes */
#define PINOT_AMD_OK 0
#define PINOT_AMD_EINVAL (-1)     /* bad argument (IllegalArgumentException / IllegalStateException) */
#define PINOT_AMD_EUNSUPPORTED (-2) /* format or query shape not supported by this build */
#define PINOT_AMD_EHIP (-3)       /* HIP runtime error */
#define PINOT_AMD_ENOMEM (-4)     /* device allocation failed */
#define PINOT_AMD_EOVERFLOW (-5)  /* result capacity exceeded */

/* FieldSpec.DataType stored types on the path (pinot-spi/.../data/FieldSpec.java) */
enum pinot_amd_data_type { PINOT_AMD_INT = 0, PINOT_AMD_LONG = 1, PINOT_AMD_FLOAT = 2, PINOT_AMD_DOUBLE = 3,
                           PINOT_AMD_STRING = 4 };

/* Forward-index encodings (local/segment/index/forward/ForwardIndexReaderFactory.java:75-115) */
enum pinot_amd_fwd_encoding {
  PINOT_AMD_FWD_FIXED_BIT = 0, /* dict-encoded SV, unsorted: FixedBitSVForwardIndexReaderV2 */
  PINOT_AMD_FWD_RAW = 1,       /* raw fixed-width SV: FixedBytePower2ChunkSV / FixedByteChunkSV (PASS_THROUGH) */
  PINOT_AMD_FWD_SORTED = 2     /* dict-encoded SV, sorted: SortedIndexReaderImpl */
};

/* Predicate types (pinot-common/.../request/context/predicate/Predicate.java Type) */
enum pinot_amd_predicate_type { PINOT_AMD_EQ = 0, PINOT_AMD_NOT_EQ = 1, PINOT_AMD_IN = 2, PINOT_AMD_NOT_IN = 3,
                                PINOT_AMD_RANGE = 4 };

/* Aggregation functions (pinot-segment-spi/.../AggregationFunctionType.java) */
enum pinot_amd_agg_type { PINOT_AMD_AGG_COUNT = 0, PINOT_AMD_AGG_SUM = 1, PINOT_AMD_AGG_MIN = 2,
                          PINOT_AMD_AGG_MAX = 3, PINOT_AMD_AGG_SUMLONG = 4, PINOT_AMD_AGG_AVG = 5,
                          /* MinMaxRangeAggregationFunction: (min, max) pair built with < / > (NaN never
                           * enters it); final result max - min */
                          PINOT_AMD_AGG_MINMAXRANGE = 6 };

/* ------------------------------------------------------------------------------------------------
 * Runtime
 * --------------------------------------------------------------------------------------------- */
int pinot_amd_abi_version(void);
const char* pinot_amd_last_error(void);
/* hipSetDevice for the calling thread; one process drives one GPU. */
int pinot_amd_set_device(int device);
/* Diagnostic: generate and hipRTC-compile a spread of query-specialised scan kernels (no device
 * needed). Returns 0 when every shape compiles; verbose != 0 prints each shape (and failures). */
int pinot_amd_jit_selftest(int verbose);
/* Bytes of slack the kernels may read past the end of a column buffer handed to the
 * low-level entry points (segments staged by pinot_amd_segment_* are padded internally). */
size_t pinot_amd_required_padding(void);

/* ------------------------------------------------------------------------------------------------
 * Segment staging: ImmutableSegmentLoader + PinotDataBuffer, HBM edition.
 * Replaces the mmap of a segment's column buffers (local/segment/index/loader/ImmutableSegmentLoader.java,
 * pinot-segment-spi/.../memory/PinotDataBuffer.java). The host buffers are the exact bytes of the
 * segment's index files (V1 files or V3 columns.psf slices); they are copied to HBM once and may be
 * released by the caller after the call returns.
 * --------------------------------------------------------------------------------------------- */
typedef struct pinot_amd_segment pinot_amd_segment;

typedef struct pinot_amd_column_spec {
  const char* name;
  int32_t stored_type;        /* pinot_amd_data_type (value type; dictionary value type for dict columns) */
  int32_t encoding;           /* pinot_amd_fwd_encoding */
  int32_t cardinality;        /* ColumnMetadata.getCardinality (dict columns) */
  int32_t bits_per_element;   /* ColumnMetadata.getBitsPerElement (fixed-bit) */
  const void* h_fwd;          /* forward index buffer */
  size_t fwd_size;
  const void* h_dictionary;   /* dictionary buffer (BE fixed width; strings NUL padded), or NULL */
  size_t dictionary_size;
  const void* h_inverted;     /* bitmap inverted index buffer (BitmapInvertedIndexWriter layout), or NULL */
  size_t inverted_size;
} pinot_amd_column_spec;

int pinot_amd_segment_create(const char* name, int64_t num_docs, pinot_amd_segment** out);
/* Raw (no-dictionary) forward indexes may use any ChunkCompressionType (ChunkCompressionType.java:22):
 * PASS_THROUGH chunks are copied; LZ4, LZ4_LENGTH_PREFIXED, SNAPPY, DELTA and DELTADELTA chunks are
 * decoded on the device (one wave per chunk, BaseChunkForwardIndexReader.decompressChunk); ZSTANDARD
 * and GZIP chunks are inflated on the host with the system libzstd / zlib. Malformed chunks fail
 * with PINOT_AMD_EINVAL. */
int pinot_amd_segment_add_column(pinot_amd_segment* seg, const pinot_amd_column_spec* spec);
int pinot_amd_segment_destroy(pinot_amd_segment* seg);
int64_t pinot_amd_segment_num_docs(const pinot_amd_segment* seg);
/* HBM bytes held by the segment (forward indexes + dictionaries + inverted indexes + directories). */
int64_t pinot_amd_segment_device_bytes(const pinot_amd_segment* seg);
/* Device pointer to a staged column's forward-index values (fixed-bit stream, raw values at
 * rawDataStart, or sorted pairs) — for the low-level entry points below. */
const void* pinot_amd_segment_column_fwd(const pinot_amd_segment* seg, const char* column);

/* ------------------------------------------------------------------------------------------------
 * Low-level operators (one per reference class), device in / device out.
 * --------------------------------------------------------------------------------------------- */

/* FixedBitSVForwardIndexReaderV2.readDictIds over a contiguous docId range
 * (local/segment/index/readers/forward/FixedBitSVForwardIndexReaderV2.java:64-103, FixedBitIntReader.read32).
 * d_packed: big-endian MSB-first bit stream; writes length int32 dictIds to d_out. */
int pinot_amd_fwd_read_dict_ids(const void* d_packed, int32_t bits, int64_t start_doc, int64_t length,
                                int32_t* d_out, void* stream);

/* FixedBitSVForwardIndexWriter (local/io/writer/impl/FixedBitSVForwardIndexWriter.java) — packs
 * num_values int32 dictIds into the big-endian bit stream (ceil(n*bits/8) bytes written). */
int pinot_amd_fwd_pack_dict_ids(const int32_t* d_values, int64_t num_values, int32_t bits, void* d_packed,
                                void* stream);

/* FixedBytePower2ChunkSVForwardIndexReader.readValuesSV on a PASS_THROUGH buffer
 * (local/segment/index/readers/forward/FixedBytePower2ChunkSVForwardIndexReader.java:48-90):
 * big-endian values at d_raw (rawDataStart) -> native little-endian values in d_out. */
int pinot_amd_fwd_read_raw(const void* d_raw, int32_t stored_type, int64_t start_doc, int64_t length, void* d_out,
                           void* stream);

/* Dense docId bitsets: bit d of word d/64 set <=> doc d matches (MutableRoaringBitmap in
 * core/operator/docidsets, expanded). num_words = ceil(num_docs / 64). */
int pinot_amd_bitset_and(const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_out, int64_t num_words, void* stream);
int pinot_amd_bitset_or(const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_out, int64_t num_words, void* stream);
int pinot_amd_bitset_not(const uint64_t* d_a, uint64_t* d_out, int64_t num_docs, void* stream);
/* BlockDocIdIterator materialisation (core/operator/dociditerators): ascending docIds of the set
 * bits, compacted with wavefront ballot + prefix sums. h_count receives the count. d_out must hold
 * num_docs int32. */
int pinot_amd_bitset_to_doc_ids(const uint64_t* d_bitset, int64_t num_docs, int32_t* d_out, int64_t* h_count,
                                void* stream);
int pinot_amd_bitset_count(const uint64_t* d_bitset, int64_t num_docs, int64_t* h_count, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Query plan: FilterPlanNode + AggregationPlanNode / GroupByPlanNode + CombinePlanNode.
 * A query is compiled once on the host (predicate evaluation per segment mirrors
 * core/operator/filter/predicate/PredicateEvaluatorProvider.java) and executed over a batch of
 * segments in one device pass (replaces ServerQueryExecutorV1Impl -> InstancePlanMakerImplV2 ->
 * per-segment operators -> GroupByCombineOperator / AggregationCombineOperator).
 * --------------------------------------------------------------------------------------------- */
typedef struct pinot_amd_query pinot_amd_query;

typedef struct pinot_amd_predicate_spec {
  const char* column;
  int32_t type;               /* pinot_amd_predicate_type */
  int32_t num_values;         /* EQ/NOT_EQ: 1; IN/NOT_IN: n; RANGE: unused */
  const int64_t* h_values_i;  /* values for INT/LONG columns */
  const double* h_values_d;   /* values for FLOAT/DOUBLE columns */
  const char* const* h_values_s; /* values for STRING columns */
  /* RANGE (RangePredicate): bounds in the column's value domain */
  int32_t lower_unbounded, upper_unbounded, lower_inclusive, upper_inclusive;
  int64_t lower_i, upper_i;
  double lower_d, upper_d;
  const char* lower_s;
  const char* upper_s;
  int32_t use_inverted_index; /* 1: evaluate through the bitmap inverted index (BitmapBasedFilterOperator) */
} pinot_amd_predicate_spec;

int pinot_amd_query_create(pinot_amd_query** out);
int pinot_amd_query_destroy(pinot_amd_query* q);
/* Filter in conjunctive normal form: clause c is the OR of its predicates; the filter is the AND of
 * all clauses (an AND/OR/NOT tree is normalised to CNF by the caller; NOT on a leaf = NOT_EQ/NOT_IN
 * or negate=1). */
int pinot_amd_query_add_predicate(pinot_amd_query* q, int32_t clause, const pinot_amd_predicate_spec* p,
                                  int32_t negate);
/* GROUP BY on dictionary-encoded columns (DictionaryBasedGroupKeyGenerator.java:116-180) or on raw
 * INT/LONG/FLOAT/DOUBLE columns (NoDictionarySingleColumnGroupKeyGenerator.java:98-143,
 * NoDictionaryMultiColumnGroupKeyGenerator: one group per distinct value, FLOAT/DOUBLE told apart by
 * floatToIntBits/doubleToLongBits). A raw column gets a derived dictionary twin staged on its segment
 * at the first such query (kept for later queries). */
int pinot_amd_query_add_group_by(pinot_amd_query* q, const char* column);
/* Aggregation function (column NULL or "*" for COUNT(*)). Returns the aggregation index via out_index. */
int pinot_amd_query_add_aggregation(pinot_amd_query* q, int32_t agg_type, const char* column, int32_t* out_index);
/* Aggregation over a binary arithmetic transform of two columns (SUM / MIN / MAX / AVG):
 * MultiplicationTransformFunction (times), SubtractionTransformFunction (minus),
 * AdditionTransformFunction (plus) in core/operator/transform/function/. Pinot evaluates these in
 * double; with two INT operands the device sums the exact int64 value (equal to the reference's
 * double sum while partial sums stay below 2^53), otherwise it computes in double as the
 * reference does. Needs the query-specialised (hipRTC) kernel; EUNSUPPORTED without it. */
enum pinot_amd_expr_op { PINOT_AMD_EXPR_COLUMN = 0, PINOT_AMD_EXPR_MUL = 1, PINOT_AMD_EXPR_SUB = 2,
                         PINOT_AMD_EXPR_ADD = 3 };
int pinot_amd_query_add_aggregation_expr(pinot_amd_query* q, int32_t agg_type, int32_t expr_op, const char* column_a,
                                         const char* column_b, int32_t* out_index);
/* Install the group key space of group-by column `column` (values in the column's stored type, any
 * order; duplicates ignored): the union of the dictionaries of every server's segments, so that the
 * dense accumulator tables of all servers index groups identically and can be merged in place
 * (the broker merges by value: GroupByDataTableReducer.java:258). Must hold every dictionary value of
 * the segments executed (EINVAL otherwise). Without it the key space is the union over the batch. */
int pinot_amd_query_set_group_key_values(pinot_amd_query* q, const char* column, int32_t stored_type, int64_t n,
                                         const int64_t* h_values_i, const double* h_values_d,
                                         const char* const* h_values_s);
/* QueryOptions numGroupsLimit (InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT = 100000). */
int pinot_amd_query_set_num_groups_limit(pinot_amd_query* q, int64_t limit);
/* The server's combine table (GroupByUtils.createIndexedTableForCombineOperator, GroupByUtils.java:104-149;
 * IndexedTable.finish): with no ORDER BY the result keeps LIMIT groups (the table stops accepting new
 * ones; here the first LIMIT in ascending key order); with ORDER BY the top
 * trimSize = max(5 * LIMIT, min_server_group_trim_size) groups by the ORDER BY, sorted (ties in ascending
 * key order). min_server_group_trim_size <= 0 disables the trim (every group kept when ordered). Replaces
 * the server-side IndexedTable of GroupByCombineOperator; not set: every group is returned. */
int pinot_amd_query_set_result_limit(pinot_amd_query* q, int64_t limit, int64_t min_server_group_trim_size,
                                     int64_t group_trim_threshold);
/* Query options of the server result's size (defaults 0 / 10000): serverReturnFinalResult (with ORDER BY and
 * no HAVING the table keeps LIMIT groups, GroupByUtils.java:134-139) and sortAggregateLimitThreshold. With
 * ORDER BY keys = GROUP BY keys (safe trim, QueryContext.java:568-580,746-747) and LIMIT below the threshold,
 * Pinot's sorted combine (CombinePlanNode.java:150-154) keeps the top LIMIT groups, exact; at or above it each
 * segment keeps its top LIMIT groups by the ORDER BY (GroupByOperator.java:157-175) and the combine table the
 * top trimSize of their union -- restated for dense key spaces (a presence pass over ORDER BY ranks, each
 * segment's LIMIT-th rank as the cutoff its docs are aggregated within) and over hash-table key spaces (the
 * (key, segment) scan table, each segment's top LIMIT entries by a radix selection over the ORDER BY). */
int pinot_amd_query_set_server_options(pinot_amd_query* q, int32_t server_return_final_result,
                                       int64_t sort_aggregate_limit_threshold);
/* QueryOptions minSegmentGroupTrimSize (default -1: CommonConstants.java:1436). With ORDER BY not equal to the
 * GROUP BY keys (an unsafe trim) and a positive value, each segment keeps its top max(value, 5 x LIMIT) groups
 * by the ORDER BY, aggregation values included (QueryContext.java:575-578, GroupByUtils.java:63-66): the (key,
 * segment) hash plan, each segment's top entries by a radix selection over the ORDER BY's final values (ties in
 * ascending group key; TableResizer leaves them unspecified). Under a safe trim the segment trim size is LIMIT
 * whatever this value (pinot_amd_query_set_server_options). */
int pinot_amd_query_set_segment_trim(pinot_amd_query* q, int64_t min_segment_group_trim_size);
/* ORDER BY key of the server table, in order of precedence: kind 0 = group-by column `index` (value
 * order), kind 1 = aggregation `index` (final value, Double.compare); ascending != 0 for ASC. */
int pinot_amd_query_add_order_by(pinot_amd_query* q, int32_t kind, int32_t index, int32_t ascending);

/* ------------------------------------------------------------------------------------------------
 * Execution and results (IntermediateResultsBlock / AggregationGroupByResult equivalents).
 * --------------------------------------------------------------------------------------------- */
typedef struct pinot_amd_result pinot_amd_result;

/* Execute q over n segments as one batched device pass on `stream`; results stay in HBM until
 * fetched. The group key space across segments is the union of their dictionaries. */
int pinot_amd_execute(pinot_amd_query* q, pinot_amd_segment* const* segs, int32_t n, void* stream,
                      pinot_amd_result** out);
/* FilterPlanNode -> BlockDocIdSet for each segment: evaluates only q's filter and keeps, per segment,
 * a dense docId bitset in HBM (bit d of word d/64 set <=> doc d matches), readable with
 * pinot_amd_result_bitset and convertible to ascending docIds with pinot_amd_bitset_to_doc_ids. */
int pinot_amd_execute_filter(pinot_amd_query* q, pinot_amd_segment* const* segs, int32_t n, void* stream,
                             pinot_amd_result** out);
/* Device pointer and word count of segment `segment_index`'s docId bitset of a filter-only result. */
int pinot_amd_result_bitset(pinot_amd_result* r, int32_t segment_index, const uint64_t** h_d_bitset,
                            int64_t* h_num_words);
/* Re-run a query whose plan was compiled by pinot_amd_execute on the same segments (no host work
 * beyond the launches): the benchmarked step. */
int pinot_amd_execute_again(pinot_amd_result* r, void* stream);
/* Release a result after synchronising its stream. Its plan is kept (idle, up to PINOT_AMD_PLAN_CACHE_BYTES of
 * plan device memory) for the next pinot_amd_execute of the same query -- every field, the same segments, the
 * same device and planner overrides -- which then only runs it; destroying a segment drops the plans over it. */
int pinot_amd_result_destroy(pinot_amd_result* r);
/* Number of docs that matched the filter across all segments (numDocsScanned). */
int pinot_amd_result_num_docs_matched(pinot_amd_result* r, int64_t* h_out);
/* Number of groups with >= 1 matching doc (1 for an aggregation-only query). */
int pinot_amd_result_num_groups(pinot_amd_result* r, int64_t* h_out);
/* numGroupsLimitReached (GroupByOperator / GroupByResultsBlock metadata): 1 when some segment reached
 * the query's numGroupsLimit. As in Pinot, each segment admits only the first numGroupsLimit groups
 * it sees in docId order (DictionaryBasedGroupKeyGenerator.java:351-363); later groups of that
 * segment are dropped, and the combine keeps the union of the admitted groups. */
int pinot_amd_result_num_groups_limit_reached(pinot_amd_result* r, int32_t* h_out);
/* Fetch up to cap groups: h_keys[g*num_group_by + j] = group-by column j's value as int64 (INT/LONG),
 * its double bits (FLOAT/DOUBLE) or its index into the merged STRING dictionary
 * (pinot_amd_result_string_key); h_values[g*num_aggs + a] = final result as double
 * (COUNT, SUM, MIN, MAX, AVG, SUMLONG, MINMAXRANGE as double; SUM of integers is the exact 128-bit
 * sum rounded once); h_values_i64 (optional) = exact COUNT / SUMLONG, and SUM on integer columns when
 * it fits int64 (INT64_MIN otherwise). Groups are ordered by ascending global key. */
int pinot_amd_result_fetch(pinot_amd_result* r, int64_t cap, int64_t* h_keys, double* h_values,
                           int64_t* h_values_i64, int64_t* h_num_fetched);
/* AggregationFunction.extractAggregationResult: the intermediate result of every aggregation, two
 * doubles per (group, aggregation) in fetch order — AVG: AvgPair (sum, count); MINMAXRANGE:
 * MinMaxRangePair (min, max); every other function: (final value, 0). What a server hands the broker
 * for the cross-server merge. */
int pinot_amd_result_fetch_intermediate(pinot_amd_result* r, int64_t cap, double* h_pairs, int64_t* h_num_fetched);
/* String value of merged-dictionary id `id` for group-by column j. */
const char* pinot_amd_result_string_key(pinot_amd_result* r, int32_t j, int64_t id);
/* The execution's self-check word (device address of one uint64; 0 = the check held). Partitioned plans
 * verify that every doc past the filter became exactly one record and reached the aggregation
 * (DefaultGroupByExecutor.java:192-219 folds each doc once); a nonzero word voids the result: every read
 * of its groups or matched count fails with PINOT_AMD_EINVAL. A multi-GPU merge carries the word through
 * its collectives (every rank then fails, none returns a table a failed rank contributed to). */
int pinot_amd_result_check_word(pinot_amd_result* r, void** h_d_word);
/* Executions of this process whose self-check failed (each also failed its result with PINOT_AMD_EINVAL). */
int64_t pinot_amd_selfcheck_failures(void);
/* Device view of the dense accumulators for a multi-GPU merge (RCCL all-reduce in place):
 * per aggregation slot an array of num_key_slots 8-byte words; op per slot: 0 = sum(int64),
 * 1 = sum(double), 2 = min(uint64 ordered), 3 = max(uint64 ordered), 4 / 5 = low / high word of an
 * exact 128-bit integer sum. EUNSUPPORTED for hash-table plans (merge those by value). */
int pinot_amd_result_accumulators(pinot_amd_result* r, int32_t* h_num_slots, int64_t* h_num_key_slots,
                                  void** h_slot_ptrs, int32_t* h_slot_ops);
/* Cross-GPU merge by value (replaces the broker's GroupByDataTableReducer merge of server DataTables,
 * pinot-core/.../query/reduce/GroupByDataTableReducer.java:258, and IndexedTable.upsert's
 * AggregationFunction.merge): for GROUP BY results of any plan (dense, partitioned, hash, trimmed).
 * export_groups writes the result's groups to device memory: h_key_words 64-bit words per group (the
 * merged key space's ids packed <= 63 bits per word) at d_keys[g * key_words], h_num_acc accumulator
 * words per group at d_acc[g * num_acc] (the library's encoding). d_keys / d_acc NULL: only the three
 * sizes. Every rank exports the same layout once the same global key space is installed
 * (pinot_amd_query_set_group_key_values). merge_groups folds n such rows (a rank's share of every
 * rank's rows, exchanged over RCCL) into one device hash table with the accumulator ops; until the next
 * execution the result's groups (num_groups / fetch / fetch_intermediate / export_groups) are the merged
 * ones, so a key-partitioned merge can export its merged share again. `stream` (NULL: the result's
 * stream) is ordered after the result's own stream by the library and used for this call only. */
int pinot_amd_result_export_groups(pinot_amd_result* r, uint64_t* d_keys, uint64_t* d_acc, int64_t cap,
                                   int32_t* h_key_words, int32_t* h_num_acc, int64_t* h_num_groups, void* stream);
int pinot_amd_result_merge_groups(pinot_amd_result* r, const uint64_t* d_keys, const uint64_t* d_acc, int64_t n,
                                  void* stream);
/* The device plan: "jit" (fused scan), "jit-partitioned", "jit-hash", "jit-hash-trim"; then "-select" /
 * "-wselect" / "-fwselect" for a selection-vector plan (filter on 4-doc tiles / on 64-doc bitset words /
 * fused with the inverted-index expansion), "+admit-seq" / "+admit" for numGroupsLimit admission
 * (sequential / first-doc), and " xN" when the batch ran as N shape launches. */
const char* pinot_amd_result_kernel_info(pinot_amd_result* r);
/* Algorithmic HBM bytes of the last execution (the roofline numerator): every decoded column once
 * (fixed-bit columns at their bit width, raw columns at their value width); under an inverted-index
 * gate only the rows that pass it; selection-vector plans: the filter columns of every doc, 16 B per
 * vector entry (written + read) and the gathered columns of the matches; plus, per inverted-index leaf,
 * the selected bitmaps' serialized bytes and -- only when the expansion writes one -- the dense docId
 * bitset written and read once (the fused -fwselect plan writes none). */
int pinot_amd_result_algorithmic_bytes(pinot_amd_result* r, double* h_bytes);
/* Host planning time of the execute that built this result, per phase, as "phase=ms;..." (raw_keys:
 * derived dictionaries of raw GROUP BY columns; leaves: per-segment predicate resolution; keys_probe:
 * merged key space + the plan-time match-count probe; plan: accumulators, plan kind, descriptors;
 * jit_alloc: kernel lookup / hipRTC compile, launch descriptors and buffers; launch: enqueueing the first
 * execution). Diagnostics for cold / cached query latency. */
const char* pinot_amd_result_plan_timing(pinot_amd_result* r);
/* Kernel timing of the last execute: device milliseconds of the fused scan kernel, measured with
 * HIP events on the execution stream. */
int pinot_amd_result_last_kernel_ms(pinot_amd_result* r, double* h_ms);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_AMD_H */
