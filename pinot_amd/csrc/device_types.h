// device_types.h — POD descriptors shared by the host planner (host.cpp) and the gfx950
// kernels (kernels.hip). Everything here is uploaded verbatim to HBM or passed as kernargs.
#pragma once
#include <stdint.h>

namespace pamd {

constexpr int kBlock = 256;                         // 4 waves of 64
constexpr int kDocsPerThread = 4;                   // 4 consecutive docs per lane
constexpr int kTileDocs = kBlock * kDocsPerThread;  // 1024 docs per block-tile
constexpr int kMaxSlots = 16;                       // distinct columns referenced by one query
constexpr int kMaxLeaves = 16;                      // predicate leaves
constexpr int kMaxClauses = 16;                     // CNF clauses (4 bits each in a 64-bit word)
constexpr int kMaxAcc = 16;                         // accumulator arrays (acc 0 = COUNT)
constexpr int kMaxGroupCols = 16;
constexpr int kMaxKeyWords = 8;                     // 64-bit words of a hash-table group key
// slack the kernels may read past the end of a column buffer (5 dwords of a bit window, a 32 B
// value vector of the last tile, and up to 3 whole padding tiles of 8-byte values behind a segment's last
// tile: the tile-level select walks steps of up to 4 tiles of one segment)
constexpr int kPadBytes = 4 * kTileDocs * 8 + 256;

// column encodings (pinot_amd_fwd_encoding)
enum : int32_t { ENC_FIXED_BIT = 0, ENC_RAW = 1, ENC_SORTED = 2 };
// value types (pinot_amd_data_type)
enum : int32_t { T_INT = 0, T_LONG = 1, T_FLOAT = 2, T_DOUBLE = 3, T_STRING = 4 };

// predicate leaf kinds (what a resolved PredicateEvaluator reduces to)
enum : int32_t {
  LEAF_DICT_RANGE = 0,  // lo_i <= dictId < hi_i     (SortedDictionaryBasedRangePredicateEvaluator)
  LEAF_DICT_SET = 1,    // bit dictId of `bits`       (DictionaryBasedIn/Eq..., unsorted range)
  LEAF_RAW_RANGE_I = 2, // lo_i <= v <= hi_i          (Int/LongRawValueBasedRangePredicateEvaluator)
  LEAF_RAW_RANGE_F = 3, // lo_d <= v <= hi_d          (Float/DoubleRawValueBasedRangePredicateEvaluator)
  LEAF_RAW_IN_I = 4,    // v in sorted in_i[0..in_n)  (Int/LongRawValueBasedInPredicateEvaluator)
  LEAF_RAW_IN_F = 5,    // v in sorted in_d[0..in_n)
  LEAF_DOC_RANGE = 6,   // lo_i <= docId <= hi_i      (SortedIndexBasedFilterOperator)
  LEAF_DOC_BITSET = 7,  // bit docId of `bits`        (BitmapBasedFilterOperator over the inverted index)
  LEAF_CONST = 8        // lo_i != 0                  (alwaysTrue / alwaysFalse evaluators)
};

// accumulator ops
//   ACC_SUM_I64   wrapping int64 sum (SUMLONG: Java long arithmetic)
//   ACC_SUM_I128  exact sum of int64 values: low word here, high word in the next array (ACC_HI),
//                 carried with the value returned by the low word's atomic (SUM / AVG on integers)
//   ACC_FIRST_DOC smallest matching docId of a (segment, key) entry (numGroupsLimit trimming)
enum : int32_t { ACC_COUNT = 0, ACC_SUM_I64 = 1, ACC_SUM_F64 = 2, ACC_MIN = 3, ACC_MAX = 4, ACC_SUM_I128 = 5,
                 ACC_HI = 6, ACC_FIRST_DOC = 7 };

struct DevColumn {
  const uint8_t* data;     // FIXED_BIT: BE bit stream | RAW: BE values | SORTED: LE int32 start docId per dictId
  const void* dict;        // dictionary values, native LE array of the value type (dict columns)
  const int32_t* remap;    // dictId -> ordinal in the query's merged key space (group-by columns)
  int32_t enc, type, bits, card;
};

struct DevLeaf {
  int32_t slot, kind, negate, clause;
  int64_t lo_i, hi_i;
  double lo_d, hi_d;
  const uint32_t* bits;    // LEAF_DICT_SET: one bit per dictId; LEAF_DOC_BITSET: one bit per docId
  const int64_t* in_i;
  const double* in_d;
  int32_t in_n, pad;
  // dictionary leaves of columns of <= 64 values: bit d set = dictId d passes (LEAF_CONST: all or none;
  // negation not applied). The accept-mask plans test a doc with one bit extract.
  uint64_t accept;
};

struct DevSegment {
  int64_t num_docs;
  int64_t tile_begin;      // first tile of this segment in its launch
  int32_t key_seg;         // index of the segment in its trim batch (hash key word of trimming plans)
  int32_t pad;             // sequential admission descriptors: 1 = the prefix is the whole segment
  DevColumn cols[kMaxSlots];
  DevLeaf leaves[kMaxLeaves];
};

// Partitioned GROUP BY (key spaces too large for an LDS table): the scan emits one record per
// matching doc into key-range partitions, then each partition is aggregated in LDS.
//   count pass:   hist[p * grid + block] = matching docs of `block` whose key falls in partition p
//   scan:         offs[p * grid + block] = exclusive prefix within partition p; part_begin = prefix
//                 of partition totals (part_begin[nparts] = all records)
//   scatter pass: record r of partition p at part_begin[p] + offs[..] + running index, staged per
//                 partition in LDS and written out in runs; a record is `rec_bytes` bytes (whole
//                 64-bit words) at rec + r * rec_bytes, bit-packed: the local key (key & (2^key_shift
//                 - 1)) in the low bits, then one field per accumulated value (JitPlan::val_bits /
//                 val_off; integers as value - vbase[j], FLOAT / DOUBLE as raw bits)
//   agg pass:     one LDS table of 2^key_shift keys per partition, flushed with global atomics
// Sampled plans (JitPlan::part_sampled) replace the count pass with a histogram over every
// sample_stride-th tile of each scatter block's range: block b gets an allotment of records of
// partition p sized from its own sample (with a margin for the sampling error); what does not fit
// goes to the overflow slab (ovf_rec / ovf_part), which pinot_part_ovf adds into the HBM table directly.
struct DevPartition {
  int32_t nparts, key_shift;
  int64_t atomic_threshold;  // records <= this: the direct-atomic scan runs instead of scatter + agg
  int64_t sample_stride;     // > 0: counts[1] x stride estimates the matches before the count pass
  unsigned long long* counts;  // [0] count-pass matches, [1] sampled matches, [2] direct-atomic scan matches
  uint32_t* hist;
  int64_t* offs;
  int64_t* part_begin;
  uint8_t* rec;
  int64_t vbase[kMaxAcc];    // packed records: integer value j is stored as value - vbase[j]
  // sampled plans (JitPlan::part_sampled): offs[c] = first record of allotment c = p * seg_grid + b
  // (partition p, scatter block b; offs[c + 1] ends it); after the scatter hist[c] = the records it
  // holds and eff_begin = their exclusive prefix, the aggregation pass's record index space
  int64_t seg_grid;
  int64_t* eff_begin;
  uint8_t* ovf_rec;          // overflow slab: records, their partitions, and the count
  uint32_t* ovf_part;
  unsigned long long* ovf_n;
  // the execution's self-check word, 0 when it holds (the result then refuses its groups, PINOT_AMD_EINVAL):
  // exact plans add every partition whose scatter-block run ends anywhere but where the count pass put the next
  // block's records; sampled plans every scatter block whose records made (docs past the filter, numGroupsLimit
  // admission and the segment trim) differ from the records it left in its allotments plus those it sent to the
  // overflow slab
  unsigned long long* check;
  // per block, 4 words: the HW_ID and XCC_ID hardware registers, the block's self-check mismatches, its records
  // (count blocks at [4 * b], scatter blocks at [4 * (count grid + b)]): a failed check names the CUs involved
  uint32_t* hw;
};
constexpr int kHwWords = 4;

// Inverted-index leaf of one segment: the selected RoaringBitmap containers (of every dictId the
// predicate selects) are OR-ed into a dense docId bitset (BitmapBasedFilterOperator's bitmap OR).
// one segment of a fused inverted-index select launch (roaring_select_kernel)
struct FusedSelSeg {
  int64_t item_begin;          // prefix of the segments' work items (chunk groups) over the launch
  int32_t seg;                 // the segment's index in the launch (the selection vector's tag)
  int32_t nitems;
  int32_t job[kMaxLeaves];     // leaf j's ExpandJob when it is an inverted-index bitset here, else -1
};

struct ExpandJob {
  const uint8_t* inv;          // staged inverted-index buffer
  const struct RoaringContainer* conts;  // container directory of the column
  const int32_t* sel;          // selected container indices, grouped by work item (expand_group() chunks)
  const int32_t* grp;          // work item k's containers: sel[grp[k] .. grp[k+1])
  unsigned long long* bitset;  // output, nwords 64-bit words (every word written each run)
  int64_t num_docs, nwords;
  int64_t sel_begin;           // prefix of nsel over the plan's jobs
  int64_t item_begin;          // prefix of nchunks over the plan's jobs (work items)
  int32_t nsel, nchunks;       // nchunks: the job's work items (groups of expand_group() 65536-doc chunks)
  // the selected containers' descriptors packed in the sel order (byte offset | min(count, 65535) << 32
  // | kind << 48), built once per plan: one load per container instead of sel -> directory; nullptr
  // when the inverted-index buffer is 4 GiB or larger
  const unsigned long long* psel;
};

// One compressed chunk of a raw forward index (BaseChunkForwardIndexWriter layout), decoded on the
// device at staging by one wave. codec: ChunkCompressionType (1 SNAPPY, 3 LZ4 -- the 4-byte length
// prefix of LZ4_LENGTH_PREFIXED already skipped by the host --, 6 DELTA, 7 DELTADELTA).
struct ChunkJob {
  uint64_t src_off;  // into the staged compressed file
  uint64_t dst_off;  // into the contiguous decoded values
  uint32_t src_len, dst_len;
  int32_t codec, pad;
};

// Hash-table group-by (key spaces a dense table cannot hold, and numGroupsLimit trimming): open
// addressing with linear probing over `cap` slots. A key is `nwords` 64-bit words (the group columns'
// merged ids packed <= 63 bits per word, or 64 when one of the word's fields can never be all ones, so no
// word is ever ~0 (host.cpp pack_key_words); trimming plans add the batch segment
// index as the last word), stored word-major at keys[w * cap + slot]; EMPTY words are ~0. A slot is
// claimed word by word with compare-and-swap: whoever sets word w decides it, a thread finding a
// different word moves on to the next slot, so a slot's key is complete once every thread that
// touched it has passed (no locks, no spinning). Accumulators live at acc[a * cap + slot].
struct DevHash {
  unsigned long long* keys;
  int64_t cap;                       // power of two
  unsigned long long* overflow;      // docs that found no free slot (the host grows the table or fails)
  int64_t max_probe;                 // > 0: a key gives up after this many slots (linear probing), 0: cap
  // Second level of a hash plan with an LDS first level (JitPlan::hash_spill): a doc whose key finds no LDS
  // slot is appended to its block's region as a spill record -- the key words, then one word per value
  // accumulator (acc order, ACC_HI skipped: the int64 value, the double's bits, or the ordered MIN / MAX
  // encoding) -- and counted in its key-hash partition (hash >> spill_shift). The spill passes (kernels.hip)
  // then group the records by partition and aggregate each partition in LDS, so the tail keys reach the HBM
  // table once per (partition chunk, key) instead of once per doc. Records past spill_cap take the HBM table.
  unsigned long long* spill;         // grid x kSpillGroups sub-regions of spill_cap records of spill_words words
  int64_t spill_cap;                 // records per sub-region
  uint32_t* spill_cnt;               // per sub-region: records appended (those past spill_cap counted too)
  uint32_t* spill_hist;              // [partition * grid + block] records kept in the region
  int32_t spill_shift;               // partitions = 2^(64 - spill_shift)
  int32_t spill_words;
  // Direct placement (JitPlan::hash_direct with direct = 1; keys without skew, no LDS first level): a record goes
  // straight to its place in the partition-major array -- dst + dbase[p * grid + b] + the block's running count of
  // partition p -- from the exact per-(partition, block) counts dcnt of an earlier region-mode execution of the same
  // plan (the doc -> (partition, block) map is fixed: no LDS level decides which docs spill). Records past a count
  // take the HBM table; a block whose count of some partition falls short of dcnt leaves holes and adds to check
  // (the result is then void: pinot_amd_result_check_word / verify).
  unsigned long long* dst;
  const int64_t* dbase;
  const uint32_t* dcnt;
  unsigned long long* check;
  int32_t direct;
};
// A key's home slot in an HBM hash table of cap (a power of two) slots: the key hash's TOP bits, so the keys of one
// spill partition (the same hash's top bits, DevHash::spill_shift) share one contiguous slice of the table and the
// spill aggregation's merges of a partition land in a few MB of the table instead of all of it
__host__ __device__ __forceinline__ uint64_t hash_home(uint64_t x, int64_t cap) {
  return cap <= 1 ? 0ull : x >> (64 - __builtin_ctzll((unsigned long long)cap));
}
constexpr int kSpillMaxParts = 2048;  // spill partitions (the scan block's LDS histogram)
// A scan block's spill region is split in kSpillGroups sub-regions by the partition's top 2 bits (sub-region
// bx * kSpillGroups + g, spill_cap records each, spill_cnt per sub-region): a chunk of the region pass then meets a
// quarter of the partitions, so its partition runs are 4x longer (whole 128-byte lines instead of ~5-record runs)
constexpr int kSpillGroups = 4;

// Segment-level group trim over a hash plan's (key, segment) scan table (GroupByOperator.java:157-175,
// TableResizer.trimInSegmentResults): each segment keeps its top `keep` groups in the ORDER BY's order. The order is
// a chain of 64-bit stage keys compared lexicographically, smaller first: kind 0 = ORDER BY group columns (merged ids
// from the packed key words, DESC ones flipped, packed into one mixed-radix value while it fits), kind 1 = an
// ORDER BY aggregation's final value (extractFinalResult, Double.compare order, DESC complemented), kind 2 = a key
// word (ties in ascending group key, the last word first). Found per segment by a radix select, 8 bits per pass.
struct SegSelStage {
  int32_t kind;
  int32_t ncols;  // kind 0
  int32_t word[kMaxGroupCols], shift[kMaxGroupCols], bits[kMaxGroupCols], flip[kMaxGroupCols];
  int64_t size[kMaxGroupCols], mul[kMaxGroupCols];
  int32_t agg_type, acc, acc2, desc;  // kind 1: pinot_amd_agg_type, its accumulator (and MINMAXRANGE's max)
  int32_t kword;                      // kind 2
};
constexpr int kSegSelMaxStages = 16;

// Group keys by value for the cross-rank merge (the broker reduce on the device): group column j's
// merged id sits in bits [shift[j], shift[j] + bits) of key word word[j] (the hash plan's packing, <= 63
// bits per word); a dense table's key decomposes as id_j = (key / stride[j]) % size[j] (mixed radix).
struct DevKeyPack {
  int32_t ncols, nw;
  int32_t word[kMaxGroupCols], shift[kMaxGroupCols];
  int64_t stride[kMaxGroupCols], size[kMaxGroupCols];
};

// Uniform per-launch plan (kernel argument of the generated scan kernels and the fixed passes).
struct DevQuery {
  int32_t nsegs;                            // segments of this launch (DevSegment array length)
  int32_t nacc;                             // accumulator arrays, acc 0 = COUNT
  int32_t acc_op[kMaxAcc];
  int64_t num_keys;                         // dense key space (1 for aggregation only; hash plans: 0)
  int64_t total_tiles;                      // 1024-doc tiles of this launch
  // selection-vector plans (late materialisation): the filter pass appends (segment << 32 | docId)
  // entries, each wave's run padded to a multiple of 4 with docId 0xFFFFFFFF; the gather pass
  // aggregates them. sel_count[0] = entries appended, sel_count[1] = runs that did not fit sel_cap
  unsigned long long* sel_entries;
  unsigned long long* sel_count;
  int64_t sel_cap;
  int32_t sel_chunk;     // vector entries a select wave reserves at a time (planner: from the expected matches)
  int32_t sel_pad;
  // numGroupsLimit admission of dense trimming plans (JitPlan::admit / firstdoc): bit `key` of segment
  // key_seg's bitmap (admit_words 32-bit words per segment) = the segment admitted that group. The
  // first-doc pass keeps first[key_seg * num_keys + key] = the key's smallest matching docId so far and
  // appends each key it sees first to that segment's list (seen[key_seg * seen_cap ..], count seen_n[key_seg])
  const uint32_t* admit;
  int64_t admit_words;
  uint32_t* first;
  uint32_t* seen;
  unsigned long long* seen_n;
  int64_t seen_cap;
  unsigned long long* admit_flag;  // numGroupsLimitReached (the sequential admission pass sets it)
  // segment-level safe trim (JitPlan::seg_ord): per segment (key_seg) the ORDER BY rank of its LIMIT-th
  // group (~0: the segment keeps every group), and the presence bitmaps over ranks (seg_words words each)
  const unsigned long long* seg_cut;
  unsigned long long* seg_bits;
  int64_t seg_words;
};

}  // namespace pamd
