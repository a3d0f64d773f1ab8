// jit.h — query-shape description and the hipRTC-compiled specialised scan kernels (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace pamd {

constexpr int kPartSub = 4;  // partition count / scatter blocks: 4 x 256 threads (one block per CU)
constexpr int kPartCountRatio = 2;  // count-pass blocks per scatter-pass block (count needs little LDS)
constexpr int64_t kAdmitSeqMaxKeys = 1 << 20;  // sequential admission: the seen-key bitmap (128 KiB) in LDS
constexpr int kAdmitSeqSlots = 2048;           // its per-tile hash table of new keys (key, first doc)
constexpr int kHashLdsProbes = 8;              // LDS first level of a hash plan: slots probed before HBM
// LDS bytes of the sequential admission kernel for a key space
inline size_t jit_admitseq_lds(int64_t num_keys) {
  return (size_t)((num_keys + 31) / 32) * 4 + kAdmitSeqSlots * 8 + 1024 * 4 + 80 * 4;
}

struct JitSlot {
  int enc;       // ENC_* (the same in every segment of the batch)
  int type;      // T_* value type
  int bits = 0;  // FIXED_BIT: bit width when every segment of the batch agrees (<= 15), else 0
  int dict_regs = 0;  // dictionary of <= 64 entries in every segment: looked up across lanes (ds_bpermute)
};
struct JitLeaf {
  int slot;        // -1: reads no column (docId range / bitset / constant)
  int clause;
  int negate;
  uint32_t kinds;  // bit k set: some segment resolves this predicate to LEAF kind k
  int bits_regs = 0;  // dictId set of <= 64 words in every segment: held one word per lane
  // dictId set of <= lds_words 32-bit words in every segment (too large for lane registers): copied
  // into LDS when the block's segment changes (256-thread blocks only: the segment is block-uniform)
  int lds_words = 0;
  // 1 / 2: the column has <= 32 / <= 64 dictIds in every segment: the leaf is DevLeaf::accept, tested
  // per doc with one bit extract, OR-ed with the clause's other mask leaves on the same column first
  int mask = 0;
  // > 0 (mask leaves of a fixed-bit column of <= 6 bits, 256-thread scan / select blocks): the clause's
  // mask group is looked up in an LDS table of 2^lut bytes, built when the block's segment changes and
  // indexed by lut bits of the packed column: 4 docs' fields (lut = 4 x bits) or 2 docs' (lut = 2 x bits)
  int lut = 0;
};
// value an accumulator reads: a column slot, or a binary arithmetic expression of two slots
// (EXPR_MUL / SUB / ADD: Pinot's times / minus / plus transforms)
enum { EXPR_COL = 0, EXPR_MUL = 1, EXPR_SUB = 2, EXPR_ADD = 3 };
struct JitVal {
  int expr = EXPR_COL;
  int slot = 0;
  int slot2 = -1;
  bool operator==(const JitVal& o) const { return expr == o.expr && slot == o.slot && slot2 == o.slot2; }
};
struct JitAcc {
  int op;    // ACC_* (an ACC_SUM_I128 is followed by its ACC_HI entry; ACC_FIRST_DOC reads no slot)
  int slot;
  int expr = EXPR_COL;
  int slot2 = -1;
  int nan_skip = 0;  // aggregation-only MIN / MAX: NaN skipped (MinMaxRangePair) instead of propagated
  // ACC_SUM_I128 into an LDS table whose per-block partial sums provably fit int64 (the column's value
  // range x the docs one block (or one aggregation block) can add to a key): the LDS word is a plain
  // int64 (ds_add_u64, no returned value to wait for) and the flush sign-extends it into the
  // 128-bit HBM sum
  int narrow = 0;
  // ACC_SUM_I128 whose whole-query sum provably fits int64 (value range x all docs of the query): the
  // per-doc (and per-block flush) adds into the HBM table are one non-returning 64-bit atomic on the low
  // word -- no returned value to wait for the carry -- and the plan sets each high word to the low word's
  // sign at its end (sext_hi_kernel), the 128-bit sum the readers expect
  int hbm_narrow = 0;
  JitVal val() const { return JitVal{expr, slot, slot2}; }
};
struct JitPlan {
  std::vector<JitSlot> slots;
  std::vector<JitLeaf> leaves;  // in DevSegment::leaves order
  int nclauses = 0;
  std::vector<std::pair<int, int64_t>> group;  // (slot, key stride)
  bool any_remap = false;
  std::vector<JitAcc> accs;  // accumulators 1..n (0 is COUNT), in DevQuery acc order
  int64_t num_keys = 1;
  bool lds = false;
  int scan_nsub = 1;           // 256-thread groups per scan block (4 for a table above 40 KiB)
  int depth = 1;               // software-pipeline depth (tiles prefetched ahead), 1..4
  int waves_per_eu = 0;        // > 0: occupancy target handed to the register allocator
  bool nt_loads = false;       // column loads with the non-temporal hint (streamed once, no cache reuse)
  bool bitset = false;
  bool aggregate = true;
  // direct-atomic scan paired with a partitioned plan: runs only when the count pass found at most
  // part.atomic_threshold matching docs (then scatter + agg exit at once); counts no docs itself
  bool atomic_gate = false;
  bool sample = false;  // match count over every part.sample_stride-th tile only (MODE_SAMPLE)
  // partitioned GROUP BY (DevPartition): count / scatter / LDS-aggregate kernels instead of one scan
  bool partitioned = false;
  int key_shift = 0;           // keys per partition = 2^key_shift
  int nparts = 0;
  std::vector<JitVal> vals;    // record values (distinct values read by accumulators)
  // Bit-packed records: the partition-local key in bits [0, key_shift), then value j's field of
  // val_bits[j] bits at bit val_off[j]. An integer field holds value - DevPartition::vbase[j] (the
  // batch's value range bounds it; val_bits 0: the value is constant), a FLOAT / DOUBLE field the raw
  // bits. Filled by jit_layout_records; val_bits may be preset by the planner (empty: natural widths).
  std::vector<int> val_bits;
  std::vector<int> val_off;
  int rec_bytes = 0;           // record size: 64-bit words x 8
  int stage_cap = 0;           // scatter: records staged per partition in LDS (0: direct writes)
  int flush_pct = 85;          // scatter: a partition is written out once this % of its staging is filled (swept: 85 best)
  int flush_every = 1;         // scatter: the staged partitions are checked (two block barriers) every n tile steps
  // scatter: the wave's ready partitions are written out lane-parallel (their runs concatenated, each lane
  // one 16 / 8 B unit, owners found by a binary search over the lanes' prefix sums) instead of one run
  // after another with the whole wave on each run
  bool flush_par = true;
  // 16-byte records: the flush copies four ready partitions per wave step, a 16-lane group each (consecutive
  // lanes store consecutive records), instead of the lane-parallel flush's per-unit owner search
  bool flush_group = false;
  // partitioned plans: 256-thread groups per count / scatter block (4: one CU-wide block per CU with all the
  // LDS for staging; 2 / 1: two / four blocks per CU, each with that share of the LDS)
  int part_sub = kPartSub;
  bool scatter_batch = true;  // scatter: a lane's staging-slot atomics issued together (PINOT_AMD_SCATTER_BATCH=0: one by one)
  // Sampled capacities instead of the exact count pass: a histogram over every sample_stride-th tile
  // sizes each partition's region (DevPartition::cap); the scatter reserves space with one global
  // atomic per flushed run, records beyond a region's capacity go to the overflow slab, aggregated
  // by pinot_part_ovf with direct HBM atomics. The paired direct-atomic scan (atomic_gate) then also
  // decides from the sample.
  bool part_sampled = false;
  // hash-table GROUP BY (DevHash): group column j's merged id goes to key word hash_pack[j].first at
  // bit hash_pack[j].second; hash_seg appends the segment's key_seg as the last word (trimming)
  bool hash = false;
  int hash_words = 0;          // key words including the segment word
  bool hash_seg = false;
  std::vector<std::pair<int, int>> hash_pack;
  // > 0: an LDS-privatised first level of hash_lds slots (a multiple of 64) in front of the HBM table: a
  // doc's key is probed in the block's LDS table first (linear probing, <= kHashLdsProbes slots); only a
  // key that finds no LDS slot goes to the HBM table directly; the block flushes its occupied slots into
  // the HBM table at the end (one HBM probe + one atomic per accumulator per slot)
  int hash_lds = 0;
  // with hash_lds: a key that finds no LDS slot is spilled (DevHash::spill: appended as a record and counted
  // per key-hash partition) instead of probing the HBM table per doc
  bool hash_spill = false;
  // with hash_spill: no LDS level (keys without skew miss it anyway); every matching doc is spilled, to its
  // block's region (DevHash::direct = 0, which leaves exact per-(partition, block) counts) or straight to its
  // place in the partition-major array (direct = 1, from those counts), the region pass then skipped
  bool hash_direct = false;
  // selection-vector plan: pinot_select (the filter over the filter columns, appending matching docIds)
  // + pinot_gather (decodes only the group-by / aggregated columns of those docs and aggregates)
  bool select = false;
  // dense numGroupsLimit trimming: the aggregation (and partition count / scatter) drops docs whose key
  // the segment did not admit (DevQuery::admit); firstdoc: the admission's first-doc pass instead of an
  // aggregation (filter + group key -> atomicMin of the docId, keys seen first appended per segment)
  bool admit = false;
  bool firstdoc = false;
  // partitioned scatter of an admission plan: the block's current segment's admission bitmap (num_keys / 8
  // bytes) is held in LDS behind the staging, reloaded when the block's tiles cross into another segment, so
  // a doc's admission test is an LDS read instead of a dependent global load per doc
  bool admit_lds = false;
  // admitseq: the admission as one block per segment walking its prefix in doc order with the segment's
  // seen-key bitmap in LDS (key spaces of <= kAdmitSeqMaxKeys keys)
  bool admitseq = false;
  // ... whose filter reads no column (docId bitsets / ranges / constants only): the select pass
  // evaluates the CNF on 64-doc words
  bool word_select = false;
  int wsel_words = 4;  // word-level select: 64-doc words per lane and step (4 or 8; 16 words are one tile)
  int sel_group = 1;   // tile-level select: 1024-doc tiles per loop step (1, 2 or 4; each segment's tile
                       // range in the launch padded to a multiple of it)
  // XCD-aware tile ranges: workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share one), so the
  // physical index is remapped to a logical one that gives each XCD one contiguous eighth of the launch's
  // tiles -- its blocks then share the few segments' per-segment tables (admission bitmaps) in their L2
  bool xcd_remap = false;
  // Filter-gated value loads (fused scans of selective filters): the filter columns of tile t + 2D are loaded
  // ahead, the whole filter is evaluated D tiles ahead into a per-lane mask, and the group-key / value columns of
  // that tile load only for lanes with a matching doc -- at a few percent selectivity most 64-byte sectors of
  // the wide value columns are never fetched (late materialisation inside the scan, no selection vector)
  bool filter_gate = false;
  // hash plans' LDS first level: a doc may insert its key into an EMPTY slot with probability 2^-hash_admit
  // (0: always) -- admission by recurrence, so the slots hold a skewed distribution's head
  int hash_admit = 0;
  int hash_probes = kHashLdsProbes;  // LDS-level slots a doc's key probes before it spills (<= kHashLdsProbes)
  // diagnostics only (PINOT_AMD_DIAG_ADMIT_OFF): the dense admission's per-doc bitmap lookup left out (wrong
  // results; isolates the lookup's traffic in A/B profiles)
  bool diag_admit_off = false;
  // diagnostics only (PINOT_AMD_DIAG_REC_WRAP = bytes, a power of two): the scatter's flushed records wrap around
  // a buffer of that many bytes (wrong results; with a small wrap the record writes stay in the Infinity Cache,
  // which measures what the record round trip through HBM costs the scatter)
  int64_t diag_rec_wrap = 0;
  // Segment-level safe trim (GroupByOperator.java:157-175 with QueryContext's effective trim size = LIMIT):
  // a dense key K's rank in the ORDER BY order is ord(K) = sum over the ORDER BY columns of id' x ostride,
  // id = (K / stride) % size (the GROUP BY column's merged id), id' = size - 1 - id for DESC. Non-empty: the
  // aggregation keeps a doc only when ord(key) <= DevQuery::seg_cut[segment] (each segment's top-LIMIT
  // cutoff); segpres: instead of aggregating, set bit ord(key) of the segment's presence bitmap
  struct OrdCol { int64_t stride, size, ostride; int flip; };
  std::vector<OrdCol> seg_ord;
  bool segpres = false;
};
// record layout of a partitioned plan (fills val_off / rec_bytes from vals and val_bits)
void jit_layout_records(JitPlan* p);
// natural field width of a record value (no range known): 32 for INT / FLOAT, else 64
int jit_val_natural_bits(const JitPlan& p, const JitVal& v);
// whether record value v is stored as an integer offset from its base (else as raw float bits)
bool jit_val_is_int(const JitPlan& p, const JitVal& v);
// LDS bytes of the scatter pass for a staging capacity
size_t jit_scatter_lds(const JitPlan& p, int cap);
// LDS-privatised table layout: accumulator -> LDS array (-1: the high word of a narrow 128-bit sum,
// kept only in HBM); *narrays = arrays the LDS table holds
std::vector<int> jit_lds_layout(const JitPlan& p, int* narrays);
struct JitKernel {
  std::vector<char> image;
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;          // pinot_scan_jit, or the partition count pass
  hipFunction_t fn_scatter = nullptr;  // partitioned: scatter pass
  hipFunction_t fn_agg = nullptr;      // partitioned: LDS aggregation of the partitions
  hipFunction_t fn_ovf = nullptr;      // sampled partitioned: the overflow slab's direct atomics
  hipFunction_t fn_gather = nullptr;   // selection-vector plans: the gather-aggregate pass (fn = select)
};
// C type / size of an accumulated value: a column's decoded value type; an expression is int64
// when both operands are INT (exact), else double (the transforms' DOUBLE result)
const char* jit_val_ctype(const JitPlan& p, const JitVal& v);
int jit_val_size(const JitPlan& p, const JitVal& v);

std::string jit_shape_key(const JitPlan& p);
std::string jit_generate(const JitPlan& p);
std::string jit_full_source(const JitPlan& p);
// compiled, loaded kernel for the plan's shape (cached); nullptr + *err when unavailable
JitKernel* jit_get(const JitPlan& p, std::string* err);

}  // namespace pamd
