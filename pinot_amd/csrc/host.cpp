// host.cpp — host side of libpinot_amd.so: segment staging into HBM, per-segment predicate
// resolution (PredicateEvaluatorProvider), query planning for the fused scan kernel, execution
// over a batch of segments and result extraction. Implements include/pinot_amd.h.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <climits>
#include <limits>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <new>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/pinot_amd.h"
#include "device_types.h"
#include "jit.h"

namespace pamd {
hipError_t launch_init_acc(uint64_t* d_acc, const DevQuery& q, int64_t num_keys, hipStream_t st);
hipError_t launch_sext_hi(uint64_t* d_acc, int64_t n, const int32_t* arrs, int32_t narr, hipStream_t st);
hipError_t launch_raw_int_minmax(const uint8_t* be, int type, int64_t n, long long* out, hipStream_t st);
hipError_t launch_fingerprint(const void* p, size_t bytes, unsigned long long* out, hipStream_t st);
hipError_t launch_trim(const unsigned long long* keys, int64_t cap, int nw_seg, const uint64_t* acc, int fd_acc,
                       int32_t nsegs, int64_t limit, const int64_t* bucket_base, uint32_t* hist,
                       unsigned long long* seg_distinct, int64_t* bstar, int64_t* rank, unsigned long long* bitmap,
                       int64_t* dstar, unsigned long long* limit_reached, hipStream_t st);
hipError_t launch_hash_merge(const unsigned long long* skeys, int64_t scap, int nw, int has_seg, const uint64_t* sacc,
                             unsigned long long* fkeys, int64_t fcap, uint64_t* facc, const DevQuery& q, int fd_acc,
                             const int64_t* dstar, unsigned long long* overflow, hipStream_t st,
                             const SegSelStage* sst = nullptr, int nst = 0, const int32_t* sdone = nullptr,
                             const uint64_t* scut = nullptr);
hipError_t launch_segsel(const unsigned long long* keys, int64_t cap, int nw, const uint64_t* acc, int fd_acc,
                         const int64_t* dstar, const DevQuery& q, const SegSelStage* sst, int nst, int32_t nsegs,
                         int64_t keep, unsigned long long* cnt, int64_t* want, int32_t* done, uint64_t* prefix,
                         uint64_t* cut, uint32_t* hist, hipStream_t st);
hipError_t launch_admit(uint32_t* first, int64_t nk, const uint32_t* seen, const unsigned long long* seen_n, int64_t cap,
                        int32_t nsegs, int64_t limit, const int64_t* bucket_base, int64_t max_buckets, uint32_t* hist,
                        int64_t* bstar, int64_t* rank, unsigned long long* bitmap, int64_t* dstar,
                        unsigned long long* limit_reached, int phase, uint32_t* admit, int64_t words, hipStream_t st);
hipError_t launch_presence_bitset(const uint64_t* count, int64_t n, unsigned long long* bits, hipStream_t st);
hipError_t launch_seg_cut(const unsigned long long* bits, int64_t words, int32_t nsegs, int64_t limit,
                          unsigned long long* cut, hipStream_t st);
hipError_t launch_spill_direct_prep(const int64_t* offs, const int64_t* part_begin, const uint32_t* hist, int P,
                                    int64_t grid, int64_t* dbase, uint32_t* dcnt, int64_t* pbeg, hipStream_t st);
hipError_t launch_spill_agg(const DevHash& H, int nw, const unsigned long long* sorted, const int64_t* part_begin,
                            const DevQuery& q, uint64_t* acc, int agg_grid, int S, uint32_t narrow, hipStream_t st);
hipError_t launch_spill_passes(const DevHash& H, int nw, int64_t grid, const uint32_t* hist_unused, int64_t* offs,
                               int64_t* part_begin, unsigned long long* sorted, const DevQuery& q, uint64_t* acc,
                               int agg_grid, int S, int sorted_scatter, uint32_t narrow, hipStream_t st);
hipError_t launch_gather_groups(const int32_t* slots, int64_t ngroups, const unsigned long long* keys, int nw,
                                int64_t cap, const uint64_t* acc, int32_t nacc, uint64_t* out_keys, uint64_t* out_acc,
                                hipStream_t st);
hipError_t launch_export_groups(const int32_t* slots, int64_t ngroups, const unsigned long long* hkeys, int64_t cap,
                                const uint64_t* acc, int32_t nacc_out, const DevKeyPack& kp, uint64_t* out_keys,
                                uint64_t* out_acc, hipStream_t st);
hipError_t launch_merge_rows(const uint64_t* keys, const uint64_t* acc, int64_t n, int nw, int nacc_in,
                             unsigned long long* fkeys, int64_t fcap, uint64_t* facc, const DevQuery& q,
                             unsigned long long* overflow, hipStream_t st);
hipError_t launch_read_dict_ids(const uint8_t* packed, int bits, int64_t start, int64_t len, int32_t* out,
                                hipStream_t st);
hipError_t launch_pack_dict_ids(const int32_t* values, int64_t n, int bits, uint8_t* packed, hipStream_t st);
size_t derive_dictionary_scratch(int64_t n);
size_t sort_rows_scratch(int64_t n);
hipError_t sort_rows_by_key(const uint64_t* keys, int nwk, const int* word_bits, const uint64_t* acc, int nacc, int64_t n,
                            void* scratch, uint64_t* keys_out, uint64_t* acc_out, hipStream_t st);
hipError_t derive_dictionary(const uint8_t* d_be, int type, int64_t n, void* d_scratch, int32_t* d_ids,
                             uint8_t* d_dict_be, int64_t* h_card, hipStream_t st);
hipError_t launch_read_raw(const uint8_t* raw, int type, int64_t start, int64_t len, uint8_t* out, hipStream_t st);
hipError_t launch_chunk_decompress(const uint8_t* src, uint8_t* dst, const void* jobs, int32_t njobs, int32_t* status,
                                   hipStream_t st);
hipError_t launch_bitset_binop(const uint64_t* a, const uint64_t* b, uint64_t* out, int64_t n, int op,
                               hipStream_t st);
hipError_t launch_bitset_not(const uint64_t* a, uint64_t* out, int64_t num_docs, hipStream_t st);
int64_t compact_num_chunks(int64_t num_docs);
hipError_t launch_bitset_count(const uint64_t* bits, int64_t num_docs, int64_t* d_chunk_counts, int64_t* d_total,
                               hipStream_t st);
hipError_t launch_bitset_compact(const uint64_t* bits, int64_t num_docs, const int64_t* d_chunk_offsets,
                                 int32_t* out, hipStream_t st);
hipError_t launch_expand_jobs(const void* d_jobs, int32_t njobs, int64_t total_items, hipStream_t st);
hipError_t launch_roaring_select(const void* d_jobs, const void* d_fs, int32_t nfs, int64_t total_items, const void* d_segs,
                                 int32_t nleaves, int32_t nclauses, unsigned long long* sel_entries,
                                 unsigned long long* sel_count, int64_t sel_cap, unsigned long long* matched_out, int clause,
                                 hipStream_t st);
hipError_t launch_pack_sel(const void* conts, const int32_t* sel, int64_t n, int group, unsigned long long* out,
                           hipStream_t st);
int expand_group();
hipError_t launch_partition_offsets(const uint32_t* d_hist, int32_t nparts, int64_t nblocks, int64_t* d_offs,
                                    int64_t* d_part_begin, hipStream_t st);
hipError_t launch_allot_prefix(const uint32_t* d_hist, int32_t P, int64_t G, int mode, int64_t stride, double scale,
                               int64_t limit, int64_t* d_ptot, int64_t* d_out, hipStream_t st);
}  // namespace pamd

using namespace pamd;

// ------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_OK(expr)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(PINOT_AMD_EHIP, "%s: %s", #expr, hipGetErrorString(e_));   \
  } while (0)

namespace {

// Runtime knobs. A default build reads only the planner overrides the test suite exercises and the server's resource
// limits (the list below); the experiment knobs of earlier rounds' sweeps (DESIGN.md records their outcomes) are
// honoured only in a diagnostics build (-DPINOT_AMD_DIAGNOSTICS), so a default build plans from the query alone.
static const std::set<std::string>& kept_knobs() {
  static const std::set<std::string> kept = {
      "PINOT_AMD_ADMIT_PREFIX",
      "PINOT_AMD_ADMIT_SEQ",
      "PINOT_AMD_ATOMIC_HANDOVER",
      "PINOT_AMD_FILTER_GATE",
      "PINOT_AMD_FLUSH_EVERY",
      "PINOT_AMD_FLUSH_GROUP",
      "PINOT_AMD_FUSED_INV_SELECT",
      "PINOT_AMD_GENERIC_BITS",
      "PINOT_AMD_GROUP_PLAN",
      "PINOT_AMD_HASH_CAP_CACHE",
      "PINOT_AMD_HASH_DIRECT",
      "PINOT_AMD_HASH_INIT_SLOTS",
      "PINOT_AMD_HASH_LDS",
      "PINOT_AMD_HASH_LDS_ADMIT",
      "PINOT_AMD_HASH_LDS_SLOTS",
      "PINOT_AMD_HASH_MAX_PROBE",
      "PINOT_AMD_HASH_SPILL",
      "PINOT_AMD_HASH_TABLE_BYTES",
      "PINOT_AMD_INV_POLICY",
      "PINOT_AMD_NARROW_SUMS",
      "PINOT_AMD_PARTITIONED",
      "PINOT_AMD_PART_CAP_SCALE",
      "PINOT_AMD_PREFETCH",
      "PINOT_AMD_SAMPLE_STRIDE",
      "PINOT_AMD_SCAN_GROUP",
      "PINOT_AMD_SELECT",
      "PINOT_AMD_SELECT_PARTITIONED",
      "PINOT_AMD_SEL_GROUP",
      "PINOT_AMD_SPILL_BYTES",
      "PINOT_AMD_SPILL_SORT",
      "PINOT_AMD_STAGE_CAP",
      "PINOT_AMD_TRIM_PLAN",
      "PINOT_AMD_WIDE_LDS",
      "PINOT_AMD_POOL_BYTES",
      "PINOT_AMD_KEY_CACHE_BYTES",
      "PINOT_AMD_SPILL_MAX_BYTES",
      "PINOT_AMD_HASH_FINAL_MAX_BYTES",
      "PINOT_AMD_ADMIT_MAX_BYTES",
      "PINOT_AMD_DENSE_MAX_KEYS",
      "PINOT_AMD_PLAN_CACHE",
      "PINOT_AMD_PLAN_CACHE_BYTES",
  };
  return kept;
}
static const char* knob(const char* name) {
#ifndef PINOT_AMD_DIAGNOSTICS
  if (!kept_knobs().count(name)) return nullptr;
#endif
  return getenv(name);
}
// every knob a default build reads, with its value: part of a prepared plan's identity (a plan built under other
// overrides is another plan); empty in a diagnostics build, whose knobs are open-ended (no plan cache there)
static std::string knob_snapshot() {
#ifdef PINOT_AMD_DIAGNOSTICS
  return std::string();
#else
  std::string out = "knobs";
  for (const std::string& k : kept_knobs())
    if (const char* v = getenv(k.c_str())) out += "|" + k + "=" + v;
  return out;
#endif
}

// ------------------------------------------------------------------------------------------------
// device buffers
// ------------------------------------------------------------------------------------------------
// Device blocks released by destroyed results are kept for the next execution instead of going back to
// hipFree: a re-issued query shape allocates the same descriptors, bitset buffers and scratch again, and
// hipMalloc / hipFree (which synchronises the device) cost tens of microseconds each -- hundreds of them per
// plan on an inverted-index filter over 100 segments. Only pinot_amd_result_destroy releases into the
// cache, after synchronising the result's stream, so a cached block is idle when it is handed out again.
// Blocks up to kPoolMaxBlock bytes, PINOT_AMD_POOL_BYTES in total per device (default 1 GiB; 0 disables).
struct DevPool {
  static constexpr size_t kPoolMaxBlock = (size_t)256 << 20;
  std::mutex mu;
  std::map<int, std::multimap<size_t, void*>> free;  // device -> (block bytes -> block)
  std::map<int, size_t> bytes;
  size_t cap = 0;
  DevPool() {
    const char* e = knob("PINOT_AMD_POOL_BYTES");
    cap = e ? (size_t)strtoull(e, nullptr, 10) : ((size_t)1 << 30);
  }
  static size_t block_size(size_t n) {  // size classes: powers of two to 4 MiB, 1 MiB steps above
    if (n <= 256) return 256;
    if (n <= ((size_t)4 << 20)) {
      size_t c = 512;
      while (c < n) c <<= 1;
      return c;
    }
    return (n + ((size_t)1 << 20) - 1) & ~(((size_t)1 << 20) - 1);
  }
  void* take(size_t bsz) {
    if (!cap || bsz > kPoolMaxBlock) return nullptr;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    auto& f = free[dev];
    auto it = f.find(bsz);
    if (it == f.end()) return nullptr;
    void* p = it->second;
    f.erase(it);
    bytes[dev] -= bsz;
    return p;
  }
  // false: not cached (the caller frees it)
  bool put(void* p, size_t bsz) {
    if (!cap || bsz > kPoolMaxBlock) return false;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    auto& f = free[dev];
    size_t& b = bytes[dev];
    while (b + bsz > cap && !f.empty()) {  // evict the largest cached blocks first
      auto last = std::prev(f.end());
      (void)hipFree(last->second);
      b -= last->first;
      f.erase(last);
    }
    if (b + bsz > cap) return false;
    f.emplace(bsz, p);
    b += bsz;
    return true;
  }
};
static DevPool& dev_pool() {
  static DevPool* pool = new DevPool();  // never destroyed: blocks outlive static destruction order
  return *pool;
}
// set by pinot_amd_result_destroy while the result's members are destroyed (its stream synchronised)
static thread_local bool g_release_to_pool = false;
static thread_local size_t g_tl_alloc_bytes = 0;  // device bytes this thread allocated (a plan's footprint)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  size_t bsz = 0;  // block bytes when the block is of a pool size class (0: an exact hipMalloc)
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p && !(g_release_to_pool && bsz && dev_pool().put(p, bsz))) (void)hipFree(p);
    p = nullptr;
    n = 0;
    bsz = 0;
  }
  int raw_alloc(size_t len) {
    n = len;
    const size_t want = len ? len : 1;
    bsz = DevPool::block_size(want);
    g_tl_alloc_bytes += bsz <= DevPool::kPoolMaxBlock ? bsz : want;
    if (bsz <= DevPool::kPoolMaxBlock) {
      if ((p = dev_pool().take(bsz))) return 0;
      if (hipMalloc(&p, bsz) == hipSuccess) return 0;
    }
    bsz = 0;
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return fail(PINOT_AMD_ENOMEM, "hipMalloc(%zu) failed", len);
    }
    return 0;
  }
  // allocate n bytes + pad (zeroed), copy `src` (len bytes) to the front
  int alloc_copy(const void* src, size_t len, size_t pad) {
    release();
    if (int rc = raw_alloc(len + pad)) return rc;
    if (!pad) {
      if (len) HIP_OK(hipMemcpy(p, src, len, hipMemcpyHostToDevice));
      else HIP_OK(hipMemset(p, 0, n));
      return 0;
    }
    if (len + pad <= ((size_t)1 << 20)) {  // one copy of the bytes and their zero padding
      std::vector<uint8_t> h(len + pad, 0);
      if (len) memcpy(h.data(), src, len);
      HIP_OK(hipMemcpy(p, h.data(), n, hipMemcpyHostToDevice));
      return 0;
    }
    HIP_OK(hipMemset((uint8_t*)p + len, 0, pad));
    if (len) HIP_OK(hipMemcpy(p, src, len, hipMemcpyHostToDevice));
    return 0;
  }
  void reset() { release(); }
  int alloc(size_t len) {
    release();
    return raw_alloc(len);
  }
  // at least len bytes, reusing the buffer when it is large enough (scratch kept across calls)
  int ensure(size_t len) {
    if (p && n >= len) return 0;
    reset();
    return alloc(len);
  }
};

// Staged forward-index buffers and their device fingerprints at staging (launch_fingerprint): the partitioned plan's
// self-check report compares them with the bytes' fingerprints at the failure (selfcheck_report).
struct StagedPrint {
  size_t bytes;
  unsigned long long print;
};
static std::mutex g_print_mu;
static std::map<const void*, StagedPrint> g_prints;

static int device_fingerprint(const void* p, size_t bytes, unsigned long long* out) {
  DevBuf h;
  if (int rc = h.alloc(8)) return rc;
  HIP_OK(hipMemset(h.p, 0, 8));
  HIP_OK(launch_fingerprint(p, bytes, (unsigned long long*)h.p, nullptr));
  HIP_OK(hipMemcpy(out, h.p, 8, hipMemcpyDeviceToHost));
  return 0;
}

static uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Java String.compareTo order (UTF-16 code units); for the BMP this equals code point order,
// which for valid UTF-8 equals byte order except for supplementary characters. Compare UTF-16.
static std::u16string to_utf16(const std::string& s) {
  std::u16string out;
  size_t i = 0;
  while (i < s.size()) {
    uint32_t c = (uint8_t)s[i];
    int extra = c < 0x80 ? 0 : c < 0xE0 ? 1 : c < 0xF0 ? 2 : 3;
    if (extra) c &= (0x3F >> extra);
    for (int k = 1; k <= extra && i + k < s.size(); ++k) c = (c << 6) | ((uint8_t)s[i + k] & 0x3F);
    i += 1 + extra;
    if (c >= 0x10000) {
      c -= 0x10000;
      out.push_back((char16_t)(0xD800 + (c >> 10)));
      out.push_back((char16_t)(0xDC00 + (c & 0x3FF)));
    } else {
      out.push_back((char16_t)c);
    }
  }
  return out;
}
// Byte order first: the first differing byte is the lead (or a continuation) byte of the first differing
// code points, and byte order = code point order = UTF-16 order unless one of them is supplementary (lead
// 0xF0-0xF4, surrogates in UTF-16) and the other in U+E000..U+FFFF (lead 0xEE / 0xEF): only then convert.
// Merging 60 segments' 1000-value STRING dictionaries converted every string on every comparison (SSB Q2.x:
// ~60 ms of planning per query).
static bool java_less(const std::string& a, const std::string& b) {
  const size_t n = std::min(a.size(), b.size());
  size_t i = 0;
  while (i < n && a[i] == b[i]) ++i;
  if (i == n) return a.size() < b.size();
  const uint8_t x = (uint8_t)a[i], y = (uint8_t)b[i];
  const uint8_t lo = std::min(x, y), hi = std::max(x, y);
  if (lo >= 0xEE && lo <= 0xEF && hi >= 0xF0) return to_utf16(a) < to_utf16(b);
  return x < y;
}

// Double.compare / Double.doubleToLongBits order: -0.0 < 0.0, every NaN equal and greatest. Group
// keys of FLOAT/DOUBLE columns are told apart this way (fastutil's Double2IntOpenHashMap compares
// doubleToLongBits; sorted dictionaries use Double.compare), so merged key columns sort by it.
static uint64_t java_double_order(double v) {
  uint64_t b;
  if (std::isnan(v)) b = 0x7ff8000000000000ull;
  else memcpy(&b, &v, 8);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
static bool java_double_less(double a, double b) { return java_double_order(a) < java_double_order(b); }

struct RoaringContainerHost {
  uint32_t key, kind, count, pad;
  uint64_t offset;
};

}  // namespace

// ------------------------------------------------------------------------------------------------
// Segment
// ------------------------------------------------------------------------------------------------
struct Column {
  std::string name;
  int32_t type = 0, enc = 0, card = 0, bits = 0;
  DevBuf fwd;            // fixed-bit stream | raw values (from rawDataStart) | sorted LE starts
  DevBuf dict;           // LE dictionary values (numeric)
  std::vector<int64_t> dict_i;  // host copies for predicate resolution / result keys
  std::vector<double> dict_d;
  std::vector<std::string> dict_s;
  std::vector<int32_t> sorted_start, sorted_end;  // sorted columns
  // INT / LONG value range (ColumnMetadata minValue / maxValue): dictionary ends, or computed over the
  // staged raw values; bounds which integer sums fit 64-bit partial accumulators
  bool has_range = false;
  int64_t vmin = 0, vmax = 0;
  // inverted index
  DevBuf inv;
  DevBuf inv_conts;
  std::vector<uint32_t> inv_dir;  // containers of dictId d: [inv_dir[d], inv_dir[d+1])
  std::vector<uint64_t> inv_bytes;  // serialized bitmap bytes of dictIds < d (prefix, card+1 entries)
  std::vector<uint16_t> inv_keys;   // container -> key (high 16 bits of its docIds)
  bool has_inv = false;
};

// A predicate leaf resolved on one segment (make_leaf_for_segment), kept on the segment: a re-issued filter
// skips the dictionary lookups, the inverted-index container selection and the descriptor uploads (the
// inverted-index leaves of configs[2]: 26-151 ms of host planning per execution over 100 segments).
struct LeafCacheEntry {
  DevLeaf L;
  bool needs_slot = false;
  std::vector<std::shared_ptr<DevBuf>> bufs;  // the device buffers the leaf points at (sets, descriptors)
  bool inv = false;                           // inverted-index leaf: a docId bitset per execution
  size_t bitset_alloc = 0;
  DevBuf *sel = nullptr, *grp = nullptr, *psel = nullptr;
  int32_t nsel = 0, nchunks = 0;
  double alg_bytes = 0, bitset_bytes = 0;
};

struct pinot_amd_segment {
  std::string name;
  int64_t num_docs = 0;
  uint64_t uid = 0;  // process-unique (never reused): keys host-side caches over segment sets
  uint64_t gen = 0;  // bumped whenever a column is added (a derived dictionary twin included)
  std::map<std::string, std::unique_ptr<Column>> cols;
  int64_t device_bytes = 0;
  // docs matching a filter (signature of its predicates -> count), counted once by the planner's
  // filter-only probe: the segment is immutable, so a filter's count never changes
  std::map<std::string, int64_t> match_cache;
  std::map<std::string, std::shared_ptr<const LeafCacheEntry>> leaf_cache;  // guarded by g_leaf_mu
};

static bool is_float(int t) { return t == T_FLOAT || t == T_DOUBLE; }
static int value_size(int t) { return (t == T_INT || t == T_FLOAT) ? 4 : 8; }

static int decode_dictionary(Column& c, const uint8_t* d, size_t n) {
  if (c.type == T_STRING) {
    if (c.card <= 0) return 0;
    size_t w = n / (size_t)c.card;
    if (w * (size_t)c.card != n) return fail(PINOT_AMD_EINVAL, "string dictionary size %zu not a multiple of %d", n, c.card);
    c.dict_s.resize(c.card);
    for (int i = 0; i < c.card; ++i) {
      // FixedByteValueReaderWriter.readUnpaddedBytes: the value ends at its first NUL byte
      const char* p = (const char*)d + (size_t)i * w;
      c.dict_s[i].assign(p, strnlen(p, w));
    }
    return 0;
  }
  const int vs = value_size(c.type);
  if (n < (size_t)c.card * vs) return fail(PINOT_AMD_EINVAL, "dictionary too small for cardinality %d", c.card);
  std::vector<uint8_t> le((size_t)c.card * vs);
  for (int i = 0; i < c.card; ++i) {
    const uint8_t* p = d + (size_t)i * vs;
    if (vs == 4) {
      uint32_t u = be32(p);
      memcpy(&le[(size_t)i * 4], &u, 4);
      if (c.type == T_INT) {
        c.dict_i.push_back((int32_t)u);
      } else {
        float f;
        memcpy(&f, &u, 4);
        c.dict_d.push_back(f);
      }
    } else {
      uint64_t u = be64(p);
      memcpy(&le[(size_t)i * 8], &u, 8);
      if (c.type == T_LONG) {
        c.dict_i.push_back((int64_t)u);
      } else {
        double f;
        memcpy(&f, &u, 8);
        c.dict_d.push_back(f);
      }
    }
  }
  return c.dict.alloc_copy(le.data(), le.size(), 64);
}

// Parse the RoaringBitmap portable format of every bitmap into a container directory (offsets are
// relative to the staged inverted-index buffer).
static int build_inverted_directory(Column& c, const uint8_t* inv, size_t n) {
  std::vector<RoaringContainerHost> conts;
  c.inv_dir.assign(1, 0);
  c.inv_bytes.assign(1, 0);
  const size_t hdr = 4 * ((size_t)c.card + 1);
  if (n < hdr) return fail(PINOT_AMD_EINVAL, "inverted index too small");
  const uint32_t first = be32(inv);
  for (int d = 0; d < c.card; ++d) {
    const uint32_t s = be32(inv + 4 * (size_t)d), e = be32(inv + 4 * ((size_t)d + 1));
    // offsets may be absolute (whole buffer) or relative to the bitmap area
    // (BitmapInvertedIndexReader.java:36-45): normalise through the first offset
    const size_t base = hdr + (size_t)(s - first);
    const size_t len = (size_t)(e - s);
    if (base + len > n || len < 4) return fail(PINOT_AMD_EINVAL, "bad bitmap %d in inverted index", d);
    const uint8_t* b = inv + base;
    const uint32_t cookie = le32(b);
    size_t pos = 4;
    int32_t size;
    const uint8_t* runbits = nullptr;
    bool has_run = false;
    if ((cookie & 0xFFFF) == 12347) {
      has_run = true;
      size = (int32_t)(cookie >> 16) + 1;
      runbits = b + pos;
      pos += (size + 7) / 8;
    } else if (cookie == 12346) {
      size = (int32_t)le32(b + pos);
      pos += 4;
    } else {
      return fail(PINOT_AMD_EUNSUPPORTED, "unknown RoaringBitmap cookie %u", cookie);
    }
    const uint8_t* header = b + pos;
    pos += 4 * (size_t)size;
    if (!has_run || size >= 4) pos += 4 * (size_t)size;
    for (int32_t i = 0; i < size; ++i) {
      RoaringContainerHost rc{};
      rc.key = le16(header + 4 * i);
      const uint32_t card = (uint32_t)le16(header + 4 * i + 2) + 1;
      const bool is_run = has_run && ((runbits[i / 8] >> (i % 8)) & 1);
      rc.offset = base + pos;
      if (is_run) {
        rc.kind = 2;
        rc.count = le16(b + pos);
        pos += 2 + 4 * (size_t)rc.count;
      } else if (card <= 4096) {
        rc.kind = 0;
        rc.count = card;
        pos += 2 * (size_t)card;
      } else {
        rc.kind = 1;
        rc.count = card;
        pos += 8192;
      }
      if (pos > len) return fail(PINOT_AMD_EINVAL, "truncated bitmap %d", d);
      conts.push_back(rc);
      c.inv_keys.push_back((uint16_t)rc.key);
    }
    c.inv_dir.push_back((uint32_t)conts.size());
    c.inv_bytes.push_back((c.inv_bytes.empty() ? 0 : c.inv_bytes.back()) + len);
  }
  int rc = c.inv.alloc_copy(inv, n, 64);
  if (rc) return rc;
  rc = c.inv_conts.alloc_copy(conts.data(), conts.size() * sizeof(RoaringContainerHost), 64);
  if (rc) return rc;
  c.has_inv = true;
  return 0;
}

// ZSTANDARD / GZIP chunks are entropy-coded (FSE/Huffman) streams with no intra-chunk parallelism
// worth a wave: they are inflated on the host at staging with the system's libzstd / zlib (the
// libraries zstd-jni and java.util.zip wrap), loaded on first use.
struct HostCodecs {
  size_t (*zstd_decompress)(void*, size_t, const void*, size_t) = nullptr;
  unsigned (*zstd_is_error)(size_t) = nullptr;
  int (*z_uncompress)(uint8_t*, unsigned long*, const uint8_t*, unsigned long) = nullptr;
  HostCodecs() {
    if (void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL)) {
      zstd_decompress = (decltype(zstd_decompress))dlsym(h, "ZSTD_decompress");
      zstd_is_error = (decltype(zstd_is_error))dlsym(h, "ZSTD_isError");
    }
    if (void* h = dlopen("libz.so.1", RTLD_NOW | RTLD_LOCAL)) z_uncompress = (decltype(z_uncompress))dlsym(h, "uncompress");
  }
};
static const HostCodecs& host_codecs() {
  static HostCodecs hc;
  return hc;
}

// ---- host chunk decoders for var-byte (STRING) chunks, decoded once at staging ----
// LZ4 block format (lz4-java LZ4FastDecompressor / LZ4SafeDecompressor, third-party: the published
// block format): sequences of (token, literals, 2-byte LE offset, match); returns bytes written or -1.
static int64_t lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  size_t ip = 0, op = 0;
  while (ip < n) {
    const uint8_t tok = src[ip++];
    size_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) return -1;
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip >= n) break;  // last sequence: literals only
    if (ip + 2 > n) return -1;
    const size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return -1;
    size_t ml = (tok & 15u) + 4;
    if ((tok & 15u) == 15) {
      uint8_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    if (op + ml > cap) return -1;
    for (size_t k = 0; k < ml; ++k, ++op) dst[op] = dst[op - off];  // overlapping copies byte by byte
  }
  return (int64_t)op;
}
// Snappy raw format (snappy-java, third-party: varint uncompressed length, then literal / copy elements)
static int64_t snappy_decode(const uint8_t* src, size_t n, std::vector<uint8_t>* out) {
  size_t ip = 0;
  uint64_t len = 0;
  for (int sh = 0; ; sh += 7) {
    if (ip >= n || sh > 35) return -1;
    const uint8_t b = src[ip++];
    len |= (uint64_t)(b & 127u) << sh;
    if (!(b & 128u)) break;
  }
  out->assign(len, 0);
  uint8_t* dst = out->data();
  size_t op = 0;
  while (ip < n) {
    const uint8_t tag = src[ip++];
    if ((tag & 3u) == 0) {  // literal
      size_t l = tag >> 2;
      if (l >= 60) {
        const size_t nb = l - 59;
        if (ip + nb > n) return -1;
        l = 0;
        for (size_t k = 0; k < nb; ++k) l |= (size_t)src[ip + k] << (8 * k);
        ip += nb;
      }
      ++l;
      if (ip + l > n || op + l > len) return -1;
      memcpy(dst + op, src + ip, l);
      ip += l;
      op += l;
      continue;
    }
    size_t l, off;
    if ((tag & 3u) == 1) {
      if (ip + 1 > n) return -1;
      l = ((tag >> 2) & 7u) + 4;
      off = ((size_t)(tag >> 5) << 8) | src[ip];
      ip += 1;
    } else if ((tag & 3u) == 2) {
      if (ip + 2 > n) return -1;
      l = (tag >> 2) + 1;
      off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return -1;
      l = (tag >> 2) + 1;
      off = (size_t)le32(src + ip);
      ip += 4;
    }
    if (off == 0 || off > op || op + l > len) return -1;
    for (size_t k = 0; k < l; ++k, ++op) dst[op] = dst[op - off];
  }
  return op == len ? (int64_t)len : -1;
}

// One var-byte chunk decompressed on the host (ChunkCompressorFactory.getDecompressor per
// ChunkCompressionType: PASS_THROUGH, SNAPPY, ZSTANDARD, LZ4, LZ4_LENGTH_PREFIXED, GZIP).
static int decode_var_chunk(int comp, const uint8_t* src, size_t n, size_t target, std::vector<uint8_t>* out) {
  switch (comp) {
    case 0: out->assign(src, src + n); return 0;
    case 1: return snappy_decode(src, n, out) < 0 ? -1 : 0;
    case 2: {
      const HostCodecs& hc = host_codecs();
      if (!hc.zstd_decompress) return -2;
      out->assign(std::max<size_t>(target, 1) * 2 + 64, 0);
      size_t got = hc.zstd_decompress(out->data(), out->size(), src, n);
      if (hc.zstd_is_error(got)) return -1;
      out->resize(got);
      return 0;
    }
    case 3:
    case 4: {
      // LZ4CompressorWithLength: 4-byte LE decompressed length, then the block (V4+ writers always
      // upgrade LZ4 to the length-prefixed form; a bare LZ4 block is bounded by the chunk target size)
      size_t want, off = 0;
      if (comp == 4) {
        if (n < 4) return -1;
        want = le32(src);
        off = 4;
      } else {
        want = std::max<size_t>(target, 1) * 2 + 64;
      }
      out->assign(want, 0);
      const int64_t got = lz4_block_decode(src + off, n - off, out->data(), want);
      if (got < 0 || (comp == 4 && (size_t)got != want)) return -1;
      out->resize((size_t)got);
      return 0;
    }
    case 5: {
      const HostCodecs& hc = host_codecs();
      if (!hc.z_uncompress) return -2;
      if (n < 4) return -1;
      unsigned long dl = be32(src + n - 4);
      out->assign(dl, 0);
      if (hc.z_uncompress(out->data(), &dl, src, n - 4) != 0) return -1;
      out->resize(dl);
      return 0;
    }
    default: return -2;
  }
}

// Raw STRING forward index (VarByteChunkForwardIndexReaderV4 / V5 / V6: BE header {version,
// targetDecompressedChunkSize, ChunkCompressionType, chunksOffset}, LE metadata {docIdOffset | huge
// bit, chunkOffset} per chunk, LE chunks {numDocs, per-doc offsets (V6 compressed: sizes), bytes}; a
// huge chunk is one value). Decoded into per-doc strings.
static int read_var_byte_strings(const char* name, const uint8_t* fwd, size_t size, int64_t num_docs,
                                 std::vector<std::string>* vals) {
  if (size < 16) return fail(PINOT_AMD_EINVAL, "column %s: var-byte header truncated", name);
  const int32_t version = (int32_t)be32(fwd), target = (int32_t)be32(fwd + 4), comp = (int32_t)be32(fwd + 8);
  const uint32_t chunks_off = be32(fwd + 12);
  if (version < 4 || version > 6)
    return fail(PINOT_AMD_EUNSUPPORTED, "column %s: raw STRING forward index version %d", name, version);
  if (chunks_off < 16 || chunks_off > size || (chunks_off - 16) % 8 != 0)
    return fail(PINOT_AMD_EINVAL, "column %s: bad var-byte metadata", name);
  const size_t nchunks = (chunks_off - 16) / 8;
  vals->clear();
  vals->reserve((size_t)num_docs);
  std::vector<uint8_t> buf;
  for (size_t k = 0; k < nchunks; ++k) {
    const uint32_t doc_word = le32(fwd + 16 + 8 * k);
    const bool huge = (doc_word & 0x80000000u) != 0;
    const uint64_t s = (uint64_t)chunks_off + le32(fwd + 16 + 8 * k + 4);
    const uint64_t e = k + 1 < nchunks ? (uint64_t)chunks_off + le32(fwd + 16 + 8 * (k + 1) + 4) : size;
    if (s > e || e > size || (doc_word & 0x7FFFFFFFu) != vals->size())
      return fail(PINOT_AMD_EINVAL, "column %s: bad var-byte chunk %zu", name, k);
    const int rc = decode_var_chunk(comp, fwd + s, (size_t)(e - s), (size_t)target, &buf);
    if (rc == -2) return fail(PINOT_AMD_EUNSUPPORTED, "column %s: chunk compression %d", name, comp);
    if (rc) return fail(PINOT_AMD_EINVAL, "column %s: var-byte chunk %zu does not decode", name, k);
    if (huge) {
      vals->emplace_back((const char*)buf.data(), buf.size());
      continue;
    }
    if (buf.size() < 4) return fail(PINOT_AMD_EINVAL, "column %s: empty var-byte chunk %zu", name, k);
    const uint32_t nd = le32(buf.data());
    if ((uint64_t)4 * (nd + 1) > buf.size()) return fail(PINOT_AMD_EINVAL, "column %s: var-byte chunk %zu header", name, k);
    const bool sizes = version == 6 && comp != 0;  // VarByteChunkForwardIndexWriterV6: delta-encoded offsets
    uint64_t pos = 4ull * (nd + 1);
    for (uint32_t i = 0; i < nd; ++i) {
      uint64_t a, b;
      if (sizes) {
        a = pos;
        b = a + le32(buf.data() + 4 + 4 * i);
      } else {
        a = le32(buf.data() + 4 + 4 * i);
        b = i + 1 < nd ? le32(buf.data() + 8 + 4 * i) : buf.size();
      }
      if (a > b || b > buf.size()) return fail(PINOT_AMD_EINVAL, "column %s: var-byte value bounds in chunk %zu", name, k);
      vals->emplace_back((const char*)buf.data() + a, (size_t)(b - a));
      pos = b;
    }
  }
  if ((int64_t)vals->size() != num_docs)
    return fail(PINOT_AMD_EINVAL, "column %s: var-byte index holds %zu of %lld docs", name, vals->size(), (long long)num_docs);
  return 0;
}

// Stage a raw forward index with compressed chunks (BaseChunkForwardIndexReader.java:60-105,150-185;
// codecs per ChunkCompressionType.java:22): LZ4, LZ4_LENGTH_PREFIXED, SNAPPY, DELTA and DELTADELTA
// chunks are decoded on the device (chunk_decompress_kernel, one wave per chunk) straight into the
// column's HBM buffer; ZSTANDARD and GZIP on the host.
static int stage_compressed_chunks(Column& c, const pinot_amd_column_spec* spec, const uint8_t* fwd, int32_t version,
                                   int32_t num_chunks, int32_t size, int32_t comp, int32_t dhs, size_t need) {
  const int32_t dpc = (int32_t)be32(fwd + 8);
  const size_t off_size = version <= 2 ? 4 : 8;
  if (dpc <= 0 || num_chunks < 0 || (size_t)dhs + (size_t)num_chunks * off_size > spec->fwd_size)
    return fail(PINOT_AMD_EINVAL, "column %s: bad chunk header", spec->name);
  if (comp < 1 || comp > 7) return fail(PINOT_AMD_EUNSUPPORTED, "column %s: chunk compression %d", spec->name, comp);
  if ((comp == 6 || comp == 7) && is_float(c.type))
    return fail(PINOT_AMD_EINVAL, "column %s: DELTA chunks on a floating-point column", spec->name);
  std::vector<ChunkJob> jobs;
  size_t op = 0;
  for (int32_t ch = 0; ch < num_chunks && op < need; ++ch) {
    const uint8_t* o = fwd + dhs + (size_t)ch * off_size;
    const uint64_t start = off_size == 4 ? be32(o) : be64(o);
    const uint64_t end = ch + 1 < num_chunks ? (off_size == 4 ? be32(o + 4) : be64(o + 8)) : spec->fwd_size;
    if (start > end || end > spec->fwd_size) return fail(PINOT_AMD_EINVAL, "column %s: bad chunk offsets", spec->name);
    ChunkJob j{};
    j.src_off = start;
    j.src_len = (uint32_t)(end - start);
    j.dst_off = op;
    j.dst_len = (uint32_t)std::min<size_t>((size_t)dpc * size, need - op);
    j.codec = comp == 4 ? 3 : comp;
    if (comp == 4) {  // LZ4CompressorWithLength: 4-byte LE decompressed length first
      if (j.src_len < 4) return fail(PINOT_AMD_EINVAL, "column %s: truncated LZ4 chunk %d", spec->name, ch);
      j.src_off += 4;
      j.src_len -= 4;
    }
    jobs.push_back(j);
    op += j.dst_len;
  }
  if (op != need) return fail(PINOT_AMD_EINVAL, "column %s: chunks hold %zu of %zu bytes", spec->name, op, need);
  if (jobs.empty()) return c.fwd.alloc_copy(nullptr, 0, kPadBytes);
  if (comp == 2 || comp == 5) {
    const HostCodecs& hc = host_codecs();
    if (comp == 2 ? !hc.zstd_decompress || !hc.zstd_is_error : !hc.z_uncompress)
      return fail(PINOT_AMD_EUNSUPPORTED, "column %s: %s not loadable for chunk compression %d", spec->name,
                  comp == 2 ? "libzstd.so.1" : "libz.so.1", comp);
    std::vector<uint8_t> out(need);
    for (size_t k = 0; k < jobs.size(); ++k) {
      const ChunkJob& j = jobs[k];
      size_t got;
      if (comp == 2) {
        got = hc.zstd_decompress(out.data() + j.dst_off, j.dst_len, fwd + j.src_off, j.src_len);
        if (hc.zstd_is_error(got)) got = (size_t)-1;
      } else {  // GzipCompressor: zlib stream, then the BE uncompressed size
        unsigned long dl = j.dst_len;
        got = j.src_len >= 4 && hc.z_uncompress(out.data() + j.dst_off, &dl, fwd + j.src_off, j.src_len - 4) == 0
                  ? (size_t)dl : (size_t)-1;
      }
      if (got != j.dst_len)
        return fail(PINOT_AMD_EINVAL, "column %s: chunk %zu of compression %d decoded to %lld of %u bytes", spec->name,
                    k, comp, (long long)(int64_t)got, j.dst_len);
    }
    return c.fwd.alloc_copy(out.data(), need, kPadBytes);
  }
  DevBuf d_src, d_jobs, d_status;
  int rc = d_src.alloc_copy(fwd, spec->fwd_size, 64);
  if (!rc) rc = d_jobs.alloc_copy(jobs.data(), jobs.size() * sizeof(ChunkJob), 0);
  if (!rc) rc = d_status.alloc_copy(nullptr, 0, jobs.size() * 4);
  if (!rc) rc = c.fwd.alloc_copy(nullptr, 0, need + kPadBytes);
  if (rc) return rc;
  HIP_OK(launch_chunk_decompress((const uint8_t*)d_src.p, (uint8_t*)c.fwd.p, d_jobs.p, (int32_t)jobs.size(),
                                 (int32_t*)d_status.p, nullptr));
  HIP_OK(hipDeviceSynchronize());
  std::vector<int32_t> st(jobs.size());
  HIP_OK(hipMemcpy(st.data(), d_status.p, st.size() * 4, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < st.size(); ++k)
    if (st[k]) return fail(PINOT_AMD_EINVAL, "column %s: chunk %zu (compression %d) is malformed", spec->name, k, comp);
  return 0;
}

// segments alive (created, not destroyed): a prepared plan goes back to the plan cache only while every segment it
// reads is alive
static std::mutex g_live_mu;
static std::set<uint64_t> g_live_uids;
static void note_segment_live(uint64_t uid, bool live) {
  std::lock_guard<std::mutex> g(g_live_mu);
  if (live) g_live_uids.insert(uid);
  else g_live_uids.erase(uid);
}
static bool segments_live(const std::vector<uint64_t>& uids) {
  std::lock_guard<std::mutex> g(g_live_mu);
  for (uint64_t u : uids)
    if (!g_live_uids.count(u)) return false;
  return true;
}

extern "C" {

int pinot_amd_abi_version(void) { return PINOT_AMD_ABI_VERSION; }
const char* pinot_amd_last_error(void) { return g_last_error.c_str(); }
int pinot_amd_set_device(int device) {
  HIP_OK(hipSetDevice(device));
  return 0;
}
size_t pinot_amd_required_padding(void) { return (size_t)kPadBytes; }

int pinot_amd_segment_create(const char* name, int64_t num_docs, pinot_amd_segment** out) {
  if (!out || num_docs < 0) return fail(PINOT_AMD_EINVAL, "segment_create: bad arguments");
  if (num_docs > (int64_t)std::numeric_limits<int32_t>::max())
    return fail(PINOT_AMD_EINVAL, "segment_create: %lld docs exceed Pinot's int docId space", (long long)num_docs);
  auto* s = new pinot_amd_segment();
  s->name = name ? name : "";
  s->num_docs = num_docs;
  static std::atomic<uint64_t> next_uid{1};
  s->uid = next_uid.fetch_add(1);
  note_segment_live(s->uid, true);
  *out = s;
  return 0;
}

static void drop_segment_caches(uint64_t uid);

int pinot_amd_segment_destroy(pinot_amd_segment* seg) {
  if (seg) note_segment_live(seg->uid, false);
  if (seg) drop_segment_caches(seg->uid);  // merged key spaces, remaps and prepared plans over it
  if (seg) {
    std::lock_guard<std::mutex> g(g_print_mu);
    for (auto& kv : seg->cols) g_prints.erase(kv.second->fwd.p);
  }
  delete seg;
  return 0;
}

int64_t pinot_amd_segment_num_docs(const pinot_amd_segment* seg) { return seg ? seg->num_docs : -1; }
int64_t pinot_amd_segment_device_bytes(const pinot_amd_segment* seg) { return seg ? seg->device_bytes : -1; }

const void* pinot_amd_segment_column_fwd(const pinot_amd_segment* seg, const char* column) {
  if (!seg || !column) return nullptr;
  auto it = seg->cols.find(column);
  return it == seg->cols.end() ? nullptr : it->second->fwd.p;
}

int pinot_amd_segment_add_column(pinot_amd_segment* seg, const pinot_amd_column_spec* spec) {
  if (!seg || !spec || !spec->name) return fail(PINOT_AMD_EINVAL, "add_column: bad arguments");
  if (seg->cols.count(spec->name)) return fail(PINOT_AMD_EINVAL, "add_column: duplicate column %s", spec->name);
  ++seg->gen;
  if (spec->encoding == ENC_RAW && spec->stored_type == T_STRING) {
    // Raw STRING column: staged dictionary-encoded, as ForwardIndexHandler's ENABLE_DICTIONARY operation
    // rewrites it on load (segment/index/loader/ForwardIndexHandler.java): the distinct values sorted in
    // String.compareTo order (the StringDictionary order), dictIds in a fixed-bit forward index. Every
    // predicate and GROUP BY then runs through the dictionary path with the same docIds and values as
    // the raw-value evaluators. A legacy raw-value inverted index is dropped, as
    // SegmentPreProcessor.removeLegacyRawValueInvertedIndexes does; the scan path covers its predicates.
    if (!spec->h_fwd) return fail(PINOT_AMD_EINVAL, "column %s: no forward index", spec->name);
    std::vector<std::string> vals;
    if (int rc = read_var_byte_strings(spec->name, (const uint8_t*)spec->h_fwd, spec->fwd_size, seg->num_docs, &vals))
      return rc;
    std::vector<std::string> uniq(vals);
    std::sort(uniq.begin(), uniq.end(), java_less);
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    const int32_t card = (int32_t)std::max<size_t>(uniq.size(), 1);
    int bits = 1;
    while ((1ll << bits) < (int64_t)card) ++bits;  // PinotDataBitSet.getNumBitsPerValue(card - 1)
    size_t width = 1;
    for (auto& u : uniq) width = std::max(width, u.size());
    std::vector<uint8_t> dict((size_t)card * width, 0);
    for (size_t i = 0; i < uniq.size(); ++i) memcpy(&dict[i * width], uniq[i].data(), uniq[i].size());
    std::vector<uint8_t> fb((size_t)((seg->num_docs * bits + 7) / 8) + 8, 0);
    uint64_t acc = 0;
    int nacc = 0;
    size_t o = 0;
    for (const std::string& v : vals) {
      const uint64_t id = (uint64_t)(std::lower_bound(uniq.begin(), uniq.end(), v, java_less) - uniq.begin());
      acc = (acc << bits) | id;
      nacc += bits;
      while (nacc >= 8) { fb[o++] = (uint8_t)(acc >> (nacc - 8)); nacc -= 8; }
    }
    if (nacc > 0) fb[o++] = (uint8_t)(acc << (8 - nacc));
    pinot_amd_column_spec d = *spec;
    d.encoding = ENC_FIXED_BIT;
    d.cardinality = card;
    d.bits_per_element = bits;
    d.h_fwd = fb.data();
    d.fwd_size = fb.size();
    d.h_dictionary = dict.data();
    d.dictionary_size = dict.size();
    d.h_inverted = nullptr;
    d.inverted_size = 0;
    return pinot_amd_segment_add_column(seg, &d);
  }
  auto c = std::make_unique<Column>();
  c->name = spec->name;
  c->type = spec->stored_type;
  c->enc = spec->encoding;
  c->card = spec->cardinality;
  c->bits = spec->bits_per_element;
  const int64_t nd = seg->num_docs;
  const uint8_t* fwd = (const uint8_t*)spec->h_fwd;
  if (c->type < T_INT || c->type > T_STRING) return fail(PINOT_AMD_EINVAL, "column %s: bad type", spec->name);
  int rc = 0;
  switch (c->enc) {
    case ENC_FIXED_BIT: {
      if (c->bits < 1 || c->bits > 31) return fail(PINOT_AMD_EINVAL, "column %s: bitsPerElement %d", spec->name, c->bits);
      const size_t need = (size_t)((nd * c->bits + 7) / 8);
      if (spec->fwd_size < need)
        return fail(PINOT_AMD_EINVAL, "column %s: fixed-bit buffer %zu < %zu bytes", spec->name, spec->fwd_size, need);
      rc = c->fwd.alloc_copy(fwd, need, kPadBytes);
      break;
    }
    case ENC_SORTED: {
      if ((size_t)c->card * 8 > spec->fwd_size) return fail(PINOT_AMD_EINVAL, "column %s: sorted index too small", spec->name);
      c->sorted_start.resize(c->card);
      c->sorted_end.resize(c->card);
      for (int i = 0; i < c->card; ++i) {
        c->sorted_start[i] = (int32_t)be32(fwd + 8 * (size_t)i);
        c->sorted_end[i] = (int32_t)be32(fwd + 8 * (size_t)i + 4);
      }
      rc = c->fwd.alloc_copy(c->sorted_start.data(), c->sorted_start.size() * 4, 64);
      break;
    }
    case ENC_RAW: {
      if (c->type == T_STRING) return fail(PINOT_AMD_EUNSUPPORTED, "column %s: raw STRING", spec->name);
      if (spec->fwd_size < 16) return fail(PINOT_AMD_EINVAL, "column %s: raw index header truncated", spec->name);
      // BaseChunkForwardIndexReader.java:60-105: version 1 files have a 16-byte header and SNAPPY
      // chunks; later versions add total docs, the ChunkCompressionType and the data header start
      const int32_t version = (int32_t)be32(fwd), num_chunks = (int32_t)be32(fwd + 4);
      const int32_t size = (int32_t)be32(fwd + 12);
      if (version < 1) return fail(PINOT_AMD_EINVAL, "column %s: raw index version %d", spec->name, version);
      if (version > 1 && spec->fwd_size < 28)
        return fail(PINOT_AMD_EINVAL, "column %s: raw index header truncated", spec->name);
      const int32_t comp = version > 1 ? (int32_t)be32(fwd + 20) : 1 /* SNAPPY */;
      const int32_t dhs = version > 1 ? (int32_t)be32(fwd + 24) : 16;
      if (size != value_size(c->type)) return fail(PINOT_AMD_EINVAL, "column %s: entry size %d", spec->name, size);
      const size_t off_size = version <= 2 ? 4 : 8;
      const size_t raw_start = (size_t)dhs + (size_t)num_chunks * off_size;
      const size_t need = (size_t)nd * size;
      if (comp == 0) {  // PASS_THROUGH: chunks are contiguous raw values
        if (spec->fwd_size < raw_start + need) return fail(PINOT_AMD_EINVAL, "column %s: raw data truncated", spec->name);
        rc = c->fwd.alloc_copy(fwd + raw_start, need, kPadBytes);
      } else {
        // compressed chunks: decoded once while staging, kept as contiguous values in HBM
        rc = stage_compressed_chunks(*c, spec, fwd, version, num_chunks, size, comp, dhs, need);
      }
      break;
    }
    default:
      return fail(PINOT_AMD_EINVAL, "column %s: bad encoding %d", spec->name, c->enc);
  }
  if (rc) return rc;
  if (c->enc != ENC_RAW) {
    // (a column without documents may have an empty dictionary)
    if (!spec->h_dictionary && !(c->card == 0 && spec->dictionary_size == 0))
      return fail(PINOT_AMD_EINVAL, "column %s: dictionary required", spec->name);
    rc = decode_dictionary(*c, (const uint8_t*)spec->h_dictionary, spec->dictionary_size);
    if (rc) return rc;
    if (!c->dict_i.empty()) {  // INT / LONG dictionaries are sorted
      c->has_range = true;
      c->vmin = *std::min_element(c->dict_i.begin(), c->dict_i.end());
      c->vmax = *std::max_element(c->dict_i.begin(), c->dict_i.end());
    }
  } else if ((c->type == T_INT || c->type == T_LONG) && nd > 0) {
    DevBuf mm;
    if (int rc2 = mm.alloc(16)) return rc2;
    const long long init[2] = {LLONG_MAX, LLONG_MIN};
    HIP_OK(hipMemcpy(mm.p, init, 16, hipMemcpyHostToDevice));
    HIP_OK(launch_raw_int_minmax((const uint8_t*)c->fwd.p, c->type, nd, (long long*)mm.p, nullptr));
    long long got[2];
    HIP_OK(hipMemcpy(got, mm.p, 16, hipMemcpyDeviceToHost));
    c->has_range = true;
    c->vmin = got[0];
    c->vmax = got[1];
  }
  if (spec->h_inverted && spec->inverted_size) {
    if (c->enc == ENC_RAW) return fail(PINOT_AMD_EUNSUPPORTED, "column %s: inverted index on raw column", spec->name);
    rc = build_inverted_directory(*c, (const uint8_t*)spec->h_inverted, spec->inverted_size);
    if (rc) return rc;
  }
  seg->device_bytes += (int64_t)(c->fwd.n + c->dict.n + c->inv.n + c->inv_conts.n);
  if (c->fwd.p) {
    StagedPrint sp{c->fwd.n, 0};
    if (int rc2 = device_fingerprint(c->fwd.p, sp.bytes, &sp.print)) return rc2;
    std::lock_guard<std::mutex> g(g_print_mu);
    g_prints[c->fwd.p] = sp;
  }
  seg->cols[c->name] = std::move(c);
  return 0;
}

// ------------------------------------------------------------------------------------------------
// low-level operators
// ------------------------------------------------------------------------------------------------
int pinot_amd_fwd_read_dict_ids(const void* d_packed, int32_t bits, int64_t start_doc, int64_t length, int32_t* d_out,
                                void* stream) {
  if (!d_packed || !d_out || bits < 1 || bits > 31 || start_doc < 0 || length < 0)
    return fail(PINOT_AMD_EINVAL, "fwd_read_dict_ids: bad arguments");
  if (length == 0) return 0;
  HIP_OK(launch_read_dict_ids((const uint8_t*)d_packed, bits, start_doc, length, d_out, (hipStream_t)stream));
  return 0;
}

int pinot_amd_fwd_pack_dict_ids(const int32_t* d_values, int64_t num_values, int32_t bits, void* d_packed,
                                void* stream) {
  if (!d_values || !d_packed || bits < 1 || bits > 31 || num_values < 0)
    return fail(PINOT_AMD_EINVAL, "fwd_pack_dict_ids: bad arguments");
  if (num_values == 0) return 0;
  HIP_OK(launch_pack_dict_ids(d_values, num_values, bits, (uint8_t*)d_packed, (hipStream_t)stream));
  return 0;
}

int pinot_amd_fwd_read_raw(const void* d_raw, int32_t stored_type, int64_t start_doc, int64_t length, void* d_out,
                           void* stream) {
  if (!d_raw || !d_out || stored_type < T_INT || stored_type > T_DOUBLE || start_doc < 0 || length < 0)
    return fail(PINOT_AMD_EINVAL, "fwd_read_raw: bad arguments");
  if (length == 0) return 0;
  HIP_OK(launch_read_raw((const uint8_t*)d_raw, stored_type, start_doc, length, (uint8_t*)d_out, (hipStream_t)stream));
  return 0;
}

int pinot_amd_bitset_and(const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_out, int64_t num_words, void* stream) {
  if (!d_a || !d_b || !d_out || num_words < 0) return fail(PINOT_AMD_EINVAL, "bitset_and: bad arguments");
  if (num_words == 0) return 0;
  HIP_OK(launch_bitset_binop(d_a, d_b, d_out, num_words, 0, (hipStream_t)stream));
  return 0;
}

int pinot_amd_bitset_or(const uint64_t* d_a, const uint64_t* d_b, uint64_t* d_out, int64_t num_words, void* stream) {
  if (!d_a || !d_b || !d_out || num_words < 0) return fail(PINOT_AMD_EINVAL, "bitset_or: bad arguments");
  if (num_words == 0) return 0;
  HIP_OK(launch_bitset_binop(d_a, d_b, d_out, num_words, 1, (hipStream_t)stream));
  return 0;
}

int pinot_amd_bitset_not(const uint64_t* d_a, uint64_t* d_out, int64_t num_docs, void* stream) {
  if (!d_a || !d_out || num_docs < 0) return fail(PINOT_AMD_EINVAL, "bitset_not: bad arguments");
  if (num_docs == 0) return 0;
  HIP_OK(launch_bitset_not(d_a, d_out, num_docs, (hipStream_t)stream));
  return 0;
}

static int bitset_count_impl(const uint64_t* d_bitset, int64_t num_docs, DevBuf& counts, DevBuf& total,
                             int64_t* h_count, hipStream_t st) {
  const int64_t nc = compact_num_chunks(num_docs);
  int rc = counts.alloc((size_t)nc * 8);
  if (rc) return rc;
  rc = total.alloc(8);
  if (rc) return rc;
  HIP_OK(launch_bitset_count(d_bitset, num_docs, (int64_t*)counts.p, (int64_t*)total.p, st));
  HIP_OK(hipMemcpyAsync(h_count, total.p, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

int pinot_amd_bitset_count(const uint64_t* d_bitset, int64_t num_docs, int64_t* h_count, void* stream) {
  if (!d_bitset || !h_count || num_docs < 0) return fail(PINOT_AMD_EINVAL, "bitset_count: bad arguments");
  if (num_docs == 0) {
    *h_count = 0;
    return 0;
  }
  DevBuf counts, total;
  return bitset_count_impl(d_bitset, num_docs, counts, total, h_count, (hipStream_t)stream);
}

int pinot_amd_bitset_to_doc_ids(const uint64_t* d_bitset, int64_t num_docs, int32_t* d_out, int64_t* h_count,
                                void* stream) {
  if (!d_bitset || !d_out || !h_count || num_docs < 0) return fail(PINOT_AMD_EINVAL, "bitset_to_doc_ids: bad arguments");
  if (num_docs == 0) {
    *h_count = 0;
    return 0;
  }
  hipStream_t st = (hipStream_t)stream;
  DevBuf counts, total;
  int rc = bitset_count_impl(d_bitset, num_docs, counts, total, h_count, st);
  if (rc) return rc;
  HIP_OK(launch_bitset_compact(d_bitset, num_docs, (const int64_t*)counts.p, d_out, st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Query
// ------------------------------------------------------------------------------------------------
struct PredSpec {
  std::string column;
  int32_t type = 0, clause = 0, negate = 0, use_inv = 0;
  std::vector<int64_t> vi;
  std::vector<double> vd;
  std::vector<std::string> vs;
  int32_t lower_unbounded = 1, upper_unbounded = 1, lower_inclusive = 1, upper_inclusive = 1;
  int64_t lower_i = 0, upper_i = 0;
  double lower_d = 0, upper_d = 0;
  std::string lower_s, upper_s;
};

static std::mutex g_match_mu;  // guards every segment's match_cache (concurrent planners)

// the filter's identity for the segments' match-count cache: every field of every predicate
static std::string preds_signature(const std::vector<PredSpec>& preds) {
  std::string sig;
  char b[96];
  for (const PredSpec& p : preds) {
    sig += p.column;
    snprintf(b, sizeof(b), "|%d.%d.%d.%d|%d%d%d%d|%lld.%lld|", p.type, p.clause, p.negate, p.use_inv, p.lower_unbounded,
             p.upper_unbounded, p.lower_inclusive, p.upper_inclusive, (long long)p.lower_i, (long long)p.upper_i);
    sig += b;
    sig.append((const char*)&p.lower_d, 8).append((const char*)&p.upper_d, 8);
    sig += p.lower_s + '\x1f' + p.upper_s + '\x1f';
    for (int64_t v : p.vi) sig.append((const char*)&v, 8);
    sig += '\x1e';
    for (double v : p.vd) sig.append((const char*)&v, 8);
    sig += '\x1e';
    for (const std::string& v : p.vs) sig += v + '\x1f';
    sig += '\x1d';
  }
  return sig;
}

struct AggSpec {
  int32_t type;
  std::string column;   // empty for COUNT(*); first operand of an expression
  int32_t expr = 0;     // pinot_amd_expr_op (PINOT_AMD_EXPR_COLUMN: the column itself)
  std::string column2;  // second operand of an expression
};

struct MergedKeyColumn {
  int32_t type = 0;
  std::vector<int64_t> vi;
  std::vector<double> vd;
  std::vector<std::string> vs;
  uint64_t id = 0;  // process-unique identity of this key space (keys the per-segment remap cache)
  size_t size() const { return type == T_STRING ? vs.size() : is_float(type) ? vd.size() : vi.size(); }
  size_t host_bytes() const {
    size_t b = sizeof(*this) + vi.size() * 8 + vd.size() * 8;
    for (const std::string& s : vs) b += sizeof(std::string) + s.size();
    return b;
  }
};
static uint64_t next_key_space_id() {
  static std::atomic<uint64_t> next{1};
  return next.fetch_add(1);
}

struct pinot_amd_query {
  std::vector<PredSpec> preds;
  std::vector<std::string> group_by;
  // group-by column -> key space installed by the caller (the union of every server's dictionaries); shared,
  // immutable once installed (every plan of the query reads the same one, never a copy)
  std::map<std::string, std::shared_ptr<const MergedKeyColumn>> key_space;
  std::vector<AggSpec> aggs;
  int64_t num_groups_limit = 100000;
  // server-level IndexedTable of the combine (GroupByUtils.createIndexedTableForCombineOperator):
  // LIMIT (-1: not set, the whole table), ORDER BY keys, minServerGroupTrimSize, groupTrimThreshold
  int64_t limit = -1;
  struct OrderBy { int kind, index, asc; };  // kind 0: group-by column `index`, 1: aggregation `index`
  std::vector<OrderBy> order_by;
  int64_t min_trim = 5000, trim_threshold = 1000000;
  // query options of the server's result sizing: serverReturnFinalResult (GroupByUtils.java:134-139) and
  // sortAggregateLimitThreshold (QueryContext.shouldSortAggregateUnderSafeTrim, default 10000)
  int server_final = 0;
  int64_t sort_agg_threshold = 10000;
  int64_t min_seg_trim = -1;  // minSegmentGroupTrimSize
};

extern "C" {

int pinot_amd_query_create(pinot_amd_query** out) {
  if (!out) return fail(PINOT_AMD_EINVAL, "query_create: null out");
  *out = new pinot_amd_query();
  return 0;
}
int pinot_amd_query_destroy(pinot_amd_query* q) {
  delete q;
  return 0;
}

int pinot_amd_query_add_predicate(pinot_amd_query* q, int32_t clause, const pinot_amd_predicate_spec* p,
                                  int32_t negate) {
  if (!q || !p || !p->column) return fail(PINOT_AMD_EINVAL, "add_predicate: bad arguments");
  if (clause < 0 || clause >= kMaxClauses) return fail(PINOT_AMD_EUNSUPPORTED, "add_predicate: clause %d", clause);
  if (q->preds.size() >= (size_t)kMaxLeaves) return fail(PINOT_AMD_EUNSUPPORTED, "add_predicate: too many predicates");
  PredSpec s;
  s.column = p->column;
  s.type = p->type;
  s.clause = clause;
  s.negate = negate ? 1 : 0;
  s.use_inv = p->use_inverted_index;
  if (p->type < PINOT_AMD_EQ || p->type > PINOT_AMD_RANGE) return fail(PINOT_AMD_EINVAL, "add_predicate: bad type");
  if (p->type != PINOT_AMD_RANGE) {
    if (p->num_values < 1) return fail(PINOT_AMD_EINVAL, "add_predicate: no values");
    if ((p->type == PINOT_AMD_EQ || p->type == PINOT_AMD_NOT_EQ) && p->num_values != 1)
      return fail(PINOT_AMD_EINVAL, "add_predicate: EQ takes one value");
    for (int i = 0; i < p->num_values; ++i) {
      if (p->h_values_i) s.vi.push_back(p->h_values_i[i]);
      if (p->h_values_d) s.vd.push_back(p->h_values_d[i]);
      if (p->h_values_s) s.vs.push_back(p->h_values_s[i] ? p->h_values_s[i] : "");
    }
  } else {
    s.lower_unbounded = p->lower_unbounded;
    s.upper_unbounded = p->upper_unbounded;
    s.lower_inclusive = p->lower_inclusive;
    s.upper_inclusive = p->upper_inclusive;
    s.lower_i = p->lower_i;
    s.upper_i = p->upper_i;
    s.lower_d = p->lower_d;
    s.upper_d = p->upper_d;
    if (p->lower_s) s.lower_s = p->lower_s;
    if (p->upper_s) s.upper_s = p->upper_s;
  }
  q->preds.push_back(std::move(s));
  return 0;
}

int pinot_amd_query_add_group_by(pinot_amd_query* q, const char* column) {
  if (!q || !column) return fail(PINOT_AMD_EINVAL, "add_group_by: bad arguments");
  if (q->group_by.size() >= (size_t)kMaxGroupCols) return fail(PINOT_AMD_EUNSUPPORTED, "add_group_by: too many columns");
  q->group_by.push_back(column);
  return 0;
}

int pinot_amd_query_add_aggregation(pinot_amd_query* q, int32_t agg_type, const char* column, int32_t* out_index) {
  if (!q) return fail(PINOT_AMD_EINVAL, "add_aggregation: null query");
  if (agg_type < PINOT_AMD_AGG_COUNT || agg_type > PINOT_AMD_AGG_MINMAXRANGE)
    return fail(PINOT_AMD_EINVAL, "add_aggregation: bad type");
  AggSpec a{agg_type, (column && strcmp(column, "*") != 0) ? column : ""};
  if (agg_type != PINOT_AMD_AGG_COUNT && a.column.empty()) return fail(PINOT_AMD_EINVAL, "add_aggregation: column required");
  if (out_index) *out_index = (int32_t)q->aggs.size();
  q->aggs.push_back(a);
  return 0;
}

int pinot_amd_query_add_aggregation_expr(pinot_amd_query* q, int32_t agg_type, int32_t expr_op, const char* column_a,
                                         const char* column_b, int32_t* out_index) {
  if (!q || !column_a || !column_b || !*column_a || !*column_b)
    return fail(PINOT_AMD_EINVAL, "add_aggregation_expr: bad arguments");
  if (expr_op < PINOT_AMD_EXPR_MUL || expr_op > PINOT_AMD_EXPR_ADD)
    return fail(PINOT_AMD_EINVAL, "add_aggregation_expr: bad expression op %d", expr_op);
  if (agg_type != PINOT_AMD_AGG_SUM && agg_type != PINOT_AMD_AGG_MIN && agg_type != PINOT_AMD_AGG_MAX &&
      agg_type != PINOT_AMD_AGG_AVG && agg_type != PINOT_AMD_AGG_MINMAXRANGE)
    return fail(PINOT_AMD_EUNSUPPORTED, "add_aggregation_expr: aggregation %d over an expression", agg_type);
  AggSpec a{agg_type, column_a, expr_op, column_b};
  if (out_index) *out_index = (int32_t)q->aggs.size();
  q->aggs.push_back(a);
  return 0;
}

int pinot_amd_query_set_group_key_values(pinot_amd_query* q, const char* column, int32_t stored_type, int64_t n,
                                         const int64_t* h_values_i, const double* h_values_d,
                                         const char* const* h_values_s) {
  if (!q || !column || n < 0 || stored_type < T_INT || stored_type > T_STRING)
    return fail(PINOT_AMD_EINVAL, "set_group_key_values: bad arguments");
  MergedKeyColumn m;
  m.type = stored_type;
  m.id = next_key_space_id();
  for (int64_t i = 0; i < n; ++i) {
    if (stored_type == T_STRING) {
      if (!h_values_s || !h_values_s[i]) return fail(PINOT_AMD_EINVAL, "set_group_key_values: null string");
      m.vs.push_back(h_values_s[i]);
    } else if (is_float(stored_type)) {
      if (!h_values_d) return fail(PINOT_AMD_EINVAL, "set_group_key_values: no values");
      m.vd.push_back(stored_type == T_FLOAT ? (double)(float)h_values_d[i] : h_values_d[i]);
    } else {
      if (!h_values_i) return fail(PINOT_AMD_EINVAL, "set_group_key_values: no values");
      m.vi.push_back(h_values_i[i]);
    }
  }
  // the caller's values in any order: sorted and deduplicated in dictionary order
  if (m.type == T_STRING) {
    std::sort(m.vs.begin(), m.vs.end(), java_less);
    m.vs.erase(std::unique(m.vs.begin(), m.vs.end()), m.vs.end());
  } else if (is_float(m.type)) {
    std::sort(m.vd.begin(), m.vd.end(), java_double_less);
    m.vd.erase(std::unique(m.vd.begin(), m.vd.end(),
                           [](double a, double b) { return java_double_order(a) == java_double_order(b); }),
               m.vd.end());
  } else {
    std::sort(m.vi.begin(), m.vi.end());
    m.vi.erase(std::unique(m.vi.begin(), m.vi.end()), m.vi.end());
  }
  q->key_space[column] = std::make_shared<const MergedKeyColumn>(std::move(m));
  return 0;
}

int pinot_amd_query_set_num_groups_limit(pinot_amd_query* q, int64_t limit) {
  if (!q || limit < 1) return fail(PINOT_AMD_EINVAL, "set_num_groups_limit: bad arguments");
  q->num_groups_limit = limit;
  return 0;
}

int pinot_amd_query_set_result_limit(pinot_amd_query* q, int64_t limit, int64_t min_server_group_trim_size,
                                     int64_t group_trim_threshold) {
  if (!q || limit < 0) return fail(PINOT_AMD_EINVAL, "set_result_limit: bad arguments");
  q->limit = limit;
  q->min_trim = min_server_group_trim_size;
  q->trim_threshold = group_trim_threshold;
  return 0;
}

int pinot_amd_query_set_server_options(pinot_amd_query* q, int32_t server_return_final_result,
                                       int64_t sort_aggregate_limit_threshold) {
  if (!q || sort_aggregate_limit_threshold <= 0) return fail(PINOT_AMD_EINVAL, "set_server_options: bad arguments");
  q->server_final = server_return_final_result ? 1 : 0;
  q->sort_agg_threshold = sort_aggregate_limit_threshold;
  return 0;
}

int pinot_amd_query_set_segment_trim(pinot_amd_query* q, int64_t min_segment_group_trim_size) {
  if (!q) return fail(PINOT_AMD_EINVAL, "set_segment_trim: null query");
  q->min_seg_trim = min_segment_group_trim_size;
  return 0;
}

int pinot_amd_query_add_order_by(pinot_amd_query* q, int32_t kind, int32_t index, int32_t ascending) {
  if (!q || (kind != 0 && kind != 1) || index < 0) return fail(PINOT_AMD_EINVAL, "add_order_by: bad arguments");
  if (kind == 0 && index >= (int32_t)q->group_by.size())
    return fail(PINOT_AMD_EINVAL, "add_order_by: group-by column %d not in the query", index);
  if (kind == 1 && index >= (int32_t)q->aggs.size())
    return fail(PINOT_AMD_EINVAL, "add_order_by: aggregation %d not in the query", index);
  q->order_by.push_back({kind, index, ascending ? 1 : 0});
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Result / compiled plan
// ------------------------------------------------------------------------------------------------
// One kernel launch of a plan: the segments of a batch that share a shape (every slot's encoding and
// fixed-bit width), with their own descriptors and query-specialised kernels. Segments whose
// columns are encoded differently (a table whose index config changed between segments) run in
// separate launches accumulating into the same table, so every launch has compile-time decoders.
struct Launch {
  std::vector<int> segs;      // indices into the query's segment list
  int batch = 0;              // hash trimming batch
  DevQuery q{};               // nsegs / total_tiles of this launch; acc ops shared
  DevBuf d_segs;
  DevBuf d_bitset_ptrs;       // filter-only plans: this launch's segments' docId bitsets
  JitKernel* jit = nullptr;         // scan, or the partitioned count / scatter / aggregate trio
  JitKernel* jit_atomic = nullptr;  // partitioned: direct-atomic scan used when few docs match
  JitKernel* jit_sample = nullptr;  // partitioned: match count over every sample_stride-th tile
  // hash plans with a second level: the scan without the LDS level (JitPlan::hash_direct), its LDS bytes, and
  // the direct placement's per-launch tables (DevHash::dbase / dcnt, the partition begins) with the partition
  // count (log2) they were made for
  std::vector<DevSegment> h_segs;  // the uploaded descriptors (self-check forensics compare the count blocks' reads)
  JitKernel* jit_direct = nullptr;
  size_t shmem_direct = 0;
  DevBuf d_dbase, d_dcnt, d_dpbeg;
  int direct_lg = -1;
  int grid = 1, atomic_grid = 1, sample_grid = 1, agg_grid = 1, scan_nsub = 1, part_sub = kPartSub;
  size_t shmem = 0, shmem_scatter = 0, shmem_agg = 0;
  DevPartition part{};
  int64_t docs = 0, tiles = 0;
  double col_bytes = 0;  // algorithmic bytes of the launch's decoded columns over all its docs
  bool gated = false;    // an inverted-index gate clause: columns are read only where it passes
  // selection-vector plan (late materialisation): select pass over the filter columns, gather pass
  bool select = false, word_select = false;
  // fused inverted-index select (roaring_select_kernel): expansion + word-level select in one launch
  bool fused = false;
  DevBuf d_fused;  // FusedSelSeg per segment of the launch
  int32_t nfused = 0, fused_leaves = 0, fused_clauses = 0;
  bool fused_clause = false;  // roaring_select_clause_kernel (no negated bitset leaf)
  int64_t fused_items = 0;
  size_t shmem_sets = 0;  // LDS dictId sets of the scan / select pass (JitLeaf::lds_words)
  int gather_grid = 1, gather_threads = 256;
  double filter_bytes = 0, value_bpr = 0;  // select: filter columns over all docs; gathered bytes per match
  bool fgate = false;  // filter-gated fused scan: filter columns over all docs, value bytes per match
  // partitioned: record size; sampled capacities (strided histogram instead of the count pass)
  int rec_bytes = 0;
  bool part_sampled = false;
  int64_t region_cap = 0;  // records the partition regions can hold
  // dense numGroupsLimit admission: the first-doc pass over each segment's prefix (d_fd_segs: the
  // launch's segments cut to their prefixes), or over whole segments (d_segs) when a prefix saw too few keys
  JitKernel* jit_fd = nullptr;
  JitKernel* jit_as = nullptr;  // the sequential admission (key spaces that fit LDS), one block per segment
  JitKernel* jit_sp = nullptr;  // segment-level safe trim: the presence pass over ORDER BY ranks
  int sp_grid = 1;
  DevBuf d_fd_segs;
  DevQuery fd_q{};
  int fd_grid = 1, fd_full_grid = 1;
};

enum PlanKind { PLAN_DENSE = 0, PLAN_PARTITIONED = 1, PLAN_HASH = 2, PLAN_FILTER = 3 };

struct pinot_amd_result {
  hipStream_t stream = nullptr;
  PlanKind kind = PLAN_DENSE;
  DevQuery q{};                  // plan-wide: nacc, acc_op, num_keys (dense)
  std::deque<Launch> launches;  // deque: Launch holds device buffers and is never moved
  std::vector<std::unique_ptr<DevBuf>> owned;  // leaf sets, remaps, bitsets
  bool filter_gate = false;  // the fused scan loads key / value columns behind its filter (JitPlan::filter_gate)
  // inverted index leaves to (re)build each execution: (segment, leaf, container selection)
  struct InvLeaf {
    int seg;
    const Column* col;
    DevBuf* bitset;
    DevBuf* sel;   // selected container indices grouped by chunk
    DevBuf* grp;   // chunk k's containers: sel[grp[k] .. grp[k+1])
    int32_t nsel, nchunks;
    int64_t num_docs;
    double alg_bytes;     // the selected bitmaps' serialized bytes (read once)
    double bitset_bytes;  // the dense docId bitset written and read once (only when the expansion runs)
    DevBuf* psel = nullptr;  // packed descriptors in sel order (ExpandJob::psel), or none
  };
  std::vector<InvLeaf> inv_leaves;
  DevBuf d_expand_jobs;        // one ExpandJob per inv_leaves entry (batched clear + expand launches)
  int64_t expand_total = 0;   // work items: (job, 65536-doc chunk) pairs
  std::vector<std::unique_ptr<DevBuf>> bitsets;  // filter-only plans: one docId bitset per segment
  std::vector<int64_t> bitset_words;
  DevBuf acc;                  // dense table, or the hash plan's final table accumulators
  // counters: 3 per launch ([0] count pass / scan matches, [1] sampled matches, [2] direct-atomic
  // scan matches), then numGroupsLimitReached, then hash overflow
  DevBuf matched;
  std::vector<std::shared_ptr<const MergedKeyColumn>> keys;  // merged dictionaries of the group-by columns
  std::vector<std::shared_ptr<DevBuf>> shared;  // device buffers shared with the planner's caches (remaps)
  std::vector<int64_t> key_stride;    // dense: mixed-radix strides
  std::vector<int32_t> agg_acc;        // aggregation -> accumulator index (AVG: sum acc; MINMAXRANGE: min acc)
  std::vector<int32_t> agg_acc2;       // MINMAXRANGE: max acc
  std::vector<int32_t> agg_type;
  int32_t num_group_by = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t ev_x = nullptr;  // orders a cross-rank call's stream after the result's (call_stream)
  std::string jit_status;
  // partitioned GROUP BY: shared work buffers (launches run one after another)
  DevBuf hist, offs, part_begin, rec;
  bool check_failed = false;  // the last execution's partitioned self-check failed (verify_partitioned)
  // hash plans with a second level: 0 = the LDS level (skewed keys), 1 = no LDS level, records to the blocks'
  // regions (counting the direct placement's allotments), 2 = direct placement; 0 -> 1 when an execution spilled
  // most matching docs (check_overflow), 1 -> 2 after a counting execution. direct_ran: the last execution placed
  // records directly (its check word then holds the blocks that fell short of their allotments)
  int hash_mode = 0;
  bool direct_ran = false;
  bool direct_place = false;  // mode 2 allowed (PINOT_AMD_HASH_DIRECT=place / force)
  // prepared-plan cache (plan_cache_*): the identity this plan was built for, the segments it reads, its device bytes
  std::string plan_key;
  std::vector<uint64_t> plan_uids;
  size_t plan_bytes = 0;
  // segment-level group trim over the (key, segment) scan table of a hash plan (SegSelStage, launch_segsel): the
  // safe trim past the dense cap (keep = LIMIT) and the unsafe trim with minSegmentGroupTrimSize (keep =
  // max(minSegmentGroupTrimSize, 5 x LIMIT)), each segment's top `keep` groups in the ORDER BY's order
  bool segsel = false;
  int64_t segsel_keep = 0;
  std::vector<SegSelStage> segsel_st;
  DevBuf d_segsel_st, ss_cnt, ss_want, ss_done, ss_prefix, ss_cut, ss_hist;
  std::string check_msg;
  DevBuf part_hw;  // per launch: the count and scatter blocks' placement and tallies (DevPartition::hw)
  DevBuf eff_begin, ovf_n, ovf_rec, ovf_part;  // sampled plans: allotment prefix, overflow slab
  // selection-vector plans: the shared vector (launches run one after another) and 2 counters per launch
  DevBuf sel, sel_ctr;
  // hash-table GROUP BY
  int nw = 0;                          // key words (group columns)
  std::vector<int> pack_word, pack_shift, pack_bits;
  DevBuf fkeys;                        // final table keys (nw x fcap)
  int64_t fcap = 0;
  // untrimmed hash plans: the table grows 4x (up to fcap_ceiling: 2 x the plan's group bound, the slot and
  // byte limits) while docs find no slot. The capacity an execution settled on is remembered per (query
  // shape, segment set) (cap_key); a plan that starts from it runs without the host synchronisation that
  // reads the overflow counter (ovf_pending: check_overflow settles it when the groups are read)
  int64_t fcap_ceiling = 0;
  std::string cap_key;
  // second level of the LDS-privatised hash plan (JitPlan::hash_spill, DevHash::spill)
  DevBuf sp_rec, sp_sorted, sp_cnt, sp_hist, sp_offs, sp_pbeg;
  int64_t spill_cap = 0, spill_grid = 0;
  int64_t spill_cap_max = 0;  // regions' ceiling: the scan blocks' docs, within PINOT_AMD_SPILL_MAX_BYTES
  int spill_words = 0, spill_slots = 0, spill_agg_grid = 1;
  uint32_t spill_narrow = 0;  // accumulators (bit a) whose integer sums fit int64 over all docs: plain LDS adds
  bool cap_known = false, ovf_pending = false;
  bool trim = false;                   // numGroupsLimit trimming (scan tables keyed by (key, segment))
  int64_t limit = 100000;
  bool limit_possible = false;         // some segment may hold >= numGroupsLimit keys
  int nbatches = 1;
  std::vector<int64_t> batch_cap;      // scan table slots per batch
  std::vector<int32_t> batch_nsegs;
  std::vector<int64_t> batch_bucket_off;  // offset of the batch's bucket_base array in d_bucket_base
  std::vector<int64_t> batch_buckets;
  DevBuf skeys, sacc;                  // trim scan table (largest batch)
  DevBuf d_bucket_base, t_hist, t_distinct, t_bstar, t_rank, t_bitmap, t_dstar;
  int fd_acc = -1;                     // ACC_FIRST_DOC accumulator index
  // dense numGroupsLimit admission (trimming over a key space a dense table holds): per segment the first
  // matching docId of every key seen in its prefix, the list of those keys, and the admission bitmaps
  bool admit = false;
  DevBuf a_first, a_seen, a_seen_n, a_bits, a_hist, a_bbase, a_bstar, a_rank, a_bitmap, a_dstar;
  // segment-level safe trim (JitPlan::seg_ord): per segment a presence bitmap over ORDER BY ranks (sp_words
  // words) and the rank of its LIMIT-th group
  bool seg_trim = false;
  DevBuf sp_bits, sp_cut;
  int64_t sp_words = 0;
  int32_t sp_nsegs = 0;
  int64_t a_cap = 0, a_words = 0, a_buckets = 0, a_max_buckets = 0;
  std::vector<int64_t> a_prefix;       // docs of each segment the first pass reads
  std::vector<int64_t> a_docs;
  // cross-rank merge by value (pinot_amd_result_merge_groups): until the next execution the result's
  // groups are those of the merged table (keys packed as the hash plan packs them)
  bool merged = false;
  DevBuf mkeys, macc, movf;
  // group compaction scratch (presence bits, chunk counts, total, slot indices, gathered keys / accumulators),
  // kept across fetches and executions: a fetch allocates nothing on the device
  DevBuf c_bits, c_counts, c_total, c_idx, c_okeys, c_oacc;
  DevBuf c_skeys, c_sacc, c_sscratch;  // hash groups sorted by key on the device (sort_rows_by_key)
  int64_t mcap = 0;
  int mnw = 0;
  // server-level IndexedTable (pinot_amd_query_set_result_limit / add_order_by), applied at compaction
  int64_t srv_limit = -1, srv_min_trim = 5000, srv_trim_threshold = 1000000;
  std::vector<pinot_amd_query::OrderBy> srv_order;
  int srv_final = 0;                   // serverReturnFinalResult
  int64_t srv_sort_threshold = 10000;  // sortAggregateLimitThreshold
  bool srv_safe = false;               // ORDER BY keys = GROUP BY keys, no HAVING (QueryContext._isUnsafeTrim false)
  bool srv_trimmed = false;
  // host planning time per phase (pinot_amd_result_plan_timing)
  std::string plan_timing;
  // result compaction cache (valid until the next execution)
  bool compacted = false;
  // HBM-table array indices of the whole-query-narrow sums' low words (JitAcc::hbm_narrow): their high
  // words are set from the low words' signs at the plan's end
  DevBuf d_sext;
  int32_t n_sext = 0;
  int64_t ngroups = 0;
  std::vector<uint64_t> ckeys, cacc;  // per group: key words (hash) or dense key; all accumulator words
  ~pinot_amd_result() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev_x) (void)hipEventDestroy(ev_x);
  }
};

namespace {

// ------------------------------------------------------------------------------------------------
// Prepared-plan cache. A server re-issues the same query over the same segments (dashboards, retries, the
// broker's per-server fan-out of a repeated query); a destroyed result's plan -- its generated kernels, device
// descriptors, leaf tables, group tables, grown capacities -- is kept, idle, under the identity it was built
// for, and the next execute of that identity takes it and only runs it (run_plan, the work execute_again does),
// skipping the host planning (predicate leaves, key spaces, plan choice, descriptor packing, buffer setup).
// Identity: the query (every field of pinot_amd_query, the installed key spaces by id), filter-only or not, the
// segments by (uid, generation), the device, and the planner overrides in the environment. A plan reading a
// destroyed segment is dropped with it (drop_segment_caches); a plan whose self-check failed is never kept.
// At most PINOT_AMD_PLAN_CACHE_BYTES (default 2 GiB) of plan device memory, 64 plans, least recently used out
// first; a plan above a quarter of the budget is freed as before. PINOT_AMD_PLAN_CACHE=0 disables the cache.
// ------------------------------------------------------------------------------------------------
struct PlanCacheEntry {
  std::unique_ptr<pinot_amd_result> r;
  uint64_t used = 0;
};
static std::mutex g_plan_mu;
static std::multimap<std::string, PlanCacheEntry> g_plans;
static size_t g_plan_bytes = 0;
static uint64_t g_plan_clock = 0;

static bool plan_cache_on() {
  static const bool on = [] {
    const char* v = knob("PINOT_AMD_PLAN_CACHE");
    return !(v && std::string(v) == "0");
  }();
  return on;
}
static size_t plan_cache_budget() {
  static const size_t b = [] {
    const char* v = knob("PINOT_AMD_PLAN_CACHE_BYTES");
    return v ? (size_t)std::max(0ll, atoll(v)) : (size_t)2 << 30;
  }();
  return b;
}

static std::string plan_identity(const pinot_amd_query& Q, const std::vector<pinot_amd_segment*>& segs, bool filter_only) {
  const std::string ks = knob_snapshot();
  if (ks.empty() || !plan_cache_on()) return std::string();
  std::string k = filter_only ? "F|" : "Q|";
  auto num = [&](long long v) { k += std::to_string(v) + ","; };
  k += preds_signature(Q.preds) + "|G";
  for (const std::string& g : Q.group_by) k += g + '\x1f';
  k += "|K";
  for (const auto& kv : Q.key_space) k += kv.first + "=" + std::to_string(kv.second ? kv.second->id : 0) + '\x1f';
  k += "|A";
  for (const AggSpec& a : Q.aggs) {
    num(a.type);
    k += a.column + '\x1f';
    num(a.expr);
    k += a.column2 + '\x1f';
  }
  k += "|O";
  for (const auto& o : Q.order_by) {
    num(o.kind);
    num(o.index);
    num(o.asc);
  }
  k += "|L";
  for (long long v : {(long long)Q.num_groups_limit, (long long)Q.limit, (long long)Q.min_trim, (long long)Q.trim_threshold,
                      (long long)Q.server_final, (long long)Q.sort_agg_threshold, (long long)Q.min_seg_trim})
    num(v);
  k += "|S";
  for (auto* sg : segs) k += std::to_string(sg->uid) + "." + std::to_string(sg->gen) + ",";
  int dev = 0;
  (void)hipGetDevice(&dev);
  k += "|D" + std::to_string(dev) + "|" + ks;
  return k;
}

// an idle plan of this identity, or null
static pinot_amd_result* plan_cache_take(const std::string& key) {
  if (key.empty()) return nullptr;
  std::lock_guard<std::mutex> g(g_plan_mu);
  auto it = g_plans.find(key);
  if (it == g_plans.end()) return nullptr;
  pinot_amd_result* r = it->second.r.release();
  g_plan_bytes -= r->plan_bytes;
  g_plans.erase(it);
  return r;
}

// true: the cache keeps r (idle: its stream synchronised by the caller)
static bool plan_cache_put(pinot_amd_result* r) {
  if (r->plan_key.empty() || r->check_failed || !segments_live(r->plan_uids)) return false;
  const size_t budget = plan_cache_budget();
  if (r->plan_bytes > budget / 4) return false;
  std::vector<std::unique_ptr<pinot_amd_result>> evicted;
  {
    std::lock_guard<std::mutex> g(g_plan_mu);
    while (!g_plans.empty() && (g_plan_bytes + r->plan_bytes > budget || g_plans.size() >= 64)) {
      auto lru = g_plans.begin();
      for (auto it = g_plans.begin(); it != g_plans.end(); ++it)
        if (it->second.used < lru->second.used) lru = it;
      g_plan_bytes -= lru->second.r->plan_bytes;
      evicted.push_back(std::move(lru->second.r));
      g_plans.erase(lru);
    }
    PlanCacheEntry e;
    e.r.reset(r);
    e.used = ++g_plan_clock;
    g_plan_bytes += r->plan_bytes;
    g_plans.emplace(r->plan_key, std::move(e));
  }
  g_release_to_pool = true;  // evicted plans are idle: their blocks go to the device pool (outside the lock)
  evicted.clear();
  g_release_to_pool = false;
  return true;
}

// plans reading segment uid (it is being destroyed)
static void plan_cache_drop_uid(uint64_t uid) {
  std::vector<std::unique_ptr<pinot_amd_result>> dropped;
  {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (auto it = g_plans.begin(); it != g_plans.end();) {
      if (std::find(it->second.r->plan_uids.begin(), it->second.r->plan_uids.end(), uid) != it->second.r->plan_uids.end()) {
        g_plan_bytes -= it->second.r->plan_bytes;
        dropped.push_back(std::move(it->second.r));
        it = g_plans.erase(it);
      } else {
        ++it;
      }
    }
  }
  g_release_to_pool = true;  // idle plans (synchronised when cached)
  dropped.clear();
  g_release_to_pool = false;
}

// Dictionary.insertionIndexOf: index if found, else -(insertionPoint + 1)
template <typename T, typename Less>
int64_t insertion_index_of(const std::vector<T>& v, const T& x, Less less) {
  auto it = std::lower_bound(v.begin(), v.end(), x, less);
  const int64_t i = it - v.begin();
  if (it != v.end() && !less(x, *it)) return i;
  return -(i + 1);
}

struct DictView {
  const Column* c;
  int64_t card() const { return c->card; }
  // insertion index of a predicate value given as int64 / double / string
  int64_t ins_i(int64_t x) const {
    if (c->type == T_STRING) return ins_s(std::to_string(x));
    if (is_float(c->type)) return ins_d((double)x);
    return insertion_index_of(c->dict_i, x, std::less<int64_t>());
  }
  int64_t ins_d(double x) const {
    if (!is_float(c->type)) {
      // integer dictionary probed with a double bound: position among integers
      const double f = std::floor(x);
      auto it = std::lower_bound(c->dict_i.begin(), c->dict_i.end(), x,
                                 [](int64_t a, double b) { return (double)a < b; });
      const int64_t i = it - c->dict_i.begin();
      if (f == x && it != c->dict_i.end() && (double)*it == x) return i;
      return -(i + 1);
    }
    return insertion_index_of(c->dict_d, x, [](double a, double b) { return a < b; });
  }
  int64_t ins_s(const std::string& x) const {
    if (c->type != T_STRING) {
      char* end = nullptr;
      if (is_float(c->type)) return ins_d(strtod(x.c_str(), &end));
      return insertion_index_of(c->dict_i, (int64_t)strtoll(x.c_str(), &end, 10), std::less<int64_t>());
    }
    return insertion_index_of(c->dict_s, x, java_less);
  }
};

// dictIds of an EQ/IN predicate's values (PredicateUtils.getDictIdSet): values absent from the
// dictionary are dropped
static std::vector<int32_t> dict_ids_of_values(const PredSpec& p, const Column& c) {
  DictView dv{&c};
  std::vector<int32_t> ids;
  const size_t n = std::max(p.vi.size(), std::max(p.vd.size(), p.vs.size()));
  for (size_t i = 0; i < n; ++i) {
    int64_t r;
    if (c.type == T_STRING)
      r = !p.vs.empty() ? dv.ins_s(p.vs[i]) : dv.ins_i(p.vi[i]);
    else if (is_float(c.type))
      r = !p.vd.empty() ? dv.ins_d(p.vd[i]) : !p.vi.empty() ? dv.ins_d((double)p.vi[i]) : dv.ins_s(p.vs[i]);
    else
      r = !p.vi.empty() ? dv.ins_i(p.vi[i]) : !p.vd.empty() ? dv.ins_d(p.vd[i]) : dv.ins_s(p.vs[i]);
    if (r >= 0) ids.push_back((int32_t)r);
  }
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  return ids;
}

// SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:115-160):
// [start, end) dictIds
static void dict_range_of(const PredSpec& p, const Column& c, int64_t* start, int64_t* end) {
  DictView dv{&c};
  auto ins = [&](bool lower) -> int64_t {
    if (c.type == T_STRING) return dv.ins_s(lower ? p.lower_s : p.upper_s);
    if (is_float(c.type)) return dv.ins_d(lower ? p.lower_d : p.upper_d);
    return dv.ins_i(lower ? p.lower_i : p.upper_i);
  };
  if (p.lower_unbounded) {
    *start = 0;
  } else {
    const int64_t i = ins(true);
    *start = i < 0 ? -(i + 1) : (p.lower_inclusive ? i : i + 1);
  }
  if (p.upper_unbounded) {
    *end = c.card;
  } else {
    const int64_t i = ins(false);
    *end = i < 0 ? -(i + 1) : (p.upper_inclusive ? i + 1 : i);
  }
}

}  // namespace

// Evaluate an EQ/IN/RANGE predicate through the bitmap inverted index or through the forward
// index? Both give the same docId set; pick the one that moves fewer bytes: the selected bitmaps
// (serialized size, ~its container payloads) plus writing and re-reading the dense bitset, against
// decoding the fixed-bit forward index (free when the column is decoded anyway for GROUP BY /
// aggregation). PINOT_AMD_INV_POLICY=always|never overrides (tests).
static bool use_inverted_for(const Column& c, int64_t num_docs, const std::vector<int32_t>& ids, bool is_range,
                             int64_t start, int64_t end, bool decoded_anyway) {
  if (const char* pol = knob("PINOT_AMD_INV_POLICY")) {
    if (strcmp(pol, "always") == 0) return true;
    if (strcmp(pol, "never") == 0) return false;
  }
  uint64_t inv = 0;
  int64_t nconts = 0;
  if (is_range) {
    inv = c.inv_bytes[end] - c.inv_bytes[start];
    nconts = (int64_t)c.inv_dir[end] - c.inv_dir[start];
  } else {
    for (int32_t d : ids) {
      inv += c.inv_bytes[d + 1] - c.inv_bytes[d];
      nconts += (int64_t)c.inv_dir[d + 1] - c.inv_dir[d];
    }
  }
  const double inv_cost = (double)inv + 64.0 * (double)nconts + 2.0 * (double)num_docs / 8.0;
  const double scan_cost = decoded_anyway ? 0.0 : (double)num_docs * c.bits / 8.0;
  return inv_cost < scan_cost;
}

// docId-bitset slack behind an inverted-index leaf's words (make_leaf_for_segment): 64 tiles
constexpr size_t kBitsetSlackBytes = 64 * kTileDocs / 8;

static int make_leaf_uncached(pinot_amd_result* r, int si, const pinot_amd_segment* seg, const PredSpec& p,
                              const Column& c, int slot, DevLeaf* L, bool* needs_slot, hipStream_t st,
                              bool decoded_anyway) {
  memset(L, 0, sizeof(*L));
  L->slot = slot;
  L->clause = p.clause;
  L->negate = p.negate;
  *needs_slot = true;
  const bool negated_type = p.type == PINOT_AMD_NOT_EQ || p.type == PINOT_AMD_NOT_IN;
  if (negated_type) L->negate ^= 1;

  if (c.enc == ENC_RAW) {
    // raw-value based evaluators
    if (p.type == PINOT_AMD_RANGE) {
      if (is_float(c.type)) {
        L->kind = LEAF_RAW_RANGE_F;
        double lo = -INFINITY, hi = INFINITY;
        if (c.type == T_FLOAT) {
          // FloatRawValueBasedRangePredicateEvaluator: Math.nextUp/nextDown in float
          if (!p.lower_unbounded) lo = p.lower_inclusive ? (double)(float)p.lower_d : (double)std::nextafter((float)p.lower_d, INFINITY);
          if (!p.upper_unbounded) hi = p.upper_inclusive ? (double)(float)p.upper_d : (double)std::nextafter((float)p.upper_d, -INFINITY);
        } else {
          if (!p.lower_unbounded) lo = p.lower_inclusive ? p.lower_d : std::nextafter(p.lower_d, INFINITY);
          if (!p.upper_unbounded) hi = p.upper_inclusive ? p.upper_d : std::nextafter(p.upper_d, -INFINITY);
        }
        L->lo_d = lo;
        L->hi_d = hi;
      } else {
        // Int/LongRawValueBasedRangePredicateEvaluator: exclusive bounds +/- 1, unbounded = type min/max
        const int64_t tmin = c.type == T_INT ? INT32_MIN : INT64_MIN, tmax = c.type == T_INT ? INT32_MAX : INT64_MAX;
        int64_t lo = tmin, hi = tmax;
        if (!p.lower_unbounded) {
          if (!p.lower_inclusive && p.lower_i == tmax) return fail(PINOT_AMD_EINVAL, "Invalid range on %s", c.name.c_str());
          lo = p.lower_inclusive ? p.lower_i : p.lower_i + 1;
        }
        if (!p.upper_unbounded) {
          if (!p.upper_inclusive && p.upper_i == tmin) return fail(PINOT_AMD_EINVAL, "Invalid range on %s", c.name.c_str());
          hi = p.upper_inclusive ? p.upper_i : p.upper_i - 1;
        }
        L->kind = LEAF_RAW_RANGE_I;
        L->lo_i = lo;
        L->hi_i = hi;
      }
      return 0;
    }
    // EQ/NOT_EQ/IN/NOT_IN: sorted value set
    auto buf = std::make_unique<DevBuf>();
    int rc;
    if (is_float(c.type)) {
      std::vector<double> v = p.vd;
      if (v.empty())
        for (int64_t x : p.vi) v.push_back((double)x);
      if (c.type == T_FLOAT)
        for (double& x : v) x = (double)(float)x;
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      L->kind = LEAF_RAW_IN_F;
      L->in_n = (int32_t)v.size();
      rc = buf->alloc_copy(v.data(), v.size() * 8, 64);
      if (rc) return rc;
      L->in_d = (const double*)buf->p;
    } else {
      std::vector<int64_t> v = p.vi;
      if (v.empty())
        for (double x : p.vd) v.push_back((int64_t)x);
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      L->kind = LEAF_RAW_IN_I;
      L->in_n = (int32_t)v.size();
      rc = buf->alloc_copy(v.data(), v.size() * 8, 64);
      if (rc) return rc;
      L->in_i = (const int64_t*)buf->p;
    }
    r->owned.push_back(std::move(buf));
    return 0;
  }

  // dictionary-based evaluators: resolve to a dictId range or dictId set in this segment
  int64_t start = 0, end = 0;
  std::vector<int32_t> ids;
  bool is_range = false;
  if (p.type == PINOT_AMD_RANGE) {
    dict_range_of(p, c, &start, &end);
    if (end < start) end = start;
    is_range = true;
  } else {
    ids = dict_ids_of_values(p, c);
    if (!ids.empty() && ids.back() - ids.front() + 1 == (int32_t)ids.size()) {
      is_range = true;
      start = ids.front();
      end = (int64_t)ids.back() + 1;
    } else if (ids.empty()) {
      is_range = true;
      start = end = 0;
    }
  }
  const bool empty = is_range ? end <= start : ids.empty();
  const bool full = is_range ? (start <= 0 && end >= c.card) : (int64_t)ids.size() == c.card;
  L->accept = 0ull;
  if (c.card <= 64) {
    if (is_range)
      for (int64_t d = std::max<int64_t>(start, 0); d < std::min<int64_t>(end, c.card); ++d) L->accept |= 1ull << d;
    else
      for (int32_t d : ids) L->accept |= 1ull << d;
  }
  if (empty || full) {  // alwaysFalse / alwaysTrue evaluators
    L->kind = LEAF_CONST;
    L->lo_i = full ? 1 : 0;
    L->accept = full ? ~0ull : 0ull;
    *needs_slot = false;
    L->slot = -1;
    return 0;
  }
  if (c.enc == ENC_SORTED && is_range) {
    // SortedIndexBasedFilterOperator: a dictId range of a sorted column is one docId range
    L->kind = LEAF_DOC_RANGE;
    L->lo_i = c.sorted_start[start];
    L->hi_i = c.sorted_end[end - 1];
    L->slot = -1;
    *needs_slot = false;
    return 0;
  }
  if (p.use_inv && c.has_inv && c.enc == ENC_FIXED_BIT &&
      use_inverted_for(c, seg->num_docs, ids, is_range, start, end, decoded_anyway)) {
    // BitmapBasedFilterOperator: OR of the inverted-index bitmaps of the matching dictIds
    if (is_range) {
      ids.clear();
      for (int64_t d = start; d < end; ++d) ids.push_back((int32_t)d);
    }
    // selected containers grouped by 65536-doc chunk (container key): the expansion builds each
    // chunk of the dense bitset in LDS from its group and writes it out once
    const int64_t tiles = (seg->num_docs + kTileDocs - 1) / kTileDocs;
    const size_t bs_bytes = (size_t)std::max<int64_t>(tiles, 1) * kTileDocs / 8 + 64;
    // work items: groups of G consecutive chunks; a group's containers in (value, chunk) order
    const int32_t nchunks = (int32_t)((bs_bytes / 8 + 1023) / 1024);
    const int32_t G = expand_group();
    const int32_t ngroups = (nchunks + G - 1) / G;
    std::vector<int32_t> grp(ngroups + 1, 0);
    for (int32_t d : ids)
      for (uint32_t k = c.inv_dir[d]; k < c.inv_dir[d + 1]; ++k)
        if (c.inv_keys[k] < nchunks) ++grp[c.inv_keys[k] / G + 1];
    for (int32_t k = 0; k < ngroups; ++k) grp[k + 1] += grp[k];
    std::vector<int32_t> sel(grp[ngroups]);
    {
      std::vector<int32_t> fillp(grp.begin(), grp.end() - 1);
      for (int32_t d : ids)
        for (uint32_t k = c.inv_dir[d]; k < c.inv_dir[d + 1]; ++k)
          if (c.inv_keys[k] < nchunks) sel[fillp[c.inv_keys[k] / G]++] = (int32_t)k;
    }
    // (+ slack: grouped scan / select steps read the word of every lane's doc0 in padding tiles and in the
    // inactive steps past a block's range -- up to (D + 1) x G + 3 tiles beyond the segment -- whose masks are
    // zero; the words are allocated so those reads stay inside the buffer)
    auto bs = std::make_unique<DevBuf>();
    int rc = bs->alloc(bs_bytes + kBitsetSlackBytes);
    if (rc) return rc;
    auto sb = std::make_unique<DevBuf>();
    rc = sb->alloc_copy(sel.data(), sel.size() * 4, 64);
    if (rc) return rc;
    auto gb = std::make_unique<DevBuf>();
    rc = gb->alloc_copy(grp.data(), grp.size() * 4, 64);
    if (rc) return rc;
    double sel_bytes = 0;
    for (int32_t d : ids) sel_bytes += (double)(c.inv_bytes[d + 1] - c.inv_bytes[d]);
    r->inv_leaves.push_back({si, &c, bs.get(), sb.get(), gb.get(), (int32_t)sel.size(), ngroups, seg->num_docs,
                             sel_bytes, 2.0 * (double)((seg->num_docs + 7) / 8)});
    if (!sel.empty() && c.inv.n < ((size_t)1 << 32)) {  // packed descriptors, built once per plan
      auto pb = std::make_unique<DevBuf>();
      rc = pb->alloc(sel.size() * 8);
      if (rc) return rc;
      HIP_OK(launch_pack_sel(c.inv_conts.p, (const int32_t*)sb->p, (int64_t)sel.size(), G, (unsigned long long*)pb->p, st));
      r->inv_leaves.back().psel = pb.get();
      r->owned.push_back(std::move(pb));
    }
    r->owned.push_back(std::move(gb));
    L->kind = LEAF_DOC_BITSET;
    L->bits = (const uint32_t*)bs->p;
    L->slot = -1;
    *needs_slot = false;
    r->owned.push_back(std::move(bs));
    r->owned.push_back(std::move(sb));
    return 0;
  }
  if (is_range) {
    L->kind = LEAF_DICT_RANGE;
    L->lo_i = start;
    L->hi_i = end;
    return 0;
  }
  std::vector<uint32_t> mask(((size_t)c.card + 31) / 32 + 1, 0u);
  for (int32_t d : ids) mask[d >> 5] |= 1u << (d & 31);
  auto buf = std::make_unique<DevBuf>();
  int rc = buf->alloc_copy(mask.data(), mask.size() * 4, 64);
  if (rc) return rc;
  L->kind = LEAF_DICT_SET;
  L->bits = (const uint32_t*)buf->p;
  r->owned.push_back(std::move(buf));
  return 0;
}

static bool env_is(const char* name, const char* val);
static std::mutex g_leaf_mu;  // guards every segment's leaf_cache
constexpr size_t kLeafCacheMax = 256;  // entries per segment (cleared when full)

// make_leaf_uncached through the segment's leaf cache. The key is everything the resolution reads: the
// predicate, the slot, whether its column is decoded anyway, and the knobs of the inverted-index policy.
static std::string leaf_cache_key(const PredSpec& p, int slot, bool decoded_anyway) {
  const char* pol = knob("PINOT_AMD_INV_POLICY");
  return preds_signature({p}) + "|" + std::to_string(slot) + "|" + (decoded_anyway ? "1" : "0") + "|" +
         std::to_string(expand_group()) + "|" + (pol ? pol : "");
}

// key: leaf_cache_key(p, slot, decoded_anyway) when the caller built it once for every segment
static int make_leaf_for_segment(pinot_amd_result* r, int si, pinot_amd_segment* seg, const PredSpec& p,
                                 const Column& c, int slot, DevLeaf* L, bool* needs_slot, hipStream_t st,
                                 bool decoded_anyway, const std::string* key_in = nullptr) {
  const bool use_cache = key_in != nullptr || !env_is("PINOT_AMD_LEAF_CACHE", "0");
  std::string key_own;
  const std::string& key = key_in ? *key_in : key_own;
  if (use_cache) {
    if (!key_in) key_own = leaf_cache_key(p, slot, decoded_anyway);
    std::shared_ptr<const LeafCacheEntry> e;
    {
      std::lock_guard<std::mutex> g(g_leaf_mu);
      auto it = seg->leaf_cache.find(key);
      if (it != seg->leaf_cache.end()) e = it->second;
    }
    if (e) {
      *L = e->L;
      *needs_slot = e->needs_slot;
      for (auto& b : e->bufs) r->shared.push_back(b);
      if (e->inv) {
        auto bs = std::make_unique<DevBuf>();
        if (int rc = bs->alloc(e->bitset_alloc)) return rc;
        L->bits = (const uint32_t*)bs->p;
        r->inv_leaves.push_back({si, &c, bs.get(), e->sel, e->grp, e->nsel, e->nchunks, seg->num_docs, e->alg_bytes,
                                 e->bitset_bytes, e->psel});
        r->owned.push_back(std::move(bs));
      }
      return 0;
    }
  }
  const size_t o0 = r->owned.size(), i0 = r->inv_leaves.size();
  if (int rc = make_leaf_uncached(r, si, seg, p, c, slot, L, needs_slot, st, decoded_anyway)) return rc;
  if (!use_cache) return 0;
  auto e = std::make_shared<LeafCacheEntry>();
  e->L = *L;
  e->needs_slot = *needs_slot;
  const DevBuf* bitset = nullptr;
  if (r->inv_leaves.size() > i0) {
    const auto& il = r->inv_leaves.back();
    e->inv = true;
    e->bitset_alloc = il.bitset->n;
    e->sel = il.sel;
    e->grp = il.grp;
    e->psel = il.psel;
    e->nsel = il.nsel;
    e->nchunks = il.nchunks;
    e->alg_bytes = il.alg_bytes;
    e->bitset_bytes = il.bitset_bytes;
    bitset = il.bitset;
    HIP_OK(hipStreamSynchronize(st));  // the packed descriptors (launch_pack_sel) are read by later streams
  }
  // the leaf's descriptor buffers move to shared ownership (same objects: the pointers above stay valid);
  // the per-execution docId bitset stays owned by this result
  std::vector<std::unique_ptr<DevBuf>> keep;
  for (size_t k = o0; k < r->owned.size(); ++k) {
    if (r->owned[k].get() == bitset) {
      keep.push_back(std::move(r->owned[k]));
      continue;
    }
    std::shared_ptr<DevBuf> sb(r->owned[k].release());
    e->bufs.push_back(sb);
    r->shared.push_back(std::move(sb));
  }
  r->owned.resize(o0);
  for (auto& k : keep) r->owned.push_back(std::move(k));
  std::lock_guard<std::mutex> g(g_leaf_mu);
  if (seg->leaf_cache.size() >= kLeafCacheMax) seg->leaf_cache.clear();
  seg->leaf_cache[key] = std::move(e);
  return 0;
}

// GROUP BY on a raw (no-dictionary) column: NoDictionarySingleColumnGroupKeyGenerator /
// NoDictionaryMultiColumnGroupKeyGenerator (pinot-core/.../query/aggregation/groupby/
// NoDictionarySingleColumnGroupKeyGenerator.java:98-143) assign group ids to distinct values through
// fastutil open hash maps (equality = value equality, doubleToLongBits for FLOAT/DOUBLE). Here the
// segment gets a derived dictionary-encoded twin of the column, built once on first use and kept
// staged next to it ("<col>$dict": sorted distinct values in the same order as a Pinot dictionary +
// a fixed-bit forward index of dictIds), so the device plan groups it exactly like a dictionary
// column: same groups, same key values, same dense mixed-radix key space.
static int derive_raw_group_dictionary(pinot_amd_segment* s, const std::string& col, std::string* out_name) {
  *out_name = col + "$dict";
  if (s->cols.count(*out_name)) return 0;
  const Column& c = *s->cols.at(col);
  if (c.type == T_STRING) return fail(PINOT_AMD_EUNSUPPORTED, "GROUP BY on raw STRING column %s", col.c_str());
  const int64_t nd = s->num_docs;
  const int vs = value_size(c.type);
  // on the device (derive.hip): order keys, radix sort, distinct values, dictIds, packed forward index
  DevBuf scratch, ids, dict_be, packed;
  if (int rc = scratch.alloc(derive_dictionary_scratch(std::max<int64_t>(nd, 1)))) return rc;
  if (int rc = ids.alloc((size_t)std::max<int64_t>(nd, 1) * 4)) return rc;
  if (int rc = dict_be.alloc((size_t)std::max<int64_t>(nd, 1) * vs)) return rc;
  int64_t card = 0;
  HIP_OK(derive_dictionary((const uint8_t*)c.fwd.p, c.type, nd, scratch.p, (int32_t*)ids.p, (uint8_t*)dict_be.p, &card,
                           nullptr));
  card = std::max<int64_t>(card, 1);
  int bits = 1;
  while (card > 1 && (1ll << bits) < card) ++bits;  // PinotDataBitSet.getNumBitsPerValue(card - 1)
  const size_t fb_bytes = (size_t)((nd * bits + 7) / 8);
  if (int rc = packed.alloc(fb_bytes + 8)) return rc;
  HIP_OK(hipMemset(packed.p, 0, packed.n));
  if (nd) HIP_OK(launch_pack_dict_ids((const int32_t*)ids.p, nd, bits, (uint8_t*)packed.p, nullptr));
  std::vector<uint8_t> fb(fb_bytes + 8, 0), dict((size_t)card * vs, 0);
  HIP_OK(hipMemcpy(fb.data(), packed.p, fb_bytes, hipMemcpyDeviceToHost));
  if (nd) HIP_OK(hipMemcpy(dict.data(), dict_be.p, dict.size(), hipMemcpyDeviceToHost));
  pinot_amd_column_spec spec{};
  spec.name = out_name->c_str();
  spec.stored_type = c.type;
  spec.encoding = ENC_FIXED_BIT;
  spec.cardinality = (int32_t)card;
  spec.bits_per_element = bits;
  spec.h_fwd = fb.data();
  spec.fwd_size = fb.size();
  spec.h_dictionary = dict.data();
  spec.dictionary_size = dict.size();
  return pinot_amd_segment_add_column(s, &spec);
}

static int build_merged_keys_uncached(const std::vector<pinot_amd_segment*>& segs, const std::string& col,
                                      MergedKeyColumn* out);

// Merged dictionaries of a group-by column over a segment set, cached per (column, segments): segments are
// immutable, and every query grouping by the column over the same batch merges the same dictionaries (SSB
// Q2.x: 60 dictionaries of 1000 brands, ~5 ms per query). Entries are shared (never copied into a plan),
// least-recently-used entries go beyond a host-byte budget (PINOT_AMD_KEY_CACHE_BYTES, default 1 GiB), and
// an entry goes with the first of its segments that is destroyed.
// Per-segment remaps (dictId -> id in a merged key space) are cached the same way, keyed by (segment, column,
// key-space id): the device array a plan reads, shared with every plan that uses it (SSB Q2.x planning spent
// ~2 ms per query, the wide-key bench ~110 ms, in binary searches over the merged dictionaries).
struct KeyCacheEntry {
  std::shared_ptr<const MergedKeyColumn> keys;
  std::vector<uint64_t> uids;
  size_t bytes = 0;
  uint64_t used = 0;
};
struct RemapCacheEntry {
  std::shared_ptr<DevBuf> buf;  // nullptr: the identity (no remap needed)
  uint64_t uid = 0, used = 0;
};
static std::mutex g_keys_mu;
static std::map<std::string, KeyCacheEntry> g_keys_cache;
static std::map<std::string, RemapCacheEntry> g_remap_cache;
static size_t g_keys_bytes = 0;
static uint64_t g_cache_clock = 0;

static void drop_segment_caches(uint64_t uid) {
  plan_cache_drop_uid(uid);
  std::lock_guard<std::mutex> g(g_keys_mu);
  for (auto it = g_keys_cache.begin(); it != g_keys_cache.end();) {
    if (std::find(it->second.uids.begin(), it->second.uids.end(), uid) != it->second.uids.end()) {
      g_keys_bytes -= it->second.bytes;
      it = g_keys_cache.erase(it);
    } else {
      ++it;
    }
  }
  for (auto it = g_remap_cache.begin(); it != g_remap_cache.end();)
    it = it->second.uid == uid ? g_remap_cache.erase(it) : std::next(it);
}

static int build_merged_keys(const std::vector<pinot_amd_segment*>& segs, const std::string& col,
                             std::shared_ptr<const MergedKeyColumn>* out) {
  std::string key = col + "|";
  for (auto* sg : segs) key += std::to_string(sg->uid) + "." + std::to_string(sg->gen) + ",";
  {
    std::lock_guard<std::mutex> g(g_keys_mu);
    auto it = g_keys_cache.find(key);
    if (it != g_keys_cache.end()) {
      it->second.used = ++g_cache_clock;
      *out = it->second.keys;
      return 0;
    }
  }
  MergedKeyColumn m;
  if (int rc = build_merged_keys_uncached(segs, col, &m)) return rc;
  m.id = next_key_space_id();
  *out = std::make_shared<const MergedKeyColumn>(std::move(m));
  KeyCacheEntry ent;
  ent.keys = *out;
  ent.bytes = (*out)->host_bytes() + key.size();
  for (auto* sg : segs) ent.uids.push_back(sg->uid);
  static const size_t budget = []() {
    const char* v = knob("PINOT_AMD_KEY_CACHE_BYTES");
    return v ? (size_t)std::max(0ll, atoll(v)) : (size_t)1 << 30;
  }();
  std::lock_guard<std::mutex> g(g_keys_mu);
  if (g_keys_cache.count(key)) return 0;  // another planner built it meanwhile
  while (!g_keys_cache.empty() && g_keys_bytes + ent.bytes > budget) {  // least recently used first
    auto lru = g_keys_cache.begin();
    for (auto it = g_keys_cache.begin(); it != g_keys_cache.end(); ++it)
      if (it->second.used < lru->second.used) lru = it;
    g_keys_bytes -= lru->second.bytes;
    g_keys_cache.erase(lru);
  }
  if (ent.bytes > budget) return 0;  // larger than the whole budget: not cached
  ent.used = ++g_cache_clock;
  g_keys_bytes += ent.bytes;
  g_keys_cache[key] = std::move(ent);
  return 0;
}

static int build_merged_keys_uncached(const std::vector<pinot_amd_segment*>& segs, const std::string& col,
                                      MergedKeyColumn* out) {
  const Column* c0 = segs[0]->cols.at(col).get();
  out->type = c0->type;
  for (auto* s : segs) {
    const Column* c = s->cols.at(col).get();
    if (c->type != c0->type) return fail(PINOT_AMD_EINVAL, "group-by column %s has different types", col.c_str());
    if (c->type == T_STRING) out->vs.insert(out->vs.end(), c->dict_s.begin(), c->dict_s.end());
    else if (is_float(c->type)) out->vd.insert(out->vd.end(), c->dict_d.begin(), c->dict_d.end());
    else out->vi.insert(out->vi.end(), c->dict_i.begin(), c->dict_i.end());
  }
  if (out->type == T_STRING) {
    std::sort(out->vs.begin(), out->vs.end(), java_less);
    out->vs.erase(std::unique(out->vs.begin(), out->vs.end()), out->vs.end());
  } else if (is_float(out->type)) {
    std::sort(out->vd.begin(), out->vd.end(), java_double_less);
    out->vd.erase(std::unique(out->vd.begin(), out->vd.end(),
                              [](double a, double b) { return java_double_order(a) == java_double_order(b); }),
                  out->vd.end());
  } else {
    std::sort(out->vi.begin(), out->vi.end());
    out->vi.erase(std::unique(out->vi.begin(), out->vi.end()), out->vi.end());
  }
  return 0;
}

static int remap_for(const Column& c, const MergedKeyColumn& m, std::vector<int32_t>* out) {
  out->resize(c.card);
  for (int32_t d = 0; d < c.card; ++d) {
    int64_t pos;
    if (c.type == T_STRING)
      pos = std::lower_bound(m.vs.begin(), m.vs.end(), c.dict_s[d], java_less) - m.vs.begin();
    else if (is_float(c.type))
      pos = std::lower_bound(m.vd.begin(), m.vd.end(), c.dict_d[d], java_double_less) - m.vd.begin();
    else
      pos = std::lower_bound(m.vi.begin(), m.vi.end(), c.dict_i[d]) - m.vi.begin();
    (*out)[d] = (int32_t)pos;
  }
  return 0;
}

// the device remap of segment s's column c into key space m (cached, shared); *out = nullptr: the identity
static int cached_remap(const pinot_amd_segment* s, const std::string& col, const Column& c, const MergedKeyColumn& m,
                        std::shared_ptr<DevBuf>* out) {
  const std::string key = std::to_string(s->uid) + "." + std::to_string(s->gen) + "|" + col + "|" + std::to_string(m.id);
  if (m.id != 0) {
    std::lock_guard<std::mutex> g(g_keys_mu);
    auto it = g_remap_cache.find(key);
    if (it != g_remap_cache.end()) {
      it->second.used = ++g_cache_clock;
      *out = it->second.buf;
      return 0;
    }
  }
  std::vector<int32_t> rm;
  remap_for(c, m, &rm);
  bool identity = (int64_t)rm.size() == (int64_t)m.size();
  for (size_t d = 0; identity && d < rm.size(); ++d) identity = rm[d] == (int32_t)d;
  out->reset();
  if (!identity) {
    auto buf = std::make_shared<DevBuf>();
    if (int rc = buf->alloc_copy(rm.data(), rm.size() * 4, 64)) return rc;
    *out = std::move(buf);
  }
  if (m.id == 0) return 0;
  std::lock_guard<std::mutex> g(g_keys_mu);
  if (g_remap_cache.size() >= 16384) {  // bounded: drop the least recently used quarter
    std::vector<uint64_t> ages;
    for (auto& kv : g_remap_cache) ages.push_back(kv.second.used);
    std::nth_element(ages.begin(), ages.begin() + ages.size() / 4, ages.end());
    const uint64_t cut = ages[ages.size() / 4];
    for (auto it = g_remap_cache.begin(); it != g_remap_cache.end();)
      it = it->second.used <= cut ? g_remap_cache.erase(it) : std::next(it);
  }
  g_remap_cache[key] = RemapCacheEntry{*out, s->uid, ++g_cache_clock};
  return 0;
}

// ------------------------------------------------------------------------------------------------
// execution
// ------------------------------------------------------------------------------------------------
static int launch_one(pinot_amd_result* r, Launch& L, size_t li, uint64_t* table, const DevHash& H) {
  hipStream_t st = r->stream;
  const DevSegment* segs = (const DevSegment*)L.d_segs.p;
  uint64_t* const* bits = r->kind == PLAN_FILTER ? (uint64_t* const*)L.d_bitset_ptrs.p : nullptr;
  unsigned long long* matched = (unsigned long long*)r->matched.p + 3 * li;
  DevHash h = H;
  void* args[] = {(void*)&segs, (void*)&L.q, (void*)&table, (void*)&bits, (void*)&matched, (void*)&L.part, (void*)&h};
  if (L.select) {  // select pass (filter columns -> selection vector), then the gather-aggregate pass
    HIP_OK(hipMemsetAsync(L.q.sel_count, 0, 16, st));
    if (L.fused)
      HIP_OK(launch_roaring_select(r->d_expand_jobs.p, L.d_fused.p, L.nfused, L.fused_items, L.d_segs.p,
                                   L.fused_leaves, L.fused_clauses, L.q.sel_entries, L.q.sel_count, L.q.sel_cap,
                                   matched, L.fused_clause ? 1 : 0, st));
    else
      // (select kernels hold their tables in static LDS)
      HIP_OK(hipModuleLaunchKernel(L.jit->fn, (unsigned)L.grid, 1, 1, kBlock, 1, 1, 0, st, args, nullptr));
    if (knob("PINOT_AMD_CHECK_SELECT")) {  // diagnostics: validate the vector on the host
      unsigned long long ctr[2];
      HIP_OK(hipMemcpyAsync(ctr, L.q.sel_count, 16, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      if (ctr[1] != 0 || ctr[0] > (unsigned long long)L.q.sel_cap || ctr[0] % 4 != 0)
        return fail(PINOT_AMD_EINVAL, "select check: count %llu overflow %llu cap %lld", ctr[0], ctr[1], (long long)L.q.sel_cap);
      std::vector<unsigned long long> ent(ctr[0]);
      if (!ent.empty()) HIP_OK(hipMemcpy(ent.data(), L.q.sel_entries, ent.size() * 8, hipMemcpyDeviceToHost));
      std::vector<DevSegment> ds(L.segs.size());
      HIP_OK(hipMemcpy(ds.data(), L.d_segs.p, ds.size() * sizeof(DevSegment), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < ent.size(); ++i) {
        const uint32_t sg = (uint32_t)(ent[i] >> 32), d = (uint32_t)ent[i];
        if (sg >= ds.size() || (d != 0xFFFFFFFFu && (int64_t)d >= ds[sg].num_docs) || (uint32_t)(ent[i & ~(size_t)3] >> 32) != sg)
          return fail(PINOT_AMD_EINVAL, "select check: entry %zu = seg %u doc %u (segments %zu)", i, sg, d, ds.size());
      }
    }
    HIP_OK(hipModuleLaunchKernel(L.jit->fn_gather, (unsigned)L.gather_grid, 1, 1, (unsigned)L.gather_threads, 1, 1,
                                 (unsigned)L.shmem, st, args, nullptr));
    return 0;
  }
  if (r->kind != PLAN_PARTITIONED) {
    const bool direct = r->hash_mode > 0 && L.jit_direct;  // (the same grid: the spill regions are sized for it)
    HIP_OK(hipModuleLaunchKernel(direct ? L.jit_direct->fn : L.jit->fn, (unsigned)L.grid, 1, 1, kBlock * L.scan_nsub, 1, 1,
                                 (unsigned)(direct ? L.shmem_direct : L.shmem), st, args, nullptr));
    return 0;
  }
  const unsigned pt = (unsigned)(kBlock * L.part_sub);
  const unsigned count_grid = (unsigned)(L.grid * kPartCountRatio);
  if (L.part_sampled) {
    // per scatter block: strided histogram -> allotments -> (direct-atomic scan | scatter) -> records
    // held per allotment -> aggregation -> overflow slab
    unsigned long long* sampled = matched + 1;
    void* sargs[] = {(void*)&segs, (void*)&L.q, (void*)&table, (void*)&bits, (void*)&sampled, (void*)&L.part, (void*)&h};
    HIP_OK(hipMemsetAsync(L.part.ovf_n, 0, 8, st));
    HIP_OK(hipModuleLaunchKernel(L.jit->fn, (unsigned)L.grid, 1, 1, pt, 1, 1, (unsigned)L.shmem, st, sargs, nullptr));
    const char* cs = knob("PINOT_AMD_PART_CAP_SCALE");  // tests: < 1 forces records into the slab
    const double cap_scale = cs ? std::max(0.0, atof(cs)) : 1.0;
    HIP_OK(launch_allot_prefix(L.part.hist, L.part.nparts, L.grid, 0, L.part.sample_stride, cap_scale, L.region_cap,
                               L.part.part_begin, L.part.offs, st));
    if (L.jit_atomic)
      HIP_OK(hipModuleLaunchKernel(L.jit_atomic->fn, (unsigned)L.atomic_grid, 1, 1, kBlock, 1, 1, 0, st, args, nullptr));
    HIP_OK(hipModuleLaunchKernel(L.jit->fn_scatter, (unsigned)L.grid, 1, 1, pt, 1, 1, (unsigned)L.shmem_scatter, st, args,
                                 nullptr));
    HIP_OK(launch_allot_prefix(L.part.hist, L.part.nparts, L.grid, 1, 1, 1.0, 0, L.part.part_begin, L.part.eff_begin, st));
    void* agg_args[] = {(void*)&L.part, (void*)&table};
    HIP_OK(hipModuleLaunchKernel(L.jit->fn_agg, (unsigned)L.agg_grid, 1, 1, 1024, 1, 1, (unsigned)L.shmem_agg, st,
                                 agg_args, nullptr));
    HIP_OK(hipModuleLaunchKernel(L.jit->fn_ovf, (unsigned)(4 * L.agg_grid), 1, 1, 256, 1, 1, 0, st, agg_args, nullptr));
    return 0;
  }
  if (L.jit_sample) {
    unsigned long long* sampled = matched + 1;
    void* sargs[] = {(void*)&segs, (void*)&L.q, (void*)&table, (void*)&bits, (void*)&sampled, (void*)&L.part, (void*)&h};
    HIP_OK(hipModuleLaunchKernel(L.jit_sample->fn, (unsigned)L.sample_grid, 1, 1, kBlock, 1, 1, 0, st, sargs, nullptr));
  }
  HIP_OK(hipModuleLaunchKernel(L.jit->fn, count_grid, 1, 1, pt, 1, 1, (unsigned)L.shmem, st, args, nullptr));
  HIP_OK(launch_partition_offsets(L.part.hist, L.part.nparts, count_grid, L.part.offs, L.part.part_begin, st));
  if (L.jit_atomic)
    HIP_OK(hipModuleLaunchKernel(L.jit_atomic->fn, (unsigned)L.atomic_grid, 1, 1, kBlock, 1, 1, 0, st, args, nullptr));
  HIP_OK(hipModuleLaunchKernel(L.jit->fn_scatter, (unsigned)L.grid, 1, 1, pt, 1, 1, (unsigned)L.shmem_scatter, st, args,
                               nullptr));
  void* agg_args[] = {(void*)&L.part, (void*)&table};
  HIP_OK(hipModuleLaunchKernel(L.jit->fn_agg, (unsigned)L.agg_grid, 1, 1, 1024, 1, 1, (unsigned)L.shmem_agg, st,
                               agg_args, nullptr));
  return 0;
}

static int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = knob(name);
  return v ? atoll(v) : dflt;
}
static bool env_is(const char* name, const char* val) {
  const char* v = knob(name);
  return v && strcmp(v, val) == 0;
}

// Dense numGroupsLimit admission, every execution: the first-doc pass over each segment's prefix, the
// limit-th first docId per segment, the admission bitmaps. A segment whose prefix saw fewer than
// numGroupsLimit keys (though the segment may hold more) is redone over whole segments (one host check).
static int run_admission(pinot_amd_result* r, unsigned long long* limit_flag) {
  hipStream_t st = r->stream;
  const int32_t n = (int32_t)r->a_prefix.size();
  const int64_t nk = r->q.num_keys;
  HIP_OK(hipMemsetAsync(r->a_seen_n.p, 0, r->a_seen_n.n, st));
  auto first_pass = [&](bool full) -> int {
    for (auto& L : r->launches) {
      const DevSegment* sg = (const DevSegment*)(full ? L.d_segs.p : L.d_fd_segs.p);
      DevQuery fq = L.fd_q;
      if (full) fq.total_tiles = L.q.total_tiles;
      if (fq.total_tiles == 0) continue;
      uint64_t* table = nullptr;
      uint64_t* const* bits = nullptr;
      unsigned long long* matched = nullptr;
      DevHash h{};
      void* args[] = {(void*)&sg, (void*)&fq, (void*)&table, (void*)&bits, (void*)&matched, (void*)&L.part, (void*)&h};
      HIP_OK(hipModuleLaunchKernel(L.jit_fd->fn, (unsigned)(full ? L.fd_full_grid : L.fd_grid), 1, 1, kBlock, 1, 1, 0, st,
                                   args, nullptr));
    }
    return 0;
  };
  auto select = [&]() -> int {
    HIP_OK(hipMemsetAsync(r->a_hist.p, 0, r->a_hist.n, st));
    HIP_OK(launch_admit((uint32_t*)r->a_first.p, nk, (const uint32_t*)r->a_seen.p, (const unsigned long long*)r->a_seen_n.p,
                        r->a_cap, n, r->limit, (const int64_t*)r->a_bbase.p, r->a_max_buckets, (uint32_t*)r->a_hist.p,
                        (int64_t*)r->a_bstar.p, (int64_t*)r->a_rank.p, nullptr, nullptr, limit_flag, 0, nullptr, 0, st));
    return 0;
  };
  bool seq = !env_is("PINOT_AMD_ADMIT_SEQ", "0");
  for (auto& L : r->launches) seq &= L.jit_as != nullptr;
  if (seq) {
    // one block per segment walks its prefix in doc order (seen keys in an LDS bitmap) and writes the
    // segment's admission bitmap; a prefix that ended below the limit (outcome 2) is walked again whole
    auto seq_pass = [&](bool full) -> int {
      for (auto& L : r->launches) {
        if (L.segs.empty()) continue;
        const DevSegment* sg = (const DevSegment*)(full ? L.d_segs.p : L.d_fd_segs.p);
        DevQuery aq = L.fd_q;
        aq.total_tiles = full ? L.q.total_tiles : L.fd_q.total_tiles;
        aq.seen_cap = r->limit;
        aq.admit_flag = limit_flag;
        uint64_t* table = nullptr;
        uint64_t* const* bits = nullptr;
        unsigned long long* matched = nullptr;
        DevHash h{};
        void* args[] = {(void*)&sg, (void*)&aq, (void*)&table, (void*)&bits, (void*)&matched, (void*)&L.part, (void*)&h};
        HIP_OK(hipModuleLaunchKernel(L.jit_as->fn, (unsigned)L.segs.size(), 1, 1, kBlock, 1, 1,
                                     (unsigned)jit_admitseq_lds(nk), st, args, nullptr));
      }
      return 0;
    };
    if (int rc = seq_pass(false)) return rc;
    std::vector<unsigned long long> out((size_t)n);
    HIP_OK(hipMemcpyAsync(out.data(), r->a_seen_n.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    bool again = false;
    for (int32_t si = 0; si < n; ++si) again |= out[si] == 2;
    if (again) {
      HIP_OK(hipMemsetAsync(limit_flag, 0, 8, st));
      if (int rc = seq_pass(true)) return rc;
    }
    return 0;
  }
  if (int rc = first_pass(false)) return rc;
  if (int rc = select()) return rc;
  std::vector<unsigned long long> seen((size_t)n);
  HIP_OK(hipMemcpyAsync(seen.data(), r->a_seen_n.p, (size_t)n * 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  bool redo = false;
  for (int32_t si = 0; si < n; ++si) {
    if (seen[si] > (unsigned long long)r->a_cap) return fail(PINOT_AMD_EOVERFLOW, "admission: key list overflow");
    redo |= r->a_prefix[si] > 0 && r->a_prefix[si] < r->a_docs[si] && (int64_t)seen[si] < r->limit;
  }
  if (redo) {  // keys beyond the prefix matter: the whole segments (atomicMin keeps what the prefix found)
    HIP_OK(hipMemsetAsync(limit_flag, 0, 8, st));
    if (int rc = first_pass(true)) return rc;
    if (int rc = select()) return rc;
  }
  HIP_OK(hipMemsetAsync(r->a_bitmap.p, 0, r->a_bitmap.n, st));
  HIP_OK(hipMemsetAsync(r->a_bits.p, 0, r->a_bits.n, st));
  HIP_OK(launch_admit((uint32_t*)r->a_first.p, nk, (const uint32_t*)r->a_seen.p, (const unsigned long long*)r->a_seen_n.p,
                      r->a_cap, n, r->limit, (const int64_t*)r->a_bbase.p, r->a_max_buckets, (uint32_t*)r->a_hist.p,
                      (int64_t*)r->a_bstar.p, (int64_t*)r->a_rank.p, (unsigned long long*)r->a_bitmap.p,
                      (int64_t*)r->a_dstar.p, limit_flag, 1, (uint32_t*)r->a_bits.p, r->a_words, st));
  return 0;
}

// Hash-table capacities that held a query's groups, per (query shape, segment set) (pinot_amd_result::cap_key):
// a re-issued query starts at the grown capacity instead of growing from PINOT_AMD_HASH_INIT_SLOTS again.
static std::mutex g_cap_mu;
static std::unordered_map<std::string, int64_t> g_cap_cache;

static void remember_hash_capacity(pinot_amd_result* r) {
  r->cap_known = true;
  if (r->cap_key.empty()) return;
  std::lock_guard<std::mutex> g(g_cap_mu);
  if (g_cap_cache.size() >= 4096) g_cap_cache.clear();
  int64_t& c = g_cap_cache[r->cap_key];
  c = std::max(c, r->fcap);
}
static int64_t known_hash_capacity(const std::string& key) {
  std::lock_guard<std::mutex> g(g_cap_mu);
  auto it = g_cap_cache.find(key);
  return it == g_cap_cache.end() ? 0 : it->second;
}

// Spill-region capacities (records per scan block) an execution of a query shape over a segment set needed
// (pinot_amd_result::cap_key): a region that overflowed sends its further records to the HBM table one doc at a
// time (correct, slow: the wide-key bench at 100 segments ran 28.2 ms instead of 22.1 with room for them), so
// a re-issued query allocates the regions the last execution needed.
static std::unordered_map<std::string, int64_t> g_spill_cache;  // guarded by g_cap_mu

static void remember_spill_capacity(const std::string& key, int64_t recs) {
  if (key.empty()) return;
  std::lock_guard<std::mutex> g(g_cap_mu);
  if (g_spill_cache.size() >= 4096) g_spill_cache.clear();
  int64_t& c = g_spill_cache[key];
  c = std::max(c, recs);
}
static int64_t known_spill_capacity(const std::string& key) {
  std::lock_guard<std::mutex> g(g_cap_mu);
  auto it = g_spill_cache.find(key);
  return it == g_spill_cache.end() ? 0 : it->second;
}

// grow an untrimmed hash plan's table 4x, at most to its ceiling (*grown false: already there)
static int grow_hash(pinot_amd_result* r, bool* grown) {
  *grown = false;
  if (r->fcap >= r->fcap_ceiling) return 0;
  const int64_t ncap = std::min(r->fcap * 4, r->fcap_ceiling);
  r->fkeys.reset();
  r->acc.reset();
  if (int rc = r->fkeys.alloc((size_t)r->nw * (size_t)ncap * 8)) return rc;
  if (int rc = r->acc.alloc((size_t)r->q.nacc * (size_t)ncap * 8)) return rc;
  r->fcap = ncap;
  r->compacted = false;
  r->cap_known = false;
  *grown = true;
  return 0;
}

static int run_plan(pinot_amd_result* r) {
  r->merged = false;
  r->check_failed = false;
  r->direct_ran = false;
  r->ovf_pending = false;
  hipStream_t st = r->stream;
  r->compacted = false;
  if (r->spill_words > 0 && !r->cap_key.empty()) {
    // an execution of this shape overflowed its spill regions since they were sized: larger regions (the old
    // ones are freed first: hipFree waits for the work still reading them)
    const int64_t want = std::min(known_spill_capacity(r->cap_key), r->spill_cap_max);
    if (want > r->spill_cap) {
      const size_t bytes = (size_t)r->spill_grid * kSpillGroups * (size_t)want * (size_t)r->spill_words * 8;
      r->sp_rec.reset();
      r->sp_sorted.reset();
      if (int rc = r->sp_rec.alloc(bytes)) return rc;
      if (int rc = r->sp_sorted.alloc(bytes)) return rc;
      r->spill_cap = want;
    }
  }
  HIP_OK(hipEventRecord(r->ev0, st));
  // inverted-index leaves: expand roaring containers into dense doc bitsets
  bool all_fused = !r->launches.empty();
  for (auto& L : r->launches) all_fused &= L.fused;
  if (!r->inv_leaves.empty() && !all_fused)
    HIP_OK(launch_expand_jobs(r->d_expand_jobs.p, (int32_t)r->inv_leaves.size(), r->expand_total, st));
  HIP_OK(hipMemsetAsync(r->matched.p, 0, r->matched.n, st));
  const size_t nl = r->launches.size();
  unsigned long long* ctr = (unsigned long long*)r->matched.p;
  unsigned long long* limit_flag = ctr + 3 * nl;
  unsigned long long* overflow = ctr + 3 * nl + 1;
  if (r->kind == PLAN_HASH) {
   for (;;) {  // untrimmed hash plans: the table grows and the plan runs again while docs found no slot
    HIP_OK(hipMemsetAsync(r->fkeys.p, 0xFF, (size_t)r->nw * (size_t)r->fcap * 8, st));  // EMPTY key words
    HIP_OK(launch_init_acc((uint64_t*)r->acc.p, r->q, r->fcap, st));
    for (int b = 0; b < r->nbatches; ++b) {
      DevHash H{};
      uint64_t* table;
      if (r->trim) {
        const int64_t cap = r->batch_cap[b];
        HIP_OK(hipMemsetAsync(r->skeys.p, 0xFF, (size_t)(r->nw + 1) * (size_t)cap * 8, st));
        HIP_OK(launch_init_acc((uint64_t*)r->sacc.p, r->q, cap, st));
        H.keys = (unsigned long long*)r->skeys.p;
        H.cap = cap;
        table = (uint64_t*)r->sacc.p;
      } else {
        H.keys = (unsigned long long*)r->fkeys.p;
        H.cap = r->fcap;
        // a probe chain this long means a crowded table: the doc counts as overflow and the table grows
        // (below) instead of degrading into long serial CAS walks
        H.max_probe = env_i64("PINOT_AMD_HASH_MAX_PROBE", 512);
        table = (uint64_t*)r->acc.p;
        if (r->spill_words > 0) {
          // spill partitions: about 4096 table slots' worth of keys each (~1-2K groups), within the scan's
          // LDS histogram; the second level's LDS table then holds a partition's keys
          int lg = 6;
          while (lg < 11 && ((int64_t)1 << lg) * 4096 < r->fcap) ++lg;
          H.spill = (unsigned long long*)r->sp_rec.p;
          H.spill_cap = r->spill_cap;
          H.spill_cnt = (uint32_t*)r->sp_cnt.p;
          H.spill_hist = (uint32_t*)r->sp_hist.p;
          H.spill_shift = 64 - lg;
          H.spill_words = r->spill_words;
        }
      }
      H.overflow = overflow;
      for (size_t li = 0; li < nl; ++li)
        if (r->launches[li].batch == b) {
          Launch& L = r->launches[li];
          DevHash HL = H;
          const bool dmode = !r->trim && r->spill_words > 0 && r->hash_mode > 0 && L.jit_direct && r->direct_place;
          const int lg = 64 - H.spill_shift;
          if (dmode && r->hash_mode == 2 && L.direct_lg == lg) {  // records straight to their places
            HL.direct = 1;
            HL.dst = (unsigned long long*)r->sp_sorted.p;
            HL.dbase = (const int64_t*)L.d_dbase.p;
            HL.dcnt = (const uint32_t*)L.d_dcnt.p;
            HL.check = ctr + 3 * nl + 2;
            r->direct_ran = true;
          }
          if (int rc = launch_one(r, L, li, table, HL)) return rc;
          if (HL.direct) {
            HIP_OK(launch_spill_agg(HL, r->nw, (const unsigned long long*)r->sp_sorted.p, (const int64_t*)L.d_dpbeg.p, r->q,
                                    (uint64_t*)r->acc.p, r->spill_agg_grid, r->spill_slots, r->spill_narrow, st));
          } else if (!r->trim && r->spill_words > 0) {
            HIP_OK(launch_spill_passes(HL, r->nw, L.grid, nullptr, (int64_t*)r->sp_offs.p, (int64_t*)r->sp_pbeg.p,
                                       (unsigned long long*)r->sp_sorted.p, r->q, (uint64_t*)r->acc.p, r->spill_agg_grid,
                                       r->spill_slots, env_is("PINOT_AMD_SPILL_SORT", "0") ? 0 : 1, r->spill_narrow, st));
            if (dmode) {  // this region-mode execution without the LDS level counted the direct placement's allotments
              const size_t cells = ((size_t)1 << lg) * (size_t)L.grid;
              if (L.d_dbase.n < cells * 8) {
                L.d_dbase.reset();
                L.d_dcnt.reset();
                if (int rc = L.d_dbase.alloc(cells * 8)) return rc;
                if (int rc = L.d_dcnt.alloc(cells * 4)) return rc;
              }
              if (L.d_dpbeg.n < (((size_t)1 << lg) + 1) * 8) {
                L.d_dpbeg.reset();
                if (int rc = L.d_dpbeg.alloc((((size_t)1 << lg) + 1) * 8)) return rc;
              }
              HIP_OK(launch_spill_direct_prep((const int64_t*)r->sp_offs.p, (const int64_t*)r->sp_pbeg.p,
                                              (const uint32_t*)r->sp_hist.p, 1 << lg, L.grid, (int64_t*)L.d_dbase.p,
                                              (uint32_t*)L.d_dcnt.p, (int64_t*)L.d_dpbeg.p, st));
              L.direct_lg = lg;
            }
          }
        }
      if (r->trim) {
        const int32_t nb = r->batch_nsegs[b];
        HIP_OK(hipMemsetAsync(r->t_hist.p, 0, (size_t)r->batch_buckets[b] * 4, st));
        HIP_OK(hipMemsetAsync(r->t_distinct.p, 0, (size_t)nb * 8, st));
        HIP_OK(hipMemsetAsync(r->t_bitmap.p, 0, (size_t)nb * 16 * 8, st));
        const int64_t* bb = (const int64_t*)r->d_bucket_base.p + r->batch_bucket_off[b];
        HIP_OK(launch_trim(H.keys, H.cap, r->nw + 1, table, r->fd_acc, nb, r->limit, bb, (uint32_t*)r->t_hist.p,
                           (unsigned long long*)r->t_distinct.p, (int64_t*)r->t_bstar.p, (int64_t*)r->t_rank.p,
                           (unsigned long long*)r->t_bitmap.p, (int64_t*)r->t_dstar.p, limit_flag, st));
        const SegSelStage* sst = nullptr;
        const int nst = (int)r->segsel_st.size();
        if (r->segsel) {  // each segment's top segsel_keep entries among the numGroupsLimit survivors
          sst = (const SegSelStage*)r->d_segsel_st.p;
          HIP_OK(launch_segsel(H.keys, H.cap, r->nw, table, r->fd_acc, (const int64_t*)r->t_dstar.p, r->q, sst, nst, nb,
                               r->segsel_keep, (unsigned long long*)r->ss_cnt.p, (int64_t*)r->ss_want.p,
                               (int32_t*)r->ss_done.p, (uint64_t*)r->ss_prefix.p, (uint64_t*)r->ss_cut.p,
                               (uint32_t*)r->ss_hist.p, st));
        }
        HIP_OK(launch_hash_merge(H.keys, H.cap, r->nw, 1, table, (unsigned long long*)r->fkeys.p, r->fcap,
                                 (uint64_t*)r->acc.p, r->q, r->fd_acc, (const int64_t*)r->t_dstar.p, overflow, st, sst, nst,
                                 (const int32_t*)r->ss_done.p, (const uint64_t*)r->ss_cut.p));
      }
    }
    if (r->trim) break;
    // The table's capacity comes from a group-count bound (docs per segment, key space); real group counts
    // are usually far lower, so the plan starts small (PINOT_AMD_HASH_INIT_SLOTS) and, like the map-based
    // holders that resize as groups arrive, grows 4x when some doc found no slot (then runs again). A
    // capacity an earlier execution of this query settled on needs no check here: no host synchronisation
    // in the execution (check_overflow reads the counter with the groups and grows then if it must).
    if (r->cap_known) {
      r->ovf_pending = true;
      break;
    }
    unsigned long long ovf = 0;
    HIP_OK(hipMemcpyAsync(&ovf, overflow, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (ovf == 0) {
      remember_hash_capacity(r);
      break;
    }
    bool grown = false;
    if (int rc = grow_hash(r, &grown)) return rc;
    if (!grown) break;  // at the ceiling: the overflow counter stays set, the result reports EOVERFLOW
    HIP_OK(hipMemsetAsync(r->matched.p, 0, r->matched.n, st));
   }
    if (r->hash_mode == 1 && r->direct_place) r->hash_mode = 2;  // allotments counted: the next execution places directly
  } else {
    if (r->admit)
      if (int rc = run_admission(r, limit_flag)) return rc;
    if (r->seg_trim) {
      // segment-level safe trim: each segment's groups marked by ORDER BY rank, then its LIMIT-th rank
      HIP_OK(hipMemsetAsync(r->sp_bits.p, 0, r->sp_bits.n, st));
      for (auto& L : r->launches) {
        if (L.q.total_tiles == 0) continue;
        const DevSegment* sg = (const DevSegment*)L.d_segs.p;
        uint64_t* table = nullptr;
        uint64_t* const* bits = nullptr;
        unsigned long long* matched = nullptr;
        DevHash h{};
        void* args[] = {(void*)&sg, (void*)&L.q, (void*)&table, (void*)&bits, (void*)&matched, (void*)&L.part, (void*)&h};
        HIP_OK(hipModuleLaunchKernel(L.jit_sp->fn, (unsigned)L.sp_grid, 1, 1, kBlock, 1, 1, 0, st, args, nullptr));
      }
      HIP_OK(launch_seg_cut((const unsigned long long*)r->sp_bits.p, r->sp_words, r->sp_nsegs, r->srv_limit,
                            (unsigned long long*)r->sp_cut.p, st));
    }
    if (r->q.nacc > 0) HIP_OK(launch_init_acc((uint64_t*)r->acc.p, r->q, r->q.num_keys, st));
    DevHash H{};
    for (size_t li = 0; li < nl; ++li)
      if (int rc = launch_one(r, r->launches[li], li, (uint64_t*)r->acc.p, H)) return rc;
  }
  if (r->n_sext > 0)
    HIP_OK(launch_sext_hi((uint64_t*)r->acc.p, r->kind == PLAN_HASH ? r->fcap : r->q.num_keys, (const int32_t*)r->d_sext.p,
                          r->n_sext, st));
  HIP_OK(hipEventRecord(r->ev1, st));
  return 0;
}

// Hash-plan key words: the group columns' merged ids packed low to high. EMPTY (~0) must stay impossible
// for every word: a word takes a field while it stays within 63 bits, or fills all 64 bits when one of its
// fields can never be all ones (a key space smaller than 2^bits: its largest id leaves a zero bit) -- the
// wide-key bench's 5 ids (15 + 15 + 15 + 10 + 9 bits) then fit one word instead of two.
static int bits_for(int64_t card);
static void pack_key_words(const std::vector<int64_t>& sizes, std::vector<int>* word, std::vector<int>* shift) {
  int w = 0, sh = 0;
  bool safe = false;  // the current word has a field that is never all ones
  word->clear();
  shift->clear();
  for (int64_t size : sizes) {
    const int b = bits_for(size);
    const bool never_ones = size < ((int64_t)1 << b);
    if (sh + b > 64 || (sh + b == 64 && !(safe || never_ones))) {
      ++w;
      sh = 0;
      safe = false;
    }
    word->push_back(w);
    shift->push_back(sh);
    sh += b;
    safe |= never_ones;
  }
}

static int64_t next_pow2(int64_t x) {
  int64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}
static int bits_for(int64_t card) {  // PinotDataBitSet.getNumBitsPerValue(card - 1), at least 1
  int b = 1;
  while (b < 62 && ((int64_t)1 << b) < card) ++b;
  return b;
}

extern "C" {

// wall-clock milliseconds of the planning phases of one execute (diagnostics: where a cold / cached
// query's host time goes)
// hipModuleOccupancyMaxActiveBlocksPerMultiprocessor per (kernel, block size, dynamic LDS), memoised: the planner
// asks for every launch of every execution, and a kernel's occupancy never changes
static hipError_t occupancy_blocks(int* out, hipFunction_t fn, int threads, size_t shmem) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t>, int> memo;
  const auto key = std::make_tuple((const void*)fn, threads, shmem);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = memo.find(key);
    if (it != memo.end()) {
      *out = it->second;
      return hipSuccess;
    }
  }
  const hipError_t e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(out, fn, threads, shmem);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> g(mu);
    memo[key] = *out;
  }
  return e;
}

struct PlanClock {
  std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
  std::string* out;
  explicit PlanClock(std::string* o) : out(o) { out->clear(); }
  double lap() {
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - last).count();
    last = now;
    return ms;
  }
  void mark(const char* phase) {
    char b[64];
    snprintf(b, sizeof(b), "%s%s=%.3f", out->empty() ? "" : ";", phase, lap());
    *out += b;
  }
};

static int execute_impl(pinot_amd_query* qq, pinot_amd_segment* const* segs_in, int32_t n, void* stream,
                        bool filter_only, pinot_amd_result** out) {
  if (!qq || !segs_in || n < 1 || !out) return fail(PINOT_AMD_EINVAL, "execute: bad arguments");
  std::vector<pinot_amd_segment*> segs(segs_in, segs_in + n);
  for (auto* s : segs)
    if (!s) return fail(PINOT_AMD_EINVAL, "execute: null segment");
  const std::string plan_key = plan_identity(*qq, segs, filter_only);
  if (pinot_amd_result* hit = plan_cache_take(plan_key)) {  // a prepared plan of this identity: run it
    std::unique_ptr<pinot_amd_result> hold(hit);
    hit->stream = (hipStream_t)stream;
    PlanClock clk(&hit->plan_timing);
    clk.mark("plan_cache");
    if (int rc = run_plan(hit)) return rc;
    clk.mark("launch");
    *out = hold.release();
    return 0;
  }
  const size_t alloc0 = g_tl_alloc_bytes;
  auto res = std::make_unique<pinot_amd_result>();
  pinot_amd_result* r = res.get();
  r->stream = (hipStream_t)stream;
  r->plan_key = plan_key;
  for (auto* sg : segs) r->plan_uids.push_back(sg->uid);
  PlanClock clk(&r->plan_timing);
  pinot_amd_query filter_q;
  if (filter_only) filter_q.preds = qq->preds;  // FilterPlanNode only: no projection, no aggregation
  const pinot_amd_query* Qp = filter_only ? &filter_q : qq;
  pinot_amd_query raw_gb_q;  // group-by columns redirected to the derived dictionary of raw columns
  for (size_t j = 0; j < Qp->group_by.size(); ++j) {
    const std::string g = Qp->group_by[j];  // a copy: the redirect below rewrites Qp->group_by[j]
    int nraw = 0;
    for (auto* s : segs) {
      auto it = s->cols.find(g);
      if (it == s->cols.end()) return fail(PINOT_AMD_EINVAL, "segment %s has no column %s", s->name.c_str(), g.c_str());
      nraw += it->second->enc == ENC_RAW;
    }
    if (nraw == 0) continue;
    if (nraw != n) return fail(PINOT_AMD_EUNSUPPORTED, "GROUP BY column %s is raw in some segments only", g.c_str());
    if (Qp != &raw_gb_q) { raw_gb_q = *Qp; Qp = &raw_gb_q; }
    for (auto* s : segs)
      if (int rc = derive_raw_group_dictionary(s, g, &raw_gb_q.group_by[j])) return rc;
  }
  const pinot_amd_query& Q = *Qp;

  clk.mark("raw_keys");
  // ---- slots: columns the kernel must decode ----
  std::vector<std::string> slot_cols;
  auto slot_of = [&](const std::string& name) -> int {
    for (size_t i = 0; i < slot_cols.size(); ++i)
      if (slot_cols[i] == name) return (int)i;
    slot_cols.push_back(name);
    return (int)slot_cols.size() - 1;
  };
  for (auto* s : segs) {
    auto need = [&](const std::string& col) -> int {
      if (!s->cols.count(col)) return fail(PINOT_AMD_EINVAL, "segment %s has no column %s", s->name.c_str(), col.c_str());
      return 0;
    };
    for (auto& p : Q.preds) if (int rc = need(p.column)) return rc;
    for (auto& g : Q.group_by) if (int rc = need(g)) return rc;
    for (auto& a : Q.aggs) {
      if (!a.column.empty()) if (int rc = need(a.column)) return rc;
      if (!a.column2.empty()) if (int rc = need(a.column2)) return rc;
    }
  }
  for (auto& g : Q.group_by) slot_of(g);
  for (auto& a : Q.aggs) {
    if (a.column.empty()) continue;
    for (const std::string* col : {&a.column, &a.column2}) {
      if (col->empty()) continue;
      for (auto* s : segs)
        if (s->cols.at(*col)->type != segs[0]->cols.at(*col)->type)
          return fail(PINOT_AMD_EINVAL, "column %s has different types across segments", col->c_str());
      if (segs[0]->cols.at(*col)->type == T_STRING) return fail(PINOT_AMD_EINVAL, "cannot aggregate STRING column %s", col->c_str());
      slot_of(*col);
    }
  }

  // ---- per-segment leaves (PredicateEvaluatorProvider per segment) ----
  const size_t np = Q.preds.size();
  std::vector<std::vector<DevLeaf>> seg_leaves(n, std::vector<DevLeaf>(np));
  std::vector<std::vector<int>> leaf_slot_col(n, std::vector<int>(np, -1));
  int nclauses = 0;
  for (size_t pi = 0; pi < np; ++pi) nclauses = std::max(nclauses, Q.preds[pi].clause + 1);
  // per predicate, once: whether its column is decoded anyway, and its leaf-cache key (the same on every segment)
  std::vector<char> pred_decoded(np, 0);
  std::vector<std::string> pred_key(np);
  for (size_t pi = 0; pi < np; ++pi) {
    const PredSpec& p = Q.preds[pi];
    bool d = std::find(Q.group_by.begin(), Q.group_by.end(), p.column) != Q.group_by.end();
    for (auto& a : Q.aggs) d |= a.column == p.column || a.column2 == p.column;
    pred_decoded[pi] = d ? 1 : 0;
    pred_key[pi] = leaf_cache_key(p, -1, d);
  }
  const bool leaf_cache = !env_is("PINOT_AMD_LEAF_CACHE", "0");
  for (int si = 0; si < n; ++si) {
    for (size_t pi = 0; pi < np; ++pi) {
      const PredSpec& p = Q.preds[pi];
      const Column& c = *segs[si]->cols.at(p.column);
      bool needs_slot = false;
      const bool decoded_anyway = pred_decoded[pi] != 0;
      int rc = make_leaf_for_segment(r, si, segs[si], p, c, -1, &seg_leaves[si][pi], &needs_slot, r->stream,
                                     decoded_anyway, leaf_cache ? &pred_key[pi] : nullptr);
      if (rc) return rc;
      if (needs_slot) leaf_slot_col[si][pi] = slot_of(p.column);
    }
  }
  if ((int)slot_cols.size() > kMaxSlots)
    return fail(PINOT_AMD_EUNSUPPORTED, "query reads %zu columns (max %d)", slot_cols.size(), kMaxSlots);
  const int nslots = (int)slot_cols.size();
  for (int sl = 0; sl < nslots; ++sl)
    for (auto* s : segs)
      if (s->cols.at(slot_cols[sl])->type != segs[0]->cols.at(slot_cols[sl])->type)
        return fail(PINOT_AMD_EINVAL, "column %s has different types across segments", slot_cols[sl].c_str());
  // leaf order is the same for all segments: leaves grouped by the slot they read where some segment
  // reads one, slot-less predicates last (segments where such a leaf resolved slot-less keep its
  // CONST/DOC kind, which ignores the values)
  std::vector<int> pred_slot(np, -1);
  for (size_t pi = 0; pi < np; ++pi)
    for (int si = 0; si < n; ++si)
      if (leaf_slot_col[si][pi] >= 0) pred_slot[pi] = leaf_slot_col[si][pi];
  std::vector<size_t> order;
  for (int sl = 0; sl < nslots; ++sl)
    for (size_t pi = 0; pi < np; ++pi)
      if (pred_slot[pi] == sl) order.push_back(pi);
  for (size_t pi = 0; pi < np; ++pi)
    if (pred_slot[pi] < 0) order.push_back(pi);

  DevQuery& q = r->q;
  memset(&q, 0, sizeof(q));

  clk.mark("leaves");
  // ---- group-by key space: merged dictionaries (union over the batch, dictionary order) ----
  r->num_group_by = (int32_t)Q.group_by.size();
  r->limit = Q.num_groups_limit;
  r->srv_limit = Q.limit;
  r->srv_order = Q.order_by;
  r->srv_min_trim = Q.min_trim;
  r->srv_trim_threshold = Q.trim_threshold;
  r->srv_final = Q.server_final;
  r->srv_sort_threshold = Q.sort_agg_threshold;
  {  // QueryContext.isSameOrderAndGroupByColumns: the ORDER BY expressions, as a set, are the GROUP BY ones
    std::vector<bool> seen(Q.group_by.size(), false);
    bool only_keys = !Q.order_by.empty();
    for (const auto& ob : Q.order_by) {
      if (ob.kind != 0) only_keys = false;
      else seen[ob.index] = true;
    }
    r->srv_safe = only_keys && std::all_of(seen.begin(), seen.end(), [](bool b) { return b; });
  }
  double dense_keys = 1;
  for (size_t j = 0; j < Q.group_by.size(); ++j) {
    const std::string& g = Q.group_by[j];
    std::shared_ptr<const MergedKeyColumn> m;
    if (int rc = build_merged_keys(segs, g, &m)) return rc;
    auto ks = qq->key_space.find(qq->group_by[j]);  // installed key space (original column name)
    if (ks != qq->key_space.end()) {
      // it must hold every value of the batch's dictionaries: the batch's merged keys are a subset (checked
      // once per (batch key space, installed key space) pair: both are immutable)
      const MergedKeyColumn& K = *ks->second;
      if (K.type != m->type) return fail(PINOT_AMD_EINVAL, "key space of %s has the wrong type", g.c_str());
      static std::mutex sub_mu;
      static std::set<std::pair<uint64_t, uint64_t>> subsets;
      bool known;
      {
        std::lock_guard<std::mutex> lk(sub_mu);
        known = subsets.count({m->id, K.id}) != 0;
      }
      if (!known) {
        bool ok = true;
        if (m->type == T_STRING) {
          for (auto& v : m->vs) ok &= std::binary_search(K.vs.begin(), K.vs.end(), v, java_less);
        } else if (is_float(m->type)) {
          for (double v : m->vd) ok &= std::binary_search(K.vd.begin(), K.vd.end(), v, java_double_less);
        } else {
          for (int64_t v : m->vi) ok &= std::binary_search(K.vi.begin(), K.vi.end(), v);
        }
        if (!ok) return fail(PINOT_AMD_EINVAL, "key space of %s misses values of the segments' dictionaries", g.c_str());
        std::lock_guard<std::mutex> lk(sub_mu);
        if (subsets.size() >= 65536) subsets.clear();
        subsets.insert({m->id, K.id});
      }
      m = ks->second;
    }
    r->key_stride.push_back((int64_t)std::min(dense_keys, 9.0e18));
    dense_keys *= (double)std::max<size_t>(m->size(), 1);
    r->keys.push_back(std::move(m));
  }
  // Matching docs per segment, counted once at plan time by a filter-only pass when a planning decision
  // needs them (numGroupsLimit trimming, the selection-vector plan); segments are immutable, so the
  // counts hold for every re-execution of the plan.
  std::vector<int64_t> seg_matched;
  auto probe_matched = [&]() -> int {
    if (!seg_matched.empty()) return 0;
    // counts cached on the segments (immutable) by an earlier probe of the same filter; the rest probed
    const std::string sig = preds_signature(Q.preds);
    seg_matched.assign(n, -1);
    std::vector<pinot_amd_segment*> todo;
    std::vector<int> todo_idx;
    std::unique_lock<std::mutex> lk(g_match_mu);
    for (int si = 0; si < n; ++si) {
      auto it = segs[si]->match_cache.find(sig);
      if (it != segs[si]->match_cache.end()) {
        seg_matched[si] = it->second;
      } else {
        todo.push_back(segs[si]);
        todo_idx.push_back(si);
      }
    }
    lk.unlock();
    if (todo.empty()) return 0;
    pinot_amd_query fq;
    fq.preds = Q.preds;
    pinot_amd_result* fr = nullptr;
    if (int rc = execute_impl(&fq, todo.data(), (int32_t)todo.size(), stream, true, &fr)) return rc;
    std::unique_ptr<pinot_amd_result> hold(fr);
    for (size_t k = 0; k < todo.size(); ++k) {
      int64_t c = 0;
      if (int rc = pinot_amd_bitset_count((const uint64_t*)fr->bitsets[k]->p, todo[k]->num_docs, &c, stream)) return rc;
      seg_matched[todo_idx[k]] = c;
      std::lock_guard<std::mutex> g(g_match_mu);
      todo[k]->match_cache[sig] = c;
    }
    return 0;
  };
  // numGroupsLimit: a segment can only reach the limit if it can hold that many keys (matching docs
  // and its own dictionaries' key space bound it); otherwise no trimming can happen
  std::vector<int64_t> seg_bound(n, 0);
  bool limit_possible = false;
  if (!Q.group_by.empty() && !filter_only) {
    for (int si = 0; si < n; ++si) {
      double b = (double)segs[si]->num_docs;
      double ks = 1;
      for (auto& g : Q.group_by) ks *= (double)std::max(segs[si]->cols.at(g)->card, 1);
      b = std::min(b, ks);
      seg_bound[si] = (int64_t)b;
      limit_possible |= seg_bound[si] >= Q.num_groups_limit;
    }
    // The key space alone allows numGroupsLimit groups somewhere: bound each segment by its matching
    // docs too (a segment's groups <= its matching docs). Counted once at plan time by a filter-only
    // pass; segments are immutable, so the counts hold for every re-execution of the plan.
    if (limit_possible && !Q.preds.empty() && !env_is("PINOT_AMD_TRIM_PROBE", "0")) {
      if (int rc = probe_matched()) return rc;
      limit_possible = false;
      for (int si = 0; si < n; ++si) {
        seg_bound[si] = std::min(seg_bound[si], seg_matched[si]);
        limit_possible |= seg_bound[si] >= Q.num_groups_limit;
      }
    }
  }
  r->limit_possible = limit_possible;
  // Safe trim with LIMIT >= sortAggregateLimitThreshold and no serverReturnFinalResult: every segment keeps its
  // top LIMIT groups by the ORDER BY (GroupByOperator.java:146-182, QueryContext.java:568-580) and the combine
  // table keeps the top trimSize of their union, so groups past the global top LIMIT carry partial results.
  // Restated on dense key spaces (seg_trim): each segment's groups are marked in a presence bitmap over their
  // ORDER BY ranks, the rank of its LIMIT-th group is the segment's cutoff, and the aggregation keeps only the
  // docs whose group ranks within it. A segment that cannot hold more than LIMIT groups trims nothing. (Below
  // the threshold, and with serverReturnFinalResult, the segments trim too, but the LIMIT groups the server
  // keeps are exact either way: server_trim.)
  bool seg_trim = false;
  if (r->srv_safe && r->srv_limit >= 0 && r->srv_limit >= r->srv_sort_threshold && !r->srv_final && !filter_only &&
      !Q.group_by.empty()) {
    auto over = [&]() {
      for (int si = 0; si < n; ++si)
        if (seg_bound[si] > r->srv_limit) return true;
      return false;
    };
    if (over() && !Q.preds.empty() && seg_matched.empty()) {
      if (int rc = probe_matched()) return rc;
      for (int si = 0; si < n; ++si) seg_bound[si] = std::min(seg_bound[si], seg_matched[si]);
    }
    seg_trim = over() && !env_is("PINOT_AMD_SEG_TRIM", "0");
    if (over() && !seg_trim)
      return fail(PINOT_AMD_EUNSUPPORTED, "server result limit: a segment-level safe trim (ORDER BY = GROUP BY, "
                                          "LIMIT %lld >= sortAggregateLimitThreshold %lld) disabled by PINOT_AMD_SEG_TRIM=0",
                  (long long)r->srv_limit, (long long)r->srv_sort_threshold);
  }
  // Unsafe trim (ORDER BY other than the GROUP BY keys) with minSegmentGroupTrimSize > 0: each segment keeps its top
  // max(minSegmentGroupTrimSize, 5 x LIMIT) groups by the ORDER BY, aggregation values included (QueryContext.java:
  // 575-578, GroupByUtils.getTableCapacity, GroupByOperator.java:157-175): the (key, segment) hash plan with the
  // per-segment selection (segsel) when some segment could hold more.
  bool segsel_unsafe = false;
  int64_t segsel_unsafe_keep = 0;
  if (!r->srv_safe && !r->srv_order.empty() && Q.min_seg_trim > 0 && r->srv_limit >= 0 && !filter_only &&
      !Q.group_by.empty()) {
    const int64_t seg_keep = std::max<int64_t>(Q.min_seg_trim, 5 * r->srv_limit);
    bool over = false;
    for (int si = 0; si < n; ++si) over |= seg_bound[si] > seg_keep;
    if (over && !Q.preds.empty() && seg_matched.empty()) {
      if (int rc = probe_matched()) return rc;
      over = false;
      for (int si = 0; si < n; ++si) over |= std::min(seg_bound[si], seg_matched[si]) > seg_keep;
    }
    segsel_unsafe = over;
    segsel_unsafe_keep = seg_keep;
  }
  // admission prefixes (dense trimming): the docs of segment si that should hold numGroupsLimit distinct
  // keys, twice the coupon-collector expectation for K uniform keys (K ln(K / (K - L)) matching docs,
  // scaled by the segment's selectivity) plus 64 Ki docs; a segment that cannot reach the limit needs
  // no pass (everything admitted). A prefix that still sees fewer keys is redone over the whole segment.
  auto admit_prefixes = [&]() {
    r->a_prefix.assign(n, 0);
    r->a_docs.assign(n, 0);
    for (int si = 0; si < n; ++si) {
      const int64_t nd = segs[si]->num_docs;
      r->a_docs[si] = nd;
      if (seg_bound[si] < Q.num_groups_limit) continue;
      double ks = 1;
      for (auto& g : Q.group_by) ks *= (double)std::max(segs[si]->cols.at(g)->card, 1);
      const double L = (double)Q.num_groups_limit;
      const double need = ks > L ? ks * std::log(ks / (ks - L)) : (double)nd;
      const double sel = (!seg_matched.empty() && nd > 0) ? std::max((double)seg_matched[si] / (double)nd, 1e-9) : 1.0;
      const double rows = 2.0 * need / sel + 65536.0;
      int64_t pfx = rows >= (double)nd ? nd : ((int64_t)rows + kTileDocs - 1) / kTileDocs * kTileDocs;
      if (const char* e = knob("PINOT_AMD_ADMIT_PREFIX")) pfx = std::min<int64_t>(nd, std::max<int64_t>(kTileDocs, atoll(e)));
      r->a_prefix[si] = std::min(pfx, nd);
    }
  };

  clk.mark("keys_probe");
  // ---- accumulators: acc 0 = COUNT; others grouped by slot; ACC_FIRST_DOC last ----
  // nan_skip: MinMaxRangePair.apply compares with < / >, so NaN never enters the pair (MIN / MAX of
  // an aggregation-only query propagate it like Math.min / Math.max)
  struct AccReq { int slot; int op; int expr; int slot2; int nan_skip; };
  std::vector<AccReq> reqs;
  std::vector<int> agg_req(Q.aggs.size(), -1), agg_req2(Q.aggs.size(), -1);
  auto find_req = [&](const AccReq& rq) -> int {
    for (size_t k = 0; k < reqs.size(); ++k)
      if (reqs[k].slot == rq.slot && reqs[k].op == rq.op && reqs[k].expr == rq.expr && reqs[k].slot2 == rq.slot2 &&
          reqs[k].nan_skip == rq.nan_skip)
        return (int)k;
    reqs.push_back(rq);
    return (int)reqs.size() - 1;
  };
  for (size_t ai = 0; ai < Q.aggs.size(); ++ai) {
    const AggSpec& a = Q.aggs[ai];
    if (a.type == PINOT_AMD_AGG_COUNT) continue;
    const Column& c = *segs[0]->cols.at(a.column);
    // SUM / AVG of integer values are summed exactly in 128 bits (SumAggregationFunction accumulates
    // in double: equal whenever partial sums stay below 2^53, and the correctly rounded exact sum
    // beyond); an expression is integer when both operands are INT (the product fits 64 bits)
    const bool expr_int = a.expr != PINOT_AMD_EXPR_COLUMN && c.type == T_INT &&
                          segs[0]->cols.at(a.column2)->type == T_INT;
    int op;
    switch (a.type) {
      case PINOT_AMD_AGG_SUM:
      case PINOT_AMD_AGG_AVG:
        if (a.expr != PINOT_AMD_EXPR_COLUMN) op = expr_int ? ACC_SUM_I128 : ACC_SUM_F64;
        else op = is_float(c.type) ? ACC_SUM_F64 : ACC_SUM_I128;
        break;
      case PINOT_AMD_AGG_SUMLONG:  // Java long arithmetic: wraps
        if (is_float(c.type)) return fail(PINOT_AMD_EINVAL, "SUMLONG on floating column %s", a.column.c_str());
        op = ACC_SUM_I64;
        break;
      case PINOT_AMD_AGG_MIN: op = ACC_MIN; break;
      case PINOT_AMD_AGG_MINMAXRANGE: op = ACC_MIN; break;  // + ACC_MAX below
      default: op = ACC_MAX; break;
    }
    const int sl = slot_of(a.column);
    const int sl2 = a.expr != PINOT_AMD_EXPR_COLUMN ? slot_of(a.column2) : -1;
    if (a.type == PINOT_AMD_AGG_MINMAXRANGE) {
      agg_req[ai] = find_req({sl, ACC_MIN, a.expr, sl2, 1});
      agg_req2[ai] = find_req({sl, ACC_MAX, a.expr, sl2, 1});
    } else {
      agg_req[ai] = find_req({sl, op, a.expr, sl2, 0});
    }
  }
  std::vector<int> req_acc(reqs.size());
  std::vector<AccReq> acc_req(kMaxAcc + 2, AccReq{0, 0, 0, -1, 0});
  int nacc = 1;
  q.acc_op[0] = ACC_COUNT;
  auto push_acc = [&](const AccReq& rq) -> int {
    if (nacc >= kMaxAcc) return fail(PINOT_AMD_EUNSUPPORTED, "too many aggregations");
    acc_req[nacc] = rq;
    q.acc_op[nacc++] = rq.op;
    return 0;
  };
  for (int sl = 0; sl < kMaxSlots; ++sl)
    for (size_t k = 0; k < reqs.size(); ++k)
      if (reqs[k].slot == sl) {
        req_acc[k] = nacc;
        if (int rc = push_acc(reqs[k])) return rc;
        if (reqs[k].op == ACC_SUM_I128)
          if (int rc = push_acc({reqs[k].slot, ACC_HI, reqs[k].expr, reqs[k].slot2, 0})) return rc;
      }
  for (size_t ai = 0; ai < Q.aggs.size(); ++ai) {
    r->agg_type.push_back(Q.aggs[ai].type);
    r->agg_acc.push_back(agg_req[ai] < 0 ? 0 : req_acc[agg_req[ai]]);
    r->agg_acc2.push_back(agg_req2[ai] < 0 ? 0 : req_acc[agg_req2[ai]]);
  }

  clk.mark("accs");
  // ---- plan kind ----
  // dense table: mixed-radix keys over the merged dictionaries; hash table: key spaces beyond the
  // dense cap (DictionaryBasedGroupKeyGenerator's Int/Long/ArrayMapBasedHolder) and numGroupsLimit
  // trimming (keys admitted per segment in first-seen order)
  // dense keys are 32-bit in the kernels (K[4]): never above 2^31, whatever the override says
  const int64_t dense_cap = std::min<int64_t>(env_i64("PINOT_AMD_DENSE_MAX_KEYS", (int64_t)1 << 28), (int64_t)1 << 31);
  if (filter_only) {
    r->kind = PLAN_FILTER;
  } else if (Q.group_by.empty()) {
    r->kind = PLAN_DENSE;
  } else if (limit_possible && dense_keys <= (double)dense_cap && !env_is("PINOT_AMD_GROUP_PLAN", "hash") &&
             !env_is("PINOT_AMD_TRIM_PLAN", "hash") && [&]() {
               // dense admission: first docIds (4 B per segment and key), key lists, bitmaps within budget;
               // a segment's 1024-doc bucket histogram within one block's LDS
               int64_t max_docs = 0;
               for (auto* sg : segs) max_docs = std::max(max_docs, sg->num_docs);
               const double cap = std::min((double)max_docs, dense_keys);
               const double bytes = (double)n * (dense_keys * 4.0 + cap * 4.0 + dense_keys / 8.0);
               return bytes <= (double)env_i64("PINOT_AMD_ADMIT_MAX_BYTES", (int64_t)8 << 30) &&
                      (max_docs + 1023) / 1024 * 4 <= 64 * 1024;
             }()) {
    r->kind = PLAN_DENSE;
    r->admit = true;
  } else if (limit_possible || dense_keys > (double)dense_cap || env_is("PINOT_AMD_GROUP_PLAN", "hash")) {
    r->kind = PLAN_HASH;
    r->trim = limit_possible;
  } else {
    r->kind = PLAN_DENSE;
  }
  // segment-level trims the dense presence pass cannot restate: the safe trim past the dense cap and the unsafe
  // trim (which orders by per-segment aggregation values): per-segment results in a (key, segment) scan table, the
  // numGroupsLimit cutoff as for any trim plan, then each segment's top `keep` (segsel)
  if ((seg_trim && r->kind != PLAN_DENSE) || segsel_unsafe) {
    r->segsel = true;
    r->segsel_keep = segsel_unsafe ? segsel_unsafe_keep : r->srv_limit;
    seg_trim = false;
    r->kind = PLAN_HASH;
    r->trim = true;
    r->admit = false;
  }
  if (r->admit) admit_prefixes();
  std::vector<JitPlan::OrdCol> seg_ord;
  if (seg_trim) {
    // ORDER BY rank of a dense key: the first ORDER BY column most significant, DESC columns flipped
    std::vector<std::pair<int, int>> ocols;  // (group column, ascending), first occurrence of each column
    for (const auto& ob : r->srv_order)
      if (std::none_of(ocols.begin(), ocols.end(), [&](const std::pair<int, int>& c) { return c.first == ob.index; }))
        ocols.push_back({ob.index, ob.asc});
    int64_t run = 1;
    for (size_t o = ocols.size(); o-- > 0;) {
      const int j = ocols[o].first;
      const int64_t size = (int64_t)std::max<size_t>(r->keys[j]->size(), 1);
      seg_ord.insert(seg_ord.begin(), JitPlan::OrdCol{std::max<int64_t>(r->key_stride[j], 1), size, run,
                                                      ocols[o].second ? 0 : 1});
      run *= size;
    }
    r->sp_words = (run + 63) / 64;
    r->seg_trim = true;
  }
  if (r->trim) {
    r->fd_acc = nacc;
    if (int rc = push_acc({-1, ACC_FIRST_DOC, 0, -1, 0})) return rc;
  }
  q.nacc = (Q.aggs.empty() && Q.group_by.empty()) ? 0 : nacc;  // filter-only: count matches
  if (filter_only) q.nacc = 0;
  const int64_t num_keys = r->kind == PLAN_HASH ? 0 : (int64_t)dense_keys;
  q.num_keys = num_keys;

  clk.mark("plan_kind");
  // ---- hash plans: key packing and table sizes ----
  const int64_t table_budget = env_i64("PINOT_AMD_HASH_TABLE_BYTES", (int64_t)4 << 30);  // per trim scan table
  std::vector<int> seg_batch(n, 0);
  if (r->kind == PLAN_HASH) {
    std::vector<int64_t> sizes;
    for (auto& m : r->keys) sizes.push_back((int64_t)std::max<size_t>(m->size(), 1));
    pack_key_words(sizes, &r->pack_word, &r->pack_shift);
    r->pack_bits.clear();
    for (int64_t sz : sizes) r->pack_bits.push_back(bits_for(sz));
    r->nw = r->pack_word.empty() ? 1 : r->pack_word.back() + 1;
    if (r->nw + (r->trim ? 1 : 0) > kMaxKeyWords)
      return fail(PINOT_AMD_EUNSUPPORTED, "group key of %d words exceeds %d", r->nw, kMaxKeyWords);
    if (r->segsel) {
      // the ORDER BY as a chain of 64-bit stage keys (SegSelStage): runs of group columns in one mixed-radix value
      // while it fits (the first column most significant, DESC ones flipped), an aggregation's final value per
      // stage, then -- unsafe trims, whose ORDER BY may tie -- the key words, the last first (ascending key)
      auto& st = r->segsel_st;
      st.clear();
      SegSelStage cur{};
      bool open = false;
      unsigned __int128 span = 1;
      auto close = [&]() {
        if (open) st.push_back(cur);
        open = false;
      };
      for (const auto& ob : r->srv_order) {
        if (ob.kind == 0) {
          const int j = ob.index;
          const int64_t size = (int64_t)std::max<size_t>(r->keys[j]->size(), 1);
          if (open && (span * (unsigned __int128)size > ((unsigned __int128)1 << 64) || cur.ncols >= kMaxGroupCols)) close();
          if (!open) {
            cur = SegSelStage{};
            cur.kind = 0;
            open = true;
            span = 1;
          }
          for (int c = 0; c < cur.ncols; ++c) cur.mul[c] *= size;
          const int c = cur.ncols++;
          cur.word[c] = r->pack_word[j];
          cur.shift[c] = r->pack_shift[j];
          cur.bits[c] = r->pack_bits[j];
          cur.flip[c] = ob.asc ? 0 : 1;
          cur.size[c] = size;
          cur.mul[c] = 1;
          span *= (unsigned __int128)size;
        } else {
          close();
          SegSelStage a{};
          a.kind = 1;
          a.agg_type = r->agg_type[ob.index];
          a.acc = r->agg_acc[ob.index];
          a.acc2 = r->agg_acc2[ob.index];
          a.desc = ob.asc ? 0 : 1;
          st.push_back(a);
        }
      }
      close();
      if (!r->srv_safe)
        for (int w = r->nw - 1; w >= 0; --w) {
          SegSelStage k{};
          k.kind = 2;
          k.kword = w;
          st.push_back(k);
        }
      if (st.empty() || (int)st.size() > kSegSelMaxStages)
        return fail(PINOT_AMD_EUNSUPPORTED, "segment group trim: %zu ORDER BY stages (at most %d)", st.size(), kSegSelMaxStages);
      if (int rc = r->d_segsel_st.alloc_copy(st.data(), st.size() * sizeof(SegSelStage), 0)) return rc;
    }
    const double keyspace = dense_keys;
    double fbound = 0;
    for (int si = 0; si < n; ++si) fbound += (double)(r->trim ? std::min<int64_t>(seg_bound[si], Q.num_groups_limit) : seg_bound[si]);
    fbound = std::min(fbound, keyspace);
    const int64_t max_cap = (int64_t)1 << 31;  // compaction indexes slots with int32
    auto bytes_of = [&](int64_t cap, int words) { return (double)cap * (double)(words + nacc) * 8.0; };
    // the final table holds every admitted group at once (it cannot be batched); untrimmed plans start at
    // most PINOT_AMD_HASH_INIT_SLOTS slots and grow when groups overflow it (run_plan)
    double want = std::min(2.0 * fbound, (double)max_cap);
    if (!r->trim) want = std::min(want, (double)env_i64("PINOT_AMD_HASH_INIT_SLOTS", (int64_t)1 << 20));
    int64_t fcap = next_pow2(std::max<int64_t>(64, (int64_t)want));
    const double max_bytes = (double)env_i64("PINOT_AMD_HASH_FINAL_MAX_BYTES", (int64_t)64 << 30);
    const double fbytes = bytes_of(fcap, r->nw);
    if (fbytes > max_bytes)
      return fail(PINOT_AMD_EUNSUPPORTED, "group table of %lld slots (%.1f GB) exceeds PINOT_AMD_HASH_FINAL_MAX_BYTES",
                  (long long)fcap, fbytes / 1e9);
    if (!r->trim) {
      // growth ceiling: 2 x the group bound as a power of two, within the slot index range and the byte budget
      int64_t ceil_cap = std::min<int64_t>(max_cap, next_pow2(std::max<int64_t>(64, (int64_t)std::min(2.0 * fbound, (double)max_cap))));
      while (ceil_cap > 64 && bytes_of(ceil_cap, r->nw) > max_bytes) ceil_cap >>= 1;
      r->fcap_ceiling = std::max(ceil_cap, fcap);
      // an earlier execution of the same query shape over the same segments settled on a capacity: start there
      std::string ck = preds_signature(Q.preds) + "\x1c";
      for (size_t j = 0; j < Q.group_by.size(); ++j) ck += Q.group_by[j] + ":" + std::to_string(r->keys[j]->id) + ",";
      ck += "\x1c";
      for (auto* sg : segs) ck += std::to_string(sg->uid) + "." + std::to_string(sg->gen) + ",";
      r->cap_key = ck;
      const int64_t known = known_hash_capacity(ck);
      if (known > 0 && !env_is("PINOT_AMD_HASH_CAP_CACHE", "0")) {
        fcap = std::min(std::max(fcap, known), r->fcap_ceiling);
        r->cap_known = true;
      }
    }
    r->fcap = fcap;
    if (r->trim) {
      // scan tables keyed by (key, segment), one batch of segments at a time
      int b = 0;
      double acc_bound = 0;
      int bsegs = 0;
      auto close_batch = [&]() {
        const int64_t cap = next_pow2(std::max<int64_t>(64, (int64_t)std::min(2.0 * acc_bound, (double)max_cap)));
        r->batch_cap.push_back(cap);
        r->batch_nsegs.push_back(bsegs);
      };
      for (int si = 0; si < n; ++si) {
        const double nb = acc_bound + (double)seg_bound[si];
        const int64_t cap = next_pow2(std::max<int64_t>(64, (int64_t)std::min(2.0 * nb, (double)max_cap)));
        if (bsegs > 0 && (bytes_of(cap, r->nw + 1) > (double)table_budget || 2.0 * nb > (double)max_cap)) {
          close_batch();
          ++b;
          acc_bound = 0;
          bsegs = 0;
        }
        seg_batch[si] = b;
        acc_bound += (double)seg_bound[si];
        ++bsegs;
      }
      close_batch();
      r->nbatches = b + 1;
      for (int64_t c : r->batch_cap)
        if ((double)c < 2.0 * 1) return fail(PINOT_AMD_EINVAL, "internal: empty trim batch");
    }
  }

  clk.mark("hash_sizes");
  // ---- device segments (one DevSegment per segment; tile_begin / key_seg set per launch) ----
  std::vector<DevSegment> hsegs(n);
  for (int si = 0; si < n; ++si) {
    DevSegment& ds = hsegs[si];
    memset(&ds, 0, sizeof(ds));
    ds.num_docs = segs[si]->num_docs;
    for (int sl = 0; sl < nslots; ++sl) {
      const Column& c = *segs[si]->cols.at(slot_cols[sl]);
      DevColumn& dc = ds.cols[sl];
      dc.data = (const uint8_t*)c.fwd.p;
      dc.dict = c.dict.p;
      dc.enc = c.enc;
      dc.type = c.type;
      dc.bits = c.bits;
      dc.card = c.card;
    }
    for (size_t j = 0; j < Q.group_by.size(); ++j) {
      const Column& c = *segs[si]->cols.at(Q.group_by[j]);
      std::shared_ptr<DevBuf> buf;
      if (int rc = cached_remap(segs[si], Q.group_by[j], c, *r->keys[j], &buf)) return rc;
      if (buf) {
        ds.cols[slot_of(Q.group_by[j])].remap = (const int32_t*)buf->p;
        r->shared.push_back(std::move(buf));
      }
    }
    for (size_t k = 0; k < order.size(); ++k) {
      DevLeaf L = seg_leaves[si][order[k]];
      L.slot = pred_slot[order[k]];
      ds.leaves[k] = L;
    }
  }
  if (!r->inv_leaves.empty()) {
    std::vector<ExpandJob> jobs(r->inv_leaves.size());
    int64_t total = 0, items = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
      const auto& il = r->inv_leaves[j];
      ExpandJob& J = jobs[j];
      memset(&J, 0, sizeof(J));
      J.inv = (const uint8_t*)il.col->inv.p;
      J.conts = (const RoaringContainer*)il.col->inv_conts.p;
      J.sel = (const int32_t*)il.sel->p;
      J.bitset = (unsigned long long*)il.bitset->p;
      J.num_docs = il.num_docs;
      J.nwords = std::max<int64_t>((il.num_docs + kTileDocs - 1) / kTileDocs, 1) * (kTileDocs / 64) + 8;  // not the slack
      J.sel_begin = total;
      J.nsel = il.nsel;
      J.grp = (const int32_t*)il.grp->p;
      J.psel = il.psel ? (const unsigned long long*)il.psel->p : nullptr;
      J.item_begin = items;
      J.nchunks = il.nchunks;
      total += il.nsel;
      items += il.nchunks;
    }
    r->expand_total = items;
    if (int rc = r->d_expand_jobs.alloc_copy(jobs.data(), jobs.size() * sizeof(ExpandJob), 0)) return rc;
  }
  std::vector<uint64_t*> bitset_ptrs(n, nullptr);
  if (filter_only) {
    for (int si = 0; si < n; ++si) {
      const int64_t words = std::max<int64_t>((segs[si]->num_docs + kTileDocs - 1) / kTileDocs, 1) * (kTileDocs / 64);
      auto b = std::make_unique<DevBuf>();
      if (int rc = b->alloc((size_t)words * 8)) return rc;
      HIP_OK(hipMemset(b->p, 0, b->n));
      bitset_ptrs[si] = (uint64_t*)b->p;
      r->bitset_words.push_back(words);
      r->bitsets.push_back(std::move(b));
    }
  }

  clk.mark("dev_segs");
  // ---- plan-level kernel choices (shared by every launch) ----
  int lds_max = 0;
  {
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) lds_max = 65536;
    lds_max = std::min(lds_max, 160 * 1024);
  }
  JitPlan base;
  base.nclauses = nclauses;
  for (size_t j = 0; j < Q.group_by.size(); ++j) {
    base.group.push_back({slot_of(Q.group_by[j]), r->kind == PLAN_HASH ? 0 : r->key_stride[j]});
    for (int si = 0; si < n; ++si) base.any_remap |= hsegs[si].cols[slot_of(Q.group_by[j])].remap != nullptr;
  }
  for (int a = 1; a < q.nacc; ++a)
    base.accs.push_back({q.acc_op[a], acc_req[a].slot, acc_req[a].expr, acc_req[a].slot2, acc_req[a].nan_skip});
  base.num_keys = num_keys;
  base.admit = r->admit;
  base.seg_ord = seg_ord;
  base.bitset = filter_only;
  base.aggregate = q.nacc > 0;
  int cus = 256;
  {
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  // Integer SUMs into an LDS table keep 64-bit partials (no high word in LDS) when |value| x (docs one
  // block adds) < 2^63 for every segment: a scan block owns ceil(tiles / grid) tiles with grid >=
  // min(CUs, tiles / kPartSub); a partition aggregation block ceil(records / agg_grid) <= ceil(docs /
  // CUs) records. Bounded with the whole batch, so every launch of the plan satisfies it.
  int64_t all_tiles = 0, all_docs = 0;
  for (auto* s : segs) {
    all_tiles += (s->num_docs + kTileDocs - 1) / kTileDocs;
    all_docs += s->num_docs;
  }
  auto set_narrow = [&](__int128 docs_bound) {
    auto maxabs = [&](int sl) -> __int128 {
      __int128 m = 0;
      for (auto* s : segs) {
        const Column& c = *s->cols.at(slot_cols[sl]);
        if (!c.has_range) return -1;
        const __int128 a = c.vmax < 0 ? -(__int128)c.vmax : (__int128)c.vmax;
        const __int128 b = c.vmin < 0 ? -(__int128)c.vmin : (__int128)c.vmin;
        m = std::max(m, std::max(a, b));
      }
      return m;
    };
    for (JitAcc& a : base.accs) {
      a.narrow = 0;
      if (a.op != ACC_SUM_I128 || env_is("PINOT_AMD_NARROW_SUMS", "0")) continue;
      __int128 m = maxabs(a.slot);
      if (m >= 0 && a.expr != EXPR_COL) {
        const __int128 m2 = maxabs(a.slot2);
        m = m2 < 0 ? -1 : a.expr == EXPR_MUL ? m * m2 : m + m2;
      }
      a.narrow = (m >= 0 && m * docs_bound <= (__int128)INT64_MAX) ? 1 : 0;
    }
  };
  auto lds_arrays = [&]() {
    int k = 0;
    jit_lds_layout(base, &k);
    return (int64_t)k;
  };
  int64_t lds_bytes = (int64_t)q.nacc * std::max<int64_t>(num_keys, 1) * 8;
  int64_t hash_lds_bytes = 0;  // hash plans: the LDS first level (JitPlan::hash_lds)
  std::vector<int64_t> part_vbase;  // partitioned plans: integer record fields' bases (DevPartition::vbase)
  if (r->kind == PLAN_DENSE && q.nacc > 0) {
    const int64_t min_grid = std::max<int64_t>(1, std::min<int64_t>(cus, all_tiles / kPartSub));
    set_narrow((__int128)((all_tiles + min_grid - 1) / min_grid) * kTileDocs);
    lds_bytes = lds_arrays() * std::max<int64_t>(num_keys, 1) * 8;
    if (lds_bytes <= 40 * 1024) {  // LDS-privatised table, four 256-thread blocks per CU
      base.lds = true;
    } else if (lds_bytes <= lds_max && !env_is("PINOT_AMD_WIDE_LDS", "0")) {
      base.lds = true;  // one CU-wide block (4 x 256 threads, 16 waves) owns the whole table
      base.scan_nsub = kPartSub;
    } else if (!env_is("PINOT_AMD_PARTITIONED", "0") && !Q.group_by.empty()) {
      // key space too large for an LDS table: partition the matching docs by key range and aggregate
      // each partition in LDS (random per-lane HBM atomics run ~17x below the coalesced rate)
      set_narrow((__int128)((all_docs + cus - 1) / cus));
      const int64_t na = lds_arrays();
      // the aggregation block's LDS: the partition's table + (sampled plans) its allotment tables,
      // 2 x 8 B per scatter block (<= 2 x CUs blocks)
      const int64_t agg_lds = lds_max - (2 * 2 * (int64_t)cus + 1) * 8;
      int shift = 16;
      while (shift > 6 && na * ((int64_t)1 << shift) * 8 > agg_lds) --shift;
      const int64_t nparts = (num_keys + ((int64_t)1 << shift) - 1) >> shift;
      if (na * ((int64_t)1 << shift) * 8 <= agg_lds && nparts <= 8192) {
        r->kind = PLAN_PARTITIONED;
        base.partitioned = true;
        base.key_shift = shift;
        base.nparts = (int)nparts;
        for (auto& a : base.accs)
          if (a.op != ACC_HI && a.op != ACC_FIRST_DOC &&
              std::find(base.vals.begin(), base.vals.end(), a.val()) == base.vals.end())
            base.vals.push_back(a.val());
        // packed record fields: an integer value is stored as value - lo in bitlen(hi - lo) bits, where
        // [lo, hi] is the batch's value range (dictionary ends / staged min-max; interval arithmetic for
        // times / minus / plus of two INT columns); without a range INT takes 32 bits above INT32_MIN,
        // LONG 64. FLOAT / DOUBLE values keep their raw bits.
        auto slot_range = [&](int sl, __int128* lo, __int128* hi) {
          bool any = false;
          for (auto* s : segs) {
            const Column& c = *s->cols.at(slot_cols[sl]);
            if (s->num_docs == 0) continue;
            if (!c.has_range) return false;
            if (!any || c.vmin < *lo) *lo = c.vmin;
            if (!any || c.vmax > *hi) *hi = c.vmax;
            any = true;
          }
          if (!any) *lo = *hi = 0;
          return true;
        };
        base.val_bits.clear();
        part_vbase.clear();
        for (const JitVal& v : base.vals) {
          auto slot_type = [&](int sl) { return segs[0]->cols.at(slot_cols[sl])->type; };
          const int t1 = slot_type(v.slot), t2 = v.expr == EXPR_COL ? T_INT : slot_type(v.slot2);
          const bool is_int = v.expr == EXPR_COL ? (t1 == T_INT || t1 == T_LONG) : (t1 == T_INT && t2 == T_INT);
          if (!is_int) {
            base.val_bits.push_back(v.expr == EXPR_COL && t1 == T_FLOAT ? 32 : 64);
            part_vbase.push_back(0);
            continue;
          }
          __int128 lo = 0, hi = 0, lo2 = 0, hi2 = 0;
          bool known = slot_range(v.slot, &lo, &hi);
          if (known && v.expr != EXPR_COL) {
            known = slot_range(v.slot2, &lo2, &hi2);
            if (v.expr == EXPR_ADD) {
              lo += lo2;
              hi += hi2;
            } else if (v.expr == EXPR_SUB) {
              const __int128 l = lo - hi2, h = hi - lo2;
              lo = l;
              hi = h;
            } else {
              const __int128 c[4] = {lo * lo2, lo * hi2, hi * lo2, hi * hi2};
              lo = *std::min_element(c, c + 4);
              hi = *std::max_element(c, c + 4);
            }
          }
          if (!known) {
            const bool narrow = v.expr == EXPR_COL && t1 == T_INT;
            base.val_bits.push_back(narrow ? 32 : 64);
            part_vbase.push_back(narrow ? INT32_MIN : 0);
            continue;
          }
          int bits = 0;
          for (unsigned __int128 w = (unsigned __int128)(hi - lo); w; w >>= 1) ++bits;
          base.val_bits.push_back(std::min(bits, 64));
          part_vbase.push_back((int64_t)lo);
        }
      }
    }
  }
  if (!base.lds && !base.partitioned)
    for (JitAcc& a : base.accs) a.narrow = 0;  // HBM tables take full 128-bit adds
  if (r->kind == PLAN_HASH) {
    base.hash = true;
    base.hash_seg = r->trim;
    base.hash_words = r->nw + (r->trim ? 1 : 0);
    for (size_t j = 0; j < Q.group_by.size(); ++j) base.hash_pack.push_back({r->pack_word[j], r->pack_shift[j]});
  }

  clk.mark("kernel_choices");
  // ---- selection-vector plan (late materialisation) ----
  // A selective filter over narrow rows: the select pass reads only the filter columns and appends the
  // matching docIds; the gather pass reads the group-by / aggregated columns of those docs only (64 B
  // sectors at random positions). Chosen when its bytes, from the exact per-segment match counts,
  // undercut the fused scan's: filter columns + 16 B per match (vector write + read) + the value columns'
  // sectors a match touches + a per-match gather cost, against every column of every doc.
  std::vector<bool> leaf_slot(nslots, false), value_slot(nslots, false);
  for (size_t pi = 0; pi < np; ++pi)
    if (pred_slot[pi] >= 0) leaf_slot[pred_slot[pi]] = true;
  for (auto& g : base.group) value_slot[g.first] = true;
  for (auto& a : base.accs)
    if (a.op != ACC_FIRST_DOC) {
      value_slot[a.slot] = true;
      if (a.expr != EXPR_COL) value_slot[a.slot2] = true;
    }
  auto slot_bpr = [](const DevColumn& c) -> double {
    return c.enc == ENC_FIXED_BIT ? c.bits / 8.0 : c.enc == ENC_RAW ? (double)value_size(c.type) : 0.0;
  };
  const char* sel_env = knob("PINOT_AMD_SELECT");
  // (a partitioned plan qualifies too: when its filter keeps few docs, the gather adds them straight into
  // the HBM table, where the partitioned plan would hand over to a fused direct-atomic scan of every row)
  const bool sel_eligible = !filter_only && q.nacc > 0 && np > 0 && !r->trim && !r->admit && !r->seg_trim &&
                            (r->kind == PLAN_DENSE || r->kind == PLAN_HASH || r->kind == PLAN_PARTITIONED) &&
                            !env_is("PINOT_AMD_SELECT_PARTITIONED", base.partitioned ? "0" : "-") &&
                            !(sel_env && !strcmp(sel_env, "never"));
  if (sel_eligible) {
    // Cost in time, not bytes: a pass over a tile costs per-doc work as well as bytes (measured on one
    // MI355X: a fused scan of narrow SSB rows and the select pass alike take ~1-1.3 ps per doc however
    // few bytes they read; a gathered doc ~30-50 ps on SSB, more for scattered raw columns), so the
    // selection-vector plan only pays when the value columns it skips are wide and few docs match.
    constexpr double kBw = 6.0e12;         // achievable HBM read rate, B/s
    constexpr double kScanDoc = 1.3e-12;   // fused scan, per doc
    constexpr double kGatedDoc = 1.25e-12; // inverted-index gated scan, per doc
    constexpr double kSelectDoc = 1.0e-12; // select pass, per doc
    constexpr double kGatherDoc = 60e-12;  // gather pass, per matching doc
    double scan_b = 0, leaf_b = 0, docs_all = 0;
    for (int si = 0; si < n; ++si) {
      docs_all += (double)segs[si]->num_docs;
      for (int sl = 0; sl < nslots; ++sl) {
        const double b = slot_bpr(hsegs[si].cols[sl]) * (double)segs[si]->num_docs;
        scan_b += b;
        if (leaf_slot[sl]) leaf_b += b;
      }
    }
    bool gated = false;  // some clause is all inverted-index bitsets: the fused scan reads columns only where it passes
    {
      std::vector<int> gate(nclauses, 1), has(nclauses, 0);
      for (size_t k = 0; k < order.size(); ++k) {
        const int c = Q.preds[order[k]].clause;
        has[c] = 1;
        for (int si = 0; si < n; ++si)
          if (hsegs[si].leaves[k].kind != LEAF_DOC_BITSET || hsegs[si].leaves[k].negate) gate[c] = 0;
      }
      for (int c = 0; c < nclauses; ++c) gated |= gate[c] && has[c];
    }
    // a filter reading no column (docId bitsets / ranges / constants) selects on 64-doc words
    bool wordy = np > 0;
    for (size_t k = 0; k < order.size(); ++k)
      for (int si = 0; si < n; ++si) {
        const int kd = hsegs[si].leaves[k].kind;
        if (kd != LEAF_DOC_BITSET && kd != LEAF_DOC_RANGE && kd != LEAF_CONST) wordy = false;
      }
    constexpr double kWordDoc = 0.1e-12;  // word-level select pass, per doc
    const double sel_doc = wordy ? kWordDoc : kSelectDoc;
    const double scan_t = std::max(scan_b / kBw, docs_all * (gated ? kGatedDoc : kScanDoc));
    const bool forced = sel_env && !strcmp(sel_env, "always");
    if (forced || std::max(leaf_b / kBw, docs_all * sel_doc) < 0.9 * scan_t) {  // the select pass alone could win
      if (int rc = probe_matched()) return rc;
      double sel_bytes = leaf_b, matches = 0;
      for (int si = 0; si < n; ++si) {
        const double m = (double)seg_matched[si], docs = (double)std::max<int64_t>(segs[si]->num_docs, 1);
        const double s = m / docs;
        matches += m;
        sel_bytes += 16.0 * m;  // vector written + read
        for (int sl = 0; sl < nslots; ++sl) {
          if (!value_slot[sl]) continue;
          const DevColumn& c = hsegs[si].cols[sl];
          const double bpr = slot_bpr(c);
          if (bpr <= 0) continue;
          const double per_sector = 64.0 / bpr;  // docs per 64-byte sector
          sel_bytes += bpr * docs * (1.0 - std::pow(1.0 - s, per_sector));
        }
      }
      const double sel_t = std::max(leaf_b / kBw, docs_all * sel_doc) + matches * kGatherDoc + (sel_bytes - leaf_b) / kBw;
      base.select = forced || sel_t < 0.9 * scan_t;
      base.word_select = base.select && wordy && !env_is("PINOT_AMD_WORD_SELECT", "0");
      base.wsel_words = (int)env_i64("PINOT_AMD_WSEL_WORDS", 4) == 8 ? 8 : 4;  // swept: 8 is 4 % faster at 0.01-0.1 %, 2 % slower at 1 %
      if (base.select && base.partitioned) {  // the gather aggregates into the dense HBM table
        r->kind = PLAN_DENSE;
        base.partitioned = false;
        base.key_shift = 0;
        base.nparts = 0;
        base.vals.clear();
        base.val_bits.clear();
        part_vbase.clear();
        for (JitAcc& a : base.accs) a.narrow = 0;  // HBM tables take full 128-bit adds
      }
    }
    // tile-level select: 1024-doc tiles per loop step (PINOT_AMD_SEL_GROUP 1 / 2 / 4); the launches'
    // segment tile ranges are padded to multiples of it below
    if (base.select && !base.word_select) {
      const int64_t g = env_i64("PINOT_AMD_SEL_GROUP", 4);
      base.sel_group = g >= 4 ? 4 : g >= 2 ? 2 : 1;
    }
  }
  // a fused scan of a dense plan with tile groups too (PINOT_AMD_SCAN_GROUP, default 4: configs[1] 3.45 -> 3.38 ms,
  // SSB Q3.1 0.896 -> 0.858 ms)
  if (!base.select && r->kind == PLAN_DENSE && !base.partitioned && !r->admit && !filter_only) {
    const int64_t g = env_i64("PINOT_AMD_SCAN_GROUP", 4);
    base.sel_group = g >= 4 ? 4 : g >= 2 ? 2 : 1;
  }
  // Filter-gated value loads (JitPlan::filter_gate) for a fused dense scan: the filter columns load ahead and
  // the group-key / value columns only for lanes with a matching doc. A lane holds 4 docs, so a 64-byte sector
  // of a B-byte column (64 / B docs) is fetched when any of its docs matches: 1 - (1 - s)^(64 / B) of it at
  // selectivity s (the segments' exact match counts). Chosen when the bytes it reads -- the filter columns, then
  // the fetched share of every column read after the filter (a filter column that is also a key or value is
  // read twice) -- are at most 3/4 of the fused scan's. Opt-in (PINOT_AMD_FILTER_GATE=auto: this model,
  // =1: forced): measured on SSB it lost to the 4-tile fused scan and to the select pass on every query but
  // Q4.1 (1.075 -> 1.038 ms; Q1.1 0.641 -> 0.790, Q3.1 0.852 -> 1.053: profiles/r05/sweep_ssb_fgate.txt) --
  // these scans run near the HBM rate already, and the gate's one tile per step and a-tile-ahead filter cost
  // more issue than the skipped sectors save.
  if (!base.select && r->kind == PLAN_DENSE && !base.partitioned && !r->admit && !filter_only && q.nacc > 0 && np > 0 &&
      (env_is("PINOT_AMD_FILTER_GATE", "1") || env_is("PINOT_AMD_FILTER_GATE", "auto"))) {
    bool ok = true;  // docId-bitset leaves gate through the inverted-index path instead
    for (size_t k = 0; k < order.size() && ok; ++k)
      for (int si = 0; si < n; ++si) ok &= hsegs[si].leaves[k].kind != LEAF_DOC_BITSET;
    const bool forced = env_is("PINOT_AMD_FILTER_GATE", "1");
    double fused_b = 0, filter_b = 0, value_b = 0;
    for (int si = 0; si < n && ok; ++si)
      for (int sl = 0; sl < nslots; ++sl) {
        const double b = slot_bpr(hsegs[si].cols[sl]) * (double)segs[si]->num_docs;
        fused_b += b;
        if (leaf_slot[sl]) filter_b += b;
        if (value_slot[sl]) value_b += b;
      }
    // worth a match-count probe only if the value columns could be skipped for a real share of the bytes
    if (ok && (forced || filter_b + 0.1 * value_b <= 0.75 * fused_b)) {
      if (int rc = probe_matched()) return rc;
      double gated_b = 0;
      for (int si = 0; si < n; ++si) {
        const double docs = (double)std::max<int64_t>(segs[si]->num_docs, 1);
        const double sel = std::min(1.0, (double)seg_matched[si] / docs);
        for (int sl = 0; sl < nslots; ++sl) {
          const double bpr = slot_bpr(hsegs[si].cols[sl]);
          if (leaf_slot[sl]) gated_b += bpr * docs;
          if (value_slot[sl] && bpr > 0) gated_b += bpr * docs * (1.0 - std::pow(1.0 - sel, 64.0 / bpr));
        }
      }
      base.filter_gate = forced || gated_b <= 0.75 * fused_b;
      r->filter_gate = base.filter_gate;
      if (base.filter_gate) base.sel_group = 1;  // gated plans take one tile per step
    }
  }
  // Narrow int64 LDS partials with tile groups: every segment's tile range is padded to a multiple of G and a
  // block takes ceil(T' / (G x grid)) x G padded tiles, so the docs one block can add are bounded from the
  // padded tile total (the G = 1 bound above used the unpadded one). If a sum's margin does not hold at that
  // bound, the plan keeps one tile per step (the G = 1 bound, the same LDS layout).
  if (base.lds && !base.select && q.nacc > 0 && base.sel_group > 1) {
    auto docs_bound = [&](int64_t G) {
      int64_t tp = 0;
      for (auto* s : segs) tp += ((s->num_docs + kTileDocs - 1) / kTileDocs + G - 1) / G * G;
      const int64_t mg = std::max<int64_t>(1, std::min<int64_t>(cus, tp / kPartSub));
      return (__int128)((tp + G * mg - 1) / (G * mg) * G) * kTileDocs;
    };
    std::vector<int> before;
    for (const JitAcc& a : base.accs) before.push_back(a.narrow);
    set_narrow(docs_bound(base.sel_group));
    bool same = true;
    for (size_t i = 0; i < base.accs.size(); ++i) same &= base.accs[i].narrow == before[i];
    if (!same) {
      set_narrow(docs_bound(1));
      base.sel_group = 1;
    }
  }
  {
    if (base.select && base.lds) {
      // gather blocks walk the selection vector grid-strided (padding included, matches unevenly spread
      // over its quads): one block may add every match of the batch to its LDS table, so the narrow
      // 64-bit partials are bounded by all the docs; keep the table within the LDS
      const int64_t scan_min_grid = std::max<int64_t>(1, std::min<int64_t>(cus, all_tiles / kPartSub));
      const __int128 scan_bound = (__int128)((all_tiles + scan_min_grid - 1) / scan_min_grid) * kTileDocs;
      const __int128 gather_bound = (__int128)all_docs;
      if (gather_bound > scan_bound) {
        set_narrow(gather_bound);
        lds_bytes = lds_arrays() * std::max<int64_t>(num_keys, 1) * 8;
        if (lds_bytes > lds_max) base.select = false;
      }
    }
  }

  // Hash-table plans (DictionaryBasedGroupKeyGenerator's map-based holders) get an LDS-privatised first
  // level: one CU-wide block (4 x 256 threads) per CU keeps up to S keys with their accumulators in LDS,
  // so repeated keys (skewed group distributions) aggregate on-die and reach the HBM table once per block
  // instead of once per doc. Not for trimming plans (their keys carry the segment) or selection-vector
  // gathers. PINOT_AMD_HASH_LDS=0 disables it, PINOT_AMD_HASH_LDS_SLOTS sets S.
  if (base.hash && !r->trim && !base.select && q.nacc > 0 && !env_is("PINOT_AMD_HASH_LDS", "0")) {
    // integer SUMs in the LDS level keep int64 partials (no high-word array) when a CU-wide block's docs x
    // |value| fit (the HBM path of the same kernel always adds 128 bits); the grid has >= min(CUs, tiles / 4)
    // blocks
    const int64_t min_grid = std::max<int64_t>(1, std::min<int64_t>(cus, all_tiles / kPartSub));
    // the second level's LDS tables may meet every doc of the batch: their integer sums stay int64 when all docs x
    // |value| fit (spill_agg_kernel's narrow mask)
    set_narrow((__int128)std::max<int64_t>(all_docs, 1));
    r->spill_narrow = 0;
    for (size_t i = 0; i < base.accs.size() && i + 1 < 32; ++i)
      if (base.accs[i].narrow) r->spill_narrow |= 1u << (i + 1);
    set_narrow((__int128)((all_tiles + min_grid - 1) / min_grid) * kTileDocs);
    const int64_t slot_bytes = (int64_t)(base.hash_words + lds_arrays()) * 8;
    // second level: the LDS misses spilled as records and aggregated per key-hash partition (kernels.hip
    // spill passes) instead of one HBM probe + atomics per doc; PINOT_AMD_HASH_SPILL=0 keeps the direct path
    int nval = 0;  // a spill record's value words (spill_agg_kernel holds at most 8 words of a record)
    for (const JitAcc& a : base.accs) nval += a.op != ACC_HI && a.op != ACC_FIRST_DOC;
    const bool spill = !env_is("PINOT_AMD_HASH_SPILL", "0") && base.hash_words + nval <= 8;
    const int64_t reserve = 1024 + (spill ? (int64_t)kSpillMaxParts * 4 + 16 : 0);
    // as many slots as the LDS holds beside the kernel's static LDS (counters), a multiple of 64
    int64_t S = env_i64("PINOT_AMD_HASH_LDS_SLOTS", 0);
    if (S <= 0) S = std::min<int64_t>(8192, (lds_max - reserve) / slot_bytes);
    S = std::max<int64_t>(64, S / 64 * 64);
    if (S * slot_bytes <= lds_max - reserve) {
      base.hash_lds = (int)S;
      base.hash_spill = spill;
      // admission by recurrence (a doc inserts its key with probability 2^-5): the wide-key bench at 100 segments
      // 22.1 -> 15.4 ms, the LDS slots then holding the Zipf head instead of the first keys seen
      // (profiles/r05/sweep_wk_cap.txt); PINOT_AMD_HASH_LDS_ADMIT=n sets 2^-n, 0 inserts every key
      base.hash_admit = (int)std::min<int64_t>(8, std::max<int64_t>(0, env_i64("PINOT_AMD_HASH_LDS_ADMIT", 5)));
      // 4 of the 8 slots a one-word key could probe at once: on the ~1M-group Zipf table 16.65 -> 15.45 ms per 1B
      // rows (2 probes: 17.0; profiles/r06/sweep_lds_probes.txt) -- a key past 4 slots spills instead of reading 4 more
      base.hash_probes = 4;
      base.scan_nsub = kPartSub;
      hash_lds_bytes = S * slot_bytes;
    } else {
      for (JitAcc& a : base.accs) a.narrow = 0;
    }
  }

  clk.mark("select_plan");
  // ---- launches: segments of a batch grouped by shape (slot encodings and fixed-bit widths) ----
  const bool generic_bits = env_is("PINOT_AMD_GENERIC_BITS", "1");
  std::vector<int32_t> key_seg(n, 0);
  {
    std::vector<int32_t> cnt(r->nbatches, 0);
    for (int si = 0; si < n; ++si) key_seg[si] = cnt[seg_batch[si]]++;
  }
  for (int b = 0; b < r->nbatches; ++b) {
    // encoding signature -> segments; within it, fixed-bit width signatures
    std::map<std::string, std::vector<int>> by_enc;
    std::vector<std::string> enc_order;
    for (int si = 0; si < n; ++si) {
      if (seg_batch[si] != b) continue;
      std::string sig;
      for (int sl = 0; sl < nslots; ++sl) sig += std::to_string(hsegs[si].cols[sl].enc) + ",";
      if (!by_enc.count(sig)) enc_order.push_back(sig);
      by_enc[sig].push_back(si);
    }
    for (const std::string& es : enc_order) {
      const std::vector<int>& group = by_enc[es];
      auto bits_sig = [&](int si) {
        std::string sig;
        for (int sl = 0; sl < nslots; ++sl)
          sig += std::to_string(hsegs[si].cols[sl].enc == ENC_FIXED_BIT && hsegs[si].cols[sl].bits <= 15 ? hsegs[si].cols[sl].bits : 0) + ",";
        return sig;
      };
      std::map<std::string, std::vector<int>> by_bits;
      std::vector<std::string> bits_order;
      for (int si : group) {
        const std::string sig = bits_sig(si);
        if (!by_bits.count(sig)) bits_order.push_back(sig);
        by_bits[sig].push_back(si);
      }
      std::vector<std::vector<int>> parts;
      if (bits_order.size() <= 3) {
        for (auto& sig : bits_order) parts.push_back(by_bits[sig]);
      } else {
        parts.push_back(group);  // many widths: one launch with run-time widths where they differ
      }
      for (auto& part_segs : parts) {
        r->launches.emplace_back();
        Launch& L = r->launches.back();
        L.segs = part_segs;
        L.batch = b;
      }
    }
  }
  // Whole-query-narrow integer sums (JitAcc::hbm_narrow): when a SUM's value range times all the query's
  // docs fits int64, its adds into the HBM table need no carry, so they are one non-returning 64-bit atomic
  // on the low word (the 128-bit add waits for the old value to carry into the high word) and the plan's
  // end sets the high words from the low words' signs. Not for trimmed hash plans: their per-segment
  // tables merge into the final table before the plan's end.
  {
    std::vector<int32_t> arrs;
    if (!r->trim && q.nacc > 0 && !env_is("PINOT_AMD_HBM_NARROW", "0")) {
      auto maxabs = [&](int sl) -> __int128 {
        __int128 m = 0;
        for (auto* s : segs) {
          const Column& c = *s->cols.at(slot_cols[sl]);
          if (!c.has_range) return -1;
          const __int128 a = c.vmax < 0 ? -(__int128)c.vmax : (__int128)c.vmax;
          const __int128 b = c.vmin < 0 ? -(__int128)c.vmin : (__int128)c.vmin;
          m = std::max(m, std::max(a, b));
        }
        return m;
      };
      for (size_t ai = 0; ai < base.accs.size(); ++ai) {
        JitAcc& a = base.accs[ai];
        a.hbm_narrow = 0;
        if (a.op != ACC_SUM_I128) continue;
        __int128 m = maxabs(a.slot);
        if (m >= 0 && a.expr != EXPR_COL) {
          const __int128 m2 = maxabs(a.slot2);
          m = m2 < 0 ? -1 : a.expr == EXPR_MUL ? m * m2 : m + m2;
        }
        if (m >= 0 && m * (__int128)std::max<int64_t>(all_docs, 1) <= (__int128)INT64_MAX) {
          a.hbm_narrow = 1;
          arrs.push_back((int32_t)ai + 1);  // HBM array of its low word (array 0 is COUNT)
        }
      }
    }
    r->n_sext = (int32_t)arrs.size();
    r->d_sext.reset();
    if (!arrs.empty())
      if (int rc = r->d_sext.alloc_copy(arrs.data(), arrs.size() * 4, 0)) return rc;
  }
  const size_t nl = r->launches.size();
  if (int rc = r->matched.alloc((3 * nl + 3) * sizeof(unsigned long long))) return rc;
  HIP_OK(hipMemset(r->matched.p, 0, r->matched.n));
  size_t max_count_cells = 0, max_rec = 0, max_slab = 0, max_slab_docs = 0;
  int64_t max_sel = 0;  // selection-vector entries of the largest select launch
  for (size_t li = 0; li < nl; ++li) {
    Launch& L = r->launches[li];
    std::vector<DevSegment> ls;
    std::vector<uint64_t*> lbits;
    int64_t tiles = 0;
    for (int si : L.segs) {
      DevSegment ds = hsegs[si];
      ds.tile_begin = tiles;
      ds.key_seg = r->admit ? si : key_seg[si];
      ds.pad = r->admit ? 1 : 0;  // sequential admission over whole segments: each one walked to its end
      // (a tile-level select with G tiles per step: the segment's range padded to a multiple of G; the
      // padding tiles match nothing and read only their columns' staging padding)
      const int64_t G = base.sel_group;
      tiles += ((segs[si]->num_docs + kTileDocs - 1) / kTileDocs + G - 1) / G * G;
      L.docs += segs[si]->num_docs;
      ls.push_back(ds);
      lbits.push_back(bitset_ptrs[si]);
    }
    L.tiles = tiles;
    L.q = q;
    L.q.nsegs = (int32_t)L.segs.size();
    L.q.total_tiles = tiles;
    if (int rc = L.d_segs.alloc_copy(ls.data(), ls.size() * sizeof(DevSegment), 0)) return rc;
    static_assert(sizeof(DevSegment) % 8 == 0, "the count pass checksums descriptors in 8-byte words");
    L.h_segs = ls;
    // fused when few docs match (measured: 0.01 % / 0.1 % of 1B rows 0.36 / 0.52 -> 0.24 / 0.42 ms; at
    // 1 % the separate expansion's occupancy wins, 1.08 vs 1.17 ms); PINOT_AMD_FUSED_INV_SELECT=1 forces it
    double lm = 0, ld = 0;
    for (int si : L.segs) {
      lm += seg_matched.empty() ? 0.0 : (double)seg_matched[si];
      ld += (double)segs[si]->num_docs;
    }
    const bool fuse = env_is("PINOT_AMD_FUSED_INV_SELECT", "1") ||
                      (!env_is("PINOT_AMD_FUSED_INV_SELECT", "0") && !seg_matched.empty() && lm <= 0.004 * ld);
    if (base.word_select && fuse) {
      // the launch's segments as work items of G-chunk groups; each inverted-index leaf mapped to its
      // expansion job (its DevLeaf::bits is the job's bitset buffer)
      const int G = expand_group();
      std::vector<FusedSelSeg> fv(ls.size());
      int64_t items = 0;
      bool ok = true, neg_bits = false;
      for (size_t k = 0; k < ls.size(); ++k) {
        FusedSelSeg& f = fv[k];
        memset(&f, 0, sizeof(f));
        f.item_begin = items;
        f.seg = (int32_t)k;
        const int64_t words = (segs[L.segs[k]]->num_docs + kTileDocs - 1) / kTileDocs * (kTileDocs / 64);
        f.nitems = (int32_t)((words + 1024 * G - 1) / (1024 * G));
        for (int j = 0; j < kMaxLeaves; ++j) f.job[j] = -1;
        for (size_t j = 0; j < order.size(); ++j) {
          if (ls[k].leaves[j].kind != LEAF_DOC_BITSET) continue;
          for (size_t ii = 0; ii < r->inv_leaves.size(); ++ii)
            if (r->inv_leaves[ii].bitset->p == (const void*)ls[k].leaves[j].bits) f.job[j] = (int32_t)ii;
          ok &= f.job[j] >= 0 && r->inv_leaves[f.job[j]].nchunks >= f.nitems;
          neg_bits |= ls[k].leaves[j].negate != 0;
        }
        items += f.nitems;
      }
      if (ok) {
        if (int rc = L.d_fused.alloc_copy(fv.data(), fv.size() * sizeof(FusedSelSeg), 0)) return rc;
        L.fused = true;
        L.nfused = (int32_t)fv.size();
        L.fused_items = items;
        L.fused_leaves = (int32_t)order.size();
        // the clause-fold variant measured 5-9 % faster (sweep_inv_fused_variant.txt); negated bitset leaves need
        // the per-leaf fold
        L.fused_clause = !neg_bits && !env_is("PINOT_AMD_FUSED_VARIANT", "leaf");
        L.fused_clauses = base.nclauses;
      }
    }
    if (filter_only)
      if (int rc = L.d_bitset_ptrs.alloc_copy(lbits.data(), lbits.size() * sizeof(uint64_t*), 0)) return rc;

    JitPlan jp = base;
    for (int sl = 0; sl < nslots; ++sl) {
      const int enc = ls[0].cols[sl].enc;
      JitSlot js{enc, ls[0].cols[sl].type, 0, 0};
      if (enc != ENC_RAW) {  // dictionary of <= 64 entries everywhere: lane-register table
        bool small = true;
        for (auto& d : ls) small &= d.cols[sl].card <= 64 && d.cols[sl].card > 0;
        js.dict_regs = small ? 1 : 0;
      }
      if (enc == ENC_FIXED_BIT) {  // width shared by the launch (<= 15): compile-time shifts
        js.bits = ls[0].cols[sl].bits;
        for (auto& d : ls)
          if (d.cols[sl].bits != js.bits) js.bits = 0;
        if (js.bits > 15 || generic_bits) js.bits = 0;
      }
      jp.slots.push_back(js);
    }
    for (size_t k = 0; k < order.size(); ++k) {
      JitLeaf jl{pred_slot[order[k]], Q.preds[order[k]].clause, ls[0].leaves[k].negate, 0u};
      bool small_sets = jl.slot >= 0;
      for (auto& d : ls) {
        jl.kinds |= 1u << d.leaves[k].kind;
        if (jl.slot >= 0) small_sets &= d.cols[jl.slot].card < 64 * 32;
      }
      jl.bits_regs = (small_sets && (jl.kinds & (1u << LEAF_DICT_SET))) ? 1 : 0;
      // accept masks: a dictionary column of <= 64 values in every segment, leaves that are dictId ranges /
      // sets / constants (one bit extract per doc instead of a range compare or a set lookup)
      {
        const uint32_t ok = (1u << LEAF_DICT_RANGE) | (1u << LEAF_DICT_SET) | (1u << LEAF_CONST);
        int64_t maxc = 0;
        bool dict = jl.slot >= 0 && ls[0].cols[jl.slot].enc != ENC_RAW;
        for (auto& d : ls) if (jl.slot >= 0) maxc = std::max<int64_t>(maxc, d.cols[jl.slot].card);
        if (dict && !(jl.kinds & ~ok) && (jl.kinds & ((1u << LEAF_DICT_RANGE) | (1u << LEAF_DICT_SET))) && maxc <= 64 &&
            !env_is("PINOT_AMD_LEAF_MASKS", "0")) {
          jl.mask = maxc <= 32 ? 1 : 2;
          jl.bits_regs = 0;
          // fixed-bit columns of <= 6 bits in 256-thread scan / select blocks: an LDS accept table per
          // (clause, column) indexed by F = 4, 2 or 1 packed fields (4 / F lookups per lane of 4 docs), the
          // table at most 2^PINOT_AMD_LUT_MAX_BITS bytes (default 12: 4 KiB, one lookup per 4 docs for <= 3
          // bits). Tables of <= 2^8 bytes (one dword per LDS bank) never conflict, but the extra lookups
          // cost more than the ~6 conflict cycles they save: SSB 8.50 -> 8.56 ms at a 2^8 cap
          // (profiles/r04/sweep_ssb_lut_cap.txt) -- the select pass is latency-bound, not LDS-bound.
          const JitSlot& js = jp.slots[jl.slot];
          static const int lut_max = (int)std::min<int64_t>(12, std::max<int64_t>(6, env_i64("PINOT_AMD_LUT_MAX_BITS", 12)));
          if (js.enc == ENC_FIXED_BIT && js.bits >= 1 && js.bits <= 6 && !jp.partitioned &&
              (jp.scan_nsub == 1 || jp.select) && !env_is("PINOT_AMD_LEAF_LUT", "0"))
            jl.lut = 4 * js.bits <= lut_max ? 4 * js.bits : 2 * js.bits <= lut_max ? 2 * js.bits : js.bits;
        }
      }
      // larger dictId sets (<= 4096 words) are read from LDS, not from global memory per doc, by the
      // 256-thread blocks of non-partitioned plans (fused scans with nsub 1, every select pass)
      if (!jl.bits_regs && !jl.mask && jl.slot >= 0 && (jl.kinds & (1u << LEAF_DICT_SET)) && !jp.partitioned &&
          (jp.scan_nsub == 1 || jp.select) && !env_is("PINOT_AMD_LDS_SETS", "0")) {
        int64_t w = 0;
        for (auto& d : ls) w = std::max<int64_t>(w, (d.cols[jl.slot].card >> 5) + 1);
        int64_t used = 0;
        for (auto& o : jp.leaves) used += o.lds_words;
        w = (w + 3) & ~(int64_t)3;
        if (w <= 4096 && used + w <= 8192) jl.lds_words = (int)w;
      }
      jp.leaves.push_back(jl);
    }
    {  // pipeline depth: ~4 KiB in flight per wave (256 docs x bytes per row)
      double bpr = 0;
      for (size_t sl = 0; sl < jp.slots.size(); ++sl) {
        if (jp.select && !leaf_slot[sl]) continue;  // a select pass streams the filter columns only
        const JitSlot& js = jp.slots[sl];
        bpr += js.enc == ENC_FIXED_BIT ? (js.bits > 0 ? js.bits : 16) / 8.0 : js.enc == ENC_RAW ? value_size(js.type) : 0.0;
      }
      jp.depth = bpr <= 0 ? 1 : (int)std::min(4.0, std::max(1.0, std::ceil(4096.0 / (256.0 * bpr))));
      // a select step of G tiles loads G tiles per register set: the same bytes in flight with 1/G the sets
      if (jp.sel_group > 1) jp.depth = std::max(1, (jp.depth + jp.sel_group - 1) / jp.sel_group);
      if (const char* pd = knob("PINOT_AMD_PREFETCH")) jp.depth = std::max(1, std::min(8, atoi(pd)));
      if (env_is("PINOT_AMD_LANE_TABLES", "0")) {
        for (auto& js : jp.slots) js.dict_regs = 0;
        for (auto& jl : jp.leaves) jl.bits_regs = 0;
      }
      if (const char* pw = knob("PINOT_AMD_WAVES_PER_EU")) jp.waves_per_eu = std::max(0, std::min(8, atoi(pw)));
      // non-temporal column loads for wide-row fused scans (configs[1]: 3.58 -> 3.51 ms per 1B rows); the
      // narrow SSB select passes measured 1-3 % slower with them, the partitioned scatter 10 % slower
      jp.nt_loads = env_is("PINOT_AMD_NT_LOADS", "1") ||
                    (!env_is("PINOT_AMD_NT_LOADS", "0") && bpr >= 16.0 && !jp.partitioned && !jp.select);
      // XCD-aware tile ranges where blocks read per-segment tables beside the columns: the admission bitmaps
      // (128 KiB per segment for configs[3]) thrashed each XCD's L2 when its blocks spanned every segment
      // (default-limit configs[3] scatter: 20.1 -> 8.8 GB fetched per 400M rows, 4.87 -> 4.15 ms per plan;
      // profiles/r05/pmc_hcdef_xcd.txt). PINOT_AMD_XCD_REMAP=0|1 pins it.
      jp.xcd_remap = env_is("PINOT_AMD_XCD_REMAP", "1") || (jp.admit && !env_is("PINOT_AMD_XCD_REMAP", "0"));
#ifdef PINOT_AMD_DIAGNOSTICS
      // measurement-only variants that void the results (round-5 profiles): built with -DPINOT_AMD_DIAGNOSTICS only
      jp.diag_admit_off = env_is("PINOT_AMD_DIAG_ADMIT_OFF", "1");
      if (jp.partitioned) {
        const int64_t w = env_i64("PINOT_AMD_DIAG_REC_WRAP", 0);
        jp.diag_rec_wrap = (w >= 4096 && (w & (w - 1)) == 0) ? w : 0;
      }
#endif
    }
    if (jp.partitioned) {
      jit_layout_records(&jp);
      // sampled allotments replace the exact count pass once the strided histogram has >= 64 tiles
      const int64_t stride = env_i64("PINOT_AMD_SAMPLE_STRIDE", 32);
      jp.part_sampled = stride > 0 && tiles >= 64 * stride && !env_is("PINOT_AMD_PART_SAMPLED", "0");
      if (jp.part_sampled) L.part.sample_stride = stride;
      // scatter staging: as many records per partition as the LDS holds (up to 64); below 4 a run is
      // too short to pay for the staging round trip and records are written directly
      // PINOT_AMD_PART_SUB: 256-thread groups per scatter block (4: one CU-wide block per CU, 2 / 1: two / four
      // blocks per CU sharing the LDS)
      jp.part_sub = (int)env_i64("PINOT_AMD_PART_SUB", kPartSub);
      if (jp.part_sub != 1 && jp.part_sub != 2) jp.part_sub = kPartSub;
      const size_t stage_lds = (size_t)lds_max / (size_t)(kPartSub / jp.part_sub);
      // admission plans: the segment's admission bitmap beside the staging (an LDS read per doc instead of a
      // dependent global load; the scatter writes only the admitted docs' records, so a short staging serves)
      jp.admit_lds = jp.admit && jp.part_sub == kPartSub && !env_is("PINOT_AMD_ADMIT_LDS", "0") &&
                     jit_scatter_lds([&] { JitPlan t = jp; t.admit_lds = true; return t; }(), 4) <= stage_lds;
      int cap = 64;
      while (cap >= 4 && jit_scatter_lds(jp, cap) > stage_lds) --cap;
      jp.stage_cap = cap >= 4 ? cap : 0;
      if (const char* sc = knob("PINOT_AMD_STAGE_CAP")) jp.stage_cap = std::min(jp.stage_cap, atoi(sc));
      jp.flush_pct = (int)std::min<int64_t>(100, std::max<int64_t>(1, env_i64("PINOT_AMD_FLUSH_PCT", 85)));
      jp.flush_every = (int)std::min<int64_t>(64, std::max<int64_t>(1, env_i64("PINOT_AMD_FLUSH_EVERY", 1)));
      jp.flush_par = !env_is("PINOT_AMD_FLUSH_PAR", "0");
      jp.flush_group = env_is("PINOT_AMD_FLUSH_GROUP", "1");
      jp.scatter_batch = !env_is("PINOT_AMD_SCATTER_BATCH", "0");
    }
    {  // algorithmic bytes: each decoded column once (fixed-bit at its width, raw at its value width)
      for (size_t k = 0; k < L.segs.size(); ++k)
        for (int sl = 0; sl < nslots; ++sl) {
          const DevColumn& dc = ls[k].cols[sl];
          const double bpr = dc.enc == ENC_FIXED_BIT ? dc.bits / 8.0 : dc.enc == ENC_RAW ? (double)value_size(dc.type) : 0.0;
          L.col_bytes += bpr * (double)ls[k].num_docs;
        }
      std::vector<int> gate(nclauses, 1), has(nclauses, 0);
      for (const JitLeaf& jl : jp.leaves) {
        has[jl.clause] = 1;
        if (jl.kinds != (1u << LEAF_DOC_BITSET) || jl.negate) gate[jl.clause] = 0;
      }
      for (int c = 0; c < nclauses; ++c) L.gated |= gate[c] && has[c];
      if (jp.filter_gate) {  // filter columns of every doc, the key / value columns of the matching docs
        L.fgate = true;
        for (size_t k = 0; k < L.segs.size(); ++k)
          for (int sl = 0; sl < nslots; ++sl) {
            const double bpr = slot_bpr(ls[k].cols[sl]);
            if (leaf_slot[sl]) L.filter_bytes += bpr * (double)ls[k].num_docs;
            if (value_slot[sl] && k == 0) L.value_bpr += bpr;
          }
      }
      // gated plans: column loads D tiles ahead of their gate, gate words 2D ahead. Measured on the
      // inverted-index sweep, deeper pipelines only add registers (the gated loop is bound by its
      // per-tile overhead, not by load latency), so the row-width depth stays unless overridden.
      if (L.gated && knob("PINOT_AMD_GATE_DEPTH"))
        jp.depth = (int)std::min<int64_t>(std::max<int64_t>(env_i64("PINOT_AMD_GATE_DEPTH", 1), 1), 4);
    }
    L.jit = jit_get(jp, &r->jit_status);
    if (!L.jit) return fail(PINOT_AMD_EUNSUPPORTED, "scan kernel unavailable: %s", r->jit_status.c_str());
    if (jp.hash && jp.hash_spill && jp.hash_lds > 0 && !env_is("PINOT_AMD_HASH_DIRECT", "0")) {
      // the same scan without the LDS level, for keys without skew (a 64-slot table stays for the shared code)
      JitPlan jd = jp;
      jd.hash_direct = true;
      jd.hash_lds = 64;
      jd.hash_admit = 0;
      std::string err;
      L.jit_direct = jit_get(jd, &err);  // absent: the LDS-level plan serves every execution
      L.shmem_direct = (size_t)(hash_lds_bytes / jp.hash_lds) * 64;
      if (L.jit_direct && env_is("PINOT_AMD_HASH_DIRECT", "force")) r->hash_mode = 1;  // (tests: from the first execution)
      r->direct_place = env_is("PINOT_AMD_HASH_DIRECT", "force") || env_is("PINOT_AMD_HASH_DIRECT", "place");
    }
    if (r->admit) {
      // the admission's first-doc pass: the launch's filter + group key over each segment's prefix
      JitPlan jf = jp;
      jf.firstdoc = true;
      jf.admit = jf.lds = jf.partitioned = jf.select = jf.word_select = jf.atomic_gate = jf.sample = false;
      jf.part_sampled = false;
      jf.aggregate = false;
      jf.scan_nsub = 1;
      jf.vals.clear();
      jf.val_bits.clear();
      jf.val_off.clear();
      jf.rec_bytes = jf.stage_cap = jf.nparts = jf.key_shift = 0;
      for (auto& lf : jf.leaves) lf.lds_words = lf.lut = 0;
      L.jit_fd = jit_get(jf, &r->jit_status);
      if (!L.jit_fd) return fail(PINOT_AMD_EUNSUPPORTED, "first-doc kernel unavailable: %s", r->jit_status.c_str());
      if (r->q.num_keys <= kAdmitSeqMaxKeys && !env_is("PINOT_AMD_ADMIT_SEQ", "0")) {
        JitPlan js = jf;
        js.firstdoc = false;
        js.admitseq = true;
        std::string err;
        L.jit_as = jit_get(js, &err);  // absent: the first-doc admission below serves
      }
      std::vector<DevSegment> fs;
      int64_t ftiles = 0;
      for (size_t k = 0; k < L.segs.size(); ++k) {
        DevSegment d = ls[k];
        d.num_docs = r->a_prefix[L.segs[k]];
        // the prefix is the whole segment, or the segment cannot reach the limit (no pass: all admitted)
        d.pad = (d.num_docs == 0 || d.num_docs >= ls[k].num_docs) ? 1 : 0;
        d.tile_begin = ftiles;
        ftiles += (d.num_docs + kTileDocs - 1) / kTileDocs;
        fs.push_back(d);
      }
      if (int rc = L.d_fd_segs.alloc_copy(fs.data(), fs.size() * sizeof(DevSegment), 0)) return rc;
      L.fd_q = L.q;
      L.fd_q.total_tiles = ftiles;
      int nf = 0;
      if (occupancy_blocks(&nf, L.jit_fd->fn, kBlock, 0) != hipSuccess || nf < 1) nf = 1;
      L.fd_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * nf, ftiles));
      L.fd_full_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * nf, tiles));
    }
    if (r->seg_trim) {
      // the segment-level safe trim's presence pass: the launch's filter (+ numGroupsLimit admission) and group
      // key, each matching doc's ORDER BY rank marked in its segment's bitmap
      JitPlan js = jp;
      js.segpres = true;
      js.lds = js.partitioned = js.select = js.word_select = js.atomic_gate = js.sample = js.part_sampled = false;
      js.aggregate = false;
      js.scan_nsub = 1;
      js.sel_group = 1;
      js.vals.clear();
      js.val_bits.clear();
      js.val_off.clear();
      js.rec_bytes = js.stage_cap = js.nparts = js.key_shift = 0;
      for (auto& lf : js.leaves) lf.lds_words = lf.lut = 0;
      L.jit_sp = jit_get(js, &r->jit_status);
      if (!L.jit_sp) return fail(PINOT_AMD_EUNSUPPORTED, "presence kernel unavailable: %s", r->jit_status.c_str());
      int ns = 0;
      if (occupancy_blocks(&ns, L.jit_sp->fn, kBlock, 0) != hipSuccess || ns < 1) ns = 1;
      L.sp_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * ns, tiles));
    }
    L.scan_nsub = jp.partitioned ? 1 : jp.scan_nsub;
    L.shmem = jp.lds && !jp.partitioned ? (size_t)lds_bytes : jp.hash_lds ? (size_t)hash_lds_bytes : 0;
    for (const JitLeaf& jl : jp.leaves) L.shmem_sets += (size_t)jl.lds_words * 4;
    {  // LDS accept tables: one per (clause, column) mask group with a lookup table (jit.cpp's layout)
      std::vector<std::pair<int, int>> groups;
      for (const JitLeaf& jl : jp.leaves) {
        if (!jl.mask || !jl.lut) continue;
        const std::pair<int, int> g{jl.clause, jl.slot};
        if (std::find(groups.begin(), groups.end(), g) != groups.end()) continue;
        groups.push_back(g);
        L.shmem_sets += (size_t)(((1 << jl.lut) + 3) / 4) * 4;
      }
    }
    if (!jp.select) L.shmem += L.shmem_sets;  // a select pass has no table: its sets start at 0
    if (L.jit_direct) L.shmem_direct += L.shmem_sets;
    int per_cu = 1;
    if (jp.partitioned) {
      JitPlan ja = jp;  // companion direct-atomic scan for batches where the filter keeps few docs
      ja.partitioned = false;
      ja.lds = false;
      ja.scan_nsub = 1;
      ja.atomic_gate = true;
      ja.vals.clear();
      ja.val_off.clear();
      ja.rec_bytes = ja.stage_cap = ja.nparts = ja.key_shift = 0;
      for (auto& a : ja.accs) a.narrow = 0;  // HBM table: full 128-bit adds
      if (!env_is("PINOT_AMD_ATOMIC_HANDOVER", "0")) {
        std::string err;
        L.jit_atomic = jit_get(ja, &err);
      }
      L.part.atomic_threshold = L.jit_atomic ? L.docs / 64 : -1;
      if (env_is("PINOT_AMD_ATOMIC_HANDOVER", "force") && L.jit_atomic) L.part.atomic_threshold = INT64_MAX;
      // selectivity sample over every 32nd tile: when the extrapolated matches fall under the threshold
      // the count pass steps aside and the direct-atomic scan is the only full pass
      const int64_t stride = env_i64("PINOT_AMD_SAMPLE_STRIDE", 32);
      if (!jp.part_sampled && L.jit_atomic && stride > 0 && tiles >= 64 * stride) {
        JitPlan js = ja;
        js.atomic_gate = false;
        js.sample = true;
        js.aggregate = false;
        std::string err;
        L.jit_sample = jit_get(js, &err);
        if (L.jit_sample) L.part.sample_stride = stride;
      }
      L.part.nparts = jp.nparts;
      L.part.key_shift = jp.key_shift;
      for (size_t j = 0; j < part_vbase.size() && j < (size_t)kMaxAcc; ++j) L.part.vbase[j] = part_vbase[j];
      L.shmem_scatter = jit_scatter_lds(jp, jp.stage_cap);
      L.shmem_agg = (size_t)lds_arrays() * ((size_t)1 << jp.key_shift) * 8;
      L.shmem = (size_t)jp.nparts * 4;
      L.rec_bytes = jp.rec_bytes;
      L.part_sampled = jp.part_sampled;
      // sampled plans: the allotments may take 1.5 x docs + 256 records per partition (scaled to fit),
      // the overflow slab every doc (it can never fill up)
      L.region_cap = L.docs + L.docs / 2 + 256 * (int64_t)jp.nparts;
      max_rec = std::max(max_rec, (size_t)(jp.part_sampled ? L.region_cap : L.docs) * jp.rec_bytes + 256);
      if (jp.part_sampled) {
        max_slab = std::max(max_slab, (size_t)L.docs * jp.rec_bytes + 256);
        max_slab_docs = std::max(max_slab_docs, (size_t)L.docs + 64);
      }
      int nb = 0;
      L.part_sub = jp.part_sub;
      if (occupancy_blocks(&nb, L.jit->fn_scatter, kBlock * jp.part_sub, L.shmem_scatter) !=
              hipSuccess || nb < 1)
        nb = 1;
      per_cu = nb;
      int na = 0;
      if (occupancy_blocks(&na, L.jit->fn_agg, 1024, L.shmem_agg) != hipSuccess || na < 1)
        na = 1;
      L.agg_grid = cus * na;
      if (L.jit_atomic) {
        int nt = 0;
        if (occupancy_blocks(&nt, L.jit_atomic->fn, kBlock, 0) != hipSuccess || nt < 1) nt = 1;
        L.atomic_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * nt, tiles));
      }
      if (L.jit_sample) {
        int ns = 0;
        if (occupancy_blocks(&ns, L.jit_sample->fn, kBlock, 0) != hipSuccess || ns < 1) ns = 1;
        const int64_t vt = (tiles + L.part.sample_stride - 1) / L.part.sample_stride;
        L.sample_grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * ns, (vt + 3) / 4));
      }
      L.part.counts = (unsigned long long*)r->matched.p + 3 * li;
      L.part.check = (unsigned long long*)r->matched.p + 3 * nl + 2;
    } else if (jp.select) {
      // select pass: plain 256-thread blocks without LDS; gather pass: the table's block size and LDS
      L.select = true;
      L.word_select = jp.word_select;
      L.scan_nsub = 1;
      L.gather_threads = jp.lds ? kBlock * jp.scan_nsub : kBlock;
      int nb = 0, ng = 0;
      if (occupancy_blocks(&nb, L.jit->fn, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
      if (occupancy_blocks(&ng, L.jit->fn_gather, L.gather_threads, L.shmem) != hipSuccess ||
          ng < 1)
        ng = 1;
      // select blocks per CU: fewer, longer-running waves reserve vector chunks on the shared counter
      // fewer times (same-address atomics serialise at the memory side). The word-level select reads
      // little per doc and is bound by those reservations: 4 per CU (swept 1/2/4/8: 1 % inverted
      // 1.42/1.31/1.27/1.38 ms); the tile-level select needs its occupancy (2 per CU: SSB Q1.2 0.65 -> 0.92 ms)
      if (jp.word_select) nb = std::min(nb, 4);
      if (const char* e = knob("PINOT_AMD_SELECT_PER_CU")) nb = std::max(1, std::min(nb, atoi(e)));
      per_cu = nb;
      L.gather_grid = cus * ng;
      if (const char* e = knob("PINOT_AMD_GATHER_BLOCKS")) L.gather_grid = std::max(1, std::min(L.gather_grid, atoi(e)));
      for (size_t k = 0; k < L.segs.size(); ++k)
        for (int sl = 0; sl < nslots; ++sl) {
          const double bpr = slot_bpr(ls[k].cols[sl]);
          if (leaf_slot[sl]) L.filter_bytes += bpr * (double)ls[k].num_docs;
          if (value_slot[sl] && k == 0) L.value_bpr += bpr;
        }
      // Vector chunk a wave reserves at a time (plan-time counts): a power of two in [256, 4096] for the
      // tile-level select, [64, 4096] for the word-level one; runs split across chunks in both.
      int64_t m = 0, mt = 0;
      for (int si : L.segs) {  // + padding: one run per 256-doc wave tile, or per lane's 256 docs
        mt += seg_matched[si];
        m += seg_matched[si] + 3 * std::min<int64_t>(seg_matched[si], (segs[si]->num_docs + 255) / 256 + 1);
      }
      const int64_t waves = (int64_t)cus * nb * 4;
      // (runs continue over chunk ends, so a chunk is filled: the only padding is each wave's last chunk's
      // tail, written by the select and read by the gather -- a quarter of the matches a wave expects
      // keeps it small without many reservations)
      // (word level: about twice the matches a wave expects, its reservations measured as its bound)
      int64_t chunk = jp.word_select ? 64 : 256;
      const int64_t want = jp.word_select ? 2 * mt / std::max<int64_t>(waves, 1) : mt / std::max<int64_t>(4 * waves, 1);
      while (chunk < 4096 && chunk < want) chunk *= 2;
      L.q.sel_chunk = (int32_t)chunk;
      const int64_t per_chunk = chunk;
      const int64_t chunks = (m + per_chunk - 1) / per_chunk + waves + 1;
      max_sel = std::max<int64_t>(max_sel, chunks * chunk + 64);
    } else {
      int nb = 0;
      if (occupancy_blocks(&nb, L.jit->fn, kBlock * L.scan_nsub, L.shmem) != hipSuccess ||
          nb < 1)
        nb = 1;
      per_cu = nb;
    }
    // persistent grid: resident blocks per CU x CUs (a larger grid would only queue a tail)
    int64_t grid = (int64_t)cus * per_cu;
    if (grid > tiles) grid = std::max<int64_t>(tiles, 1);
    {
      const int sub = jp.partitioned ? jp.part_sub : L.scan_nsub;  // tiles a block takes per step
      if (sub > 1 && grid * sub > tiles) grid = std::max<int64_t>((tiles + sub - 1) / sub, 1);
    }
    if (L.part_sampled) {  // allotment tables of <= 2 x CUs scatter blocks sit behind the aggregation table
      grid = std::min<int64_t>(grid, 2 * (int64_t)cus);
      L.shmem_agg += (size_t)(2 * grid + 1) * 8;
    }
    L.grid = (int)grid;
    if (jp.partitioned) max_count_cells = std::max(max_count_cells, (size_t)jp.nparts * (size_t)grid * kPartCountRatio);
  }
  // partitioned work buffers, shared by the launches (they run one after another)
  if (r->kind == PLAN_PARTITIONED) {
    int maxp = 0;
    for (auto& L : r->launches) maxp = std::max(maxp, L.part.nparts);
    if (int rc = r->hist.alloc(max_count_cells * 4)) return rc;
    if (int rc = r->offs.alloc(max_count_cells * 8)) return rc;
    if (int rc = r->part_begin.alloc(((size_t)maxp + 1) * 8)) return rc;
    if (int rc = r->rec.alloc(max_rec)) return rc;
    int64_t hw_blocks = 0;  // per launch: count grid + scatter grid entries
    for (auto& L : r->launches) hw_blocks = std::max<int64_t>(hw_blocks, (int64_t)L.grid * (kPartCountRatio + 1));
    if (int rc = r->part_hw.alloc((size_t)hw_blocks * r->launches.size() * kHwWords * 4)) return rc;
    HIP_OK(hipMemset(r->part_hw.p, 0, r->part_hw.n));
    for (size_t li = 0; li < r->launches.size(); ++li)
      r->launches[li].part.hw = (uint32_t*)r->part_hw.p + (size_t)li * hw_blocks * kHwWords;
    if (max_slab > 0) {
      if (int rc = r->eff_begin.alloc(max_count_cells * 8 + 8)) return rc;
      if (int rc = r->ovf_n.alloc(8)) return rc;
      if (int rc = r->ovf_rec.alloc(max_slab)) return rc;
      if (int rc = r->ovf_part.alloc(max_slab_docs * 4)) return rc;
    }
    for (auto& L : r->launches) {
      L.part.hist = (uint32_t*)r->hist.p;
      L.part.offs = (int64_t*)r->offs.p;
      L.part.part_begin = (int64_t*)r->part_begin.p;
      L.part.rec = (uint8_t*)r->rec.p;
      if (L.part_sampled) {
        L.part.seg_grid = L.grid;
        L.part.ovf_n = (unsigned long long*)r->ovf_n.p;
        L.part.eff_begin = (int64_t*)r->eff_begin.p;
        L.part.ovf_rec = (uint8_t*)r->ovf_rec.p;
        L.part.ovf_part = (uint32_t*)r->ovf_part.p;
      }
    }
  }
  // selection vector + per-launch counters (entries appended, runs that did not fit)
  if (max_sel > 0) {
    if (int rc = r->sel.alloc((size_t)max_sel * 8)) return rc;
    if (int rc = r->sel_ctr.alloc(r->launches.size() * 16)) return rc;
    for (size_t li = 0; li < r->launches.size(); ++li) {
      Launch& L = r->launches[li];
      L.q.sel_entries = (unsigned long long*)r->sel.p;
      L.q.sel_count = (unsigned long long*)r->sel_ctr.p + 2 * li;
      L.q.sel_cap = max_sel;
    }
  }
  // accumulator tables
  if (r->kind == PLAN_HASH) {
    if (int rc = r->fkeys.alloc((size_t)r->nw * (size_t)r->fcap * 8)) return rc;
    if (int rc = r->acc.alloc((size_t)q.nacc * (size_t)r->fcap * 8)) return rc;
    if (base.hash_spill) {
      // spill regions: one per scan block, each holding up to the block's docs (every doc may miss), within
      // PINOT_AMD_SPILL_BYTES (default 8 GiB) for the regions and as much for their partition-major copy;
      // records past a region's capacity take the HBM table directly
      int64_t gmax = 1, per_max = 1;
      for (auto& L : r->launches) {
        gmax = std::max<int64_t>(gmax, L.grid);
        per_max = std::max<int64_t>(per_max, (L.q.total_tiles + L.grid - 1) / std::max(L.grid, 1));
      }
      int nval = 0;
      for (const JitAcc& a : base.accs) nval += a.op != ACC_HI && a.op != ACC_FIRST_DOC;
      r->spill_words = r->nw + nval;
      // (sizes per sub-region: a block's region is kSpillGroups of them, one per partition group -- a quarter of the
      // block's docs each when the spilled keys hash evenly, with a quarter more for the spread)
      const double budget = (double)env_i64("PINOT_AMD_SPILL_BYTES", (int64_t)8 << 30);
      const int64_t block_docs = per_max * kTileDocs;
      const int64_t sub_docs = block_docs / kSpillGroups + block_docs / (4 * kSpillGroups) + 256;
      r->spill_cap = std::max<int64_t>(64, std::min<int64_t>(std::min(sub_docs, block_docs),
          (int64_t)(budget / ((double)gmax * kSpillGroups * r->spill_words * 8.0))));
      // an earlier execution of this query shape over these segments needed more (its regions overflowed): up to
      // PINOT_AMD_SPILL_MAX_BYTES (default 32 GiB per copy); run_plan grows them the same way later
      const double maxb = (double)env_i64("PINOT_AMD_SPILL_MAX_BYTES", (int64_t)32 << 30);
      r->spill_cap_max = std::max<int64_t>(64, std::min<int64_t>(block_docs,
          (int64_t)(maxb / ((double)gmax * kSpillGroups * r->spill_words * 8.0))));
      if (const int64_t known = known_spill_capacity(r->cap_key))
        r->spill_cap = std::max(r->spill_cap, std::min(known, r->spill_cap_max));
      r->spill_grid = gmax;
      const size_t region_bytes = (size_t)gmax * kSpillGroups * (size_t)r->spill_cap * (size_t)r->spill_words * 8;
      if (int rc = r->sp_rec.alloc(region_bytes)) return rc;
      if (int rc = r->sp_sorted.alloc(region_bytes)) return rc;
      if (int rc = r->sp_cnt.alloc((size_t)gmax * kSpillGroups * 4)) return rc;
      if (int rc = r->sp_hist.alloc((size_t)kSpillMaxParts * (size_t)gmax * 4)) return rc;
      if (int rc = r->sp_offs.alloc((size_t)kSpillMaxParts * (size_t)gmax * 8)) return rc;
      if (int rc = r->sp_pbeg.alloc(((size_t)kSpillMaxParts + 1) * 8)) return rc;
      // second-level LDS table: every slot's key words and accumulator arrays in one CU's LDS
      r->spill_slots = (int)std::min<int64_t>(8192, (lds_max - 64) / ((int64_t)(r->nw + q.nacc) * 8));
      r->spill_agg_grid = cus;
    }
    if (r->trim) {
      const int64_t scap = *std::max_element(r->batch_cap.begin(), r->batch_cap.end());
      if (int rc = r->skeys.alloc((size_t)(r->nw + 1) * (size_t)scap * 8)) return rc;
      if (int rc = r->sacc.alloc((size_t)q.nacc * (size_t)scap * 8)) return rc;
      // per batch: bucket_base (1024-doc buckets of first docIds per segment)
      std::vector<int64_t> bb;
      int32_t maxnb = 0;
      int64_t maxbk = 0;
      for (int b = 0; b < r->nbatches; ++b) {
        r->batch_bucket_off.push_back((int64_t)bb.size());
        int64_t acc_b = 0;
        for (int si = 0; si < n; ++si) {
          if (seg_batch[si] != b) continue;
          bb.push_back(acc_b);
          acc_b += (segs[si]->num_docs + 1023) / 1024;
        }
        bb.push_back(acc_b);
        r->batch_buckets.push_back(acc_b);
        maxnb = std::max(maxnb, r->batch_nsegs[b]);
        maxbk = std::max(maxbk, acc_b);
      }
      if (int rc = r->d_bucket_base.alloc_copy(bb.data(), bb.size() * 8, 0)) return rc;
      if (int rc = r->t_hist.alloc((size_t)std::max<int64_t>(maxbk, 1) * 4)) return rc;
      if (int rc = r->t_distinct.alloc((size_t)maxnb * 8)) return rc;
      if (int rc = r->t_bstar.alloc((size_t)maxnb * 8)) return rc;
      if (int rc = r->t_rank.alloc((size_t)maxnb * 8)) return rc;
      if (int rc = r->t_dstar.alloc((size_t)maxnb * 8)) return rc;
      if (int rc = r->t_bitmap.alloc((size_t)maxnb * 16 * 8)) return rc;
      if (r->segsel) {
        const size_t E = r->segsel_st.size();
        if (int rc = r->ss_cnt.alloc((size_t)maxnb * 8)) return rc;
        if (int rc = r->ss_want.alloc((size_t)maxnb * 8)) return rc;
        if (int rc = r->ss_done.alloc((size_t)maxnb * 4)) return rc;
        if (int rc = r->ss_prefix.alloc((size_t)maxnb * 8)) return rc;
        if (int rc = r->ss_cut.alloc((size_t)maxnb * E * 8)) return rc;
        if (int rc = r->ss_hist.alloc((size_t)maxnb * 256 * 4)) return rc;
      }
    }
  } else {
    if (int rc = r->acc.alloc((size_t)std::max(q.nacc, 1) * (size_t)std::max<int64_t>(num_keys, 1) * 8)) return rc;
  }
  if (r->admit) {
    int64_t max_docs = 0;
    std::vector<int64_t> bb;
    for (int si = 0; si < n; ++si) {
      bb.push_back(r->a_buckets);
      const int64_t nb = (segs[si]->num_docs + 1023) / 1024 + 1;
      r->a_buckets += nb;
      r->a_max_buckets = std::max(r->a_max_buckets, nb);
      max_docs = std::max(max_docs, segs[si]->num_docs);
    }
    bb.push_back(r->a_buckets);
    r->a_cap = std::max<int64_t>(1, std::min<int64_t>(max_docs, num_keys));
    r->a_words = (num_keys + 31) / 32;
    if (int rc = r->a_first.alloc((size_t)n * (size_t)num_keys * 4)) return rc;
    HIP_OK(hipMemset(r->a_first.p, 0xFF, r->a_first.n));  // unseen; the admission resets what it touches
    if (int rc = r->a_seen.alloc((size_t)n * (size_t)r->a_cap * 4)) return rc;
    if (int rc = r->a_seen_n.alloc((size_t)n * 8)) return rc;
    if (int rc = r->a_bits.alloc((size_t)n * (size_t)r->a_words * 4)) return rc;
    if (int rc = r->a_hist.alloc((size_t)r->a_buckets * 4)) return rc;
    if (int rc = r->a_bbase.alloc_copy(bb.data(), bb.size() * 8, 0)) return rc;
    if (int rc = r->a_bstar.alloc((size_t)n * 8)) return rc;
    if (int rc = r->a_rank.alloc((size_t)n * 8)) return rc;
    if (int rc = r->a_dstar.alloc((size_t)n * 8)) return rc;
    if (int rc = r->a_bitmap.alloc((size_t)n * 16 * 8)) return rc;
    for (auto& L : r->launches) {
      for (DevQuery* dq : {&L.q, &L.fd_q}) {
        dq->admit = (const uint32_t*)r->a_bits.p;
        dq->admit_words = r->a_words;
        dq->first = (uint32_t*)r->a_first.p;
        dq->seen = (uint32_t*)r->a_seen.p;
        dq->seen_n = (unsigned long long*)r->a_seen_n.p;
        dq->seen_cap = r->a_cap;
      }
    }
  }
  if (r->seg_trim) {
    r->sp_nsegs = n;
    if (int rc = r->sp_bits.alloc((size_t)n * (size_t)r->sp_words * 8)) return rc;
    if (int rc = r->sp_cut.alloc((size_t)n * 8)) return rc;
    for (auto& L : r->launches) {
      L.q.seg_cut = (const unsigned long long*)r->sp_cut.p;
      L.q.seg_bits = (unsigned long long*)r->sp_bits.p;
      L.q.seg_words = r->sp_words;
    }
  }
  clk.mark("jit_alloc");
  HIP_OK(hipEventCreate(&r->ev0));
  HIP_OK(hipEventCreate(&r->ev1));
  const bool cap_from_cache = r->cap_known;
  if (int rc = run_plan(r)) return rc;
  clk.mark("launch");
  r->plan_bytes = g_tl_alloc_bytes - alloc0;
  if (r->kind == PLAN_HASH && !r->trim) {  // diagnostics: the table's slots, and whether an earlier execution sized it
    char b[96];
    snprintf(b, sizeof(b), ";hash_slots=%lld;hash_slots_remembered=%d", (long long)r->fcap, cap_from_cache ? 1 : 0);
    r->plan_timing += b;
  }
  *out = res.release();
  return 0;
}

// No C++ exception may cross the C ABI: a host allocation failure (a huge dense key space, a derived
// dictionary of a huge segment) comes back as PINOT_AMD_ENOMEM like a failed hipMalloc.
extern "C++" {
template <class F>
static int no_throw(const char* what, F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return fail(PINOT_AMD_ENOMEM, "%s: host allocation failed", what);
  } catch (const std::exception& e) {
    return fail(PINOT_AMD_EINVAL, "%s: %s", what, e.what());
  }
}
}

int pinot_amd_execute(pinot_amd_query* qq, pinot_amd_segment* const* segs_in, int32_t n, void* stream,
                      pinot_amd_result** out) {
  return no_throw("execute", [&] { return execute_impl(qq, segs_in, n, stream, false, out); });
}

int pinot_amd_execute_filter(pinot_amd_query* qq, pinot_amd_segment* const* segs_in, int32_t n, void* stream,
                             pinot_amd_result** out) {
  return no_throw("execute_filter", [&] { return execute_impl(qq, segs_in, n, stream, true, out); });
}

int pinot_amd_result_bitset(pinot_amd_result* r, int32_t segment_index, const uint64_t** h_d_bitset,
                            int64_t* h_num_words) {
  if (!r || !h_d_bitset || !h_num_words) return fail(PINOT_AMD_EINVAL, "result_bitset: bad arguments");
  if (r->bitsets.empty()) return fail(PINOT_AMD_EINVAL, "result_bitset: not a filter-only result");
  if (segment_index < 0 || segment_index >= (int32_t)r->bitsets.size())
    return fail(PINOT_AMD_EINVAL, "result_bitset: segment index %d out of range", segment_index);
  HIP_OK(hipStreamSynchronize(r->stream));
  *h_d_bitset = (const uint64_t*)r->bitsets[segment_index]->p;
  *h_num_words = r->bitset_words[segment_index];
  return 0;
}

int pinot_amd_execute_again(pinot_amd_result* r, void* stream) {
  if (!r) return fail(PINOT_AMD_EINVAL, "execute_again: null result");
  r->stream = (hipStream_t)stream;
  return run_plan(r);
}

int pinot_amd_result_destroy(pinot_amd_result* r) {
  if (!r) return 0;
  // the result's work is finished before its blocks go to the device pool (a caller still reading a
  // pinot_amd_result_bitset buffer on another stream must order that read before this call)
  const bool idle = hipStreamSynchronize(r->stream) == hipSuccess;
  if (idle && plan_cache_put(r)) return 0;  // kept for the next execute of its identity
  g_release_to_pool = idle;
  delete r;
  g_release_to_pool = false;
  return 0;
}

static int read_counters(pinot_amd_result* r, std::vector<unsigned long long>* c) {
  c->resize(r->matched.n / 8);
  HIP_OK(hipMemcpyAsync(c->data(), r->matched.p, r->matched.n, hipMemcpyDeviceToHost, r->stream));
  HIP_OK(hipStreamSynchronize(r->stream));
  return 0;
}

// Executions whose partitioned self-check failed, process-wide (pinot_amd_selfcheck_failures): the test suite fails
// its session on a nonzero count, so a caller that swallowed the error still shows up.
static std::atomic<long long> g_selfcheck_failures{0};

// One line per scatter block that failed the partitioned self-check: its hardware placement (XCC, SE, SH, CU from
// HW_ID / XCC_ID), the records it made and the records its count blocks counted (exact plans), and where those
// count blocks ran -- the evidence a failure leaves, whichever process hits it.
static std::string selfcheck_report(pinot_amd_result* r) {
  std::string out;
  for (size_t li = 0; li < r->launches.size(); ++li) {
    const Launch& L = r->launches[li];
    if (!L.part.hw || L.grid <= 0) continue;
    const int64_t cg = (int64_t)L.grid * kPartCountRatio, P = L.part.nparts;
    std::vector<uint32_t> hw((size_t)(cg + L.grid) * kHwWords);
    if (hipMemcpy(hw.data(), L.part.hw, hw.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) continue;
    std::vector<uint32_t> hist;  // (the launches share the histogram buffer: it holds the last launch's)
    if (!L.part_sampled && li + 1 == r->launches.size()) {
      hist.resize((size_t)P * cg);
      if (hipMemcpy(hist.data(), L.part.hist, hist.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) hist.clear();
    }
    auto where = [&](int64_t e) {
      const uint32_t id = hw[(size_t)e * kHwWords], x = hw[(size_t)e * kHwWords + 1];
      char b[96];
      snprintf(b, sizeof(b), "xcc %u se %u sh %u cu %u", x, (id >> 13) & 7u, (id >> 12) & 1u, (id >> 8) & 15u);
      return std::string(b);
    };
    int shown = 0;
    for (int64_t b = 0; b < L.grid && shown < 8; ++b) {
      const int64_t e = cg + b;
      if (hw[(size_t)e * kHwWords + 2] == 0) continue;
      ++shown;
      char line[256];
      snprintf(line, sizeof(line), "\n  launch %zu scatter block %lld (%s): %u %s, %u records made", li, (long long)b,
               where(e).c_str(), hw[(size_t)e * kHwWords + 2], L.part_sampled ? "records unaccounted" : "partition runs off",
               hw[(size_t)e * kHwWords + 3]);
      out += line;
      if (!hist.empty()) {
        int64_t counted = 0;
        for (int64_t c = b * kPartCountRatio; c < (b + 1) * kPartCountRatio && c < cg; ++c) {
          for (int64_t q = 0; q < P; ++q) counted += hist[(size_t)q * cg + c];
          out += "; count block " + std::to_string(c) + " (" + where(c) + ")";
          // the descriptors it read (checksummed as it read them) against the plan's upload
          const uint32_t rng = hw[(size_t)c * kHwWords + 3];
          const int s0 = (int)(rng >> 16), s1 = (int)(rng & 0xFFFFu);
          if (rng != 0 || hw[(size_t)c * kHwWords + 2] != 0) {
            uint64_t dk = 0xcbf29ce484222325ull;
            for (int k = s0; k <= s1 && k < (int)L.h_segs.size(); ++k) {
              const uint64_t* w = (const uint64_t*)&L.h_segs[(size_t)k];
              for (size_t i = 0; i < sizeof(DevSegment) / 8; ++i) dk = (dk ^ w[i]) * 0x100000001b3ull;
            }
            const bool same = (uint32_t)(dk ^ (dk >> 32)) == hw[(size_t)c * kHwWords + 2];
            out += std::string(same ? ", read its descriptors as planned" : ", READ DESCRIPTORS OTHER THAN THE PLAN'S") +
                   " (segments " + std::to_string(s0) + "-" + std::to_string(s1) + ")";
          }
        }
        out += "; counted " + std::to_string(counted);
      }
    }
    // the columns' HBM bytes against their fingerprints at staging: changed bytes vs a misread of intact ones
    std::vector<DevSegment> ds(L.segs.size());
    if (!ds.empty() &&
        hipMemcpy(ds.data(), L.d_segs.p, ds.size() * sizeof(DevSegment), hipMemcpyDeviceToHost) == hipSuccess) {
      int checked = 0, changed = 0;
      std::string which;
      for (size_t k = 0; k < ds.size(); ++k)
        for (int c = 0; c < kMaxSlots; ++c) {
          const void* d = ds[k].cols[c].data;
          StagedPrint sp{};
          {
            std::lock_guard<std::mutex> g(g_print_mu);
            auto it = g_prints.find(d);
            if (!d || it == g_prints.end()) continue;
            sp = it->second;
          }
          unsigned long long now = 0;
          if (device_fingerprint(d, sp.bytes, &now)) continue;
          ++checked;
          if (now != sp.print) {
            ++changed;
            if (changed <= 4) which += " (segment " + std::to_string(k) + " slot " + std::to_string(c) + ")";
          }
        }
      out += "\n  launch " + std::to_string(li) + ": " + std::to_string(changed) + " of " + std::to_string(checked) +
             " staged column buffers changed since staging" + which;
    }
    // the count pass run again on the same inputs (exact plans): does it reproduce its first histogram?
    if (!L.part_sampled && !hist.empty()) {
      DevBuf h2, m2, hw2;
      if (h2.alloc(hist.size() * 4) || m2.alloc(64) || hw2.alloc((size_t)cg * kHwWords * 4)) continue;
      (void)hipMemset(m2.p, 0, 64);
      DevPartition pc = L.part;
      pc.hist = (uint32_t*)h2.p;
      pc.hw = (uint32_t*)hw2.p;
      const DevSegment* segs = (const DevSegment*)L.d_segs.p;
      uint64_t* table = nullptr;
      uint64_t* const* bits = nullptr;
      unsigned long long* matched = (unsigned long long*)m2.p;
      DevHash h{};
      DevQuery q = L.q;
      void* args[] = {(void*)&segs, (void*)&q, (void*)&table, (void*)&bits, (void*)&matched, (void*)&pc, (void*)&h};
      std::vector<uint32_t> again(hist.size());
      if (hipModuleLaunchKernel(L.jit->fn, (unsigned)cg, 1, 1, (unsigned)(kBlock * L.part_sub), 1, 1, (unsigned)L.shmem,
                                nullptr, args, nullptr) != hipSuccess ||
          hipMemcpy(again.data(), h2.p, again.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
        continue;
      int64_t cells = 0, blocks = 0;
      std::string ex;
      for (int64_t c = 0; c < cg; ++c) {
        int64_t d = 0, t1 = 0, t2 = 0;
        for (int64_t q2 = 0; q2 < P; ++q2) {
          const size_t i = (size_t)q2 * cg + c;
          d += hist[i] != again[i];
          t1 += hist[i];
          t2 += again[i];
        }
        cells += d;
        if (d) {
          ++blocks;
          if (blocks <= 4)
            ex += " (count block " + std::to_string(c) + ": " + std::to_string(t1) + " -> " + std::to_string(t2) + ")";
        }
      }
      out += "\n  launch " + std::to_string(li) + ": the count pass run again differs in " + std::to_string(cells) +
             " cells of " + std::to_string(blocks) + " count blocks" + ex;
    }
  }
  return out;
}

// A partitioned execution whose self-check failed (DevPartition::check) fails its result: its groups and matched
// counts are never read. There is no re-execution: the cause of the round-5 misreads is gone (module loads, jit.cpp
// jit_get), and any future failure must surface, with the blocks' placement, instead of being retried away.
static int verify_partitioned(pinot_amd_result* r, const std::vector<unsigned long long>& c) {
  if (r->check_failed) return fail(PINOT_AMD_EINVAL, "%s", r->check_msg.c_str());
  if (r->kind == PLAN_HASH && r->direct_ran) {  // direct placement: every block filled its allotments
    const unsigned long long bad = c[3 * r->launches.size() + 2];
    if (bad == 0) return 0;
    r->check_failed = true;
    ++g_selfcheck_failures;
    r->check_msg = "hash plan direct placement: " + std::to_string(bad) +
                   " (partition, block) allotments got fewer records than the counting execution made; the result is void";
    fprintf(stderr, "pinot_amd: %s\n", r->check_msg.c_str());
    return fail(PINOT_AMD_EINVAL, "%s", r->check_msg.c_str());
  }
  if (r->kind != PLAN_PARTITIONED) return 0;
  const unsigned long long bad = c[3 * r->launches.size() + 2];
  if (bad == 0) return 0;
  r->check_failed = true;
  ++g_selfcheck_failures;
  r->check_msg = "partitioned plan self-check failed (" + std::to_string(bad) +
                 (r->launches.empty() || !r->launches[0].part_sampled ? " partition runs off their counted records"
                                                                       : " scatter blocks with unaccounted records") +
                 "); the result is void" + selfcheck_report(r);
  fprintf(stderr, "pinot_amd: %s\n", r->check_msg.c_str());
  return fail(PINOT_AMD_EINVAL, "%s", r->check_msg.c_str());
}

int pinot_amd_result_num_docs_matched(pinot_amd_result* r, int64_t* h_out) {
  if (!r || !h_out) return fail(PINOT_AMD_EINVAL, "num_docs_matched: bad arguments");
  std::vector<unsigned long long> c;
  if (int rc = read_counters(r, &c)) return rc;
  if (int rc = verify_partitioned(r, c)) return rc;
  // per launch: the scan / count pass and the direct-atomic scan both count every matching doc;
  // whichever ran has the total (partitioned plans run one of them)
  int64_t total = 0;
  for (size_t li = 0; li < r->launches.size(); ++li) total += (int64_t)std::max(c[3 * li], c[3 * li + 2]);
  *h_out = total;
  return 0;
}

int pinot_amd_result_algorithmic_bytes(pinot_amd_result* r, double* h_bytes) {
  if (!r || !h_bytes) return fail(PINOT_AMD_EINVAL, "algorithmic_bytes: bad arguments");
  std::vector<unsigned long long> c;
  if (int rc = read_counters(r, &c)) return rc;
  double b = 0;
  // inverted leaves: the selected bitmaps' bytes; the dense bitset written and read back only when the
  // expansion kernel runs (the fused inverted select of -fwselect plans keeps its words on-die)
  bool all_fused = !r->launches.empty();
  for (const auto& L : r->launches) all_fused &= L.fused;
  for (const auto& il : r->inv_leaves) b += il.alg_bytes + (all_fused ? 0.0 : il.bitset_bytes);
  for (size_t li = 0; li < r->launches.size(); ++li) {
    const Launch& L = r->launches[li];
    if (L.select) {  // filter columns of every doc, the vector written and read, the gathered columns
      const double m = (double)c[3 * li];
      b += L.filter_bytes + m * (16.0 + L.value_bpr);
    } else if (L.fgate) {
      b += L.filter_bytes + (double)std::max(c[3 * li], c[3 * li + 2]) * L.value_bpr;
    } else if (!L.gated || L.docs == 0) {
      b += L.col_bytes;
    } else {  // gated: only the rows that pass the filter need their column bytes
      const double m = (double)std::max(c[3 * li], c[3 * li + 2]);
      b += L.col_bytes * m / (double)L.docs;
    }
  }
  *h_bytes = b;
  return 0;
}

const char* pinot_amd_result_kernel_info(pinot_amd_result* r) {
  if (!r) return "";
  static thread_local std::string info;
  switch (r->kind) {
    case PLAN_PARTITIONED: info = "jit-partitioned"; break;
    case PLAN_HASH: info = r->trim ? "jit-hash-trim" : "jit-hash"; break;
    default: info = "jit";
  }
  // the hash plan's second level: the LDS level dropped, counting (region) or placing directly -- as of the next
  // execution for the counting step (the mode advances at the end of an execution)
  if (r->kind == PLAN_HASH && r->hash_mode > 0) info += r->direct_ran ? "+direct" : "+nolds";
  for (const auto& L : r->launches)
    if (L.select) {
      // wselect: the filter ran on 64-doc words; fwselect: fused with the inverted-index expansion
      info += L.fused ? "-fwselect" : L.word_select ? "-wselect" : "-select";
      break;
    }
  if (r->filter_gate) info += "+fgate";
  if (r->admit) {
    bool seq = !env_is("PINOT_AMD_ADMIT_SEQ", "0");
    for (auto& L : r->launches) seq &= L.jit_as != nullptr;
    info += seq ? "+admit-seq" : "+admit";
  }
  if (r->launches.size() > 1) info += " x" + std::to_string(r->launches.size());
  return info.c_str();
}

int pinot_amd_result_last_kernel_ms(pinot_amd_result* r, double* h_ms) {
  if (!r || !h_ms) return fail(PINOT_AMD_EINVAL, "last_kernel_ms: bad arguments");
  HIP_OK(hipEventSynchronize(r->ev1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, r->ev0, r->ev1));
  *h_ms = ms;
  return 0;
}

// Compact the non-empty groups on the device (presence bitset -> ballot / prefix-sum compaction ->
// gather) and copy only those rows to the host; hash-table groups are then put in key order.
// the execution's overflow counters: a full hash table or selection vector fails the result
static int check_overflow(pinot_amd_result* r) {
  hipStream_t st = r->stream;
  std::vector<unsigned long long> c;
  if (int rc = read_counters(r, &c)) return rc;
  if (r->ovf_pending) {
    // an execution at a remembered capacity skipped its overflow check: if some doc found no slot after all,
    // grow and run the plan again (it then checks, and grows further, itself)
    r->ovf_pending = false;
    if (c[3 * r->launches.size() + 1] != 0) {
      bool grown = false;
      if (int rc = grow_hash(r, &grown)) return rc;
      if (grown) {
        if (int rc = run_plan(r)) return rc;
        if (int rc = read_counters(r, &c)) return rc;
      }
    }
  }
  if (int rc = verify_partitioned(r, c)) return rc;
  if (c[3 * r->launches.size() + 1] != 0)
    return fail(PINOT_AMD_EOVERFLOW, "group hash table full (%lld docs without a slot); raise PINOT_AMD_HASH_TABLE_BYTES",
                (long long)c[3 * r->launches.size() + 1]);
  if (r->spill_words > 0 && r->spill_grid > 0 && !r->cap_key.empty()) {
    // the last launch's per-block record counts: a region that ran out sizes the next execution's regions
    std::vector<uint32_t> cnt((size_t)r->spill_grid * kSpillGroups);
    HIP_OK(hipMemcpyAsync(cnt.data(), r->sp_cnt.p, cnt.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const int64_t mx = (int64_t)*std::max_element(cnt.begin(), cnt.end());
    if (mx > r->spill_cap) remember_spill_capacity(r->cap_key, mx + mx / 8);
    // most matching docs missed the LDS level (keys without skew): the next executions drop it -- one counting the
    // blocks' records per partition, then direct placement (no region pass)
    bool all_direct = !r->launches.empty();
    for (const Launch& L : r->launches) all_direct &= L.jit_direct != nullptr;
    const size_t last = r->launches.size() - 1;
    int64_t spilled = 0;
    for (uint32_t x : cnt) spilled += x;
    if (r->hash_mode == 0 && all_direct && c[3 * last] > 0 && 2 * spilled >= (int64_t)c[3 * last]) r->hash_mode = 1;
  }
  if (r->sel_ctr.n) {
    std::vector<unsigned long long> sc(r->sel_ctr.n / 8);
    HIP_OK(hipMemcpyAsync(sc.data(), r->sel_ctr.p, r->sel_ctr.n, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (size_t li = 0; li < sc.size() / 2; ++li)
      if (sc[2 * li + 1] != 0)
        return fail(PINOT_AMD_EOVERFLOW, "selection vector of launch %zu overflowed (%llu runs dropped)", li, sc[2 * li + 1]);
  }
  return 0;
}

// the group table of the result: the plan's (dense or hash) or, after a cross-rank merge, the merged one
struct GroupTable {
  bool hash;
  int64_t slots;
  int nwk;
  const unsigned long long* keys;  // hash tables: nwk x slots key words
  const uint64_t* acc;
};
static GroupTable group_table(const pinot_amd_result* r) {
  if (r->merged) return {true, r->mcap, r->mnw, (const unsigned long long*)r->mkeys.p, (const uint64_t*)r->macc.p};
  if (r->kind == PLAN_HASH) return {true, r->fcap, r->nw, (const unsigned long long*)r->fkeys.p, (const uint64_t*)r->acc.p};
  return {false, r->q.num_keys, 1, nullptr, (const uint64_t*)r->acc.p};
}

// device compaction of a group table's non-empty slots (COUNT != 0), ascending: slot indices in r->c_idx
static int compact_slots(pinot_amd_result* r, const GroupTable& T, hipStream_t st, int64_t* ng) {
  DevBuf &bits = r->c_bits, &counts = r->c_counts, &total = r->c_total, &idx = r->c_idx;
  if (int rc = bits.ensure((size_t)((T.slots + 63) / 64 + 1) * 8)) return rc;
  HIP_OK(launch_presence_bitset(T.acc, T.slots, (unsigned long long*)bits.p, st));
  const int64_t nc = compact_num_chunks(T.slots);
  if (int rc = counts.ensure((size_t)nc * 8)) return rc;
  if (int rc = total.ensure(8)) return rc;
  HIP_OK(launch_bitset_count((const uint64_t*)bits.p, T.slots, (int64_t*)counts.p, (int64_t*)total.p, st));
  HIP_OK(hipMemcpyAsync(ng, total.p, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (*ng > 0) {
    if (int rc = idx.ensure((size_t)*ng * 4)) return rc;
    HIP_OK(launch_bitset_compact((const uint64_t*)bits.p, T.slots, (const int64_t*)counts.p, (int32_t*)idx.p, st));
  }
  return 0;
}

static int server_trim(pinot_amd_result* r);

static int compact_groups(pinot_amd_result* r) {
  if (r->compacted) return 0;
  hipStream_t st = r->stream;
  const int nacc = std::max(r->q.nacc, 1);
  if (int rc = check_overflow(r)) return rc;
  if (r->num_group_by == 0 || r->q.nacc == 0) {
    r->ngroups = 1;
    r->ckeys.assign(1, 0);
    r->cacc.assign((size_t)nacc, 0);
    if (r->q.nacc > 0) {
      HIP_OK(hipMemcpyAsync(r->cacc.data(), r->acc.p, (size_t)nacc * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    }
    r->compacted = true;
    return 0;
  }
  const GroupTable T = group_table(r);
  const bool hash = T.hash;
  const int nwk = T.nwk;
  DevBuf &idx = r->c_idx, &okeys = r->c_okeys, &oacc = r->c_oacc;
  int64_t ng = 0;
  if (int rc = compact_slots(r, T, st, &ng)) return rc;
  r->ngroups = ng;
  r->ckeys.resize((size_t)ng * nwk);
  r->cacc.resize((size_t)ng * nacc);
  if (ng > 0) {
    if (int rc = okeys.ensure((size_t)ng * nwk * 8)) return rc;
    if (int rc = oacc.ensure((size_t)ng * nacc * 8)) return rc;
    HIP_OK(launch_gather_groups((const int32_t*)idx.p, ng, T.keys, nwk, T.slots, T.acc, nacc, (uint64_t*)okeys.p,
                                (uint64_t*)oacc.p, st));
    const void* src_keys = okeys.p;
    const void* src_acc = oacc.p;
    if (hash && ng > 1) {
      // ascending global key (column ids compared from the last column to the first) = the packed key words
      // as one integer, word nwk - 1 most significant: a stable LSD radix sort over the words on the device
      // (derive.hip), then the sorted rows cross PCIe. (A host sort of 1.34M two-column keys took ~0.4 s.)
      std::vector<int> word_bits(nwk, 1);
      for (int j = 0; j < r->num_group_by; ++j)
        word_bits[r->pack_word[j]] = std::max(word_bits[r->pack_word[j]], r->pack_shift[j] + r->pack_bits[j]);
      DevBuf &sk = r->c_skeys, &sa = r->c_sacc, &ss = r->c_sscratch;
      if (int rc = sk.ensure((size_t)ng * nwk * 8)) return rc;
      if (int rc = sa.ensure((size_t)ng * nacc * 8)) return rc;
      if (int rc = ss.ensure(sort_rows_scratch(ng))) return rc;
      HIP_OK(sort_rows_by_key((const uint64_t*)okeys.p, nwk, word_bits.data(), (const uint64_t*)oacc.p, nacc, ng, ss.p,
                              (uint64_t*)sk.p, (uint64_t*)sa.p, st));
      src_keys = sk.p;
      src_acc = sa.p;
    }
    HIP_OK(hipMemcpyAsync(r->ckeys.data(), src_keys, r->ckeys.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(r->cacc.data(), src_acc, r->cacc.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  if (int rc = server_trim(r)) return rc;
  r->compacted = true;
  return 0;
}

int pinot_amd_result_num_groups_limit_reached(pinot_amd_result* r, int32_t* h_out) {
  if (!r || !h_out) return fail(PINOT_AMD_EINVAL, "num_groups_limit_reached: bad arguments");
  *h_out = 0;
  // without a segment that can hold numGroupsLimit keys the flag is false; otherwise the trim pass
  // computed GroupByOperator's numGroups >= numGroupsLimit per segment
  if (r->num_group_by == 0 || !r->limit_possible) return 0;
  std::vector<unsigned long long> c;
  if (int rc = read_counters(r, &c)) return rc;
  if (int rc = verify_partitioned(r, c)) return rc;  // a void execution reports no flag either
  *h_out = c[3 * r->launches.size()] != 0 ? 1 : 0;
  return 0;
}

int pinot_amd_result_num_groups(pinot_amd_result* r, int64_t* h_out) {
  if (!r || !h_out) return fail(PINOT_AMD_EINVAL, "num_groups: bad arguments");
  if (r->num_group_by == 0) {
    *h_out = 1;
    return 0;
  }
  if (int rc = compact_groups(r)) return rc;
  *h_out = r->ngroups;
  return 0;
}

static double decode_ordered(uint64_t u, int op) {
  if (op == ACC_MIN && u == ~0ull) return INFINITY;
  if (op == ACC_MAX && u == 0ull) return -INFINITY;
  const uint64_t b = (u >> 63) ? (u & 0x7FFFFFFFFFFFFFFFull) : ~u;
  double d;
  memcpy(&d, &b, 8);
  return d;
}

// final value of aggregation a from a group's accumulator words A (AggregationFunction.extractFinalResult):
// *v as double, *vi the exact int64 for COUNT / SUMLONG / integer SUM within int64
static void final_value(const pinot_amd_result* r, const uint64_t* A, int a, double* v_out, int64_t* vi_out) {
  const int acc = r->agg_acc[a];
  const int op = r->q.acc_op[acc];
  const uint64_t w = A[acc];
  const uint64_t cnt = r->q.nacc ? A[0] : 0;
  double v;
  int64_t vi = 0;
  // exact 128-bit integer sum (lo, hi) -> correctly rounded double
  auto sum128 = [&](int64_t* exact) -> double {
    const __int128 s = (__int128)(((unsigned __int128)A[acc + 1] << 64) | (unsigned __int128)w);
    *exact = (s >= (__int128)INT64_MIN && s <= (__int128)INT64_MAX) ? (int64_t)s : INT64_MIN;
    return (double)s;
  };
  switch (r->agg_type[a]) {
    case PINOT_AMD_AGG_COUNT:
      vi = (int64_t)cnt;
      v = (double)vi;
      break;
    case PINOT_AMD_AGG_AVG: {
      int64_t ex;
      const double s = op == ACC_SUM_F64 ? ([&] { double d; memcpy(&d, &w, 8); return d; })() : sum128(&ex);
      v = cnt ? s / (double)cnt : -INFINITY;  // AvgAggregationFunction: empty -> DEFAULT_FINAL_RESULT
      break;
    }
    case PINOT_AMD_AGG_MIN:
    case PINOT_AMD_AGG_MAX:
      v = decode_ordered(w, op);
      break;
    case PINOT_AMD_AGG_MINMAXRANGE:  // MinMaxRangeAggregationFunction.extractFinalResult: max - min
      v = decode_ordered(A[r->agg_acc2[a]], ACC_MAX) - decode_ordered(w, ACC_MIN);
      break;
    default:
      if (op == ACC_SUM_F64) {
        memcpy(&v, &w, 8);
      } else if (op == ACC_SUM_I128) {
        v = sum128(&vi);
      } else {
        vi = (int64_t)w;
        v = (double)vi;
      }
  }
  *v_out = v;
  *vi_out = vi;
}

// merged-key id of group column j of compacted group g
static int64_t group_key_id(const pinot_amd_result* r, int64_t g, int j) {
  const bool hash = r->kind == PLAN_HASH || r->merged;
  if (hash) {
    const int nwk = r->merged ? r->mnw : r->nw;
    return (int64_t)((r->ckeys[(size_t)g * nwk + r->pack_word[j]] >> r->pack_shift[j]) & (((uint64_t)1 << r->pack_bits[j]) - 1));
  }
  const int64_t sz = (int64_t)std::max<size_t>(r->keys[j]->size(), 1);
  return ((int64_t)r->ckeys[(size_t)g] / std::max<int64_t>(r->key_stride[j], 1)) % sz;
}

// Double.compare: -0.0 < 0.0, NaN above everything (the order TableResizer's comparators give doubles)
static int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  const uint64_t ka = java_double_order(a), kb = java_double_order(b);
  return ka < kb ? -1 : ka > kb ? 1 : 0;
}

// The combine's IndexedTable at the server (GroupByUtils.java:104-149, IndexedTable.finish): without
// ORDER BY the table stops taking new groups at LIMIT (the first LIMIT groups it receives; here the first
// in ascending key order, which is Pinot's order for one segment with an array-based holder); with ORDER
// BY it keeps the top trimSize = max(5 * LIMIT, minServerGroupTrimSize) groups by the ORDER BY (ties:
// ascending key), sorted. Pinot additionally trims to trimSize whenever its table passes trimThreshold =
// max(groupTrimThreshold, 2 * trimSize) groups while merging segments; with more groups than that the
// surviving set depends on its merge order (the device result keeps the exact top trimSize).
static int server_trim(pinot_amd_result* r) {
  r->srv_trimmed = false;
  if (r->srv_limit < 0 || r->num_group_by == 0) return 0;
  const int nacc = std::max(r->q.nacc, 1);
  const bool hash = r->kind == PLAN_HASH || r->merged;
  const int nwk = r->merged ? r->mnw : hash ? r->nw : 1;
  int64_t keep;
  if (r->srv_order.empty()) {
    keep = r->srv_limit;
  } else if ((r->srv_safe && r->srv_limit < r->srv_sort_threshold) || r->srv_final) {
    // safe trim with a small LIMIT: the sorted combine (SortedGroupByCombineOperator, CombinePlanNode.java:
    // 150-154) merges the segments' top-LIMIT records keeping LIMIT (GroupByUtils.getSortedReduceMerger);
    // every group of the global top LIMIT is in each of its segments' top LIMIT, so those are exact.
    // serverReturnFinalResult without HAVING: the IndexedTable's result size is LIMIT (GroupByUtils.java:134)
    keep = r->srv_limit;
  } else {
    keep = r->srv_min_trim > 0 ? std::max<int64_t>(r->srv_limit * 5, r->srv_min_trim) : INT64_MAX;
  }
  const int64_t ng = r->ngroups;
  if (ng <= keep && r->srv_order.empty()) return 0;
  std::vector<int64_t> perm((size_t)ng);
  for (int64_t g = 0; g < ng; ++g) perm[(size_t)g] = g;
  if (!r->srv_order.empty()) {
    // sort keys per group: merged-key ids for group columns (dictionary order = value order), final values
    const size_t no = r->srv_order.size();
    std::vector<double> fv((size_t)ng * no);
    std::vector<int64_t> kid((size_t)ng * no);
    for (int64_t g = 0; g < ng; ++g)
      for (size_t o = 0; o < no; ++o) {
        const auto& ob = r->srv_order[o];
        if (ob.kind == 0) {
          kid[(size_t)g * no + o] = group_key_id(r, g, ob.index);
        } else {
          int64_t vi;
          final_value(r, &r->cacc[(size_t)g * nacc], ob.index, &fv[(size_t)g * no + o], &vi);
        }
      }
    auto less = [&](int64_t a, int64_t b) {
      for (size_t o = 0; o < no; ++o) {
        const auto& ob = r->srv_order[o];
        int c;
        if (ob.kind == 0) {
          const int64_t x = kid[(size_t)a * no + o], y = kid[(size_t)b * no + o];
          c = x < y ? -1 : x > y ? 1 : 0;
        } else {
          c = java_double_compare(fv[(size_t)a * no + o], fv[(size_t)b * no + o]);
        }
        if (c != 0) return ob.asc ? c < 0 : c > 0;
      }
      return a < b;  // ascending key (compacted order)
    };
    if (keep < ng) {
      std::nth_element(perm.begin(), perm.begin() + keep, perm.end(), less);
      perm.resize((size_t)keep);
    }
    std::sort(perm.begin(), perm.end(), less);
  } else {
    perm.resize((size_t)keep);
  }
  std::vector<uint64_t> k2(perm.size() * nwk), a2(perm.size() * nacc);
  for (size_t i = 0; i < perm.size(); ++i) {
    std::copy_n(&r->ckeys[(size_t)perm[i] * nwk], nwk, &k2[i * nwk]);
    std::copy_n(&r->cacc[(size_t)perm[i] * nacc], nacc, &a2[i * nacc]);
  }
  r->ckeys.swap(k2);
  r->cacc.swap(a2);
  r->srv_trimmed = (int64_t)perm.size() < ng;
  r->ngroups = (int64_t)perm.size();
  return 0;
}

int pinot_amd_result_fetch(pinot_amd_result* r, int64_t cap, int64_t* h_keys, double* h_values, int64_t* h_values_i64,
                           int64_t* h_num_fetched) {
  if (!r || cap < 0 || !h_num_fetched) return fail(PINOT_AMD_EINVAL, "fetch: bad arguments");
  if (int rc = no_throw("fetch", [&] { return compact_groups(r); })) return rc;
  const int na = (int)r->agg_type.size();
  const int nacc = std::max(r->q.nacc, 1);
  const bool hash = r->kind == PLAN_HASH || r->merged;
  const int nwk = r->merged ? r->mnw : hash ? r->nw : 1;
  if (r->ngroups > cap) return fail(PINOT_AMD_EOVERFLOW, "fetch: %lld groups exceed capacity %lld", (long long)r->ngroups,
                                    (long long)cap);
  // the groups converted in slices on up to 8 host threads (1M groups: key decode + final values)
  auto convert = [&](int64_t g0, int64_t g1) {
  for (int64_t g = g0; g < g1; ++g) {
    const uint64_t* A = &r->cacc[(size_t)g * nacc];
    if (h_keys) {
      int64_t rem = hash ? 0 : (int64_t)r->ckeys[(size_t)g];
      for (int j = 0; j < r->num_group_by; ++j) {
        const MergedKeyColumn& m = *r->keys[j];
        int64_t id;
        if (hash) {
          id = (int64_t)((r->ckeys[(size_t)g * nwk + r->pack_word[j]] >> r->pack_shift[j]) & (((uint64_t)1 << r->pack_bits[j]) - 1));
        } else {
          const int64_t sz = (int64_t)std::max<size_t>(m.size(), 1);
          id = rem % sz;
          rem /= sz;
        }
        int64_t o;
        if (m.type == T_STRING) o = id;
        else if (is_float(m.type)) memcpy(&o, &m.vd[id], 8);
        else o = m.vi[id];
        h_keys[g * r->num_group_by + j] = o;
      }
    }
    for (int a = 0; a < na; ++a) {
      double v;
      int64_t vi;
      final_value(r, A, a, &v, &vi);
      if (h_values) h_values[g * na + a] = v;
      if (h_values_i64) h_values_i64[g * na + a] = vi;
    }
  }
  };
  const int64_t ng = r->ngroups;
  const int nt = ng >= (1 << 17) ? (int)std::min<unsigned>(8u, std::max(1u, std::thread::hardware_concurrency())) : 1;
  if (nt <= 1) {
    convert(0, ng);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(convert, ng * t / nt, ng * (t + 1) / nt);
    for (auto& t : th) t.join();
  }
  *h_num_fetched = r->ngroups;
  return 0;
}

int pinot_amd_result_fetch_intermediate(pinot_amd_result* r, int64_t cap, double* h_pairs, int64_t* h_num_fetched) {
  if (!r || cap < 0 || !h_pairs || !h_num_fetched) return fail(PINOT_AMD_EINVAL, "fetch_intermediate: bad arguments");
  if (int rc = no_throw("fetch_intermediate", [&] { return compact_groups(r); })) return rc;
  if (r->ngroups > cap)
    return fail(PINOT_AMD_EOVERFLOW, "fetch_intermediate: %lld groups exceed capacity %lld", (long long)r->ngroups,
                (long long)cap);
  const int na = (int)r->agg_type.size();
  const int nacc = std::max(r->q.nacc, 1);
  std::vector<double> v((size_t)r->ngroups * na);
  std::vector<int64_t> vi((size_t)r->ngroups * na);
  int64_t got = 0;
  if (int rc = pinot_amd_result_fetch(r, r->ngroups, nullptr, v.data(), vi.data(), &got)) return rc;
  for (int64_t g = 0; g < r->ngroups; ++g) {
    const uint64_t* A = &r->cacc[(size_t)g * nacc];
    for (int a = 0; a < na; ++a) {
      double* out = h_pairs + ((size_t)g * na + a) * 2;
      const int acc = r->agg_acc[a];
      switch (r->agg_type[a]) {
        case PINOT_AMD_AGG_AVG: {  // AvgPair(sum, count)
          const double cnt = (double)(r->q.nacc ? A[0] : 0);
          if (r->q.acc_op[acc] == ACC_SUM_F64) memcpy(&out[0], &A[acc], 8);
          else out[0] = (double)(__int128)(((unsigned __int128)A[acc + 1] << 64) | (unsigned __int128)A[acc]);
          out[1] = cnt;
          break;
        }
        case PINOT_AMD_AGG_MINMAXRANGE:  // MinMaxRangePair(min, max)
          out[0] = decode_ordered(A[acc], ACC_MIN);
          out[1] = decode_ordered(A[r->agg_acc2[a]], ACC_MAX);
          break;
        default:
          out[0] = v[(size_t)g * na + a];
          out[1] = 0;
      }
    }
  }
  *h_num_fetched = r->ngroups;
  return 0;
}

const char* pinot_amd_result_string_key(pinot_amd_result* r, int32_t j, int64_t id) {
  if (!r || j < 0 || j >= r->num_group_by) return nullptr;
  const MergedKeyColumn& m = *r->keys[j];
  if (m.type != T_STRING || id < 0 || id >= (int64_t)m.vs.size()) return nullptr;
  return m.vs[id].c_str();
}

int pinot_amd_result_check_word(pinot_amd_result* r, void** h_d_word) {
  if (!r || !h_d_word) return fail(PINOT_AMD_EINVAL, "check_word: bad arguments");
  *h_d_word = (unsigned long long*)r->matched.p + 3 * r->launches.size() + 2;
  return 0;
}

int64_t pinot_amd_selfcheck_failures(void) { return (int64_t)g_selfcheck_failures.load(); }

int pinot_amd_result_accumulators(pinot_amd_result* r, int32_t* h_num_slots, int64_t* h_num_key_slots,
                                  void** h_slot_ptrs, int32_t* h_slot_ops) {
  if (!r || !h_num_slots || !h_num_key_slots) return fail(PINOT_AMD_EINVAL, "accumulators: bad arguments");
  if (r->kind == PLAN_HASH || r->merged)
    return fail(PINOT_AMD_EUNSUPPORTED, "accumulators: hash-table (and merged) results merge by value "
                                        "(pinot_amd_result_export_groups / pinot_amd_result_merge_groups)");
  *h_num_slots = r->q.nacc;
  *h_num_key_slots = r->q.num_keys;
  for (int a = 0; a < r->q.nacc; ++a) {
    if (h_slot_ptrs) h_slot_ptrs[a] = (uint8_t*)r->acc.p + (size_t)a * r->q.num_keys * 8;
    if (h_slot_ops) {
      switch (r->q.acc_op[a]) {
        case ACC_SUM_F64: h_slot_ops[a] = 1; break;
        case ACC_MIN: h_slot_ops[a] = 2; break;
        case ACC_MAX: h_slot_ops[a] = 3; break;
        case ACC_SUM_I128: h_slot_ops[a] = 4; break;
        case ACC_HI: h_slot_ops[a] = 5; break;
        default: h_slot_ops[a] = 0;  // COUNT, SUM_I64
      }
    }
  }
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Cross-rank merge by value (the broker reduce, GroupByDataTableReducer.java:258, on the device)
// ------------------------------------------------------------------------------------------------
// The hash plan's key packing over the result's merged key space (identical on every rank once the
// global key space is installed), and the dense table's mixed-radix strides.
static int key_pack(const pinot_amd_result* r, DevKeyPack* kp) {
  memset(kp, 0, sizeof(*kp));
  kp->ncols = r->num_group_by;
  if (kp->ncols > kMaxGroupCols) return fail(PINOT_AMD_EUNSUPPORTED, "export: %d group columns", kp->ncols);
  std::vector<int64_t> sizes;
  for (int j = 0; j < kp->ncols; ++j) sizes.push_back((int64_t)std::max<size_t>(r->keys[j]->size(), 1));
  std::vector<int> word, shift;
  pack_key_words(sizes, &word, &shift);  // the hash plan's packing
  for (int j = 0; j < kp->ncols; ++j) {
    kp->word[j] = word[j];
    kp->shift[j] = shift[j];
    kp->size[j] = sizes[j];
    kp->stride[j] = j < (int)r->key_stride.size() ? std::max<int64_t>(r->key_stride[j], 1) : 1;
  }
  kp->nw = word.empty() ? 1 : word.back() + 1;
  if (kp->nw > kMaxKeyWords) return fail(PINOT_AMD_EUNSUPPORTED, "group key of %d words exceeds %d", kp->nw, kMaxKeyWords);
  return 0;
}

// accumulators exported per group: every array but the trimming plans' first-docId (always last)
static int export_nacc(const pinot_amd_result* r) { return r->fd_acc >= 0 ? r->fd_acc : r->q.nacc; }

// the stream a cross-rank call runs on: the caller's (ordered after the result's own stream through an
// event, whatever the caller did), or the result's; r->stream itself is never replaced
static int call_stream(pinot_amd_result* r, void* stream, hipStream_t* out) {
  *out = r->stream;
  if (!stream || (hipStream_t)stream == r->stream) return 0;
  if (!r->ev_x) HIP_OK(hipEventCreateWithFlags(&r->ev_x, hipEventDisableTiming));
  HIP_OK(hipEventRecord(r->ev_x, r->stream));
  HIP_OK(hipStreamWaitEvent((hipStream_t)stream, r->ev_x, 0));
  *out = (hipStream_t)stream;
  return 0;
}

int pinot_amd_result_export_groups(pinot_amd_result* r, uint64_t* d_keys, uint64_t* d_acc, int64_t cap,
                                   int32_t* h_key_words, int32_t* h_num_acc, int64_t* h_num_groups, void* stream) {
  if (!r || !h_key_words || !h_num_acc || !h_num_groups || cap < 0)
    return fail(PINOT_AMD_EINVAL, "export_groups: bad arguments");
  return no_throw("export_groups", [&]() -> int {
    if (r->num_group_by == 0 || r->q.nacc == 0)
      return fail(PINOT_AMD_EUNSUPPORTED, "export_groups: not a GROUP BY result with aggregations");
    hipStream_t st;
    if (int rc = call_stream(r, stream, &st)) return rc;
    DevKeyPack kp;
    if (int rc = key_pack(r, &kp)) return rc;
    // a merged result exports its merged table (keys already packed this way: a key-partitioned
    // cross-rank merge exports each rank's merged share again)
    if (!r->merged && r->kind == PLAN_HASH && kp.nw != r->nw)
      return fail(PINOT_AMD_EINVAL, "export_groups: key packing mismatch");
    if (r->merged && kp.nw != r->mnw) return fail(PINOT_AMD_EINVAL, "export_groups: merged key packing mismatch");
    if (int rc = check_overflow(r)) return rc;
    const GroupTable T = group_table(r);
    const DevBuf& idx = r->c_idx;
    int64_t ng = 0;
    if (int rc = compact_slots(r, T, st, &ng)) return rc;
    *h_key_words = kp.nw;
    *h_num_acc = export_nacc(r);
    *h_num_groups = ng;
    if (!d_keys || !d_acc) return 0;  // sizing call
    if (ng > cap) return fail(PINOT_AMD_EOVERFLOW, "export_groups: %lld groups exceed capacity %lld", (long long)ng,
                              (long long)cap);
    HIP_OK(launch_export_groups((const int32_t*)idx.p, ng, T.keys, T.slots, T.acc, export_nacc(r), kp, d_keys, d_acc, st));
    HIP_OK(hipStreamSynchronize(st));
    return 0;
  });
}

int pinot_amd_result_merge_groups(pinot_amd_result* r, const uint64_t* d_keys, const uint64_t* d_acc, int64_t n,
                                  void* stream) {
  if (!r || n < 0 || (n > 0 && (!d_keys || !d_acc))) return fail(PINOT_AMD_EINVAL, "merge_groups: bad arguments");
  return no_throw("merge_groups", [&]() -> int {
    if (r->num_group_by == 0 || r->q.nacc == 0)
      return fail(PINOT_AMD_EUNSUPPORTED, "merge_groups: not a GROUP BY result with aggregations");
    hipStream_t st;
    if (int rc = call_stream(r, stream, &st)) return rc;
    DevKeyPack kp;
    if (int rc = key_pack(r, &kp)) return rc;
    r->merged = false;
    const int64_t mcap = next_pow2(std::max<int64_t>(64, 2 * n));
    if (mcap > ((int64_t)1 << 31)) return fail(PINOT_AMD_EUNSUPPORTED, "merge_groups: %lld rows", (long long)n);
    // the merged table's buffers grow and are reused across merges (one per step in a multi-GPU loop)
    if (int rc = r->mkeys.ensure((size_t)mcap * kp.nw * 8)) return rc;
    if (int rc = r->macc.ensure((size_t)mcap * r->q.nacc * 8)) return rc;
    if (int rc = r->movf.ensure(8)) return rc;
    r->mcap = mcap;
    r->mnw = kp.nw;
    HIP_OK(hipMemsetAsync(r->mkeys.p, 0xFF, (size_t)mcap * kp.nw * 8, st));
    HIP_OK(hipMemsetAsync(r->movf.p, 0, 8, st));
    HIP_OK(launch_init_acc((uint64_t*)r->macc.p, r->q, mcap, st));
    HIP_OK(launch_merge_rows(d_keys, d_acc, n, kp.nw, export_nacc(r), (unsigned long long*)r->mkeys.p, mcap,
                             (uint64_t*)r->macc.p, r->q, (unsigned long long*)r->movf.p, st));
    unsigned long long ovf = 0;
    HIP_OK(hipMemcpyAsync(&ovf, r->movf.p, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (ovf) return fail(PINOT_AMD_EOVERFLOW, "merge_groups: %llu rows without a slot", ovf);
    if (r->kind != PLAN_HASH) {  // fetch decodes merged keys with the hash plan's packing
      r->pack_word.assign(kp.word, kp.word + kp.ncols);
      r->pack_shift.assign(kp.shift, kp.shift + kp.ncols);
      r->pack_bits.clear();
      for (int j = 0; j < kp.ncols; ++j) r->pack_bits.push_back(bits_for(kp.size[j]));
    }
    r->merged = true;
    r->compacted = false;
    return 0;
  });
}

const char* pinot_amd_result_plan_timing(pinot_amd_result* r) { return r ? r->plan_timing.c_str() : ""; }
