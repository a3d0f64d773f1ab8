// kernels.hip — gfx950 kernels for Pinot's segment scan / filter / aggregation / group-by.
//
// Layout in HBM: every column keeps the bytes Pinot writes for it — the fixed-bit
// forward index as the big-endian MSB-first bit stream, raw values big-endian — so nothing is
// transcoded at staging time; the kernels byte-swap in registers (v_perm_b32).
//
// The fused scan (filter + group key + aggregation) is generated per query shape and compiled with
// hipRTC (jit.cpp); this file holds the fixed kernels around it: accumulator initialisation, the
// hash-table trimming / merge / result compaction passes, the low-level operators (forward-index
// decode, bitsets, docId compaction), inverted-index expansion and raw-chunk decompression.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "device_types.h"
#include "../../include/pinot_amd.h"

namespace pamd {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap64(uint32_t hi_word_be, uint32_t lo_word_be) {
  // bytes as stored: hi_word_be holds the first 4 bytes (most significant in BE order)
  return ((uint64_t)bswap32(hi_word_be) << 32) | bswap32(lo_word_be);
}
__device__ __forceinline__ double u64_as_double(uint64_t u) { return __longlong_as_double((long long)u); }

__device__ __forceinline__ uint32_t sel4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
}

// 4 consecutive values of a big-endian MSB-first bit stream starting at doc0 (FixedBitIntReader /
// PinotDataBitSet.readInt semantics). A 5-dword window always covers 4 values of <= 31 bits.
__device__ __forceinline__ void load_fixed_bit4(const uint8_t* data, int bits, int64_t doc0, int64_t out[4]) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(data);
  const int64_t bit0 = doc0 * bits;
  const int64_t w0 = bit0 >> 5;
  const uint32_t r = (uint32_t)(bit0 & 31);
  const uint32_t x0 = bswap32(w[w0]), x1 = bswap32(w[w0 + 1]), x2 = bswap32(w[w0 + 2]),
                 x3 = bswap32(w[w0 + 3]), x4 = bswap32(w[w0 + 4]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t p = r + (uint32_t)(k * bits);
    const uint32_t i = p >> 5, sh = p & 31;
    const uint64_t win = ((uint64_t)sel4(i, x0, x1, x2, x3) << 32) | sel4(i, x1, x2, x3, x4);
    out[k] = (int64_t)((win << sh) >> (64 - bits));
  }
}

// ------------------------------------------------------------------------------------------------
// wave reductions (64 lanes)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
// accumulator update at a table word (LDS or HBM; generic address space resolves both); an
// ACC_SUM_I128 low word carries into `hi` (the next array's word)
__device__ __forceinline__ void acc_apply(int32_t op, uint64_t* p, uint64_t* hi, uint64_t bits, uint64_t hbits) {
  switch (op) {
    case ACC_COUNT:
    case ACC_SUM_I64:
      atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
    case ACC_SUM_I128: {
      const uint64_t old = (uint64_t)atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      const uint64_t h = hbits + (uint64_t)(old + bits < old);
      if (h) atomicAdd(reinterpret_cast<unsigned long long*>(hi), (unsigned long long)h);
      break;
    }
    case ACC_HI:
      break;
    case ACC_SUM_F64:
      unsafeAtomicAdd(reinterpret_cast<double*>(p), u64_as_double(bits));
      break;
    case ACC_MAX:
      atomicMax(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
    default:  // ACC_MIN, ACC_FIRST_DOC
      atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
  }
}

__device__ __forceinline__ uint64_t acc_identity(int32_t op) {
  if (op == ACC_MIN || op == ACC_FIRST_DOC) return ~0ull;
  return 0ull;  // COUNT/SUM: 0 (also +0.0 for f64); MAX: ordered 0 is below every double
}

__global__ void init_acc_kernel(uint64_t* acc, int64_t num_keys, DevQuery q) {
  const int64_t n = (int64_t)q.nacc * num_keys;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc[i] = acc_identity(q.acc_op[i / num_keys]);
}

// The plan's end for whole-query-narrow 128-bit sums (JitAcc::hbm_narrow): their low words were added mod
// 2^64 with non-returning atomics (no carries), and the true sums fit int64, so each high word is the low
// word's sign. acc[lo * n + i] / acc[(lo + 1) * n + i] for every array index lo in arrs.
__global__ void sext_hi_kernel(uint64_t* acc, int64_t n, const int32_t* arrs, int32_t narr) {
  for (int32_t a = 0; a < narr; ++a) {
    const uint64_t* lo = acc + (int64_t)arrs[a] * n;
    uint64_t* hi = acc + (int64_t)(arrs[a] + 1) * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
      hi[i] = (int64_t)lo[i] < 0 ? ~0ull : 0ull;
  }
}

// ------------------------------------------------------------------------------------------------
// Hash-table GROUP BY passes (DevHash layout; the scan itself is the JIT kernel)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
// slot of the nw-word key kw in a table (inserted if absent; lock-free word-by-word CAS, see
// DevHash), -1 when every slot holds another key
// max_probe > 0: give up after that many slots (a crowded table: the caller counts the doc as overflow and the
// host grows the table) -- unbounded, every new key of a full table walked all of it (a cold wide-key execution
// whose first table was too small spent 68 s in one spill aggregation)
__device__ int64_t hash_find_rt(unsigned long long* keys, int64_t cap, int nw, const uint64_t* kw, int64_t max_probe = 0) {
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int w = 0; w < nw; ++w) x = fmix64(x ^ kw[w]);
  const uint64_t mask = (uint64_t)cap - 1ull;
  uint64_t i = hash_home(x, cap);
  const int64_t lim = max_probe > 0 && max_probe < cap ? max_probe : cap;
  for (int64_t n = 0; n < lim; ++n) {
    bool ok = true;
    for (int w = 0; w < nw && ok; ++w) {
      unsigned long long* pw = keys + (uint64_t)w * (uint64_t)cap + i;
      unsigned long long cur = __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == ~0ull) {
        cur = atomicCAS(pw, ~0ull, (unsigned long long)kw[w]);
        if (cur == ~0ull) cur = kw[w];
      }
      ok = cur == kw[w];
    }
    if (ok) return (int64_t)i;
    i = (i + 1ull) & mask;
  }
  return -1;
}

// numGroupsLimit trimming (DictionaryBasedGroupKeyGenerator.java:351-363 / the map holders'
// getGroupId(rawKey, numGroupsLimit)): within a segment Pinot admits group keys in the order their
// first matching doc appears, until numGroupsLimit keys are held; later keys are dropped. The trim
// scan table is keyed by (key, segment) and tracks each entry's first matching docId; first docIds
// of one segment are distinct (one key per doc), so the admitted keys are exactly those whose first
// docId is <= the limit-th smallest first docId of the segment (dstar). Found in four passes:
//   1. per segment: distinct entries, and a histogram of first docIds in 1024-doc buckets
//   2. per segment: the bucket holding the limit-th first docId and its rank inside the bucket
//   3. the first docIds of that bucket as a 1024-bit map
//   4. the rank-th set bit -> dstar
__global__ void trim_count_kernel(const unsigned long long* keys, int64_t cap, int nw_seg, const uint64_t* acc,
                                  int fd_acc, const int64_t* bucket_base, uint32_t* hist,
                                  unsigned long long* seg_distinct) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    if (acc[i] == 0ull) continue;
    const int64_t s = (int64_t)keys[(uint64_t)(nw_seg - 1) * (uint64_t)cap + i];
    const uint64_t fd = acc[(uint64_t)fd_acc * (uint64_t)cap + i];
    atomicAdd(&seg_distinct[s], 1ull);
    atomicAdd(&hist[bucket_base[s] + (int64_t)(fd >> 10)], 1u);
  }
}

// one block per segment; bstar[s] = -1: the segment holds <= limit keys (nothing trimmed)
// strict (dense admission over a segment prefix): a segment holding exactly `limit` keys is cut at the
// limit-th first docId too, since keys beyond the prefix may exist; otherwise <= limit keys admit all
__global__ void __launch_bounds__(256) trim_select_kernel(int64_t limit, const int64_t* bucket_base,
                                                          const uint32_t* hist, const unsigned long long* seg_distinct,
                                                          int64_t* bstar, int64_t* rank,
                                                          unsigned long long* limit_reached, int strict) {
  __shared__ int64_t wtot[4];
  __shared__ int64_t carry;
  const int s = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nd = (int64_t)seg_distinct[s];
  // GroupByOperator.java:133: numGroupsLimitReached = numGroups >= numGroupsLimit
  if (threadIdx.x == 0 && nd >= limit) atomicOr(limit_reached, 1ull);
  if (strict ? nd < limit : nd <= limit) {
    if (threadIdx.x == 0) bstar[s] = -1;
    return;
  }
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int64_t b0 = bucket_base[s], b1 = bucket_base[s + 1];
  for (int64_t base = b0; base < b1; base += 256) {
    const int64_t i = base + threadIdx.x;
    const int64_t x = i < b1 ? (int64_t)hist[i] : 0;
    int64_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int w = 0; w < wave; ++w) before += wtot[w];
    const int64_t c_incl = before + incl, c_excl = c_incl - x;
    if (i < b1 && c_excl < limit && c_incl >= limit) {
      bstar[s] = i - b0;
      rank[s] = limit - c_excl;  // 1-based rank of dstar among the bucket's first docIds
    }
    __syncthreads();
    if (threadIdx.x == 255) carry = c_incl;
    __syncthreads();
    if (carry >= limit) break;
  }
}

__global__ void trim_bitmap_kernel(const unsigned long long* keys, int64_t cap, int nw_seg, const uint64_t* acc,
                                   int fd_acc, const int64_t* bstar, unsigned long long* bitmap) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    if (acc[i] == 0ull) continue;
    const int64_t s = (int64_t)keys[(uint64_t)(nw_seg - 1) * (uint64_t)cap + i];
    const uint64_t fd = acc[(uint64_t)fd_acc * (uint64_t)cap + i];
    if (bstar[s] >= 0 && (int64_t)(fd >> 10) == bstar[s])
      atomicOr(&bitmap[s * 16 + (int64_t)((fd & 1023) >> 6)], 1ull << (fd & 63));
  }
}

__global__ void trim_cutoff_kernel(int32_t nsegs, const int64_t* bstar, const int64_t* rank,
                                   const unsigned long long* bitmap, int64_t* dstar) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  if (bstar[s] < 0) {
    dstar[s] = INT64_MAX;
    return;
  }
  int64_t r = rank[s];
  int64_t out = -1;
  for (int w = 0; w < 16 && out < 0; ++w) {
    uint64_t m = bitmap[(int64_t)s * 16 + w];
    const int c = __popcll(m);
    if (r > c) {
      r -= c;
      continue;
    }
    while (--r > 0) m &= m - 1;
    out = bstar[s] * 1024 + w * 64 + __builtin_ctzll(m);
  }
  dstar[s] = out;
}

// Dense numGroupsLimit admission (key spaces a dense table holds; the same first-seen semantics as the
// hash trimming above, DictionaryBasedGroupKeyGenerator.java:351-363). The first-doc pass (JIT,
// MODE_FIRSTDOC) over a prefix of each segment leaves first[s * nk + key] = the key's first matching
// docId and the list seen[s * cap ..] of the keys it saw (seen_n[s] of them). Then, over those lists only:
//   admit_hist:   histogram of first docIds in 1024-doc buckets per segment (LDS, one block per chunk)
//   trim_select:  the bucket and rank of the limit-th first docId (strict: exactly `limit` keys seen in a
//                 prefix still cut there)
//   admit_bucket: that bucket's first docIds as a 1024-bit map; trim_cutoff: the limit-th first docId dstar
//   admit_bits:   bit key of segment s's bitmap = first <= dstar[s] (all ones when nothing is cut), and
//                 first[] reset to "unseen" for the next execution
__global__ void __launch_bounds__(256) admit_hist_kernel(const uint32_t* first, int64_t nk, const uint32_t* seen,
                                                         const unsigned long long* seen_n, int64_t cap, int64_t chunk,
                                                         const int64_t* bucket_base, uint32_t* hist) {
  extern __shared__ uint32_t lh[];
  const int s = blockIdx.y;
  const int64_t n = (int64_t)min((unsigned long long)cap, seen_n[s]);
  const int64_t b0 = bucket_base[s], nb = bucket_base[s + 1] - b0;
  const int64_t i0 = (int64_t)blockIdx.x * chunk;
  if (i0 >= n) return;
  const int64_t i1 = min(n, i0 + chunk);
  for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = 0u;
  __syncthreads();
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint32_t f = first[(int64_t)s * nk + seen[(int64_t)s * cap + i]];
    atomicAdd(&lh[min((int64_t)(f >> 10), nb - 1)], 1u);
  }
  __syncthreads();
  for (int64_t b = threadIdx.x; b < nb; b += blockDim.x)
    if (lh[b]) atomicAdd(&hist[b0 + b], lh[b]);
}

__global__ void admit_bucket_kernel(const uint32_t* first, int64_t nk, const uint32_t* seen,
                                    const unsigned long long* seen_n, int64_t cap, int32_t nsegs, const int64_t* bstar,
                                    unsigned long long* bitmap) {
  const int s = blockIdx.y;
  if (s >= nsegs || bstar[s] < 0) return;
  const int64_t n = (int64_t)min((unsigned long long)cap, seen_n[s]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = first[(int64_t)s * nk + seen[(int64_t)s * cap + i]];
    if ((int64_t)(f >> 10) == bstar[s]) atomicOr(&bitmap[(int64_t)s * 16 + ((f & 1023u) >> 6)], 1ull << (f & 63u));
  }
}

// one block row per segment: untrimmed segments get every bit; trimmed ones the keys whose first docId
// is <= dstar (words zeroed by the host first); first[] entries of the listed keys go back to unseen
__global__ void admit_bits_kernel(uint32_t* first, int64_t nk, const uint32_t* seen, const unsigned long long* seen_n,
                                  int64_t cap, const int64_t* dstar, uint32_t* admit, int64_t words) {
  const int s = blockIdx.y;
  uint32_t* A = admit + (int64_t)s * words;
  const int64_t n = (int64_t)min((unsigned long long)cap, seen_n[s]);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (dstar[s] == INT64_MAX) {
    for (int64_t w = t; w < words; w += stride) A[w] = ~0u;
  }
  for (int64_t i = t; i < n; i += stride) {
    const uint32_t key = seen[(int64_t)s * cap + i];
    uint32_t* f = first + (int64_t)s * nk + key;
    if (dstar[s] != INT64_MAX && (int64_t)*f <= dstar[s]) atomicOr(&A[key >> 5], 1u << (key & 31u));
    *f = 0xFFFFFFFFu;
  }
}

// ------------------------------------------------------------------------------------------------
// Segment-level group trim over a hash plan's (key, segment) scan table (SegSelStage; GroupByOperator.java:
// 157-175): per segment, the `keep` smallest entries in the chain of stage keys. Stage by stage, 8 bits per pass,
// each segment's candidates (entries tied with the cutoff on every earlier stage) are histogrammed on the current
// digit (segsel_hist) and the digit holding the wanted rank is picked (segsel_pick); a stage whose cutoff value
// holds exactly the wanted count ends the segment's selection there (done = stage), else its ties go on.
// ------------------------------------------------------------------------------------------------
// exact (lo, hi) two's complement 128-bit integer -> double, rounded to nearest even (as the host's
// (double)(__int128) in final_value)
__device__ __forceinline__ double i128_to_double_rn(uint64_t lo, uint64_t hi) {
  const bool neg = (int64_t)hi < 0;
  if (neg) {
    lo = ~lo + 1ull;
    hi = ~hi + (lo == 0ull ? 1ull : 0ull);
  }
  if (hi == 0ull && lo < (1ull << 53)) {
    const double d = (double)lo;
    return neg ? -d : d;
  }
  int e;  // bit index of the leading one
  uint64_t m, rest;
  if (hi) {
    const int lz = __clzll((long long)hi);
    e = 127 - lz;
    m = lz ? (hi << lz) | (lo >> (64 - lz)) : hi;
    rest = lz ? lo << lz : lo;
  } else {
    const int lz = __clzll((long long)lo);
    e = 63 - lz;
    m = lo << lz;
    rest = 0ull;
  }
  uint64_t mant = m >> 11;
  const uint64_t r = m & 0x7FFull;
  if (r > 0x400ull || (r == 0x400ull && (rest != 0ull || (mant & 1ull)))) mant += 1ull;
  const double d = ldexp((double)mant, e - 52);
  return neg ? -d : d;
}
__device__ __forceinline__ double decode_ordered_dev(uint64_t u, int op) {
  if (op == ACC_MIN && u == ~0ull) return __builtin_inf();
  if (op == ACC_MAX && u == 0ull) return -__builtin_inf();
  const uint64_t b = (u >> 63) ? (u & 0x7FFFFFFFFFFFFFFFull) : ~u;
  return __longlong_as_double((long long)b);
}
// Double.compare order as an unsigned key (every NaN one value above +inf, -0.0 below 0.0)
__device__ __forceinline__ uint64_t java_double_key(double d) {
  uint64_t b = d != d ? 0x7FF8000000000000ull : (uint64_t)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// extractFinalResult of a SegSelStage's aggregation from scan-table slot i (host.cpp final_value)
__device__ double segsel_final(const SegSelStage& g, const DevQuery& q, const uint64_t* acc, int64_t cap, int64_t i) {
  auto A = [&](int a) { return acc[(uint64_t)a * (uint64_t)cap + (uint64_t)i]; };
  const int op = q.acc_op[g.acc];
  const uint64_t w = A(g.acc);
  const uint64_t cnt = A(0);
  auto sum = [&]() -> double {
    if (op == ACC_SUM_F64) return u64_as_double(w);
    if (op == ACC_SUM_I128) return i128_to_double_rn(w, A(g.acc + 1));
    return i128_to_double_rn(w, (int64_t)w < 0 ? ~0ull : 0ull);
  };
  switch (g.agg_type) {
    case PINOT_AMD_AGG_COUNT: return (double)cnt;
    case PINOT_AMD_AGG_AVG: return cnt ? sum() / (double)cnt : -__builtin_inf();
    case PINOT_AMD_AGG_MIN:
    case PINOT_AMD_AGG_MAX: return decode_ordered_dev(w, op);
    case PINOT_AMD_AGG_MINMAXRANGE: return decode_ordered_dev(A(g.acc2), ACC_MAX) - decode_ordered_dev(w, ACC_MIN);
    default: return sum();
  }
}
__device__ uint64_t segsel_key(const SegSelStage& g, const DevQuery& q, const unsigned long long* keys,
                               const uint64_t* acc, int64_t cap, int64_t i) {
  if (g.kind == 2) return keys[(uint64_t)g.kword * (uint64_t)cap + (uint64_t)i];
  if (g.kind == 1) {
    const uint64_t k = java_double_key(segsel_final(g, q, acc, cap, i));
    return g.desc ? ~k : k;
  }
  uint64_t u = 0ull;
  for (int c = 0; c < g.ncols; ++c) {
    const uint64_t w = keys[(uint64_t)g.word[c] * (uint64_t)cap + (uint64_t)i];
    uint64_t id = (w >> g.shift[c]) & (g.bits[c] >= 64 ? ~0ull : ((1ull << g.bits[c]) - 1ull));
    if (g.flip[c]) id = (uint64_t)g.size[c] - 1ull - id;
    u += id * (uint64_t)g.mul[c];
  }
  return u;
}
// a present entry of the scan table that the numGroupsLimit cutoff admitted; its segment (batch index)
__device__ __forceinline__ bool segsel_entry(const unsigned long long* keys, int64_t cap, int nw, const uint64_t* acc,
                                             int fd_acc, const int64_t* dstar, int64_t i, int64_t* s) {
  if (acc[i] == 0ull) return false;
  *s = (int64_t)keys[(uint64_t)nw * (uint64_t)cap + (uint64_t)i];
  return !dstar || acc[(uint64_t)fd_acc * (uint64_t)cap + (uint64_t)i] <= (uint64_t)dstar[*s];
}
// entry i against its segment's cutoffs on stages [0, upto): -1 below, 0 tied on all, 1 above
__device__ __forceinline__ int segsel_cmp(const SegSelStage* st, const DevQuery& q, const unsigned long long* keys,
                                          const uint64_t* acc, int64_t cap, int64_t i, const uint64_t* cut, int upto) {
  for (int j = 0; j < upto; ++j) {
    const uint64_t u = segsel_key(st[j], q, keys, acc, cap, i);
    if (u != cut[j]) return u < cut[j] ? -1 : 1;
  }
  return 0;
}

__global__ void segsel_count_kernel(const unsigned long long* keys, int64_t cap, int nw, const uint64_t* acc, int fd_acc,
                                    const int64_t* dstar, unsigned long long* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s;
    if (segsel_entry(keys, cap, nw, acc, fd_acc, dstar, i, &s)) atomicAdd(&cnt[s], 1ull);
  }
}
// want[s] = keep; done[s] = -2 when the segment holds <= keep candidates (nothing trimmed), else -1 (selecting)
__global__ void segsel_init_kernel(int32_t nsegs, int64_t keep, const unsigned long long* cnt, int64_t* want, int32_t* done,
                                   uint64_t* prefix) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  want[s] = keep;
  done[s] = (int64_t)cnt[s] <= keep ? -2 : -1;
  prefix[s] = 0ull;
}
__global__ void segsel_hist_kernel(const unsigned long long* keys, int64_t cap, int nw, const uint64_t* acc, int fd_acc,
                                   const int64_t* dstar, DevQuery q, const SegSelStage* st, int nst, int j, int d,
                                   const int32_t* done, const uint64_t* prefix, const uint64_t* cut, uint32_t* hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s;
    if (!segsel_entry(keys, cap, nw, acc, fd_acc, dstar, i, &s) || done[s] != -1) continue;
    if (j > 0 && segsel_cmp(st, q, keys, acc, cap, i, cut + s * nst, j) != 0) continue;
    const uint64_t u = segsel_key(st[j], q, keys, acc, cap, i);
    if (d < 7 && (u >> (8 * (d + 1))) != (prefix[s] >> (8 * (d + 1)))) continue;
    atomicAdd(&hist[s * 256 + (int64_t)((u >> (8 * d)) & 255ull)], 1u);
  }
}
__global__ void segsel_pick_kernel(int32_t nsegs, int nst, int j, int d, const uint32_t* hist, int64_t* want, int32_t* done,
                                   uint64_t* prefix, uint64_t* cut) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs || done[s] != -1) return;
  int64_t cum = 0;
  for (int b = 0; b < 256; ++b) {
    const int64_t h = hist[(int64_t)s * 256 + b];
    if (cum + h < want[s]) {
      cum += h;
      continue;
    }
    prefix[s] |= (uint64_t)b << (8 * d);
    want[s] -= cum;
    if (d == 0) {  // the stage's cutoff value; h candidates hold it exactly
      cut[(int64_t)s * nst + j] = prefix[s];
      prefix[s] = 0ull;
      if (h == want[s] || j + 1 >= nst) done[s] = j;
    }
    return;
  }
}

// Fold a scan table into the final table: every present entry (admitted by the trim cutoff when
// dstar != nullptr; the segment word is dropped from the key) is inserted by key and its
// accumulators applied with the plan's ops (AggregationFunction.merge of the combine).
__global__ void hash_merge_kernel(const unsigned long long* skeys, int64_t scap, int nw, int has_seg,
                                  const uint64_t* sacc, unsigned long long* fkeys, int64_t fcap, uint64_t* facc,
                                  DevQuery q, int fd_acc, const int64_t* dstar, unsigned long long* overflow,
                                  const SegSelStage* st, int nst, const int32_t* sdone, const uint64_t* scut) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < scap; i += (int64_t)gridDim.x * blockDim.x) {
    if (sacc[i] == 0ull) continue;
    if (dstar) {
      const int64_t s = (int64_t)skeys[(uint64_t)nw * (uint64_t)scap + i];
      if (sacc[(uint64_t)fd_acc * (uint64_t)scap + i] > (uint64_t)dstar[s]) continue;
      // segment-level trim: only the segment's top entries (lexicographically <= its cutoffs up to its last stage)
      if (st && sdone[s] >= 0 && segsel_cmp(st, q, skeys, sacc, scap, i, scut + s * nst, sdone[s] + 1) > 0) continue;
    }
    uint64_t kw[kMaxKeyWords];
    for (int w = 0; w < nw; ++w) kw[w] = skeys[(uint64_t)w * (uint64_t)scap + i];
    const int64_t slot = hash_find_rt(fkeys, fcap, nw, kw);
    if (slot < 0) {
      atomicAdd(overflow, 1ull);
      continue;
    }
    for (int a = 0; a < q.nacc; ++a) {
      const uint64_t v = sacc[(uint64_t)a * (uint64_t)scap + i];
      const uint64_t vh = a + 1 < q.nacc ? sacc[(uint64_t)(a + 1) * (uint64_t)scap + i] : 0ull;
      acc_apply(q.acc_op[a], facc + (uint64_t)a * (uint64_t)fcap + slot,
                facc + (uint64_t)(a + 1 < q.nacc ? a + 1 : a) * (uint64_t)fcap + slot, v, vh);
    }
    (void)has_seg;
  }
}

// ------------------------------------------------------------------------------------------------
// Hash-plan second level (DevHash::spill, JitPlan::hash_spill): the scan's LDS first level keeps a skewed
// key distribution's head on-die; the tail keys' docs were appended to their block's region as records (key
// words, then one value word per value accumulator). Here they are grouped by key-hash partition (so every
// record of a key meets in one partition) and each partition is aggregated in one block's LDS hash table,
// then merged into the HBM table: one probe + one atomic per accumulator per (partition chunk, key) instead
// of per doc -- the map-based holders' group-id lookups (DictionaryBasedGroupKeyGenerator.java:444-900)
// with their per-doc random accesses moved on-die.
// ------------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) unsigned long long LdsU64;

__device__ __forceinline__ uint64_t key_hash_rt(const uint64_t* kw, int nw) {
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int w = 0; w < nw; ++w) x = fmix64(x ^ kw[w]);
  return x;
}

// block b moves its region's records to their partitions' places: part_begin[p] + offs[p * grid + b] + the
// block's running count of partition p (LDS cursors)
__global__ void __launch_bounds__(1024) spill_scatter_kernel(DevHash H, int nw, int64_t grid, const int64_t* offs,
                                                             const int64_t* part_begin, unsigned long long* out) {
  extern __shared__ uint32_t cur[];
  const int64_t sr = blockIdx.x, b = sr / kSpillGroups;  // sub-region sr of scan block b (one partition group)
  const int P = 1 << (64 - H.spill_shift), W = H.spill_words;
  for (int i = threadIdx.x; i < P; i += blockDim.x) cur[i] = 0u;
  __syncthreads();
  const int64_t n = min((int64_t)H.spill_cnt[sr], H.spill_cap);
  const unsigned long long* reg = H.spill + sr * H.spill_cap * W;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long* r = reg + i * W;
    uint64_t kw[kMaxKeyWords];
    for (int w = 0; w < nw; ++w) kw[w] = r[w];
    const int p = (int)(key_hash_rt(kw, nw) >> H.spill_shift);
    const int64_t pos = part_begin[p] + offs[(int64_t)p * grid + b] + atomicAdd(&cur[p], 1u);
    unsigned long long* o = out + pos * W;
    for (int w = 0; w < W; ++w) o[w] = r[w];
  }
}

// LDS-sorted variant (PINOT_AMD_SPILL_SORT=1): the block counting-sorts chunks of C records of its region by
// partition in LDS, then writes the chunk word by word in partition order -- consecutive lanes store
// consecutive words of a partition's run, instead of one 8-byte store per lane and word into 64 scattered
// runs. C = 1024 x per records (per = 1..kSortPerMax per thread, as many as the LDS holds: with ~1K partitions a
// chunk of 2048 records gave each partition 2-record runs, partial 128-B lines written back 1.6x over). The chunk is
// read from HBM once, coalesced, into LDS in record order; the sort only permutes indices (srt) -- reading each
// record again for the copy fetched the chunk twice once chunks outgrew the L2 (FETCH 15.6 GB for 7.9 GB of records).
constexpr int kSortPerMax = 8;
constexpr int kSortPrefWords = 12;  // a chunk's first words per thread prefetched into registers (W = 3: all)
// Workgroup barrier ordering LDS only (waits for the wave's LDS operations, not for its global loads in flight:
// __syncthreads()'s fence waits vmcnt(0), which would drain a prefetch at every barrier)
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ void __launch_bounds__(1024) spill_scatter_sorted_kernel(DevHash H, int nw, int64_t grid, const int64_t* offs,
                                                                    const int64_t* part_begin, unsigned long long* out,
                                                                    int per) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sh_[];
  __shared__ uint32_t wsum[16];
  const int P = 1 << (64 - H.spill_shift), W = H.spill_words, C = 1024 * per;
  unsigned long long* stage = sh_;                                // C x W words
  long long* base = (long long*)(stage + (size_t)C * W);          // P: partition p's next output record
  uint32_t* cnt = (uint32_t*)(base + P);                          // P: the chunk's records per partition
  uint32_t* start = cnt + P;                                      // P: their exclusive prefix
  uint16_t* pid = (uint16_t*)(start + P);                         // C: partition of each sorted slot
  uint16_t* srt = pid + C;                                        // C: chunk record index of each sorted slot
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // j / W as a multiply-high by ceil(2^32 / W) (W > 1): exact for j < 2^16 (chunk words: C * W <= 8192 * 8), W <= 8
  const uint32_t wmagic = (uint32_t)((0x100000000ull + (uint64_t)W - 1) / (uint64_t)W);
  const int64_t sr = blockIdx.x, b = sr / kSpillGroups;  // sub-region sr of scan block b: a quarter of the partitions
  for (int i = tid; i < P; i += 1024) base[i] = part_begin[i] + offs[(int64_t)i * grid + b];
  const int64_t n = min((int64_t)H.spill_cnt[sr], H.spill_cap);
  const unsigned long long* reg = H.spill + sr * H.spill_cap * W;
  // the next chunk's first kSortPrefWords words per thread are loaded into registers as soon as the current chunk
  // is staged, so those HBM reads overlap this chunk's sort and write phases (the CU holds one block: its phases
  // would otherwise run serially; the loop's barriers order LDS only, so they do not wait for the loads); a chunk of
  // more words loads the rest when it is staged
  unsigned long long nx[kSortPrefWords];
  const auto load_chunk = [&](int64_t c) {
    const int mw = (int)min((int64_t)C, n - c) * W;
    const unsigned long long* rb = reg + c * W;
#pragma unroll
    for (int i = 0; i < kSortPrefWords; ++i) {
      const uint32_t j = (uint32_t)tid + (uint32_t)i * 1024u;
      if ((int)j < mw) nx[i] = rb[j];
    }
  };
  if (n > 0) load_chunk(0);
  for (int64_t c0 = 0; c0 < n; c0 += C) {
    const int m = (int)min((int64_t)C, n - c0);
    for (int i = tid; i < P; i += 1024) cnt[i] = 0u;
#pragma unroll
    for (int i = 0; i < kSortPrefWords; ++i) {  // the chunk's words, record order: the prefetched ones, the rest
      const int j = tid + i * 1024;
      if (j < m * W) stage[j] = nx[i];
    }
    for (int j = tid + kSortPrefWords * 1024; j < m * W; j += 1024) stage[j] = reg[c0 * W + j];
    lds_sync();
    if (c0 + C < n) load_chunk(c0 + C);
    uint32_t prk[kSortPerMax];  // a record's partition (high half) and rank in it (low half); ~0 = none
#pragma unroll
    for (int h = 0; h < kSortPerMax; ++h) prk[h] = ~0u;
#pragma unroll
    for (int h = 0; h < kSortPerMax; ++h) {
      if (h >= per) break;
      const int i = tid + h * 1024;
      if (i >= m) continue;
      uint64_t kw[kMaxKeyWords];
      for (int w = 0; w < nw; ++w) kw[w] = stage[(size_t)i * W + w];
      const uint32_t pr = (uint32_t)(key_hash_rt(kw, nw) >> H.spill_shift);
      prk[h] = (pr << 16) | atomicAdd(&cnt[pr], 1u);
    }
    lds_sync();
    {  // exclusive prefix of the counts (P <= 2048: two entries per thread)
      const int i0 = tid * 2;
      const uint32_t a = i0 < P ? cnt[i0] : 0u, a2 = i0 + 1 < P ? cnt[i0 + 1] : 0u;
      uint32_t x = a + a2;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) wsum[wv] = x;
      lds_sync();
      uint32_t off = 0;
      for (int k = 0; k < wv; ++k) off += wsum[k];
      const uint32_t ex = off + x - (a + a2);
      if (i0 < P) start[i0] = ex;
      if (i0 + 1 < P) start[i0 + 1] = ex + a;
    }
    lds_sync();
#pragma unroll
    for (int h = 0; h < kSortPerMax; ++h) {
      if (h >= per || prk[h] == ~0u) continue;
      const uint32_t pr = prk[h] >> 16;
      const int i = tid + h * 1024, pos = (int)start[pr] + (int)(prk[h] & 0xFFFFu);
      srt[pos] = (uint16_t)i;
      pid[pos] = (uint16_t)pr;
    }
    lds_sync();
    for (int j = tid; j < m * W; j += 1024) {
      const int pos = (W == 1 ? j : (int)__umulhi((uint32_t)j, wmagic)), w = j - pos * W, p = pid[pos];
      out[(size_t)(base[p] + (pos - (int)start[p])) * W + w] = stage[(size_t)srt[pos] * W + w];
    }
    lds_sync();
    for (int i = tid; i < P; i += 1024) base[i] += cnt[i];
    lds_sync();
  }
}

// apply record value word v to accumulator a (op) at p / its high word ph: COUNT is applied by the caller
__device__ __forceinline__ void spill_apply(int32_t op, uint64_t* p, uint64_t* ph, uint64_t v) {
  if (op == ACC_SUM_I128) acc_apply(op, p, ph, v, (int64_t)v < 0 ? ~0ull : 0ull);
  else acc_apply(op, p, ph, v, 0ull);
}

// Blocks take contiguous record ranges of the partition-major array; per partition a block meets, an LDS
// open-addressing table of S slots (key words, then every accumulator array of the plan) aggregates the
// records (a key that finds no slot within 64 probes goes to the HBM table directly), then every occupied
// slot is merged into the HBM table (AggregationFunction.merge: counts and sums add, MIN / MAX by the ordered
// encoding) and the table is cleared for the next partition.
__device__ __forceinline__ uint64_t spill_sext(int64_t v) { return v < 0 ? ~0ull : 0ull; }
// spill_agg_kernel: records per thread and step, as many as ~24 record words of registers allow (4 for every width
// before the kernel was templated on it)
constexpr int spill_pre_u(int ww) { return 24 / ww < 2 ? 2 : 24 / ww > 8 ? 8 : 24 / ww; }
constexpr int kSpillPreW = 8;  // record words at most (launch_spill_* require spill_words <= 8)
// WW = the record's words (spill_words), a template parameter so a step's records take WW registers each, not 8
template <int WW>
__global__ void __launch_bounds__(1024) spill_agg_kernel(const unsigned long long* recs, const int64_t* part_begin,
                                                         int P, int nw, int W, int S, DevQuery q, DevHash H,
                                                         uint64_t* acc, uint32_t narrow) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lt[];
  unsigned long long* LK = lt;                         // nw x S key words
  uint64_t* LA = (uint64_t*)(lt + (int64_t)nw * S);    // q.nacc x S accumulators
  const int tid = threadIdx.x;
  const int64_t total = part_begin[P];
  const int64_t per = (total + gridDim.x - 1) / gridDim.x;
  int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = min(total, r0 + per);
  if (r0 >= r1) return;
  int pi = 0;
  {
    int lo = 0, hi = P - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (part_begin[mid] <= r0) lo = mid; else hi = mid - 1;
    }
    pi = lo;
  }
  const int nacc = q.nacc;
  __shared__ int WJ[kMaxAcc];  // record word of accumulator a's value (acc order, ACC_HI skipped)
  if (tid == 0) {
    int j = nw;
    for (int a = 0; a < nacc && a < kMaxAcc; ++a) WJ[a] = (a == 0 || q.acc_op[a] == ACC_HI) ? -1 : j++;
  }
  __syncthreads();
  while (r0 < r1) {
    while (part_begin[pi + 1] <= r0) ++pi;
    const int64_t pe = min(r1, part_begin[pi + 1]);
    for (int i = tid; i < nw * S; i += blockDim.x) LK[i] = ~0ull;
    for (int i = tid; i < nacc * S; i += blockDim.x) LA[i] = acc_identity(q.acc_op[i / S]);
    __syncthreads();
    // one record (its words in rw, statically indexed) into the partition's LDS table, or the HBM table
    auto agg_one = [&](const uint64_t (&rw)[WW]) {
      uint64_t kw[kMaxKeyWords];
#pragma unroll
      for (int w = 0; w < WW; ++w)
        if (w < nw) kw[w] = rw[w];
      const uint64_t x = key_hash_rt(kw, nw);
      uint32_t s = (uint32_t)(((x & 0xFFFFFFFFull) * (uint64_t)(uint32_t)S) >> 32);
      int ls = -1;
      for (int n = 0; n < 64; ++n) {
        bool ok = true;
        for (int w = 0; w < nw && ok; ++w) {
          // the table word through an LDS pointer: a volatile access through the generic one compiled to a
          // volatile flat load and a vmcnt(0) wait per probe
          LdsU64* pw = (LdsU64*)(LK + (uint32_t)w * (uint32_t)S + s);
          unsigned long long c = __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (c == ~0ull) {
            __hip_atomic_compare_exchange_strong(pw, &c, (unsigned long long)kw[w], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            if (c == ~0ull) c = kw[w];
          }
          ok = c == kw[w];
        }
        if (ok) {
          ls = (int)s;
          break;
        }
        s = s + 1u == (uint32_t)S ? 0u : s + 1u;
      }
      auto word = [&](int j) {  // record word j through selects (no dynamic register indexing)
        uint64_t v = 0ull;
#pragma unroll
        for (int w = 0; w < WW; ++w) v = w == j ? rw[w] : v;
        return v;
      };
      if (ls >= 0) {  // the LDS slot (the accumulator words addressed from the shared array: LDS atomics)
        atomicAdd(reinterpret_cast<unsigned long long*>(LA + ls), 1ull);
        for (int a = 1; a < nacc; ++a) {
          const int32_t op = q.acc_op[a];
          if (op == ACC_HI) continue;
          if ((narrow >> a) & 1u)  // a narrow integer SUM: an int64 partial in LDS, no carry (no returning atomic)
            atomicAdd(reinterpret_cast<unsigned long long*>(LA + (int64_t)a * S + ls), (unsigned long long)word(WJ[a]));
          else
            spill_apply(op, LA + (int64_t)a * S + ls, LA + (int64_t)(a + 1 < nacc ? a + 1 : a) * S + ls, word(WJ[a]));
        }
        return;
      }
      // no LDS slot: straight into the HBM table
      const int64_t slot = hash_find_rt(H.keys, H.cap, nw, kw, H.max_probe);
      if (slot < 0) {
        atomicAdd(H.overflow, 1ull);
        return;
      }
      uint64_t* base = acc + slot;
      const int64_t stride = H.cap;
      atomicAdd(reinterpret_cast<unsigned long long*>(base), 1ull);
      for (int a = 1; a < nacc; ++a) {
        const int32_t op = q.acc_op[a];
        if (op == ACC_HI) continue;
        spill_apply(op, base + (int64_t)a * stride, base + (int64_t)(a + 1 < nacc ? a + 1 : a) * stride, word(WJ[a]));
      }
    };
    // spill_pre_u(WW) records per thread and step, every word loaded before any is aggregated (the loads of a step
    // overlap instead of each record's waiting behind the previous one's LDS atomics)
    for (int64_t i0 = r0; i0 < pe; i0 += (int64_t)spill_pre_u(WW) * blockDim.x) {
      uint64_t rw[spill_pre_u(WW)][WW];
#pragma unroll
      for (int u = 0; u < spill_pre_u(WW); ++u) {
        const int64_t i = i0 + (int64_t)u * blockDim.x + tid;
        const unsigned long long* r = recs + (i < pe ? i : r0) * W;
#pragma unroll
        for (int w = 0; w < WW; ++w) rw[u][w] = r[w];
      }
#pragma unroll
      for (int u = 0; u < spill_pre_u(WW); ++u)
        if (i0 + (int64_t)u * blockDim.x + tid < pe) agg_one(rw[u]);
    }
    __syncthreads();
    for (int ls = tid; ls < S; ls += blockDim.x) {
      const uint64_t c = LA[ls];
      if (c == 0ull) continue;
      uint64_t kw[kMaxKeyWords];
      for (int w = 0; w < nw; ++w) kw[w] = LK[(int64_t)w * S + ls];
      const int64_t slot = hash_find_rt(H.keys, H.cap, nw, kw, H.max_probe);
      if (slot < 0) {
        atomicAdd(H.overflow, c);
        continue;
      }
      for (int a = 0; a < nacc; ++a) {
        const uint64_t v = LA[(int64_t)a * S + ls];
        const uint64_t vh = ((narrow >> a) & 1u) ? spill_sext((int64_t)v) : a + 1 < nacc ? LA[(int64_t)(a + 1) * S + ls] : 0ull;
        acc_apply(q.acc_op[a], acc + (uint64_t)a * (uint64_t)H.cap + slot,
                  acc + (uint64_t)(a + 1 < nacc ? a + 1 : a) * (uint64_t)H.cap + slot, v, vh);
      }
    }
    __syncthreads();
    r0 = pe;
    ++pi;
  }
}

// Result compaction (GroupKeyGenerator.getGroupKeys on the device): bit i of `bits` = table slot i
// holds a group (its COUNT accumulator is non-zero); one wave ballot per 64 slots.
__global__ void presence_bitset_kernel(const uint64_t* count, int64_t n, unsigned long long* bits) {
  const int64_t nw = (n + 63) / 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw * 64; i += (int64_t)gridDim.x * blockDim.x) {
    const bool present = i < n && count[i] != 0ull;
    const unsigned long long m = __ballot(present);
    if ((threadIdx.x & 63) == 0) bits[i >> 6] = m;
  }
}

// Segment-level safe trim (GroupByOperator.java:157-175: a segment holding more than trimSize = LIMIT groups
// keeps its top LIMIT by the ORDER BY): block s finds the ORDER BY rank of segment s's LIMIT-th group in its
// presence bitmap over ranks -- per-thread popcounts over contiguous word runs, a block prefix, then the
// thread whose run holds the LIMIT-th set bit walks it. cut[s] = that rank, or ~0 when the segment holds
// <= LIMIT groups (nothing trimmed).
__global__ void __launch_bounds__(1024) seg_cut_kernel(const unsigned long long* bits, int64_t words, int64_t limit,
                                                       unsigned long long* cut) {
  __shared__ long long pre[1024];
  const int s = blockIdx.x, tid = threadIdx.x;
  const unsigned long long* b = bits + (int64_t)s * words;
  const int64_t per = (words + 1023) / 1024;
  const int64_t w0 = min(words, (int64_t)tid * per), w1 = min(words, w0 + per);
  long long c = 0;
  for (int64_t w = w0; w < w1; ++w) c += __popcll(b[w]);
  pre[tid] = c;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive prefix (Hillis-Steele)
    const long long y = tid >= o ? pre[tid - o] : 0;
    __syncthreads();
    pre[tid] += y;
    __syncthreads();
  }
  const long long total = pre[1023], ex = pre[tid] - c;
  if (total <= limit) {
    if (tid == 0) cut[s] = ~0ull;
    return;
  }
  const long long want = limit - 1;  // 0-based index of the LIMIT-th group
  if (ex <= want && want < ex + c) {
    long long r = want - ex;
    for (int64_t w = w0; w < w1; ++w) {
      unsigned long long x = b[w];
      const long long pc = __popcll(x);
      if (r < pc) {
        for (long long i = 0; i < r; ++i) x &= x - 1ull;  // drop the r lowest set bits
        cut[s] = (unsigned long long)(w * 64 + __ffsll((long long)x) - 1);
        return;
      }
      r -= pc;
    }
  }
}

// gather the compacted groups: key words (hash tables) and every accumulator word, row-major
__global__ void gather_groups_kernel(const int32_t* slots, int64_t ngroups, const unsigned long long* keys, int nw,
                                     int64_t cap, const uint64_t* acc, int32_t nacc, uint64_t* out_keys,
                                     uint64_t* out_acc) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t slot = (uint64_t)(uint32_t)slots[g];
    for (int w = 0; w < nw; ++w) out_keys[g * nw + w] = keys ? keys[(uint64_t)w * (uint64_t)cap + slot] : slot;
    for (int a = 0; a < nacc; ++a) out_acc[g * nacc + a] = acc[(uint64_t)a * (uint64_t)cap + slot];
  }
}

// Cross-rank merge by value (GroupByDataTableReducer's merge of every server's groups, here every
// GPU's): each rank exports its compacted groups as (packed key words, accumulator words), the ranks
// all-gather them over RCCL, and every rank folds all rows into one hash table with the accumulator
// ops (AggregationFunction.merge) -- whatever plan (dense, partitioned, hash, trimmed) each rank ran.
__global__ void export_groups_kernel(const int32_t* slots, int64_t ngroups, const unsigned long long* hkeys,
                                     int64_t cap, const uint64_t* acc, int32_t nacc_out, DevKeyPack kp,
                                     uint64_t* out_keys, uint64_t* out_acc) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t slot = (uint64_t)(uint32_t)slots[g];
    if (hkeys) {
      for (int w = 0; w < kp.nw; ++w) out_keys[g * kp.nw + w] = hkeys[(uint64_t)w * (uint64_t)cap + slot];
    } else {
      uint64_t kw[kMaxKeyWords];
      for (int w = 0; w < kp.nw; ++w) kw[w] = 0ull;
      for (int j = 0; j < kp.ncols; ++j) {
        const uint64_t id = (slot / (uint64_t)kp.stride[j]) % (uint64_t)kp.size[j];
        kw[kp.word[j]] |= id << kp.shift[j];
      }
      for (int w = 0; w < kp.nw; ++w) out_keys[g * kp.nw + w] = kw[w];
    }
    for (int a = 0; a < nacc_out; ++a) out_acc[g * nacc_out + a] = acc[(uint64_t)a * (uint64_t)cap + slot];
  }
}

__global__ void merge_rows_kernel(const uint64_t* keys, const uint64_t* acc, int64_t n, int nw, int nacc_in,
                                  unsigned long long* fkeys, int64_t fcap, uint64_t* facc, DevQuery q,
                                  unsigned long long* overflow) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t kw[kMaxKeyWords];
    for (int w = 0; w < nw; ++w) kw[w] = keys[i * nw + w];
    const int64_t slot = hash_find_rt(fkeys, fcap, nw, kw);
    if (slot < 0) {
      atomicAdd(overflow, 1ull);
      continue;
    }
    for (int a = 0; a < nacc_in; ++a) {
      const uint64_t v = acc[i * nacc_in + a];
      const uint64_t vh = a + 1 < nacc_in ? acc[i * nacc_in + a + 1] : 0ull;
      acc_apply(q.acc_op[a], facc + (uint64_t)a * (uint64_t)fcap + slot,
                facc + (uint64_t)(a + 1 < nacc_in ? a + 1 : a) * (uint64_t)fcap + slot, v, vh);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Low-level operators
// ------------------------------------------------------------------------------------------------

// FixedBitSVForwardIndexReaderV2.readDictIds over [start, start+len): 4 docs per lane
__global__ void read_dict_ids_kernel(const uint8_t* packed, int bits, int64_t start, int64_t len, int32_t* out) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= len) return;
  int64_t v[4];
  const int64_t doc0 = start + i0;
  // doc0 need not be 4-aligned here; the 5-dword window covers any start
  load_fixed_bit4(packed, bits, doc0, v);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + k < len) out[i0 + k] = (int32_t)v[k];
}

// FixedBitSVForwardIndexWriter: each lane packs 8 values = exactly `bits` bytes, no overlap
__global__ void pack_dict_ids_kernel(const int32_t* values, int64_t n, int bits, uint8_t* packed) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // group of 8 values
  const int64_t v0 = g * 8;
  if (v0 >= n) return;
  // stream the 8 values MSB-first through a 64-bit window (<= 8 + 31 live bits)
  const int64_t total_bytes = (n * bits + 7) / 8;
  const int64_t byte0 = g * bits;
  const uint32_t mask = (1u << bits) - 1u;
  uint64_t acc = 0;
  int live = 0, ob = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t x = v0 + k < n ? ((uint32_t)values[v0 + k] & mask) : 0u;
    acc = (acc << bits) | x;
    live += bits;
    while (live >= 8) {
      live -= 8;
      if (byte0 + ob < total_bytes) packed[byte0 + ob] = (uint8_t)(acc >> live);
      ++ob;
      acc &= (1ull << live) - 1ull;
    }
  }
}

// raw BE values -> native LE values
__global__ void read_raw_kernel(const uint8_t* raw, int type, int64_t start, int64_t len, uint8_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  if (type == T_INT || type == T_FLOAT) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(raw + (start + i) * 4);
    reinterpret_cast<uint32_t*>(out)[i] = bswap32(x);
  } else {
    const uint2 x = *reinterpret_cast<const uint2*>(raw + (start + i) * 8);
    reinterpret_cast<uint64_t*>(out)[i] = bswap64(x.x, x.y);
  }
}

__global__ void bitset_binop_kernel(const uint64_t* a, const uint64_t* b, uint64_t* out, int64_t n, int op) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = op == 0 ? (a[i] & b[i]) : (a[i] | b[i]);
}

__global__ void bitset_not_kernel(const uint64_t* a, uint64_t* out, int64_t num_docs) {
  const int64_t nw = (num_docs + 63) / 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t w = ~a[i];
    if (i == nw - 1 && (num_docs & 63)) w &= (1ull << (num_docs & 63)) - 1;
    out[i] = w;
  }
}

// Compaction, pass 1: popcount per 1024-word chunk (65536 docs)
constexpr int kCompactWords = 1024;
__global__ void bitset_chunk_count_kernel(const uint64_t* bits, int64_t nwords, int64_t* chunk_counts) {
  __shared__ int64_t wsum[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kCompactWords;
  int64_t c = 0;
  for (int i = threadIdx.x; i < kCompactWords; i += kBlock) {
    const int64_t w = base + i;
    if (w < nwords) c += __popcll(bits[w]);
  }
  c = wave_sum_i64(c);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int i = 0; i < kBlock / 64; ++i) t += wsum[i];
    chunk_counts[blockIdx.x] = t;
  }
}

// pass 2: exclusive scan of chunk counts (single block, sequential over groups of 256)
__global__ void exclusive_scan_kernel(int64_t* counts, int64_t n, int64_t* total) {
  __shared__ int64_t buf[kBlock];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const int64_t x = i < n ? counts[i] : 0;
    buf[threadIdx.x] = x;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {
      const int64_t y = threadIdx.x >= o ? buf[threadIdx.x - o] : 0;
      __syncthreads();
      buf[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < n) counts[i] = carry + buf[threadIdx.x] - x;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry += buf[kBlock - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// Sampled partitioned plans (JitPlan::part_sampled), allotment c = p * G + b (partition p, scatter
// block b). Two launches of P blocks turn per-allotment sizes into their exclusive prefix (P * G + 1
// entries): the first writes each partition's local prefix over b and its total, the second adds the
// partition's base (sum of the totals before it) and, if the whole exceeds `limit`, scales the prefix
// down to fit (floor of a monotone prefix stays monotone, so every size stays >= 0).
//   mode 0 (allotments): size = (e + e/16 + 3 x stride x (sqrt(s) + 1)) x scale from the strided
//          histogram hist[c] = s (e = stride x s: a 3-sigma margin on the sampling error);
//   mode 1 (after the scatter): size = hist[c], the records allotment c holds.
__device__ __forceinline__ int64_t allot_size(const uint32_t* hist, int64_t c, int mode, int64_t stride, double scale) {
  const double sm = (double)hist[c];
  if (mode) return (int64_t)hist[c];
  const double e = sm * (double)stride;
  return (int64_t)min((e + e / 16.0 + 3.0 * (double)stride * (sqrt(sm) + 1.0)) * scale, 4.0e9);
}

__global__ void __launch_bounds__(256) allot_local_kernel(const uint32_t* hist, int64_t G, int mode, int64_t stride,
                                                         double scale, int64_t* out, int64_t* ptot) {
  __shared__ int64_t carry;
  __shared__ int64_t wsum[4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t p = blockIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < G; b0 += 256) {
    const int64_t b = b0 + t;
    const int64_t x = b < G ? allot_size(hist, p * G + b, mode, stride, scale) : 0;
    int64_t incl = x;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < w; ++k) before += wsum[k];
    if (b < G) out[p * G + b] = before + incl - x;
    __syncthreads();
    if (t == 255) carry = before + incl;
    __syncthreads();
  }
  if (t == 0) ptot[p] = carry;
}

__global__ void __launch_bounds__(256) allot_base_kernel(const int64_t* ptot, int32_t P, int64_t G, int64_t limit,
                                                        int64_t* out) {
  __shared__ int64_t red[256];
  const int t = threadIdx.x;
  const int64_t p = blockIdx.x;
  int64_t base = 0, all = 0;
  for (int64_t q = t; q < P; q += 256) {
    all += ptot[q];
    if (q < p) base += ptot[q];
  }
  red[t] = base;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  base = red[0];
  __syncthreads();
  red[t] = all;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  all = red[0];
  const double f = (limit > 0 && all > limit) ? (double)limit / (double)all : 1.0;
  for (int64_t b = t; b < G; b += 256) {
    const int64_t v = base + out[p * G + b];
    out[p * G + b] = f < 1.0 ? (int64_t)((double)v * f) : v;
  }
  if (p == P - 1 && t == 0) out[(int64_t)P * G] = f < 1.0 ? (int64_t)((double)all * f) : all;
}

// Partitioned GROUP BY offsets (DevPartition): row p of hist holds the per-block record counts of
// partition p; one block per row turns it into exclusive per-block offsets and the row total.
__global__ void partition_row_scan_kernel(const uint32_t* hist, int64_t nblocks, int64_t* offs, int64_t* row_total) {
  __shared__ int64_t wtot[kBlock / 64];
  __shared__ int64_t carry;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = blockIdx.x;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nblocks; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const int64_t x = i < nblocks ? (int64_t)hist[row * nblocks + i] : 0;
    int64_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int w = 0; w < wave; ++w) before += wtot[w];
    if (i < nblocks) offs[row * nblocks + i] = before + incl - x;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) row_total[row] = carry;
}

// pass 3: each wave compacts 64 words (4096 docs) per step with ballot + mbcnt style prefix sums
__global__ void bitset_compact_kernel(const uint64_t* bits, int64_t nwords, const int64_t* chunk_offsets,
                                      int32_t* out) {
  __shared__ int64_t wtot[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kCompactWords;
  int64_t off = chunk_offsets[blockIdx.x];
  // the block walks its chunk in steps of 256 words (one word per lane)
  for (int step = 0; step < kCompactWords; step += kBlock) {
    const int64_t w = base + step + threadIdx.x;
    const uint64_t word = w < nwords ? bits[w] : 0ull;
    const int cnt = __popcll(word);
    // inclusive scan of cnt across the wave
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int64_t wave_off = 0;
    for (int i = 0; i < wave; ++i) wave_off += wtot[i];
    int64_t pos = off + wave_off + incl - cnt;
    uint64_t x = word;
    while (x) {
      const int b = __builtin_ctzll(x);
      out[pos++] = (int32_t)(w * 64 + b);
      x &= x - 1;
    }
    int64_t step_total = 0;
    for (int i = 0; i < kBlock / 64; ++i) step_total += wtot[i];
    off += step_total;
    __syncthreads();
  }
}

// Inverted index expansion: one block per (dictId, container) entry of a container directory
// built at staging time. Sets the container's docs in the dense bitset (atomicOr: containers of
// different dictIds share 64-bit words).
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));  // 16-byte load, dword-aligned

struct RoaringContainer {
  uint32_t key;      // high 16 bits of the docIds
  uint32_t kind;     // 0 array, 1 bitmap, 2 run
  uint32_t count;    // array: cardinality, run: number of runs
  uint32_t pad;
  uint64_t offset;   // byte offset of the container payload inside the staged inverted index
};

// a job's device pointers as global-address-space pointers: loads through the generic ones compiled to flat
// loads, which also count against lgkmcnt -- every wait for the expansion's LDS atomics then waited for them
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}

// descriptor of the container at position ci of a job's selection
__device__ __forceinline__ RoaringContainer expand_desc(const ExpandJob& J, int32_t ci) {
  if (J.psel) {
    const unsigned long long d = gptr(J.psel)[ci];
    RoaringContainer c;
    c.key = (uint32_t)(d >> 50) & 7u;  // the chunk within the item's chunk group
    c.kind = (uint32_t)(d >> 48) & 3u;
    c.count = (uint32_t)((d >> 32) & 0xFFFFu);
    c.pad = 0u;
    c.offset = d & 0xFFFFFFFFull;
    return c;
  }
  const __attribute__((address_space(1))) RoaringContainer* cp = gptr(J.conts) + gptr(J.sel)[ci];
  RoaringContainer c;
  c.key = cp->key;
  c.kind = cp->kind;
  c.count = cp->count;
  c.pad = cp->pad;
  c.offset = cp->offset;
  return c;
}

// Plan time: pack the selected containers' descriptors in sel order (ExpandJob::psel): byte offset |
// min(count, 65535) << 32 | kind << 48 | (key mod group) << 50
__global__ void pack_sel_kernel(const RoaringContainer* conts, const int32_t* sel, int64_t n, int group,
                                unsigned long long* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const RoaringContainer c = conts[sel[i]];
    out[i] = c.offset | ((unsigned long long)min(c.count, 65535u) << 32) | ((unsigned long long)c.kind << 48) |
             ((unsigned long long)(c.key % (uint32_t)group) << 50);
  }
}

// Batched expansion: every (segment, inverted-index leaf) of a plan is one ExpandJob; a work item
// is a group of G consecutive 65536-doc chunks of one job. A block builds the group's G x 8 KiB of
// bitset in LDS from its selected containers (LDS atomics, no global atomics), then writes all its
// words once (chunks with no container write zeros, so no separate clear pass). Small array
// containers are expanded one per lane; bitmap, run and large array containers by a whole wave.
// The group's containers are ordered by value, then chunk: a value's containers of consecutive chunks
// are adjacent in the serialized bitmap (payloads in key order), so neighbouring lanes read neighbouring
// bytes -- with a few docs per container (selective IN lists), one chunk per item made every container
// its own cache-line fetch.
constexpr int kExpandPer = 4;  // containers per lane per round: their loads are independent (latency overlap)

// The selected containers of work item k of job J ORed into lbits (G x 2048 words, zeroed by the
// caller); bigq / nbig: LDS queue of the containers a whole wave expands (nbig = 0 on entry). Called by
// the whole block (it synchronises).
template <int G, int kPer = kExpandPer>
__device__ __forceinline__ void expand_item(const ExpandJob& J, int32_t k, uint32_t* lbits, int32_t* bigq, int32_t* nbig) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t g0 = gptr(J.grp)[k], g1 = gptr(J.grp)[k + 1];
  for (int32_t base = g0; base < g1; base += kBlock * kPer) {
    // every load of the round first (selected index, descriptor, small-array payload), then the LDS work
    int32_t si[kPer];  // position in the job's sel order, -1: none
    RoaringContainer c[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int32_t ci = base + u * kBlock + tid;
      si[u] = ci < g1 ? ci : -1;
      if (si[u] >= 0) c[u] = expand_desc(J, ci);
    }
    // a small array's <= 16 two-byte entries with 3 dword-aligned 16-byte loads (48 bytes from the
    // dword holding the first entry; the staged buffer's zero padding keeps the tail in bounds)
    uint32_t v[kPer][16];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const bool small = si[u] >= 0 && c[u].kind == 0 && c[u].count <= 16;
      uint32_t w[12];
      const uint32_t odd = (uint32_t)(c[u].offset >> 1) & 1u;  // entry 0 in the dword's high half
      if (small) {
        // only the 16-byte pieces the entries reach (halfwords odd .. odd + count - 1): with a few docs per
        // container (selective IN lists) one piece, so the neighbouring containers' pieces share lines
        const __attribute__((address_space(1))) u32x4a4* p4 = gptr(reinterpret_cast<const u32x4a4*>(J.inv + (c[u].offset & ~3ull)));
        const uint32_t reach = odd + c[u].count;
        const u32x4a4 a = p4[0];
        u32x4a4 b = (u32x4a4)(0u), d = (u32x4a4)(0u);
        if (reach > 8u) b = p4[1];
        if (reach > 16u) d = p4[2];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y;
        w[6] = b.z; w[7] = b.w; w[8] = d.x; w[9] = d.y; w[10] = d.z; w[11] = d.w;
      }
#pragma unroll
      for (uint32_t e = 0; e < 16; ++e) {
        // 16-bit entry e is halfword e + odd of the aligned dwords (compile-time indices: e is unrolled)
        const uint32_t x0 = (e & 1u) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xFFFFu);
        const uint32_t x1 = ((e + 1) & 1u) ? (w[(e + 1) >> 1] >> 16) : (w[(e + 1) >> 1] & 0xFFFFu);
        const uint32_t x = odd ? x1 : x0;
        v[u][e] = small && e < c[u].count ? x : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      if (si[u] < 0) continue;
      if (c[u].kind == 0 && c[u].count <= 16) {
        uint32_t* lb = lbits + 2048 * (G == 1 ? 0u : c[u].key % (uint32_t)G);
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e)
          if (e < c[u].count) atomicOr(&lb[v[u][e] >> 5], 1u << (v[u][e] & 31));
      } else {
        bigq[atomicAdd(nbig, 1)] = si[u];
      }
    }
    __syncthreads();
    const int nb = *nbig;
    for (int qi = wave; qi < nb; qi += kBlock / 64) {
      const RoaringContainer c = expand_desc(J, bigq[qi]);
      const __attribute__((address_space(1))) uint8_t* p = gptr(J.inv) + c.offset;
      uint32_t* lb = lbits + 2048 * (G == 1 ? 0u : c.key % (uint32_t)G);
      if (c.kind == 1) {
        for (int i = lane; i < 1024; i += 64) {
          const uint64_t w = *reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(p + 8 * i);  // LE
          if (w) {
            atomicOr(&lb[2 * i], (uint32_t)w);
            atomicOr(&lb[2 * i + 1], (uint32_t)(w >> 32));
          }
        }
      } else if (c.kind == 0) {
        const __attribute__((address_space(1))) uint16_t* p16 = reinterpret_cast<const __attribute__((address_space(1))) uint16_t*>(p);
        for (uint32_t e = lane; e < c.count; e += 64) {
          const uint32_t d = p16[e];
          atomicOr(&lb[d >> 5], 1u << (d & 31));
        }
      } else {
        for (uint32_t r = 0; r < c.count; ++r) {
          const __attribute__((address_space(1))) uint8_t* q = p + 2 + 4 * r;
          const uint32_t s0 = q[0] | (q[1] << 8);
          const uint32_t e0 = s0 + (q[2] | (q[3] << 8));  // inclusive, < 65536
          const uint32_t w0 = s0 >> 5, w1 = e0 >> 5;
          for (uint32_t w = w0 + lane; w <= w1; w += 64) {
            uint32_t m = ~0u;
            if (w == w0) m &= ~0u << (s0 & 31);
            if (w == w1) m &= ~0u >> (31 - (e0 & 31));
            atomicOr(&lb[w], m);
          }
        }
      }
    }
    __syncthreads();
    if (tid == 0) *nbig = 0;
    __syncthreads();
  }
}

template <int G>
__global__ void __launch_bounds__(kBlock) roaring_expand_chunks_kernel(const ExpandJob* jobs, int32_t njobs,
                                                                      int64_t total_items) {
  __shared__ uint32_t lbits[2048 * G];
  __shared__ int32_t bigq[kBlock * kExpandPer];
  __shared__ int32_t nbig;
  const int tid = threadIdx.x;
  for (int64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    const ExpandJob& J = jobs[lo];
    const int32_t k = (int32_t)(item - J.item_begin);
    for (int i = tid; i < 2048 * G; i += kBlock) lbits[i] = 0u;
    if (tid == 0) nbig = 0;
    __syncthreads();
    expand_item<G>(J, k, lbits, bigq, &nbig);
    // write the group (docs >= num_docs are never set: bitmaps hold only the segment's docIds)
    const int64_t w_begin = (int64_t)k * 1024 * G;
    for (int i = tid; i < 1024 * G; i += kBlock) {
      const int64_t w = w_begin + i;
      if (w < J.nwords)
        ((__attribute__((address_space(1))) unsigned long long*)J.bitset)[w] =
            (unsigned long long)lbits[2 * i] | ((unsigned long long)lbits[2 * i + 1] << 32);
    }
    __syncthreads();
  }
}

// Fused inverted-index select (word-level select plans whose every leaf is an inverted-index docId
// bitset, a sorted-index docId range or a constant): a work item is a group of G chunks of one segment.
// Per clause, the block expands each bitset leaf's containers for the group into LDS and ORs the words
// into per-thread clause words (4G 64-bit words per thread), then ANDs the clause into the match words;
// the group's matching docIds go straight to the selection vector (one reservation per item, padded to a
// quad: an item is one segment). No dense bitset is written to or read back from HBM, and the expansion
// and the word-level select are one launch.
template <int G>
__global__ void __launch_bounds__(kBlock) roaring_select_kernel(const ExpandJob* jobs, const FusedSelSeg* fs, int32_t nfs,
                                                               int64_t total_items, const DevSegment* segs,
                                                               int32_t nleaves, int32_t nclauses,
                                                               unsigned long long* sel_entries, unsigned long long* sel_count,
                                                               int64_t sel_cap, unsigned long long* matched_out) {
  __shared__ uint32_t lbits[2048 * G];
  __shared__ int32_t bigq[kBlock * kExpandPer];
  __shared__ int32_t nbig;
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ unsigned long long sbase;
  constexpr int NW = 4 * G;  // 64-bit words per thread: word tid + 256 i of the group's 1024 G
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    int lo = 0, hi = nfs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (fs[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    const FusedSelSeg& F = fs[lo];
    const int32_t k = (int32_t)(item - F.item_begin);
    const DevSegment& sg = segs[F.seg];
    const int64_t w0 = (int64_t)k * 1024 * G;  // the group's first 64-doc word in the segment
    uint64_t mt[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int64_t d0 = (w0 + tid + 256 * i) * 64;
      mt[i] = d0 >= sg.num_docs ? 0ull : sg.num_docs - d0 >= 64 ? ~0ull : ((1ull << (sg.num_docs - d0)) - 1ull);
    }
    for (int c = 0; c < nclauses; ++c) {
      uint64_t ac[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) ac[i] = 0ull;
      for (int j = 0; j < nleaves; ++j) {
        const DevLeaf& L = sg.leaves[j];
        if (L.clause != c) continue;
        uint64_t x[NW];
        if (L.kind == LEAF_DOC_BITSET && F.job[j] >= 0) {
          for (int i = tid; i < 2048 * G; i += kBlock) lbits[i] = 0u;
          if (tid == 0) nbig = 0;
          __syncthreads();
          expand_item<G>(jobs[F.job[j]], k, lbits, bigq, &nbig);
          __syncthreads();
#pragma unroll
          for (int i = 0; i < NW; ++i) {
            const int w = tid + 256 * i;
            x[i] = (uint64_t)lbits[2 * w] | ((uint64_t)lbits[2 * w + 1] << 32);
          }
          __syncthreads();  // the region is refilled by the next leaf
        } else if (L.kind == LEAF_DOC_RANGE) {
#pragma unroll
          for (int i = 0; i < NW; ++i) {
            const int64_t d0 = (w0 + tid + 256 * i) * 64;
            const int64_t a = max(L.lo_i - d0, (int64_t)0), b = min(L.hi_i - d0, (int64_t)63);
            x[i] = a > b ? 0ull : ((~0ull >> (63 - (b - a))) << a);
          }
        } else {  // LEAF_CONST
#pragma unroll
          for (int i = 0; i < NW; ++i) x[i] = L.lo_i ? ~0ull : 0ull;
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) ac[i] |= L.negate ? ~x[i] : x[i];
      }
#pragma unroll
      for (int i = 0; i < NW; ++i) mt[i] &= ac[i];
    }
    // block prefix of the match counts, one vector reservation per item
    uint32_t cnt = 0u;
#pragma unroll
    for (int i = 0; i < NW; ++i) cnt += (uint32_t)__popcll(mt[i]);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(incl, o, 64); if (lane >= o) incl += y; }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
    for (int w = 0; w < kBlock / 64; ++w) { if (w < wave) before += wsum[w]; total += wsum[w]; }
    const uint32_t padded = (total + 3u) & ~3u;
    if (tid == 0) {
      unsigned long long b = ~0ull;
      if (total) {
        b = atomicAdd(sel_count, (unsigned long long)padded);
        if (b + padded > (unsigned long long)sel_cap) { atomicAdd(sel_count + 1, 1ull); b = ~0ull; }
        atomicAdd(matched_out, (unsigned long long)total);
      }
      sbase = b;
    }
    __syncthreads();
    const unsigned long long base = sbase;
    if (total && base != ~0ull) {
      const unsigned long long tag = (unsigned long long)(uint32_t)F.seg << 32;
      unsigned long long p = base + before + incl - cnt;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        uint64_t m = mt[i];
        const int64_t d0 = (w0 + tid + 256 * i) * 64;
        while (m) {
          const int bt = __builtin_ctzll(m);
          m &= m - 1ull;
          sel_entries[p++] = tag | (unsigned long long)(uint32_t)(d0 + bt);
        }
      }
      if (tid < (int)(padded - total)) sel_entries[base + total + tid] = tag | 0xFFFFFFFFull;
    }
    __syncthreads();  // wsum / sbase reused by the next item
  }
}

// The same selection with a clause's non-negated bitset leaves expanded together into the LDS region (the
// expansion ORs) and only the match words live across the expansion. The default for filters without
// negated bitset leaves (5-9 % faster than the per-leaf fold at 0.01-0.1 %); PINOT_AMD_FUSED_VARIANT=leaf
// forces the per-leaf kernel above.
template <int G>
__global__ void __launch_bounds__(kBlock) roaring_select_clause_kernel(const ExpandJob* jobs, const FusedSelSeg* fs,
                                                                      int32_t nfs, int64_t total_items,
                                                                      const DevSegment* segs, int32_t nleaves,
                                                                      int32_t nclauses, unsigned long long* sel_entries,
                                                                      unsigned long long* sel_count, int64_t sel_cap,
                                                                      unsigned long long* matched_out) {
  __shared__ uint32_t lbits[2048 * G];
  __shared__ int32_t bigq[kBlock * kExpandPer];
  __shared__ int32_t nbig;
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ unsigned long long sbase;
  constexpr int NW = 4 * G;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    int lo = 0, hi = nfs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (fs[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    const FusedSelSeg& F = fs[lo];
    const int32_t k = (int32_t)(item - F.item_begin);
    const DevSegment& sg = segs[F.seg];
    const int64_t w0 = (int64_t)k * 1024 * G;
    uint64_t mt[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int64_t d0 = (w0 + tid + 256 * i) * 64;
      mt[i] = d0 >= sg.num_docs ? 0ull : sg.num_docs - d0 >= 64 ? ~0ull : ((1ull << (sg.num_docs - d0)) - 1ull);
    }
    for (int c = 0; c < nclauses; ++c) {
      for (int i = tid; i < 2048 * G; i += kBlock) lbits[i] = 0u;
      if (tid == 0) nbig = 0;
      __syncthreads();
      bool any = false, other = false;
      for (int j = 0; j < nleaves; ++j) {
        const DevLeaf& L = sg.leaves[j];
        if (L.clause != c) continue;
        if (L.kind == LEAF_DOC_BITSET && F.job[j] >= 0) {
          expand_item<G>(jobs[F.job[j]], k, lbits, bigq, &nbig);
          any = true;
        } else {
          other = true;
        }
      }
      __syncthreads();
      uint64_t a[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const int w = tid + 256 * i;
        a[i] = any ? ((uint64_t)lbits[2 * w] | ((uint64_t)lbits[2 * w + 1] << 32)) : 0ull;
      }
      if (other)
        for (int j = 0; j < nleaves; ++j) {
          const DevLeaf& L = sg.leaves[j];
          if (L.clause != c || (L.kind == LEAF_DOC_BITSET && F.job[j] >= 0)) continue;
          const uint64_t neg = L.negate ? ~0ull : 0ull;
          if (L.kind == LEAF_DOC_RANGE) {
#pragma unroll
            for (int i = 0; i < NW; ++i) {
              const int64_t d0 = (w0 + tid + 256 * i) * 64;
              const int64_t x0 = max(L.lo_i - d0, (int64_t)0), x1 = min(L.hi_i - d0, (int64_t)63);
              a[i] |= (x0 > x1 ? 0ull : ((~0ull >> (63 - (x1 - x0))) << x0)) ^ neg;
            }
          } else {
#pragma unroll
            for (int i = 0; i < NW; ++i) a[i] |= (L.lo_i ? ~0ull : 0ull) ^ neg;
          }
        }
#pragma unroll
      for (int i = 0; i < NW; ++i) mt[i] &= a[i];
      __syncthreads();  // the region is refilled by the next clause
    }
    uint32_t cnt = 0u;
#pragma unroll
    for (int i = 0; i < NW; ++i) cnt += (uint32_t)__popcll(mt[i]);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const uint32_t y = __shfl_up(incl, o, 64); if (lane >= o) incl += y; }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0u, total = 0u;
    for (int w = 0; w < kBlock / 64; ++w) { if (w < wave) before += wsum[w]; total += wsum[w]; }
    const uint32_t padded = (total + 3u) & ~3u;
    if (tid == 0) {
      unsigned long long b = ~0ull;
      if (total) {
        b = atomicAdd(sel_count, (unsigned long long)padded);
        if (b + padded > (unsigned long long)sel_cap) { atomicAdd(sel_count + 1, 1ull); b = ~0ull; }
        atomicAdd(matched_out, (unsigned long long)total);
      }
      sbase = b;
    }
    __syncthreads();
    const unsigned long long base = sbase;
    if (total && base != ~0ull) {
      const unsigned long long tag = (unsigned long long)(uint32_t)F.seg << 32;
      unsigned long long p = base + before + incl - cnt;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        uint64_t m = mt[i];
        const int64_t d0 = (w0 + tid + 256 * i) * 64;
        while (m) {
          const int bt = __builtin_ctzll(m);
          m &= m - 1ull;
          sel_entries[p++] = tag | (unsigned long long)(uint32_t)(d0 + bt);
        }
      }
      if (tid < (int)(padded - total)) sel_entries[base + total + tid] = tag | 0xFFFFFFFFull;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// launchers (called from host.cpp)
// ------------------------------------------------------------------------------------------------
static inline unsigned grid_for(int64_t n, int per_block) {
  int64_t g = (n + per_block - 1) / per_block;
  return (unsigned)(g < 1 ? 1 : g);
}

// ------------------------------------------------------------------------------------------------
// Raw-chunk decompression at staging (BaseChunkForwardIndexReader.decompressChunk,
// BaseChunkForwardIndexReader.java:150-185, with the codecs of io/compression/*Decompressor.java).
// One wave per chunk: the (sequential) token stream is parsed wave-uniformly, every literal run and
// match is copied by all 64 lanes. A match with offset < length repeats the `off` bytes before it,
// so byte i of the match is dst[op - off + i % off] -- no byte-serial copy. Stores of one step become
// visible to the wave's later loads through a workgroup-scope fence (the block is one wave).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

__device__ __forceinline__ void wave_match_copy(uint8_t* dst, int64_t op, int64_t off, int64_t ml, int lane) {
  if (off >= ml) {
    for (int64_t i = lane; i < ml; i += 64) dst[op + i] = dst[op - off + i];
  } else {
    for (int64_t i = lane; i < ml; i += 64) dst[op + i] = dst[op - off + i % off];
  }
}

// LZ4 block (lz4-java LZ4SafeDecompressor semantics); returns bytes written or -1
__device__ int64_t wave_lz4(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int lane) {
  int64_t ip = 0, op = 0;
  while (ip < n) {
    const uint32_t token = src[ip++];
    int64_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) return -1;
    for (int64_t i = lane; i < lit; i += 64) dst[op + i] = src[ip + i];
    ip += lit;
    op += lit;
    if (ip >= n) break;  // last sequence: literals only
    if (ip + 2 > n) return -1;
    const int64_t off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
    ip += 2;
    int64_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= n) return -1;
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > op || op + ml > cap) return -1;
    wave_fence();
    wave_match_copy(dst, op, off, ml, lane);
    wave_fence();
    op += ml;
  }
  return op;
}

// Snappy raw block (snappy-java Snappy.uncompress); returns bytes written or -1
__device__ int64_t wave_snappy(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int lane) {
  int64_t ip = 0, op = 0;
  uint64_t len = 0;
  for (int sh = 0;; sh += 7) {
    if (ip >= n || sh > 28) return -1;
    const uint32_t b = src[ip++];
    len |= (uint64_t)(b & 0x7F) << sh;
    if (!(b & 0x80)) break;
  }
  if ((int64_t)len > cap) return -1;
  while (ip < n) {
    const uint32_t tag = src[ip++];
    int64_t l, off;
    if ((tag & 3) == 0) {
      l = (tag >> 2) + 1;
      if (l > 60) {
        const int nb = (int)l - 60;
        if (ip + nb > n) return -1;
        l = 0;
        for (int k = 0; k < nb; ++k) l |= (int64_t)src[ip + k] << (8 * k);
        l += 1;
        ip += nb;
      }
      if (ip + l > n || op + l > (int64_t)len) return -1;
      for (int64_t i = lane; i < l; i += 64) dst[op + i] = src[ip + i];
      ip += l;
      op += l;
      continue;
    }
    if ((tag & 3) == 1) {
      if (ip + 1 > n) return -1;
      l = 4 + ((tag >> 2) & 7);
      off = ((int64_t)(tag >> 5) << 8) | src[ip];
      ip += 1;
    } else if ((tag & 3) == 2) {
      if (ip + 2 > n) return -1;
      l = (tag >> 2) + 1;
      off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return -1;
      l = (tag >> 2) + 1;
      off = (int64_t)((uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8) | ((uint32_t)src[ip + 2] << 16) |
                      ((uint32_t)src[ip + 3] << 24));
      ip += 4;
    }
    if (off == 0 || off > op || op + l > (int64_t)len) return -1;
    wave_fence();
    wave_match_copy(dst, op, off, l, lane);
    wave_fence();
    op += l;
  }
  return op == (int64_t)len ? op : -1;
}

// inclusive prefix sum (Java wrapping arithmetic) over the W-byte big-endian values v[first..cnt)
template <typename U>
__device__ void wave_prefix_be(uint8_t* v, int64_t first, int64_t cnt, int lane) {
  U carry = 0;
  for (int64_t base = first; base < cnt; base += 64) {
    const int64_t i = base + lane;
    U x = 0;
    if (i < cnt) {
      // 4-byte accesses only: a chunk of an INT column may use the 8-byte layout at a 4-aligned offset
      const uint32_t* q = (const uint32_t*)(v + i * sizeof(U));
      if constexpr (sizeof(U) == 4) x = __builtin_bswap32(q[0]);
      else x = ((uint64_t)__builtin_bswap32(q[0]) << 32) | __builtin_bswap32(q[1]);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const U y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    x += carry;
    if (i < cnt) {
      uint32_t* q = (uint32_t*)(v + i * sizeof(U));
      if constexpr (sizeof(U) == 4) {
        q[0] = __builtin_bswap32(x);
      } else {
        q[0] = __builtin_bswap32((uint32_t)(x >> 32));
        q[1] = __builtin_bswap32((uint32_t)x);
      }
    }
    carry = __shfl(x, 63, 64);
  }
}

// DELTA / DELTADELTA chunk (DeltaDecompressor.java, DeltaDeltaDecompressor.java): flag byte
// (1 = LONG layout), BE count, BE first value, BE LZ4 size, LZ4 block of BE (delta-of-)deltas
__device__ int64_t wave_delta(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, bool dd, int lane) {
  if (n < 5) return -1;
  const int w = src[0] == 1 ? 8 : 4;
  const int64_t cnt = (int32_t)(((uint32_t)src[1] << 24) | ((uint32_t)src[2] << 16) | ((uint32_t)src[3] << 8) | src[4]);
  if (cnt < 0 || cnt * w > cap) return -1;
  if (cnt == 0) return 0;
  if (n < 5 + w) return -1;
  for (int i = lane; i < w; i += 64) dst[i] = src[5 + i];  // first value, as stored
  if (cnt == 1) return w;
  if (n < 9 + w) return -1;
  const uint8_t* p = src + 5 + w;
  const int64_t cs = (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
  if (cs < 0 || 9 + w + cs > n) return -1;
  if (wave_lz4(p + 4, cs, dst + w, (cnt - 1) * w, lane) != (cnt - 1) * w) return -1;
  wave_fence();
  if (w == 8) {
    if (dd) {
      wave_prefix_be<uint64_t>(dst, 1, cnt, lane);
      wave_fence();
    }
    wave_prefix_be<uint64_t>(dst, 0, cnt, lane);
  } else {
    if (dd) {
      wave_prefix_be<uint32_t>(dst, 1, cnt, lane);
      wave_fence();
    }
    wave_prefix_be<uint32_t>(dst, 0, cnt, lane);
  }
  return cnt * w;
}

// status[j]: 0 decoded to exactly dst_len bytes, 1 malformed or wrong size, 2 unknown codec
__global__ void __launch_bounds__(64) chunk_decompress_kernel(const uint8_t* __restrict__ src, uint8_t* dst,
                                                              const ChunkJob* __restrict__ jobs, int32_t njobs,
                                                              int32_t* __restrict__ status) {
  const int lane = threadIdx.x;
  for (int32_t j = blockIdx.x; j < njobs; j += gridDim.x) {
    const ChunkJob jb = jobs[j];
    const uint8_t* s = src + jb.src_off;
    uint8_t* d = dst + jb.dst_off;
    int64_t got;
    switch (jb.codec) {
      case 1: got = wave_snappy(s, jb.src_len, d, jb.dst_len, lane); break;
      case 3: got = wave_lz4(s, jb.src_len, d, jb.dst_len, lane); break;
      case 6: got = wave_delta(s, jb.src_len, d, jb.dst_len, false, lane); break;
      case 7: got = wave_delta(s, jb.src_len, d, jb.dst_len, true, lane); break;
      default: got = -2;
    }
    if (lane == 0) status[j] = got == (int64_t)jb.dst_len ? 0 : got == -2 ? 2 : 1;
  }
}

hipError_t launch_chunk_decompress(const uint8_t* src, uint8_t* dst, const void* jobs, int32_t njobs, int32_t* status,
                                   hipStream_t st) {
  if (njobs <= 0) return hipSuccess;
  const int grid = njobs < 65536 ? njobs : 65536;
  hipLaunchKernelGGL(chunk_decompress_kernel, dim3(grid), dim3(64), 0, st, src, dst, (const ChunkJob*)jobs, njobs,
                     status);
  return hipGetLastError();
}

// ColumnMetadata minValue / maxValue of a raw INT / LONG column (SegmentColumnarIndexCreator writes them
// into metadata.properties): min and max of the staged big-endian values, grid-stride with a wave
// reduction and one 64-bit atomic pair per wave. out[0] / out[1] start at INT64_MAX / INT64_MIN.
__global__ void raw_int_minmax_kernel(const uint8_t* __restrict__ be, int type, int64_t n, long long* out) {
  long long mn = LLONG_MAX, mx = LLONG_MIN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long long v;
    if (type == T_INT) {
      v = (long long)(int32_t)__builtin_bswap32(*reinterpret_cast<const uint32_t*>(be + 4 * i));
    } else {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(be + 8 * i);
      v = (long long)(((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]));
    }
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(out, mn);
    atomicMax(out + 1, mx);
  }
}

// Order-independent 64-bit fingerprint of a device buffer (word i mixed with its index, summed): taken when a column
// is staged and again when a partitioned plan's self-check fails, it tells a column whose HBM bytes changed since
// staging apart from a misread of intact bytes (host.cpp selfcheck_report).
__global__ void fingerprint_kernel(const uint64_t* p, int64_t nwords, unsigned long long* out) {
  uint64_t h = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = p[i] ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    h += x;
  }
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(out, (unsigned long long)h);
}

hipError_t launch_fingerprint(const void* p, size_t bytes, unsigned long long* out, hipStream_t st) {
  const int64_t nw = (int64_t)(bytes / 8);
  if (nw <= 0) return hipSuccess;
  unsigned g = grid_for(nw, kBlock);
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(fingerprint_kernel, dim3(g), dim3(kBlock), 0, st, (const uint64_t*)p, nw, out);
  return hipGetLastError();
}

hipError_t launch_raw_int_minmax(const uint8_t* be, int type, int64_t n, long long* out, hipStream_t st) {
  unsigned g = grid_for(n, kBlock);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(raw_int_minmax_kernel, dim3(g), dim3(kBlock), 0, st, be, type, n, out);
  return hipGetLastError();
}

hipError_t launch_sext_hi(uint64_t* d_acc, int64_t n, const int32_t* arrs, int32_t narr, hipStream_t st) {
  unsigned g = grid_for(n, kBlock);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(sext_hi_kernel, dim3(g), dim3(kBlock), 0, st, d_acc, n, arrs, narr);
  return hipGetLastError();
}

hipError_t launch_init_acc(uint64_t* d_acc, const DevQuery& q, int64_t num_keys, hipStream_t st) {
  const int64_t n = (int64_t)q.nacc * num_keys;
  unsigned g = grid_for(n, kBlock);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(init_acc_kernel, dim3(g), dim3(kBlock), 0, st, d_acc, num_keys, q);
  return hipGetLastError();
}

static inline unsigned grid_cap(int64_t n, int per_block, unsigned cap) {
  const unsigned g = grid_for(n, per_block);
  return g > cap ? cap : g;
}

hipError_t launch_trim(const unsigned long long* keys, int64_t cap, int nw_seg, const uint64_t* acc, int fd_acc,
                       int32_t nsegs, int64_t limit, const int64_t* bucket_base, uint32_t* hist,
                       unsigned long long* seg_distinct, int64_t* bstar, int64_t* rank, unsigned long long* bitmap,
                       int64_t* dstar, unsigned long long* limit_reached, hipStream_t st) {
  const unsigned g = grid_cap(cap, kBlock, 8192);
  hipLaunchKernelGGL(trim_count_kernel, dim3(g), dim3(kBlock), 0, st, keys, cap, nw_seg, acc, fd_acc, bucket_base, hist,
                     seg_distinct);
  hipLaunchKernelGGL(trim_select_kernel, dim3((unsigned)nsegs), dim3(256), 0, st, limit, bucket_base, hist,
                     seg_distinct, bstar, rank, limit_reached, 0);
  hipLaunchKernelGGL(trim_bitmap_kernel, dim3(g), dim3(kBlock), 0, st, keys, cap, nw_seg, acc, fd_acc, bstar, bitmap);
  hipLaunchKernelGGL(trim_cutoff_kernel, dim3(grid_for(nsegs, kBlock)), dim3(kBlock), 0, st, nsegs, bstar, rank, bitmap,
                     dstar);
  return hipGetLastError();
}

hipError_t launch_admit(uint32_t* first, int64_t nk, const uint32_t* seen, const unsigned long long* seen_n, int64_t cap,
                        int32_t nsegs, int64_t limit, const int64_t* bucket_base, int64_t max_buckets, uint32_t* hist,
                        int64_t* bstar, int64_t* rank, unsigned long long* bitmap, int64_t* dstar,
                        unsigned long long* limit_reached, int phase, uint32_t* admit, int64_t words, hipStream_t st) {
  if (nsegs <= 0) return hipSuccess;
  if (phase == 0) {  // histogram + the limit-th bucket per segment (seen_n doubles as the distinct count)
    const int64_t chunk = 8192;
    const unsigned cx = (unsigned)std::max<int64_t>(1, (cap + chunk - 1) / chunk);
    hipLaunchKernelGGL(admit_hist_kernel, dim3(cx, (unsigned)nsegs), dim3(256), (size_t)max_buckets * 4, st, first, nk,
                       seen, seen_n, cap, chunk, bucket_base, hist);
    hipLaunchKernelGGL(trim_select_kernel, dim3((unsigned)nsegs), dim3(256), 0, st, limit, bucket_base, hist, seen_n, bstar,
                       rank, limit_reached, 1);
    return hipGetLastError();
  }
  const unsigned cx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((cap + 255) / 256, 64));
  hipLaunchKernelGGL(admit_bucket_kernel, dim3(cx, (unsigned)nsegs), dim3(256), 0, st, first, nk, seen, seen_n, cap, nsegs,
                     bstar, bitmap);
  hipLaunchKernelGGL(trim_cutoff_kernel, dim3(grid_for(nsegs, kBlock)), dim3(kBlock), 0, st, nsegs, bstar, rank, bitmap,
                     dstar);
  const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((std::max(cap, words) + 255) / 256, 64));
  hipLaunchKernelGGL(admit_bits_kernel, dim3(bx, (unsigned)nsegs), dim3(256), 0, st, first, nk, seen, seen_n, cap, dstar,
                     admit, words);
  return hipGetLastError();
}

hipError_t launch_hash_merge(const unsigned long long* skeys, int64_t scap, int nw, int has_seg, const uint64_t* sacc,
                             unsigned long long* fkeys, int64_t fcap, uint64_t* facc, const DevQuery& q, int fd_acc,
                             const int64_t* dstar, unsigned long long* overflow, hipStream_t st, const SegSelStage* sst,
                             int nst, const int32_t* sdone, const uint64_t* scut) {
  hipLaunchKernelGGL(hash_merge_kernel, dim3(grid_cap(scap, kBlock, 8192)), dim3(kBlock), 0, st, skeys, scap, nw, has_seg,
                     sacc, fkeys, fcap, facc, q, fd_acc, dstar, overflow, sst, nst, sdone, scut);
  return hipGetLastError();
}

// the segment-level trim's selection over one trim batch's scan table (after launch_trim: dstar admits the
// numGroupsLimit survivors): per segment `keep` entries, cutoffs per stage in cut (nsegs x nst), done per segment
// (-2: nothing trimmed; j: selection ended at stage j). hist: nsegs x 256 words, zeroed per pass here.
hipError_t launch_segsel(const unsigned long long* keys, int64_t cap, int nw, const uint64_t* acc, int fd_acc,
                         const int64_t* dstar, const DevQuery& q, const SegSelStage* sst, int nst, int32_t nsegs,
                         int64_t keep, unsigned long long* cnt, int64_t* want, int32_t* done, uint64_t* prefix,
                         uint64_t* cut, uint32_t* hist, hipStream_t st) {
  if (nsegs <= 0 || nst <= 0) return hipSuccess;
  const unsigned g = grid_cap(cap, kBlock, 8192), gs = grid_for(nsegs, kBlock);
  hipError_t e = hipMemsetAsync(cnt, 0, (size_t)nsegs * 8, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(segsel_count_kernel, dim3(g), dim3(kBlock), 0, st, keys, cap, nw, acc, fd_acc, dstar, cnt);
  hipLaunchKernelGGL(segsel_init_kernel, dim3(gs), dim3(kBlock), 0, st, nsegs, keep, cnt, want, done, prefix);
  for (int j = 0; j < nst; ++j)
    for (int d = 7; d >= 0; --d) {
      if ((e = hipMemsetAsync(hist, 0, (size_t)nsegs * 256 * 4, st)) != hipSuccess) return e;
      hipLaunchKernelGGL(segsel_hist_kernel, dim3(g), dim3(kBlock), 0, st, keys, cap, nw, acc, fd_acc, dstar, q, sst, nst, j,
                         d, done, prefix, cut, hist);
      hipLaunchKernelGGL(segsel_pick_kernel, dim3(gs), dim3(kBlock), 0, st, nsegs, nst, j, d, hist, want, done, prefix, cut);
    }
  return hipGetLastError();
}

// spill_agg_kernel<W> for the record's width
template <int WW>
static hipError_t launch_spill_agg_w(const DevHash& H, int nw, const unsigned long long* sorted, const int64_t* part_begin,
                                     int P, const DevQuery& q, uint64_t* acc, int agg_grid, int S, uint32_t narrow,
                                     hipStream_t st) {
  const size_t lds = (size_t)S * (size_t)(nw + q.nacc) * 8;
  (void)hipFuncSetAttribute((const void*)spill_agg_kernel<WW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(spill_agg_kernel<WW>, dim3((unsigned)agg_grid), dim3(1024), lds, st, sorted, part_begin, P, nw, WW,
                     S, q, H, acc, narrow);
  return hipGetLastError();
}
static hipError_t launch_spill_agg_kernel(const DevHash& H, int nw, const unsigned long long* sorted,
                                          const int64_t* part_begin, int P, const DevQuery& q, uint64_t* acc,
                                          int agg_grid, int S, uint32_t narrow, hipStream_t st) {
  switch (H.spill_words) {
    case 1: return launch_spill_agg_w<1>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 2: return launch_spill_agg_w<2>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 3: return launch_spill_agg_w<3>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 4: return launch_spill_agg_w<4>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 5: return launch_spill_agg_w<5>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 6: return launch_spill_agg_w<6>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 7: return launch_spill_agg_w<7>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    case 8: return launch_spill_agg_w<8>(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_spill_passes(const DevHash& H, int nw, int64_t grid, const uint32_t* hist_unused, int64_t* offs,
                               int64_t* part_begin, unsigned long long* sorted, const DevQuery& q, uint64_t* acc,
                               int agg_grid, int S, int sorted_scatter, uint32_t narrow, hipStream_t st) {
  (void)hist_unused;
  const int P = 1 << (64 - H.spill_shift);
  // offsets of (partition, block) runs, partition-major (the histogram the scan left in H.spill_hist)
  hipLaunchKernelGGL(partition_row_scan_kernel, dim3((unsigned)P), dim3(kBlock), 0, st, H.spill_hist, grid, offs, part_begin);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(kBlock), 0, st, part_begin, (int64_t)P, part_begin + P);
  const auto sorted_lds = [&](int per) {
    return (size_t)1024 * per * H.spill_words * 8 + (size_t)P * (8 + 4 + 4) + (size_t)1024 * per * 2 * 2;
  };
  int per = kSortPerMax;
  // (one block per CU with the largest chunk: halving the LDS for two blocks per CU, 2x shorter runs, measured
  // 6.08 -> 6.57 ms per 400M uniform rows)
  const size_t lds_cap = (size_t)150 * 1024;
  while (per > 1 && sorted_lds(per) > lds_cap) --per;
  if (sorted_scatter && sorted_lds(per) <= lds_cap) {
    (void)hipFuncSetAttribute((const void*)spill_scatter_sorted_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sorted_lds(per));
    hipLaunchKernelGGL(spill_scatter_sorted_kernel, dim3((unsigned)(grid * kSpillGroups)), dim3(1024), sorted_lds(per), st, H, nw, grid,
                       (const int64_t*)offs, (const int64_t*)part_begin, sorted, per);
  } else {
    hipLaunchKernelGGL(spill_scatter_kernel, dim3((unsigned)(grid * kSpillGroups)), dim3(1024), (size_t)P * 4, st, H, nw, grid,
                       (const int64_t*)offs, (const int64_t*)part_begin, sorted);
  }
  return launch_spill_agg_kernel(H, nw, (const unsigned long long*)sorted, (const int64_t*)part_begin, P, q, acc, agg_grid,
                                 S, narrow, st);
}

// Direct placement's tables (DevHash::direct) from a region-mode execution's spill passes: record place
// dbase[p * grid + b] = part_begin[p] + offs[p * grid + b], its count dcnt = the block's records of partition p, and
// the partition begins the aggregation reads (part_begin is shared by the launches of a plan; these are per launch)
__global__ void spill_direct_prep_kernel(const int64_t* offs, const int64_t* part_begin, const uint32_t* hist, int P,
                                         int64_t grid, int64_t* dbase, uint32_t* dcnt, int64_t* pbeg) {
  const int64_t n = (int64_t)P * grid;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    dbase[i] = part_begin[i / grid] + offs[i];
    dcnt[i] = hist[i];
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= P; i += (int64_t)gridDim.x * blockDim.x)
    pbeg[i] = part_begin[i];
}

hipError_t launch_spill_direct_prep(const int64_t* offs, const int64_t* part_begin, const uint32_t* hist, int P,
                                    int64_t grid, int64_t* dbase, uint32_t* dcnt, int64_t* pbeg, hipStream_t st) {
  hipLaunchKernelGGL(spill_direct_prep_kernel, dim3(grid_cap((int64_t)P * grid, kBlock, 4096)), dim3(kBlock), 0, st, offs,
                     part_begin, hist, P, grid, dbase, dcnt, pbeg);
  return hipGetLastError();
}

// the second level's aggregation alone: records already partition-major (direct placement)
hipError_t launch_spill_agg(const DevHash& H, int nw, const unsigned long long* sorted, const int64_t* part_begin,
                            const DevQuery& q, uint64_t* acc, int agg_grid, int S, uint32_t narrow, hipStream_t st) {
  const int P = 1 << (64 - H.spill_shift);
  return launch_spill_agg_kernel(H, nw, sorted, part_begin, P, q, acc, agg_grid, S, narrow, st);
}

hipError_t launch_seg_cut(const unsigned long long* bits, int64_t words, int32_t nsegs, int64_t limit,
                          unsigned long long* cut, hipStream_t st) {
  if (nsegs <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_cut_kernel, dim3((unsigned)nsegs), dim3(1024), 0, st, bits, words, limit, cut);
  return hipGetLastError();
}

hipError_t launch_presence_bitset(const uint64_t* count, int64_t n, unsigned long long* bits, hipStream_t st) {
  const int64_t nw = (n + 63) / 64;
  hipLaunchKernelGGL(presence_bitset_kernel, dim3(grid_cap(nw * 64, kBlock, 8192)), dim3(kBlock), 0, st, count, n, bits);
  return hipGetLastError();
}

hipError_t launch_gather_groups(const int32_t* slots, int64_t ngroups, const unsigned long long* keys, int nw,
                                int64_t cap, const uint64_t* acc, int32_t nacc, uint64_t* out_keys, uint64_t* out_acc,
                                hipStream_t st) {
  if (ngroups <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_groups_kernel, dim3(grid_cap(ngroups, kBlock, 8192)), dim3(kBlock), 0, st, slots, ngroups,
                     keys, nw, cap, acc, nacc, out_keys, out_acc);
  return hipGetLastError();
}

hipError_t launch_export_groups(const int32_t* slots, int64_t ngroups, const unsigned long long* hkeys, int64_t cap,
                                const uint64_t* acc, int32_t nacc_out, const DevKeyPack& kp, uint64_t* out_keys,
                                uint64_t* out_acc, hipStream_t st) {
  if (ngroups <= 0) return hipSuccess;
  hipLaunchKernelGGL(export_groups_kernel, dim3(grid_cap(ngroups, kBlock, 8192)), dim3(kBlock), 0, st, slots, ngroups,
                     hkeys, cap, acc, nacc_out, kp, out_keys, out_acc);
  return hipGetLastError();
}

hipError_t launch_merge_rows(const uint64_t* keys, const uint64_t* acc, int64_t n, int nw, int nacc_in,
                             unsigned long long* fkeys, int64_t fcap, uint64_t* facc, const DevQuery& q,
                             unsigned long long* overflow, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_rows_kernel, dim3(grid_cap(n, kBlock, 8192)), dim3(kBlock), 0, st, keys, acc, n, nw, nacc_in,
                     fkeys, fcap, facc, q, overflow);
  return hipGetLastError();
}

hipError_t launch_read_dict_ids(const uint8_t* packed, int bits, int64_t start, int64_t len, int32_t* out,
                                hipStream_t st) {
  hipLaunchKernelGGL(read_dict_ids_kernel, dim3(grid_for((len + 3) / 4, kBlock)), dim3(kBlock), 0, st, packed, bits,
                     start, len, out);
  return hipGetLastError();
}

hipError_t launch_pack_dict_ids(const int32_t* values, int64_t n, int bits, uint8_t* packed, hipStream_t st) {
  hipLaunchKernelGGL(pack_dict_ids_kernel, dim3(grid_for((n + 7) / 8, kBlock)), dim3(kBlock), 0, st, values, n, bits,
                     packed);
  return hipGetLastError();
}

hipError_t launch_read_raw(const uint8_t* raw, int type, int64_t start, int64_t len, uint8_t* out, hipStream_t st) {
  hipLaunchKernelGGL(read_raw_kernel, dim3(grid_for(len, kBlock)), dim3(kBlock), 0, st, raw, type, start, len, out);
  return hipGetLastError();
}

hipError_t launch_bitset_binop(const uint64_t* a, const uint64_t* b, uint64_t* out, int64_t n, int op,
                               hipStream_t st) {
  unsigned g = grid_for(n, kBlock);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(bitset_binop_kernel, dim3(g), dim3(kBlock), 0, st, a, b, out, n, op);
  return hipGetLastError();
}

hipError_t launch_bitset_not(const uint64_t* a, uint64_t* out, int64_t num_docs, hipStream_t st) {
  unsigned g = grid_for((num_docs + 63) / 64, kBlock);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(bitset_not_kernel, dim3(g), dim3(kBlock), 0, st, a, out, num_docs);
  return hipGetLastError();
}

int64_t compact_num_chunks(int64_t num_docs) { return ((num_docs + 63) / 64 + kCompactWords - 1) / kCompactWords; }

hipError_t launch_bitset_count(const uint64_t* bits, int64_t num_docs, int64_t* d_chunk_counts, int64_t* d_total,
                               hipStream_t st) {
  const int64_t nw = (num_docs + 63) / 64;
  const int64_t nc = compact_num_chunks(num_docs);
  hipLaunchKernelGGL(bitset_chunk_count_kernel, dim3((unsigned)nc), dim3(kBlock), 0, st, bits, nw, d_chunk_counts);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(kBlock), 0, st, d_chunk_counts, nc, d_total);
  return hipGetLastError();
}

hipError_t launch_bitset_compact(const uint64_t* bits, int64_t num_docs, const int64_t* d_chunk_offsets,
                                 int32_t* out, hipStream_t st) {
  const int64_t nw = (num_docs + 63) / 64;
  const int64_t nc = compact_num_chunks(num_docs);
  hipLaunchKernelGGL(bitset_compact_kernel, dim3((unsigned)nc), dim3(kBlock), 0, st, bits, nw, d_chunk_offsets, out);
  return hipGetLastError();
}


hipError_t launch_partition_offsets(const uint32_t* d_hist, int32_t nparts, int64_t nblocks, int64_t* d_offs,
                                    int64_t* d_part_begin, hipStream_t st) {
  if (nparts <= 0) return hipSuccess;
  hipLaunchKernelGGL(partition_row_scan_kernel, dim3((unsigned)nparts), dim3(kBlock), 0, st, d_hist, nblocks, d_offs,
                     d_part_begin);
  hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(kBlock), 0, st, d_part_begin, (int64_t)nparts,
                     d_part_begin + nparts);
  return hipGetLastError();
}

hipError_t launch_allot_prefix(const uint32_t* d_hist, int32_t P, int64_t G, int mode, int64_t stride, double scale,
                               int64_t limit, int64_t* d_ptot, int64_t* d_out, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  hipLaunchKernelGGL(allot_local_kernel, dim3((unsigned)P), dim3(256), 0, st, d_hist, G, mode, stride, scale, d_out, d_ptot);
  hipLaunchKernelGGL(allot_base_kernel, dim3((unsigned)P), dim3(256), 0, st, d_ptot, P, G, limit, d_out);
  return hipGetLastError();
}

hipError_t launch_pack_sel(const void* conts, const int32_t* sel, int64_t n, int group, unsigned long long* out,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_sel_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const RoaringContainer*)conts, sel, n,
                     group, out);
  return hipGetLastError();
}

// the chunk-group size (1, 2, 4 or 8 chunks per work item; the planner groups the containers the same way).
// Swept on configs[2] (profiles/r03/sweep_inv_expand_group.txt): 4 beats 8 (a 64 KiB LDS bitset halves
// the blocks per CU) and 1 (every small container its own line fetch)
int expand_group() {
#ifdef PINOT_AMD_DIAGNOSTICS  // the sweep's knob (diagnostics builds only)
  static const int g = [] {
    const char* e = getenv("PINOT_AMD_EXPAND_GROUP");
    const int v = e ? atoi(e) : 4;
    return v >= 8 ? 8 : v >= 4 ? 4 : v >= 2 ? 2 : 1;
  }();
  return g;
#else
  return 4;
#endif
}

hipError_t launch_roaring_select(const void* d_jobs, const void* d_fs, int32_t nfs, int64_t total_items, const void* d_segs,
                                 int32_t nleaves, int32_t nclauses, unsigned long long* sel_entries,
                                 unsigned long long* sel_count, int64_t sel_cap, unsigned long long* matched_out, int clause,
                                 hipStream_t st) {
  if (nfs <= 0 || total_items <= 0) return hipSuccess;
  const ExpandJob* jobs = reinterpret_cast<const ExpandJob*>(d_jobs);
  const FusedSelSeg* fs = reinterpret_cast<const FusedSelSeg*>(d_fs);
  const DevSegment* segs = reinterpret_cast<const DevSegment*>(d_segs);
  const int64_t blocks = std::min<int64_t>(total_items, 16384);
  if (clause) {
    switch (expand_group()) {
      case 8: hipLaunchKernelGGL(roaring_select_clause_kernel<8>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
      case 4: hipLaunchKernelGGL(roaring_select_clause_kernel<4>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
      case 2: hipLaunchKernelGGL(roaring_select_clause_kernel<2>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
      default: hipLaunchKernelGGL(roaring_select_clause_kernel<1>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
    }
    return hipGetLastError();
  }
  switch (expand_group()) {  // the jobs' container grouping
    case 8: hipLaunchKernelGGL(roaring_select_kernel<8>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
    case 4: hipLaunchKernelGGL(roaring_select_kernel<4>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
    case 2: hipLaunchKernelGGL(roaring_select_kernel<2>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
    default: hipLaunchKernelGGL(roaring_select_kernel<1>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, fs, nfs, total_items, segs, nleaves, nclauses, sel_entries, sel_count, sel_cap, matched_out); break;
  }
  return hipGetLastError();
}

hipError_t launch_expand_jobs(const void* d_jobs, int32_t njobs, int64_t total_items, hipStream_t st) {
  if (njobs <= 0 || total_items <= 0) return hipSuccess;
  const ExpandJob* jobs = reinterpret_cast<const ExpandJob*>(d_jobs);
  const int64_t blocks = std::min<int64_t>(total_items, 16384);
  switch (expand_group()) {
    case 8: hipLaunchKernelGGL(roaring_expand_chunks_kernel<8>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, njobs, total_items); break;
    case 4: hipLaunchKernelGGL(roaring_expand_chunks_kernel<4>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, njobs, total_items); break;
    case 2: hipLaunchKernelGGL(roaring_expand_chunks_kernel<2>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, njobs, total_items); break;
    default: hipLaunchKernelGGL(roaring_expand_chunks_kernel<1>, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, njobs, total_items); break;
  }
  return hipGetLastError();
}

}  // namespace pamd
