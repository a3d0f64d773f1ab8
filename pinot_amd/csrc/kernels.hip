// kernels.hip — gfx950 kernels for Pinot's segment scan / filter / aggregation / group-by.
//
// Layout in HBM: every column keeps the bytes Pinot writes for it — the fixed-bit
// forward index as the big-endian MSB-first bit stream, raw values big-endian — so nothing is
// transcoded at staging time; the kernels byte-swap in registers (v_perm_b32).
//
// Work decomposition: a block of 256 threads (4 wave64) owns a contiguous range of 1024-doc tiles
// across the whole segment batch; each lane owns 4 consecutive docs of a tile, so a raw INT column
// is one 16 B load per lane (1 KiB per wave instruction, fully coalesced) and a LONG/DOUBLE column
// two. Filter, group-key and aggregation are fused in one pass; group accumulators live in LDS
// when the key space fits and are merged into HBM with atomics once per block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "device_types.h"

namespace pamd {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint64_t bswap64(uint32_t hi_word_be, uint32_t lo_word_be) {
  // bytes as stored: hi_word_be holds the first 4 bytes (most significant in BE order)
  return ((uint64_t)bswap32(hi_word_be) << 32) | bswap32(lo_word_be);
}
__device__ __forceinline__ uint64_t ordered_from_double(double d) {
  uint64_t u = (uint64_t)__double_as_longlong(d);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
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

// dictId of a doc of a sorted column: last dictId whose first doc <= doc (SortedIndexReaderImpl).
__device__ __forceinline__ int32_t sorted_dict_id(const int32_t* starts, int32_t card, int64_t doc) {
  int32_t lo = 0, hi = card - 1;
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if ((int64_t)starts[mid] <= doc) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// A lane's raw words for one column of one tile: fetched early (prefetch), decoded later.
struct Raw {
  uint4 a, b;
};

// Issue the loads of a column's 4 docs at doc0: fixed-bit = 5-dword window, raw 4 B = one 16 B
// load, raw 8 B = two 16 B loads. Sorted columns are decoded by dependent lookups (no fetch).
// Every path assigns both vectors whole so the words stay in registers.
__device__ __forceinline__ Raw fetch_slot(const DevColumn& c, int64_t doc0) {
  Raw r;
  if (c.enc == ENC_FIXED_BIT) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(c.data) + ((doc0 * c.bits) >> 5);
    r.a = make_uint4(w[0], w[1], w[2], w[3]);
    r.b = make_uint4(w[4], 0u, 0u, 0u);
  } else if (c.enc == ENC_RAW) {
    if (c.type == T_INT || c.type == T_FLOAT) {
      r.a = *reinterpret_cast<const uint4*>(c.data + doc0 * 4);
      r.b = make_uint4(0u, 0u, 0u, 0u);
    } else {
      r.a = *reinterpret_cast<const uint4*>(c.data + doc0 * 8);
      r.b = *reinterpret_cast<const uint4*>(c.data + doc0 * 8 + 16);
    }
  } else {
    r.a = make_uint4(0u, 0u, 0u, 0u);
    r.b = r.a;
  }
  return r;
}

// Decoded per-slot representation: dictIds (dict columns), INT/LONG values, or FLOAT/DOUBLE as
// double bits.
__device__ __forceinline__ void decode_slot(const DevColumn& c, int64_t doc0, const Raw& r, int64_t v[4]) {
  if (c.enc == ENC_FIXED_BIT) {
    const int bits = c.bits;
    const uint32_t rr = (uint32_t)((doc0 * bits) & 31);
    const uint32_t x0 = bswap32(r.a.x), x1 = bswap32(r.a.y), x2 = bswap32(r.a.z), x3 = bswap32(r.a.w),
                   x4 = bswap32(r.b.x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t p = rr + (uint32_t)(k * bits);
      const uint32_t i = p >> 5, sh = p & 31;
      const uint64_t win = ((uint64_t)sel4(i, x0, x1, x2, x3) << 32) | sel4(i, x1, x2, x3, x4);
      v[k] = (int64_t)((win << sh) >> (64 - bits));
    }
  } else if (c.enc == ENC_RAW) {
    if (c.type == T_INT) {
      v[0] = (int64_t)(int32_t)bswap32(r.a.x);
      v[1] = (int64_t)(int32_t)bswap32(r.a.y);
      v[2] = (int64_t)(int32_t)bswap32(r.a.z);
      v[3] = (int64_t)(int32_t)bswap32(r.a.w);
    } else if (c.type == T_FLOAT) {
      v[0] = __double_as_longlong((double)__uint_as_float(bswap32(r.a.x)));
      v[1] = __double_as_longlong((double)__uint_as_float(bswap32(r.a.y)));
      v[2] = __double_as_longlong((double)__uint_as_float(bswap32(r.a.z)));
      v[3] = __double_as_longlong((double)__uint_as_float(bswap32(r.a.w)));
    } else {
      v[0] = (int64_t)bswap64(r.a.x, r.a.y);
      v[1] = (int64_t)bswap64(r.a.z, r.a.w);
      v[2] = (int64_t)bswap64(r.b.x, r.b.y);
      v[3] = (int64_t)bswap64(r.b.z, r.b.w);
    }
  } else {  // ENC_SORTED
    const int32_t* starts = reinterpret_cast<const int32_t*>(c.data);
    int32_t id = sorted_dict_id(starts, c.card, doc0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      while (id + 1 < c.card && (int64_t)starts[id + 1] <= doc0 + k) ++id;
      v[k] = id;
    }
  }
}

// value of slot element as int64 (for SUM on integer columns) — dict columns go through the
// dictionary (BlockValSet.getLongValuesSV over Dictionary.readLongValues)
__device__ __forceinline__ int64_t slot_value_i64(const DevColumn& c, int64_t x) {
  if (c.enc == ENC_RAW) return x;
  return c.type == T_INT ? (int64_t) reinterpret_cast<const int32_t*>(c.dict)[x]
                         : reinterpret_cast<const int64_t*>(c.dict)[x];
}
// value as double (SUM on FLOAT/DOUBLE, MIN, MAX: Pinot aggregates these in double)
__device__ __forceinline__ double slot_value_f64(const DevColumn& c, int64_t x) {
  if (c.enc == ENC_RAW) {
    return (c.type == T_INT || c.type == T_LONG) ? (double)x : __longlong_as_double(x);
  }
  switch (c.type) {
    case T_INT: return (double)reinterpret_cast<const int32_t*>(c.dict)[x];
    case T_LONG: return (double)reinterpret_cast<const int64_t*>(c.dict)[x];
    case T_FLOAT: return (double)reinterpret_cast<const float*>(c.dict)[x];
    default: return reinterpret_cast<const double*>(c.dict)[x];
  }
}

__device__ __forceinline__ bool in_sorted_i64(const int64_t* a, int32_t n, int64_t v) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == v;
}
__device__ __forceinline__ bool in_sorted_f64(const double* a, int32_t n, double v) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == v;
}

// one predicate leaf over the lane's 4 docs -> 4-bit mask
__device__ __forceinline__ uint32_t eval_leaf(const DevLeaf& L, const int64_t v[4], int64_t doc0) {
  uint32_t m = 0;
  switch (L.kind) {
    case LEAF_DICT_RANGE:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= (uint32_t)(v[k] >= L.lo_i && v[k] < L.hi_i) << k;
      break;
    case LEAF_DICT_SET:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= ((L.bits[v[k] >> 5] >> (v[k] & 31)) & 1u) << k;
      break;
    case LEAF_RAW_RANGE_I:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= (uint32_t)(v[k] >= L.lo_i && v[k] <= L.hi_i) << k;
      break;
    case LEAF_RAW_RANGE_F:
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double d = __longlong_as_double(v[k]);
        m |= (uint32_t)(d >= L.lo_d && d <= L.hi_d) << k;
      }
      break;
    case LEAF_RAW_IN_I:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= (uint32_t)in_sorted_i64(L.in_i, L.in_n, v[k]) << k;
      break;
    case LEAF_RAW_IN_F:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= (uint32_t)in_sorted_f64(L.in_d, L.in_n, __longlong_as_double(v[k])) << k;
      break;
    case LEAF_DOC_RANGE:
#pragma unroll
      for (int k = 0; k < 4; ++k) m |= (uint32_t)(doc0 + k >= L.lo_i && doc0 + k <= L.hi_i) << k;
      break;
    case LEAF_DOC_BITSET: {
      // doc0 is a multiple of 4: the 4 bits sit in one 32-bit word
      m = (L.bits[doc0 >> 5] >> (doc0 & 31)) & 0xFu;
      break;
    }
    default:  // LEAF_CONST
      m = L.lo_i ? 0xFu : 0u;
      break;
  }
  return L.negate ? (~m & 0xFu) : m;
}

// ------------------------------------------------------------------------------------------------
// wave reductions (64 lanes)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_sum_i64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ double wave_sum_f64(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(x, o, 64);
    x = y > x ? y : x;
  }
  return x;
}

// accumulator update at a table word (LDS or HBM; generic address space resolves both)
__device__ __forceinline__ void acc_apply(int32_t op, uint64_t* p, uint64_t bits) {
  switch (op) {
    case ACC_COUNT:
    case ACC_SUM_I64:
      atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
    case ACC_SUM_F64:
      unsafeAtomicAdd(reinterpret_cast<double*>(p), u64_as_double(bits));
      break;
    case ACC_MIN:
      atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
    default:
      atomicMax(reinterpret_cast<unsigned long long*>(p), (unsigned long long)bits);
      break;
  }
}

__device__ __forceinline__ uint64_t acc_identity(int32_t op) {
  if (op == ACC_MIN) return ~0ull;
  return 0ull;  // COUNT/SUM: 0 (also +0.0 for f64); MAX: ordered 0 is below every double
}

// ------------------------------------------------------------------------------------------------
// Fused filter + group-by + aggregation over a batch of segments.
//   kBitset: also write the filter's docId bitset (per segment, at bitset_out[s] words)
//   kLds:    accumulate into an LDS-privatised table of q.lds_keys keys, flushed once per block
// ------------------------------------------------------------------------------------------------
template <int NS, bool kLds, bool kBitset>
__global__ void __launch_bounds__(kBlock) scan_kernel(const DevSegment* __restrict__ segs, const DevQuery q,
                                                      uint64_t* __restrict__ acc,      // [nacc][num_keys]
                                                      uint64_t* const* __restrict__ bitset_out,
                                                      unsigned long long* __restrict__ matched_out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_table[];  // [nacc][lds_keys]
  const int tid = threadIdx.x;
  const int lane = tid & 63;

  if constexpr (kLds) {
    const int n = q.nacc * q.lds_keys;
    for (int i = tid; i < n; i += kBlock) lds_table[i] = acc_identity(q.acc_op[i / q.lds_keys]);
    __syncthreads();
  }
  uint64_t* const table = kLds ? lds_table : acc;
  const int64_t tstride = kLds ? (int64_t)q.lds_keys : q.num_keys;

  // contiguous tile range of this block
  const int64_t per = (q.total_tiles + gridDim.x - 1) / gridDim.x;
  const int64_t t_begin = (int64_t)blockIdx.x * per;
  const int64_t t_end = min(q.total_tiles, t_begin + per);
  int64_t matched = 0;

  int s = 0;
  if (t_begin < t_end) {
    // last segment whose tile_begin <= t_begin (wave-uniform binary search)
    int lo = 0, hi = q.nsegs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs[mid].tile_begin <= t_begin) lo = mid; else hi = mid - 1;
    }
    s = lo;
  }

  auto doc_of = [&](int seg_idx, int64_t t) -> int64_t {
    return (t - segs[seg_idx].tile_begin) * kTileDocs + (int64_t)tid * kDocsPerThread;
  };
  // software pipeline: the next tile's column words are in flight while this tile is processed
  Raw rc[NS];
#pragma unroll
  for (int sl = 0; sl < NS; ++sl) {
    rc[sl].a = make_uint4(0u, 0u, 0u, 0u);
    rc[sl].b = rc[sl].a;
    if (t_begin < t_end && sl < q.nslots) rc[sl] = fetch_slot(segs[s].cols[sl], doc_of(s, t_begin));
  }

  for (int64_t t = t_begin; t < t_end; ++t) {
    const DevSegment& seg = segs[s];
    const int64_t doc0 = doc_of(s, t);
    const int64_t nd = seg.num_docs;
    uint32_t match = doc0 + 4 <= nd ? 0xFu : doc0 >= nd ? 0u : (0xFu >> (4 - (nd - doc0)));

    int s_next = s;
    while (s_next + 1 < q.nsegs && segs[s_next + 1].tile_begin <= t + 1) ++s_next;
    Raw rn[NS];
    const int64_t doc_n = doc_of(s_next, t + 1);
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      rn[sl].a = make_uint4(0u, 0u, 0u, 0u);
      rn[sl].b = rn[sl].a;
      if (t + 1 < t_end && sl < q.nslots) rn[sl] = fetch_slot(segs[s_next].cols[sl], doc_n);
    }

    // ---- decode every referenced column (compile-time slot indices only) ----
    int64_t v[NS][4];
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      if (sl < q.nslots) decode_slot(seg.cols[sl], doc0, rc[sl], v[sl]);
    }

    // ---- filter: AND over clauses of OR over leaves ----
    if (q.nleaves > 0) {
      uint64_t clause_bits = 0;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        if (sl < q.nslots) {
          for (int l = q.slot_leaf_begin[sl]; l < q.slot_leaf_begin[sl + 1]; ++l) {
            const DevLeaf& L = seg.leaves[l];
            clause_bits |= (uint64_t)eval_leaf(L, v[sl], doc0) << (4 * L.clause);
          }
        }
      }
      for (int l = q.slotless_leaf_begin; l < q.slotless_leaf_end; ++l) {
        const DevLeaf& L = seg.leaves[l];
        clause_bits |= (uint64_t)eval_leaf(L, v[0], doc0) << (4 * L.clause);
      }
      for (int c = 0; c < q.nclauses; ++c) match &= (uint32_t)(clause_bits >> (4 * c)) & 0xFu;
    }

    if constexpr (kBitset) {
      // lane l holds bits for docs doc0..doc0+3 = bits 4*(l%16).. of word (tile*16 + tid/16)
      uint64_t w = (uint64_t)match << (4 * (lane & 15));
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) w |= __shfl_xor(w, o, 64);
      if ((lane & 15) == 0) bitset_out[s][(doc0 >> 6)] = w;
    }

    matched += __builtin_popcount(match);
    do {  // aggregation; `break` leaves it, the pipeline rotation below always runs
    if (q.nacc == 0) break;

    // ---- group key per doc ----
    int64_t key[4] = {0, 0, 0, 0};
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      if (sl < q.nslots && q.slot_group_stride[sl] > 0) {
        const int32_t* remap = seg.cols[sl].remap;
        const int64_t st = q.slot_group_stride[sl];
#pragma unroll
        for (int k = 0; k < 4; ++k) key[k] += (int64_t)(remap ? remap[v[sl][k]] : (int32_t)v[sl][k]) * st;
      }
    }

    // ---- aggregation ----
    // wave-uniform key fast path: every matching doc of the wave falls in one group (always true
    // for aggregation-only queries; common for sorted time columns)
    const bool lane_has = match != 0;
    const int first_k = lane_has ? __builtin_ctz(match) : 0;
    const int64_t kA = key[first_k];
    bool lane_uniform = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) lane_uniform &= !((match >> k) & 1) || key[k] == kA;
    const unsigned long long has_mask = __ballot(lane_has);
    if (has_mask == 0) break;
    const int src = __ffsll((long long)has_mask) - 1;
    const int64_t kW = __shfl(kA, src, 64);
    const bool wave_uniform = __ballot(lane_has && (!lane_uniform || kA != kW)) == 0;

    if (wave_uniform) {
      uint64_t* row = table + kW;
      const int64_t cnt = wave_sum_i64(__builtin_popcount(match));
      if (lane == 0) acc_apply(ACC_COUNT, row, (uint64_t)cnt);
#pragma unroll
      for (int sl = 0; sl < NS; ++sl) {
        if (sl < q.nslots) {
          const DevColumn& col = seg.cols[sl];
          for (int a = q.slot_acc_begin[sl]; a < q.slot_acc_begin[sl + 1]; ++a) {
            const int32_t op = q.acc_op[a];
            uint64_t r;
            if (op == ACC_SUM_I64) {
              int64_t p = 0;
#pragma unroll
              for (int k = 0; k < 4; ++k) p += ((match >> k) & 1) ? slot_value_i64(col, v[sl][k]) : 0;
              r = (uint64_t)wave_sum_i64(p);
            } else if (op == ACC_SUM_F64) {
              double p = 0.0;
#pragma unroll
              for (int k = 0; k < 4; ++k) p += ((match >> k) & 1) ? slot_value_f64(col, v[sl][k]) : 0.0;
              r = (uint64_t)__double_as_longlong(wave_sum_f64(p));
            } else if (op == ACC_MIN) {
              uint64_t p = ~0ull;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const double d = slot_value_f64(col, v[sl][k]);
                // NaN: skipped by the group-by `value < min`, ordered below everything (decodes
                // back to NaN) for aggregation-only Math.min
                const uint64_t o = d == d ? ordered_from_double(d) : q.agg_only ? 0ull : ~0ull;
                if (((match >> k) & 1) && o < p) p = o;
              }
              r = wave_min_u64(p);
            } else {
              uint64_t p = 0;
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const double d = slot_value_f64(col, v[sl][k]);
                const uint64_t o = d == d ? ordered_from_double(d) : q.agg_only ? ~0ull : 0ull;
                if (((match >> k) & 1) && o > p) p = o;
              }
              r = wave_max_u64(p);
            }
            if (lane == 0) acc_apply(op, row + (int64_t)a * tstride, r);
          }
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((match >> k) & 1) {
          uint64_t* row = table + key[k];
          acc_apply(ACC_COUNT, row, 1);
#pragma unroll
          for (int sl = 0; sl < NS; ++sl) {
            if (sl < q.nslots) {
              const DevColumn& col = seg.cols[sl];
              for (int a = q.slot_acc_begin[sl]; a < q.slot_acc_begin[sl + 1]; ++a) {
                const int32_t op = q.acc_op[a];
                uint64_t r;
                if (op == ACC_SUM_I64) {
                  r = (uint64_t)slot_value_i64(col, v[sl][k]);
                } else {
                  const double d = slot_value_f64(col, v[sl][k]);
                  if (op != ACC_SUM_F64 && d != d) {
                    if (!q.agg_only) continue;  // group-by MIN/MAX skip NaN (`value < min`)
                    r = op == ACC_MIN ? 0ull : ~0ull;  // Math.min/max propagate NaN
                  } else {
                    r = op == ACC_SUM_F64 ? (uint64_t)__double_as_longlong(d) : ordered_from_double(d);
                  }
                }
                acc_apply(op, row + (int64_t)a * tstride, r);
              }
            }
          }
        }
      }
    }
    } while (0);

#pragma unroll
    for (int sl = 0; sl < NS; ++sl) rc[sl] = rn[sl];
    s = s_next;
  }

  // ---- per-block results ----
  {
    const int64_t wm = wave_sum_i64(matched);
    if (lane == 0 && wm) atomicAdd(matched_out, (unsigned long long)wm);
  }
  if constexpr (kLds) {
    __syncthreads();
    for (int g = tid; g < q.lds_keys; g += kBlock) {
      if (lds_table[g] == 0) continue;  // no matching doc in this block for key g
      for (int a = 0; a < q.nacc; ++a)
        acc_apply(q.acc_op[a], acc + (int64_t)a * q.num_keys + g, lds_table[(int64_t)a * q.lds_keys + g]);
    }
  }
}

__global__ void init_acc_kernel(uint64_t* acc, int64_t num_keys, DevQuery q) {
  const int64_t n = (int64_t)q.nacc * num_keys;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc[i] = acc_identity(q.acc_op[i / num_keys]);
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
struct RoaringContainer {
  uint32_t key;      // high 16 bits of the docIds
  uint32_t kind;     // 0 array, 1 bitmap, 2 run
  uint32_t count;    // array: cardinality, run: number of runs
  uint32_t pad;
  uint64_t offset;   // byte offset of the container payload inside the staged inverted index
};

// Batched expansion: every (segment, inverted-index leaf) of a plan is one ExpandJob; a work item
// is one 65536-doc chunk of one job. A block builds its chunk's 8 KiB of bitset in LDS from the
// chunk's selected containers (LDS atomics, no global atomics), then writes all 1024 words once
// (chunks with no container write zeros, so no separate clear pass). Small array containers are
// expanded one per lane; bitmap, run and large array containers by a whole wave.
__global__ void __launch_bounds__(kBlock) roaring_expand_chunks_kernel(const ExpandJob* jobs, int32_t njobs,
                                                                      int64_t total_items) {
  __shared__ uint32_t lbits[2048];
  __shared__ int32_t bigq[kBlock];
  __shared__ int32_t nbig;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].item_begin <= item) lo = mid; else hi = mid - 1;
    }
    const ExpandJob& J = jobs[lo];
    const int32_t k = (int32_t)(item - J.item_begin);
    for (int i = tid; i < 2048; i += kBlock) lbits[i] = 0u;
    if (tid == 0) nbig = 0;
    __syncthreads();
    const int32_t g0 = J.grp[k], g1 = J.grp[k + 1];
    for (int32_t base = g0; base < g1; base += kBlock) {
      const int32_t ci = base + tid;
      if (ci < g1) {
        const RoaringContainer c = J.conts[J.sel[ci]];
        const uint8_t* p = J.inv + c.offset;
        if (c.kind == 0 && c.count <= 16) {
          for (uint32_t e = 0; e < c.count; ++e) {
            const uint32_t d = p[2 * e] | (p[2 * e + 1] << 8);
            atomicOr(&lbits[d >> 5], 1u << (d & 31));
          }
        } else {
          bigq[atomicAdd(&nbig, 1)] = J.sel[ci];
        }
      }
      __syncthreads();
      const int nb = nbig;
      for (int qi = wave; qi < nb; qi += kBlock / 64) {
        const RoaringContainer c = J.conts[bigq[qi]];
        const uint8_t* p = J.inv + c.offset;
        if (c.kind == 1) {
          for (int i = lane; i < 1024; i += 64) {
            const uint64_t w = *reinterpret_cast<const uint64_t*>(p + 8 * i);  // LE
            if (w) {
              atomicOr(&lbits[2 * i], (uint32_t)w);
              atomicOr(&lbits[2 * i + 1], (uint32_t)(w >> 32));
            }
          }
        } else if (c.kind == 0) {
          for (uint32_t e = lane; e < c.count; e += 64) {
            const uint32_t d = p[2 * e] | (p[2 * e + 1] << 8);
            atomicOr(&lbits[d >> 5], 1u << (d & 31));
          }
        } else {
          for (uint32_t r = 0; r < c.count; ++r) {
            const uint8_t* q = p + 2 + 4 * r;
            const uint32_t s0 = q[0] | (q[1] << 8);
            const uint32_t e0 = s0 + (q[2] | (q[3] << 8));  // inclusive, < 65536
            const uint32_t w0 = s0 >> 5, w1 = e0 >> 5;
            for (uint32_t w = w0 + lane; w <= w1; w += 64) {
              uint32_t m = ~0u;
              if (w == w0) m &= ~0u << (s0 & 31);
              if (w == w1) m &= ~0u >> (31 - (e0 & 31));
              atomicOr(&lbits[w], m);
            }
          }
        }
      }
      __syncthreads();
      if (tid == 0) nbig = 0;
      __syncthreads();
    }
    // write the chunk (docs >= num_docs are never set: bitmaps hold only the segment's docIds)
    const int64_t w_begin = (int64_t)k * 1024;
    for (int i = tid; i < 1024; i += kBlock) {
      const int64_t w = w_begin + i;
      if (w < J.nwords) J.bitset[w] = (unsigned long long)lbits[2 * i] | ((unsigned long long)lbits[2 * i + 1] << 32);
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

template <int NS>
static hipError_t launch_scan_ns(const DevSegment* d_segs, const DevQuery& q, uint64_t* d_acc,
                                 uint64_t* const* d_bitsets, unsigned long long* d_matched, int grid, size_t shmem,
                                 hipStream_t st) {
  if (d_bitsets)  // filter-only plan (FilterPlanNode -> docId set): no accumulators
    hipLaunchKernelGGL((scan_kernel<NS, false, true>), dim3(grid), dim3(kBlock), 0, st, d_segs, q, d_acc, d_bitsets,
                       d_matched);
  else if (q.lds_keys > 0)
    hipLaunchKernelGGL((scan_kernel<NS, true, false>), dim3(grid), dim3(kBlock), shmem, st, d_segs, q, d_acc, nullptr,
                       d_matched);
  else
    hipLaunchKernelGGL((scan_kernel<NS, false, false>), dim3(grid), dim3(kBlock), shmem, st, d_segs, q, d_acc,
                       nullptr, d_matched);
  return hipGetLastError();
}

// slot-count variant: decoded values live in NS x 4 registers, so a 4-column query does not pay
// the register cost (and occupancy) of the 8-column kernel
static inline int ns_for(int nslots) { return nslots <= 1 ? 1 : nslots <= 2 ? 2 : nslots <= 4 ? 4 : 8; }

hipError_t launch_scan(const DevSegment* d_segs, const DevQuery& q, uint64_t* d_acc, uint64_t* const* d_bitsets,
                       unsigned long long* d_matched, int grid, hipStream_t st) {
  const size_t shmem = q.lds_keys > 0 ? (size_t)q.nacc * q.lds_keys * 8 : 0;
  if (d_bitsets && q.nacc > 0) return hipErrorNotSupported;
  switch (ns_for(q.nslots)) {
    case 1: return launch_scan_ns<1>(d_segs, q, d_acc, d_bitsets, d_matched, grid, shmem, st);
    case 2: return launch_scan_ns<2>(d_segs, q, d_acc, d_bitsets, d_matched, grid, shmem, st);
    case 4: return launch_scan_ns<4>(d_segs, q, d_acc, d_bitsets, d_matched, grid, shmem, st);
    default: return launch_scan_ns<8>(d_segs, q, d_acc, d_bitsets, d_matched, grid, shmem, st);
  }
}

template <int NS>
static int occupancy_ns(bool lds, size_t shmem) {
  int n = 0;
  const hipError_t e = lds ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<NS, true, false>, kBlock, shmem)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scan_kernel<NS, false, false>, kBlock, shmem);
  return (e == hipSuccess && n > 0) ? n : 1;
}

int scan_blocks_per_cu(int nslots, bool lds, size_t shmem) {
  switch (ns_for(nslots)) {
    case 1: return occupancy_ns<1>(lds, shmem);
    case 2: return occupancy_ns<2>(lds, shmem);
    case 4: return occupancy_ns<4>(lds, shmem);
    default: return occupancy_ns<8>(lds, shmem);
  }
}

hipError_t launch_init_acc(uint64_t* d_acc, const DevQuery& q, hipStream_t st) {
  const int64_t n = (int64_t)q.nacc * q.num_keys;
  unsigned g = grid_for(n, kBlock);
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(init_acc_kernel, dim3(g), dim3(kBlock), 0, st, d_acc, q.num_keys, q);
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

hipError_t launch_expand_jobs(const void* d_jobs, int32_t njobs, int64_t total_items, hipStream_t st) {
  if (njobs <= 0 || total_items <= 0) return hipSuccess;
  const ExpandJob* jobs = reinterpret_cast<const ExpandJob*>(d_jobs);
  const int64_t blocks = std::min<int64_t>(total_items, 16384);
  hipLaunchKernelGGL(roaring_expand_chunks_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, jobs, njobs,
                     total_items);
  return hipGetLastError();
}

}  // namespace pamd
