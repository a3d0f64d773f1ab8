// derive.hip — dictionary twin of a raw INT / LONG / FLOAT / DOUBLE column, derived on the device
// (GROUP BY on a raw column groups by value: NoDictionarySingleColumnGroupKeyGenerator.java:98-143
// keeps a value -> group id map per segment; here each segment gets, once, a sorted dictionary of its
// distinct values and a fixed-bit dictId forward index, so raw group-by columns take the dictionary
// plans). Values are compared by Java's identity for FLOAT / DOUBLE (Float.floatToIntBits /
// Double.doubleToLongBits equality: every NaN one value, -0.0 != 0.0) and ordered by Double.compare.
//
//   1. order_keys_kernel:   big-endian staged values -> order-preserving uint64 keys
//   2. rocprim radix sort of the keys (a copy)
//   3. unique_flags_kernel + exclusive scan: distinct keys in order, their count = cardinality
//   4. dict_ids_kernel:     per doc, the dictId (binary search in the distinct keys)
//   5. dict_values_kernel:  distinct keys -> big-endian dictionary values (the staged dictionary format)
// The fixed-bit packing reuses pack_dict_ids_kernel (kernels.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "device_types.h"

namespace pamd {

__device__ __forceinline__ uint64_t java_double_order_dev(double v) {
  // Double.compare order: NaN (canonical, above +inf); -0.0 < 0.0
  uint64_t b = (uint64_t)__double_as_longlong(v);
  if (v != v) b = 0x7FF8000000000000ull;
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void order_keys_kernel(const uint8_t* be, int type, int64_t n, uint64_t* keys) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    uint64_t k;
    if (type == T_INT || type == T_FLOAT) {
      const uint32_t u = __builtin_bswap32(reinterpret_cast<const uint32_t*>(be)[d]);
      if (type == T_INT) k = (uint64_t)(int64_t)(int32_t)u ^ (1ull << 63);
      else k = java_double_order_dev((double)__uint_as_float(u));
    } else {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(be) + 2 * d;
      const uint64_t u = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
      k = type == T_LONG ? (u ^ (1ull << 63)) : java_double_order_dev(__longlong_as_double((long long)u));
    }
    keys[d] = k;
  }
}

__global__ void unique_flags_kernel(const uint64_t* sorted, int64_t n, uint32_t* flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = (i == 0 || sorted[i] != sorted[i - 1]) ? 1u : 0u;
}

__global__ void scatter_unique_kernel(const uint64_t* sorted, const uint32_t* flags, const uint32_t* pos, int64_t n,
                                      uint64_t* uniq) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (flags[i]) uniq[pos[i]] = sorted[i];
}

__global__ void dict_ids_kernel(const uint64_t* keys, int64_t n, const uint64_t* uniq, int64_t card, int32_t* ids) {
  for (int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; d < n; d += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[d];
    int64_t lo = 0, hi = card - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (uniq[mid] < k) lo = mid + 1; else hi = mid;
    }
    ids[d] = (int32_t)lo;
  }
}

// distinct keys -> dictionary values, big-endian fixed width (4 B INT / FLOAT, 8 B LONG / DOUBLE)
__global__ void dict_values_kernel(const uint64_t* uniq, int64_t card, int type, uint8_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < card; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = uniq[i];
    uint64_t u;
    if (type == T_INT || type == T_LONG) {
      u = k ^ (1ull << 63);
    } else {
      const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
      if (type == T_FLOAT) {
        const float f = (float)__longlong_as_double((long long)b);
        u = (uint64_t)__float_as_uint(f);
      } else {
        u = b;
      }
    }
    if (type == T_INT || type == T_FLOAT) {
      reinterpret_cast<uint32_t*>(out)[i] = __builtin_bswap32((uint32_t)u);
    } else {
      reinterpret_cast<uint32_t*>(out)[2 * i] = __builtin_bswap32((uint32_t)(u >> 32));
      reinterpret_cast<uint32_t*>(out)[2 * i + 1] = __builtin_bswap32((uint32_t)u);
    }
  }
}

static unsigned grid_of(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}

// scratch: caller-provided device buffers sized by derive_dictionary_scratch (keys, sorted keys, flags,
// positions, distinct keys: n entries each, plus the sort / scan temporary storage)
size_t derive_dictionary_scratch(int64_t n) {
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_keys(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (unsigned int)n, 0,
                                 64);
  (void)rocprim::exclusive_scan(nullptr, scan_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n,
                                rocprim::plus<uint32_t>());
  const size_t tmp = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
  return (size_t)n * (8 + 8 + 4 + 4 + 8) + tmp + 256;
}

// -> *h_card distinct values; d_ids[n] the docs' dictIds; d_dict_be[card * value size] the dictionary
hipError_t derive_dictionary(const uint8_t* d_be, int type, int64_t n, void* d_scratch, int32_t* d_ids,
                             uint8_t* d_dict_be, int64_t* h_card, hipStream_t st) {
  if (n <= 0) {
    *h_card = 0;
    return hipSuccess;
  }
  uint8_t* p = reinterpret_cast<uint8_t*>(d_scratch);
  uint64_t* keys = reinterpret_cast<uint64_t*>(p);
  uint64_t* sorted = keys + n;
  uint32_t* flags = reinterpret_cast<uint32_t*>(sorted + n);
  uint32_t* pos = flags + n;
  uint64_t* uniq = reinterpret_cast<uint64_t*>(pos + n);
  void* tmp = reinterpret_cast<void*>(((uintptr_t)(uniq + n) + 255) & ~(uintptr_t)255);
  size_t sort_bytes = 0, scan_bytes = 0;
  hipError_t e = rocprim::radix_sort_keys(nullptr, sort_bytes, keys, sorted, (unsigned int)n, 0, 64, st);
  if (e != hipSuccess) return e;
  e = rocprim::exclusive_scan(nullptr, scan_bytes, flags, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(order_keys_kernel, dim3(grid_of(n)), dim3(256), 0, st, d_be, type, n, keys);
  e = rocprim::radix_sort_keys(tmp, sort_bytes, keys, sorted, (unsigned int)n, 0, 64, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(unique_flags_kernel, dim3(grid_of(n)), dim3(256), 0, st, sorted, n, flags);
  e = rocprim::exclusive_scan(tmp, scan_bytes, flags, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
  if (e != hipSuccess) return e;
  uint32_t last[2];
  e = hipMemcpyAsync(&last[0], pos + n - 1, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(&last[1], flags + n - 1, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return e;
  const int64_t card = (int64_t)last[0] + last[1];
  hipLaunchKernelGGL(scatter_unique_kernel, dim3(grid_of(n)), dim3(256), 0, st, sorted, flags, pos, n, uniq);
  hipLaunchKernelGGL(dict_ids_kernel, dim3(grid_of(n)), dim3(256), 0, st, keys, n, uniq, card, d_ids);
  hipLaunchKernelGGL(dict_values_kernel, dim3(grid_of(card)), dim3(256), 0, st, uniq, card, type, d_dict_be);
  *h_card = card;
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Compacted hash-table groups in ascending key order (the order a dense table's groups come in): a
// hash plan's packed key words compare, as one (nwk x 64)-bit integer with word nwk - 1 most
// significant, exactly as the group columns' merged ids from the last column to the first, so a stable
// LSD radix sort over the words -- least significant word first, each pass sorting (word, row) pairs in
// the order the previous passes left -- yields the permutation; the rows are then gathered.
// ------------------------------------------------------------------------------------------------
__global__ void key_word_kernel(const uint64_t* keys, int nwk, int w, const uint32_t* idx, int64_t n, uint64_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = keys[(idx ? (int64_t)idx[i] : i) * nwk + w];
}
__global__ void iota_kernel(uint32_t* idx, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = (uint32_t)i;
}
__global__ void gather_rows_kernel(const uint64_t* src, int width, const uint32_t* idx, int64_t n, uint64_t* dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * width; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / width, c = i - r * width;
    dst[i] = src[(int64_t)idx[r] * width + c];
  }
}

size_t sort_rows_scratch(int64_t n) {
  size_t sort_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (unsigned int)n, 0, 64);
  return (size_t)n * (8 + 8 + 4 + 4) + sort_bytes + 512;
}

// keys: n rows of nwk words (row-major), acc: n rows of nacc words; word_bits[w]: bits word w can use.
// Rows written to keys_out / acc_out in ascending key order.
hipError_t sort_rows_by_key(const uint64_t* keys, int nwk, const int* word_bits, const uint64_t* acc, int nacc, int64_t n,
                            void* scratch, uint64_t* keys_out, uint64_t* acc_out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  uint8_t* p = reinterpret_cast<uint8_t*>(scratch);
  uint64_t* kw = reinterpret_cast<uint64_t*>(p);
  uint64_t* kw2 = kw + n;
  uint32_t* idx = reinterpret_cast<uint32_t*>(kw2 + n);
  uint32_t* idx2 = idx + n;
  void* tmp = reinterpret_cast<void*>(((uintptr_t)(idx2 + n) + 255) & ~(uintptr_t)255);
  size_t sort_bytes = 0;
  hipError_t e = rocprim::radix_sort_pairs(nullptr, sort_bytes, kw, kw2, idx, idx2, (unsigned int)n, 0, 64, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(iota_kernel, dim3(grid_of(n)), dim3(256), 0, st, idx, n);
  for (int w = 0; w < nwk; ++w) {
    hipLaunchKernelGGL(key_word_kernel, dim3(grid_of(n)), dim3(256), 0, st, keys, nwk, w, (const uint32_t*)idx, n, kw);
    const unsigned end_bit = (unsigned)(word_bits[w] < 1 ? 1 : word_bits[w] > 64 ? 64 : word_bits[w]);
    e = rocprim::radix_sort_pairs(tmp, sort_bytes, kw, kw2, idx, idx2, (unsigned int)n, 0u, end_bit, st);
    if (e != hipSuccess) return e;
    uint32_t* t = idx;  // the sorted permutation becomes the next pass's input order
    idx = idx2;
    idx2 = t;
  }
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_of(n * nwk)), dim3(256), 0, st, keys, nwk, (const uint32_t*)idx, n, keys_out);
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_of(n * nacc)), dim3(256), 0, st, acc, nacc, (const uint32_t*)idx, n, acc_out);
  return hipGetLastError();
}

}  // namespace pamd
