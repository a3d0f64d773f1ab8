// FETCH_SIZE calibration for the access shapes of the selective plans (round-5 verdict: profiles/summarize.py
// doubled FETCH_SIZE for every kernel, while MI355X_MICROARCH.md states the 1/2 under-count only for wide coalesced
// streaming reads). Kernels reading a KNOWN set of bytes, each launch behind a 1 GiB write that pushes the earlier
// data out of the 256 MiB Infinity Cache:
//   probe_stream16   16 B per lane, coalesced, grid-stride (the guide's calibrated case)
//   probe_idx        a sorted docId list read 4 B per lane (the selection vector alone)
//   probe_gather4    the docId list, then a 4-byte value per docId (pinot_gather's fixed-bit / raw INT reads)
//   probe_gather8    the same with 8-byte values (raw LONG / DOUBLE)
//   probe_chunks     one wave per variable-length contiguous span of 16-4096 B (roaring array containers)
// Host side: for every launch, the bytes it needs at 32-, 64- and 128-byte granularity (distinct sectors / lines
// touched), printed as one JSON line per launch in launch order; profiles/fetch_probe.py joins them with the
// rocprofv3 --pmc dispatches and gives FETCH_SIZE x 1024 / known bytes per shape.
//   hipcc --offload-arch=gfx950 -O3 -o build/fetch_probe profiles/fetch_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__global__ void __launch_bounds__(256) probe_flush(uint4* buf, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    buf[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

__global__ void __launch_bounds__(256) probe_stream16(const uint4* a, size_t n, unsigned* out) {
  unsigned x = 0u;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9E3779B9u) out[0] = x;  // keeps the loads; practically never stores
}

__global__ void __launch_bounds__(256) probe_idx(const uint32_t* idx, size_t m, unsigned* out) {
  unsigned x = 0u;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) x ^= idx[i];
  if (x == 0x9E3779B9u) out[0] = x;
}

__global__ void __launch_bounds__(256) probe_gather4(const uint32_t* col, const uint32_t* idx, size_t m, unsigned* out) {
  unsigned x = 0u;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x)
    x ^= col[idx[i]];
  if (x == 0x9E3779B9u) out[0] = x;
}

__global__ void __launch_bounds__(256) probe_gather8(const uint64_t* col, const uint32_t* idx, size_t m, unsigned* out) {
  unsigned long long x = 0ull;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x)
    x ^= col[idx[i]];
  if (x == 0x9E3779B97F4A7C15ull) out[0] = (unsigned)x;
}

// one wave per span: lanes read the span's 16-byte words (a span of 16-4096 B: 1-256 words)
__global__ void __launch_bounds__(256) probe_chunks(const uint4* a, const uint64_t* starts, const uint32_t* words,
                                                    int nspans, unsigned* out) {
  const int lane = threadIdx.x & 63;
  unsigned x = 0u;
  for (int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < nspans; s += (gridDim.x * blockDim.x) >> 6) {
    const uint64_t b = starts[s];
    for (uint32_t w = lane; w < words[s]; w += 64) {
      const uint4 v = a[b + w];
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (x == 0x9E3779B9u) out[0] = x;
}

struct Known {
  uint64_t b32 = 0, b64 = 0, b128 = 0;
};

// distinct 32 / 64 / 128-byte units of the byte addresses [a, a + len) over a sorted list
static Known units(const std::vector<std::pair<uint64_t, uint64_t>>& spans) {
  Known k;
  uint64_t l32 = ~0ull, l64 = ~0ull, l128 = ~0ull;
  for (auto [a, len] : spans) {
    for (uint64_t u = a >> 5; u <= (a + len - 1) >> 5; ++u)
      if (u != l32) { ++k.b32; l32 = u; }
    for (uint64_t u = a >> 6; u <= (a + len - 1) >> 6; ++u)
      if (u != l64) { ++k.b64; l64 = u; }
    for (uint64_t u = a >> 7; u <= (a + len - 1) >> 7; ++u)
      if (u != l128) { ++k.b128; l128 = u; }
  }
  k.b32 *= 32;
  k.b64 *= 64;
  k.b128 *= 128;
  return k;
}

static void report(const char* kernel, const char* shape, double param, uint64_t bytes, const Known& k,
                   uint64_t meta = 0) {
  printf("{\"kernel\": \"%s\", \"shape\": \"%s\", \"param\": %g, \"bytes\": %llu, \"b32\": %llu, \"b64\": %llu, "
         "\"b128\": %llu, \"meta\": %llu}\n",
         kernel, shape, param, (unsigned long long)bytes, (unsigned long long)k.b32, (unsigned long long)k.b64,
         (unsigned long long)k.b128, (unsigned long long)meta);
  fflush(stdout);
}

int main() {
  const size_t N4 = (size_t)1 << 28;  // 1 GiB of 4-byte values
  const size_t N8 = (size_t)1 << 27;  // 1 GiB of 8-byte values
  const size_t FL = ((size_t)1 << 30) / 16;
  uint4 *flush, *stream;
  uint32_t *col4, *idx;
  uint64_t* col8;
  unsigned* out;
  CK(hipMalloc(&flush, FL * 16));
  CK(hipMalloc(&stream, FL * 16));
  CK(hipMalloc(&col4, N4 * 4));
  CK(hipMalloc(&col8, N8 * 8));
  CK(hipMalloc(&idx, N4 * 4));  // a docId list of up to every row
  CK(hipMalloc(&out, 64));
  CK(hipMemset(stream, 1, FL * 16));
  CK(hipMemset(col4, 2, N4 * 4));
  CK(hipMemset(col8, 3, N8 * 8));
  const int grid = 256 * 8 * 4;
  auto flush_l3 = [&]() {
    hipLaunchKernelGGL(probe_flush, dim3(grid), dim3(256), 0, 0, flush, FL);
    CK(hipDeviceSynchronize());
  };
  // 1. streaming 16 B per lane
  flush_l3();
  hipLaunchKernelGGL(probe_stream16, dim3(grid), dim3(256), 0, 0, stream, FL, out);
  CK(hipDeviceSynchronize());
  report("probe_stream16", "stream16", 0, FL * 16, units({{0, FL * 16}}));
  // 2. sorted docId lists at several selectivities, over the 4- and 8-byte columns
  std::mt19937_64 rng(7);
  for (double sel : {0.001, 0.01, 0.1, 0.5}) {
    for (int w : {4, 8}) {
      const size_t n = w == 4 ? N4 : N8;
      std::vector<uint32_t> h;
      h.reserve((size_t)(n * sel * 1.1) + 16);
      std::bernoulli_distribution pick(sel);
      for (size_t d = 0; d < n; ++d)
        if (pick(rng)) h.push_back((uint32_t)d);
      const size_t m = h.size();
      CK(hipMemcpy(idx, h.data(), m * 4, hipMemcpyHostToDevice));
      std::vector<std::pair<uint64_t, uint64_t>> sp;
      sp.reserve(m);
      for (uint32_t d : h) sp.push_back({(uint64_t)d * w, (uint64_t)w});
      const Known kv = units(sp);
      const Known ki = units({{0, m * 4}});
      flush_l3();
      hipLaunchKernelGGL(probe_idx, dim3(grid), dim3(256), 0, 0, idx, m, out);
      CK(hipDeviceSynchronize());
      report("probe_idx", w == 4 ? "idx_for_gather4" : "idx_for_gather8", sel, m * 4, ki);
      flush_l3();
      if (w == 4) hipLaunchKernelGGL(probe_gather4, dim3(grid), dim3(256), 0, 0, col4, idx, m, out);
      else hipLaunchKernelGGL(probe_gather8, dim3(grid), dim3(256), 0, 0, col8, idx, m, out);
      CK(hipDeviceSynchronize());
      report(w == 4 ? "probe_gather4" : "probe_gather8", w == 4 ? "gather4_values" : "gather8_values", sel, m * w, kv);
    }
  }
  // 3. variable-length contiguous spans (roaring containers): 16-4096 B at random 16-byte-aligned places, sorted
  for (int avg : {64, 512, 2048}) {
    const int nspans = (int)std::min<size_t>(400000, (size_t)512 * 1024 * 1024 / avg);
    std::vector<uint64_t> st(nspans);
    std::vector<uint32_t> wd(nspans);
    std::uniform_int_distribution<uint64_t> pos(0, FL - 300);
    std::uniform_int_distribution<uint32_t> len(1, (uint32_t)std::max(1, avg / 8));
    for (int s = 0; s < nspans; ++s) st[s] = pos(rng);
    std::sort(st.begin(), st.end());
    uint64_t bytes = 0;
    std::vector<std::pair<uint64_t, uint64_t>> sp;
    for (int s = 0; s < nspans; ++s) {
      wd[s] = std::min<uint32_t>(256, len(rng));
      if (s + 1 < nspans && st[s] + wd[s] > st[s + 1]) wd[s] = (uint32_t)std::max<uint64_t>(1, st[s + 1] - st[s]);
      bytes += (uint64_t)wd[s] * 16;
      sp.push_back({st[s] * 16, (uint64_t)wd[s] * 16});
    }
    uint64_t* dst;
    uint32_t* dwd;
    CK(hipMalloc(&dst, nspans * 8));
    CK(hipMalloc(&dwd, nspans * 4));
    CK(hipMemcpy(dst, st.data(), nspans * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwd, wd.data(), nspans * 4, hipMemcpyHostToDevice));
    flush_l3();
    hipLaunchKernelGGL(probe_chunks, dim3(grid), dim3(256), 0, 0, stream, dst, dwd, nspans, out);
    CK(hipDeviceSynchronize());
    report("probe_chunks", "spans", avg, bytes, units(sp), (uint64_t)nspans * 12);  // + the span list, streamed
    CK(hipFree(dst));
    CK(hipFree(dwd));
  }
  return 0;
}
