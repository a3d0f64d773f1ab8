// module_unload_probe.hip -- round 6: do device buffers allocated and uploaded after a code object was loaded
// and unloaded (hipModuleLoadData + hipModuleUnload, the on-disk JIT cache's validity probe before round 6) read
// back correctly on every XCD?
//
// Per trial: allocate `nbuf` buffers and upload a distinct pattern into each through hipMemcpy from pageable host
// memory (the library's staging path), [optionally] load + unload the code object given on the command line (never
// launched), load it again and keep it (the cache's real load), then read every buffer back on every XCD
// (64 blocks, each reading all of it), counting words that differ from the pattern. Control: the same trials
// without the load + unload.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/module_unload_probe scripts/module_unload_probe.hip
//   ./build/module_unload_probe build/part.co [trials] [nbuf] [kib]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(2);                                                                                 \
    }                                                                                          \
  } while (0)

__host__ __device__ inline uint32_t pat(uint64_t i, uint32_t salt) {
  uint32_t h = (uint32_t)i * 2654435761u ^ salt;
  h ^= h >> 15;
  h *= 0x2c1b3c6du;
  h ^= h >> 12;
  return h | 1u;
}

__device__ inline uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xFu;
}

// out[b * 4 + 0..3]: stale words seen by block b, first stale index, its value, the block's XCC id
__global__ void k_check(const uint32_t* x, size_t n, uint32_t salt, unsigned long long* out) {
  __shared__ unsigned long long bad, first, val;
  if (threadIdx.x == 0) {
    bad = 0;
    first = ~0ull;
    val = 0;
  }
  __syncthreads();
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = x[i];
    if (v != pat(i, salt)) {
      atomicAdd(&bad, 1ull);
      if (atomicMin(&first, (unsigned long long)i) > i) val = v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = bad;
    out[blockIdx.x * 4 + 1] = first;
    out[blockIdx.x * 4 + 2] = val;
    out[blockIdx.x * 4 + 3] = xcc_id();
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s code_object [trials] [nbuf] [kib]\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string image = ss.str();
  const int trials = argc > 2 ? atoi(argv[2]) : 20;
  const int nbuf = argc > 3 ? atoi(argv[3]) : 32;
  const size_t bytes = (size_t)(argc > 4 ? atoi(argv[4]) : 128) << 10;
  const size_t n = bytes / 4;
  const int kBlocks = 64;
  unsigned long long* d_out = nullptr;
  CK(hipMalloc(&d_out, kBlocks * 4 * 8));
  std::vector<unsigned long long> h_out(kBlocks * 4);
  std::vector<uint32_t> host(n);
  int total[2] = {0, 0};
  for (int mode = 0; mode < 2; ++mode) {  // 0: control (no load / unload), 1: probe load + unload, then load
    std::vector<hipModule_t> kept;
    unsigned long long stale_words = 0, stale_bufs = 0, bufs = 0, pre_stale = 0;
    for (int t = 0; t < trials; ++t) {
      // the data first (the failing test stages its segments before it plans), then the module loads
      std::vector<uint32_t*> xs(nbuf, nullptr);
      for (int b = 0; b < nbuf; ++b) {
        CK(hipMalloc(&xs[b], bytes));
        const uint32_t salt = 0x5000u + 977u * (uint32_t)(t * nbuf + b) + 131u * (uint32_t)mode;
        for (size_t i = 0; i < n; ++i) host[i] = pat(i, salt);
        CK(hipMemcpy(xs[b], host.data(), bytes, hipMemcpyHostToDevice));
      }
      for (int b = 0; b < nbuf; ++b) {  // read once before the module work (the test's first query scans the segments)
        const uint32_t salt = 0x5000u + 977u * (uint32_t)(t * nbuf + b) + 131u * (uint32_t)mode;
        k_check<<<kBlocks, 256>>>(xs[b], n, salt, d_out);
        CK(hipGetLastError());
        CK(hipMemcpy(h_out.data(), d_out, h_out.size() * 8, hipMemcpyDeviceToHost));
        for (int blk = 0; blk < kBlocks; ++blk) pre_stale += h_out[blk * 4];
      }
      if (mode == 1) {
        hipModule_t m = nullptr;
        CK(hipModuleLoadData(&m, image.data()));
        CK(hipModuleUnload(m));
      }
      hipModule_t k = nullptr;
      CK(hipModuleLoadData(&k, image.data()));
      kept.push_back(k);
      for (int b = 0; b < nbuf; ++b) {
        const uint32_t salt = 0x5000u + 977u * (uint32_t)(t * nbuf + b) + 131u * (uint32_t)mode;
        k_check<<<kBlocks, 256>>>(xs[b], n, salt, d_out);
        CK(hipGetLastError());
        CK(hipMemcpy(h_out.data(), d_out, h_out.size() * 8, hipMemcpyDeviceToHost));
        ++bufs;
        bool any = false;
        for (int blk = 0; blk < kBlocks; ++blk) {
          if (!h_out[blk * 4]) continue;
          stale_words += h_out[blk * 4];
          if (!any && stale_bufs < 4)
            printf("  STALE mode %d trial %d buf %d (%p) block %d xcc %llu: %llu words, first index %llu = %08llx "
                   "(expected %08x)\n",
                   mode, t, b, (void*)xs[b], blk, h_out[blk * 4 + 3], h_out[blk * 4], h_out[blk * 4 + 1],
                   h_out[blk * 4 + 2], pat(h_out[blk * 4 + 1], salt));
          any = true;
        }
        stale_bufs += any;
      }
      for (int b = 0; b < nbuf; ++b) CK(hipFree(xs[b]));
    }
    for (auto k : kept) CK(hipModuleUnload(k));
    printf("mode %d (%s): %llu / %llu buffers read stale somewhere, %llu stale words (%llu before the module work)\n",
           mode, mode ? "probe load + unload before each real load" : "control: real load only", stale_bufs, bufs,
           stale_words, pre_stale);
    fflush(stdout);
    total[mode] = (int)stale_bufs;
  }
  printf("SUMMARY control %d probe %d\n", total[0], total[1]);
  return 0;
}
