// coherence_probe.hip -- does a host-to-device copy into device memory that kernels have read or written
// before become visible to every XCD's next kernel? (round 6: the partitioned-plan misread investigation)
//
// Per scenario and buffer size, `trials` times: put an old pattern into the buffer (a kernel write over the whole
// chip, or an upload), let blocks on every XCD read it (their L2s then hold its lines), overwrite it with a new
// pattern through hipMemcpy from host memory (the library's staging path: pageable, null stream), and read it
// back on every XCD, counting the words that still hold something other than the new pattern (per XCC id).
//
//   hipcc --offload-arch=gfx950 -O2 -o gpurun_out/coherence_probe scripts/coherence_probe.hip
//   ./gpurun_out/coherence_probe [trials]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
  return h | 1u;  // never 0
}

__device__ inline uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xFu;
}

__global__ void k_write(uint32_t* x, size_t n, uint32_t salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = pat(i, salt);
}

// every block reads the whole buffer (grids of 8k blocks: every XCD's L2 ends up holding it)
__global__ void k_touch(const uint32_t* x, size_t n, uint32_t* sink) {
  uint32_t s = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  if (s == 0x9e3779b9u) sink[0] = s;
}

// out[b * 4 + 0] = words of the buffer block b read that differ from pat(., salt); [1] the first such index;
// [2] its value; [3] the block's XCC id
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

struct Tally {
  unsigned long long runs = 0, bad_runs = 0, bad_words = 0, per_xcc[8] = {0};
};

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 20;
  const int kBlocks = 64;  // 8 per XCD
  uint32_t* sink = nullptr;
  unsigned long long* d_out = nullptr;
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&d_out, kBlocks * 4 * 8));
  std::vector<unsigned long long> h_out(kBlocks * 4);
  const size_t sizes[] = {(size_t)16 << 10, (size_t)256 << 10, (size_t)1 << 20, (size_t)3 << 20};
  const char* names[] = {"kernel-write+touch, upload over it (same buffer)",
                         "upload+touch, upload over it (same buffer)",
                         "kernel-write+touch, hipFree, hipMalloc, upload",
                         "kernel-write+touch, upload from pinned memory",
                         "kernel-write+touch, hipMemcpyAsync on a non-blocking stream + sync"};
  const int nscen = 5;
  hipStream_t nb;
  CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
  int total_bad = 0;
  for (int sc = 0; sc < nscen; ++sc) {
    for (size_t bytes : sizes) {
      Tally T;
      const size_t n = bytes / 4;
      std::vector<uint32_t> host(n);
      uint32_t* pinned = nullptr;
      if (sc == 3) CK(hipHostMalloc(&pinned, bytes));
      uint32_t* x = nullptr;
      CK(hipMalloc(&x, bytes));
      for (int t = 0; t < trials; ++t) {
        const uint32_t s_old = 0x1000u + 2u * (uint32_t)t + (uint32_t)sc * 7919u, s_new = s_old + 1u;
        if (sc == 1) {
          for (size_t i = 0; i < n; ++i) host[i] = pat(i, s_old);
          CK(hipMemcpy(x, host.data(), bytes, hipMemcpyHostToDevice));
        } else {
          k_write<<<1024, 256>>>(x, n, s_old);
          CK(hipGetLastError());
        }
        k_touch<<<kBlocks, 256>>>(x, n, sink);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        if (sc == 2) {
          uint32_t* old = x;
          CK(hipFree(x));
          CK(hipMalloc(&x, bytes));
          (void)old;
        }
        for (size_t i = 0; i < n; ++i) host[i] = pat(i, s_new);
        if (sc == 3) {
          memcpy(pinned, host.data(), bytes);
          CK(hipMemcpy(x, pinned, bytes, hipMemcpyHostToDevice));
        } else if (sc == 4) {
          CK(hipMemcpyAsync(x, host.data(), bytes, hipMemcpyHostToDevice, nb));
          CK(hipStreamSynchronize(nb));
        } else {
          CK(hipMemcpy(x, host.data(), bytes, hipMemcpyHostToDevice));
        }
        k_check<<<kBlocks, 256>>>(x, n, s_new, d_out);
        CK(hipGetLastError());
        CK(hipMemcpy(h_out.data(), d_out, h_out.size() * 8, hipMemcpyDeviceToHost));
        ++T.runs;
        bool any = false;
        for (int b = 0; b < kBlocks; ++b) {
          const unsigned long long bad = h_out[b * 4];
          if (!bad) continue;
          any = true;
          T.bad_words += bad;
          T.per_xcc[h_out[b * 4 + 3] & 7] += bad;
          if (T.bad_runs < 3)
            fprintf(stdout, "  BAD scen %d size %zu trial %d block %d xcc %llu: %llu words, first %llu = %08llx (old %08x new %08x)\n",
                    sc, bytes, t, b, h_out[b * 4 + 3], bad, h_out[b * 4 + 1], h_out[b * 4 + 2],
                    pat(h_out[b * 4 + 1], s_old), pat(h_out[b * 4 + 1], s_new));
        }
        if (any) ++T.bad_runs;
      }
      CK(hipFree(x));
      if (pinned) CK(hipHostFree(pinned));
      printf("scenario %d (%s) size %zu: %llu / %llu runs stale, %llu stale words; per xcc:", sc, names[sc], bytes,
             T.bad_runs, T.runs, T.bad_words);
      for (int k = 0; k < 8; ++k) printf(" %llu", T.per_xcc[k]);
      printf("\n");
      fflush(stdout);
      total_bad += (int)T.bad_runs;
    }
  }
  printf("SUMMARY stale runs %d\n", total_bad);
  return 0;
}
