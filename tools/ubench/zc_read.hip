// Zero-copy read bandwidth: a kernel streaming pinned host memory over PCIe
// (16 B per lane, grid-stride), vs the SDMA copy.  Measurement only.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void k_read(const uint4* __restrict__ src, size_t n, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Gather of variable-length records (JWS tokens, ~630 B) from pinned host
// memory in a shuffled order into a packed device buffer: one record per wave
// step, 16 B per lane -- the access pattern a class-major stream would need.
__global__ void k_gather(const uint8_t* __restrict__ src, const uint32_t* __restrict__ off,
                         const uint32_t* __restrict__ dst_off, int nrec, int len, uint8_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int r = wave; r < nrec; r += nw) {
    const uint8_t* s = src + off[r];
    uint8_t* d = dst + dst_off[r];
    for (int b = lane * 16; b < len; b += 64 * 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(s + b);
      *reinterpret_cast<uint4*>(d + b) = v;
    }
  }
}

int main() {
  const size_t bytes = 384ull << 20;
  void* h;
  unsigned* d;
  if (hipHostMalloc(&h, bytes, hipHostMallocPortable) != hipSuccess) return 1;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  memset(h, 1, bytes);
  for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
    double best = 1e9;
    for (int it = 0; it < 4; ++it) {
      const auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, (const uint4*)h, bytes / 16, d);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    printf("zero-copy kernel read, %5d blocks x 256: %.1f GB/s\n", blocks, bytes / best / 1e9);
  }
  // gather: 600k records of 640 B (16-B aligned) in a shuffled order
  {
    const int nrec = 600000, len = 640;
    uint32_t *hoff = nullptr, *hdo = nullptr, *doff, *ddo;
    uint8_t* ddst;
    hoff = (uint32_t*)malloc(sizeof(uint32_t) * nrec);
    hdo = (uint32_t*)malloc(sizeof(uint32_t) * nrec);
    for (int i = 0; i < nrec; ++i) { hoff[i] = (uint32_t)i * len; hdo[i] = (uint32_t)i * len; }
    unsigned x = 12345;
    for (int i = nrec - 1; i > 0; --i) {            // shuffle the source order
      x = x * 1103515245u + 12345u;
      const int j = (int)((x >> 8) % (unsigned)(i + 1));
      const uint32_t t = hoff[i]; hoff[i] = hoff[j]; hoff[j] = t;
    }
    if (hipMalloc(&doff, sizeof(uint32_t) * nrec) || hipMalloc(&ddo, sizeof(uint32_t) * nrec) ||
        hipMalloc(&ddst, (size_t)nrec * len))
      return 3;
    (void)hipMemcpy(doff, hoff, sizeof(uint32_t) * nrec, hipMemcpyHostToDevice);
    (void)hipMemcpy(ddo, hdo, sizeof(uint32_t) * nrec, hipMemcpyHostToDevice);
    for (int blocks : {512, 1024, 2048, 4096}) {
      double best = 1e9;
      for (int it = 0; it < 4; ++it) {
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, (const uint8_t*)h, doff, ddo, nrec, len, ddst);
        if (hipDeviceSynchronize() != hipSuccess) return 4;
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      printf("zero-copy gather, %d x 640-B records, %5d blocks x 256: %.1f GB/s\n", nrec, blocks,
             (double)nrec * len / best / 1e9);
    }
    // the SDMA engine on the same bytes (contiguous), for reference
    double best = 1e9;
    for (int it = 0; it < 4; ++it) {
      const auto t0 = std::chrono::steady_clock::now();
      (void)hipMemcpy(ddst, h, (size_t)nrec * len, hipMemcpyHostToDevice);
      best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    printf("SDMA hipMemcpy H2D of the same %.0f MB: %.1f GB/s\n", nrec * (double)len / 1e6, nrec * (double)len / best / 1e9);
  }
  return 0;
}
