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
  return 0;
}
