// FETCH_SIZE calibration for the point kernel's access pattern (measurement
// only).  MI355X_MICROARCH.md: FETCH_SIZE is calibrated (x2) for 16-B/lane
// coalesced streaming reads only; "calibrate on a known byte count in your own
// access pattern".  Two kernels over a 7.6 GB table (far past the 256 MiB
// Infinity Cache), each run once under rocprofv3 --pmc FETCH_SIZE:
//   k_gather: 1M lanes x 22 random 80-byte entries (5 x dwordx4 per entry,
//             16-B aligned, the comb-table layout of ecdsa.hip): 1.85 GB requested
//   k_stream: 16 B/lane coalesced read of 1 GiB (the guide's x2 reference)
// FETCH_SIZE x 1024 / requested bytes = the counter's bytes per requested byte.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t ENT_WORDS = 20;                    // 80-byte entries
constexpr size_t NENT = (size_t)95 << 20;           // 7.97 GB
constexpr int GATHERS = 22;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void __launch_bounds__(64) k_gather(const uint32_t* __restrict__ tab, uint32_t* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  uint32_t acc = 0;
  for (int g = 0; g < GATHERS; ++g) {
    const uint64_t e = (uint64_t)mix(i * 64u + (uint32_t)g) % NENT;
    const uint4* p = reinterpret_cast<const uint4*>(tab + e * ENT_WORDS);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint4 v = p[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// the packed P-256 layout (ecdsa.hpp JG_EC_PACK64): 64-byte entries, 64-B
// aligned, 4 x dwordx4 -- each entry half of one 128-B line
__global__ void __launch_bounds__(64) k_gather64(const uint32_t* __restrict__ tab, uint32_t* out) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  uint32_t acc = 0;
  for (int g = 0; g < GATHERS; ++g) {
    const uint64_t e = (uint64_t)mix(i * 64u + (uint32_t)g + 0x5bd1e995u) % (NENT * ENT_WORDS / 16);
    const uint4* p = reinterpret_cast<const uint4*>(tab + e * 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = p[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

__global__ void k_stream(const uint4* __restrict__ src, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main() {
  uint32_t* tab = nullptr;
  uint32_t* out = nullptr;
  const size_t bytes = NENT * ENT_WORDS * 4;
  if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  if (hipMemset(tab, 1, bytes) != hipSuccess) return 1;
  const unsigned lanes = 1u << 20;
  hipLaunchKernelGGL(k_gather, dim3(lanes / 64), dim3(64), 0, 0, tab, out);
  hipLaunchKernelGGL(k_gather64, dim3(lanes / 64), dim3(64), 0, 0, tab, out);
  const size_t sbytes = (size_t)1 << 30;
  hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)tab, sbytes / 16, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("{\"gather_requested_bytes\": %zu, \"gather64_requested_bytes\": %zu, \"stream_requested_bytes\": %zu, "
              "\"entry_bytes\": 80, \"gathers\": %zu}\n", (size_t)lanes * GATHERS * 80, (size_t)lanes * GATHERS * 64,
              sbytes, (size_t)lanes * GATHERS);
  (void)hipFree(tab);
  (void)hipFree(out);
  return 0;
}
