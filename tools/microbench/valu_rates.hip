// Issue rate of the VALU instructions the big-integer kernels are made of
// (gfx950): each kernel runs 8 independent dependency chains of ONE
// instruction kind per lane, 8 waves per SIMD, so the result is throughput,
// not latency.  Printed as lane-operations per second and as a fraction of the
// full rate by clock (256 CUs x 64 lanes x clock).  The value of each chain is
// passed through an empty asm statement every step so the compiler cannot fold
// the repeated operation into one.
//   build: hipcc -O3 --offload-arch=gfx950 -o valu_rates valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int CH = 8, U = 8;

template <int OP>
__global__ void __launch_bounds__(256) k_rate(uint64_t* out, int iters, uint32_t seed) {
  uint32_t a[CH];
  uint64_t h[CH];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int c = 0; c < CH; ++c) { a[c] = t * 7u + c + seed; h[c] = ((uint64_t)a[c] << 20) | c; }
  const uint32_t b = seed | 1u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (OP == 0) a[c] = a[c] + b;                              // v_add_u32
        if constexpr (OP == 1) a[c] = a[c] * 19u;                            // v_mul_lo_u32
        if constexpr (OP == 2) h[c] = (uint64_t)(uint32_t)h[c] * b + h[c];    // v_mad_u64_u32
        if constexpr (OP == 3) h[c] = h[c] >> 26;                            // v_lshrrev_b64
        if constexpr (OP == 4) h[c] = (h[c] << 3) + (uint64_t)b;             // v_lshl_add_u64
        if constexpr (OP == 5) a[c] = (a[c] << 4) + b;                       // v_lshl_add_u32
        if constexpr (OP == 6) h[c] = h[c] + (uint64_t)b;                    // 64-bit add (v_add_co + v_addc)
        if constexpr (OP == 7) a[c] = __builtin_amdgcn_alignbit(a[c], b, 7); // v_alignbit_b32
        if constexpr (OP == 0 || OP == 1 || OP == 5 || OP == 7) asm volatile("" : "+v"(a[c]));
        else asm volatile("" : "+v"(h[c]));
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += h[c] + a[c];
  out[t] = s;
}

template <int OP>
int run(const char* name, hipDeviceProp_t& p, uint64_t* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);   // warm-up
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 5u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 256 * iters * U * CH;
  const double full = (double)p.multiProcessorCount * 64 * (p.clockRate * 1e3);
  std::printf("%-16s %8.3f ms  %7.2f T lane-op/s  %.3f of full rate by clock\n", name, ms, ops / ms / 1e9,
              ops / (ms * 1e-3) / full);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  std::printf("%s: %d CUs, clock %.0f MHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate / 1e3);
  const int blocks = p.multiProcessorCount * 8, iters = 2048;       // 8 waves per SIMD
  uint64_t* out;
  CHK(hipMalloc(&out, sizeof(uint64_t) * blocks * 256));
  run<0>("v_add_u32", p, out, blocks, iters);
  run<1>("v_mul_lo_u32", p, out, blocks, iters);
  run<2>("v_mad_u64_u32", p, out, blocks, iters);
  run<3>("v_lshrrev_b64", p, out, blocks, iters);
  run<4>("v_lshl_add_u64", p, out, blocks, iters);
  run<5>("v_lshl_add_u32", p, out, blocks, iters);
  run<6>("add u64", p, out, blocks, iters);
  run<7>("v_alignbit_b32", p, out, blocks, iters);
  CHK(hipFree(out));
  return 0;
}
