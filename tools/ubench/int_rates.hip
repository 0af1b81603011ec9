// Instruction-throughput microbenchmark for the integer / fp64 ops the
// multi-precision verify kernels are built from (gfx950).  Each thread runs
// 8 independent chains of one instruction; rate = lane-ops / second.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHAINS 8

#define DEF_KERNEL(NAME, BODY)                                              \
__global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) { \
  uint32_t a[CHAINS]; uint64_t c[CHAINS]; double d[CHAINS];                 \
  for (int k = 0; k < CHAINS; ++k) { a[k] = seed * (threadIdx.x + k + 1);   \
    c[k] = a[k] ^ 0x12345678ull; d[k] = (double)a[k]; }                     \
  uint32_t b = seed + blockIdx.x;  double db = (double)b * 1e-9;            \
  for (int it = 0; it < ITERS; ++it) {                                      \
    _Pragma("unroll") for (int k = 0; k < CHAINS; ++k) { BODY; }            \
  }                                                                         \
  uint64_t s = 0; double ds = 0;                                            \
  for (int k = 0; k < CHAINS; ++k) { s += c[k] + a[k]; ds += d[k]; }        \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s + (uint32_t)ds;  \
}

DEF_KERNEL(k_mad_u64_u32,
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c[k]) : "v"(a[k]), "v"(b) : "vcc"))
DEF_KERNEL(k_mad_u64_u32_sgpr,
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c[k]) : "v"(a[k]), "s"(b) : "vcc"))
DEF_KERNEL(k_mul_lo_u32,
  asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_mul_hi_u32,
  asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_mad_u32_u24,
  asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_mul_hi_u32_u24,
  asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_add_co_u32,
  asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(b) : "vcc"))
DEF_KERNEL(k_addc_co_u32,
  asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc"))
DEF_KERNEL(k_add3_u32,
  asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_lshl_add_u32,
  asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_fma_f64,
  asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d[k]) : "v"(db)))
DEF_KERNEL(k_lshl_add_u64,
  asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(c[k]) : "v"((uint64_t)b)))
DEF_KERNEL(k_lshrrev_b64,
  asm volatile("v_lshrrev_b64 %0, 28, %0" : "+v"(c[k])))
DEF_KERNEL(k_and_b32,
  asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_alignbit_b32,
  asm volatile("v_alignbit_b32 %0, %0, %1, 28" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_bitop3_b32,
  asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[k]) : "v"(b)))
DEF_KERNEL(k_mad_u64_u32_dep,
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c[0]) : "v"(a[k]), "v"(b) : "vcc"))

// 8 MADs per asm statement: the compiler's conservative s_nop between inline
// asm statements is paid once per 8 instead of once per MAD
#define MAD8(c, a, b) asm volatile(                                     \
  "v_mad_u64_u32 %0, s[100:101], %8, %9, %0\n"                          \
  "v_mad_u64_u32 %1, s[100:101], %8, %9, %1\n"                          \
  "v_mad_u64_u32 %2, s[100:101], %8, %9, %2\n"                          \
  "v_mad_u64_u32 %3, s[100:101], %8, %9, %3\n"                          \
  "v_mad_u64_u32 %4, s[100:101], %8, %9, %4\n"                          \
  "v_mad_u64_u32 %5, s[100:101], %8, %9, %5\n"                          \
  "v_mad_u64_u32 %6, s[100:101], %8, %9, %6\n"                          \
  "v_mad_u64_u32 %7, s[100:101], %8, %9, %7"                             \
  : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]) \
  : "v"(a), "v"(b) : "s100", "s101")
DEF_KERNEL(k_mad_block8, if (k == 0) { MAD8(c, a[1], b); })

struct K { const char* name; void (*fn)(uint32_t*, uint32_t); };

int main() {
  K ks[] = {
    {"v_mad_u64_u32", k_mad_u64_u32}, {"v_mad_u64_u32(sgpr)", k_mad_u64_u32_sgpr},
    {"v_mad_u64_u32(dep chain)", k_mad_u64_u32_dep}, {"v_mad_u64_u32(8 per asm)", k_mad_block8},
    {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_hi_u32", k_mul_hi_u32},
    {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
    {"v_add_co_u32", k_add_co_u32}, {"v_addc_co_u32", k_addc_co_u32},
    {"v_add3_u32", k_add3_u32}, {"v_lshl_add_u32", k_lshl_add_u32},
    {"v_lshl_add_u64", k_lshl_add_u64}, {"v_fma_f64", k_fma_f64},
    {"v_lshrrev_b64", k_lshrrev_b64}, {"v_and_b32", k_and_b32},
    {"v_alignbit_b32", k_alignbit_b32}, {"v_bitop3_b32", k_bitop3_b32},
  };
  int occ[] = {1, 2, 4, 8};  // waves per SIMD
  uint32_t* out; hipMalloc(&out, 256 * 8 * 4 * 256 * sizeof(uint32_t) * 2);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("{\"cus\": %d, \"rates\": [\n", ncu);
  bool first = true;
  for (auto& k : ks) {
    for (int w : occ) {
      int blocks = ncu * w;  // 256 threads = 4 waves = one per SIMD
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double ops = 5.0 * blocks * 256.0 * ITERS * CHAINS;
      double rate = ops / (ms * 1e-3);
      printf("%s {\"inst\": \"%s\", \"waves_per_simd\": %d, \"Tlane_ops_per_s\": %.3f, \"lane_ops_per_clk_per_cu_at_2.4GHz\": %.2f}",
             first ? "" : ",\n", k.name, w, rate / 1e12, rate / ncu / 2.4e9);
      first = false;
    }
  }
  printf("\n]}\n");
  return 0;
}
