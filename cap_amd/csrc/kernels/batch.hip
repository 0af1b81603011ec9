// batch.hip -- batch-level helper kernels: the device half of a pipeline
// chunk's dispatch plan, and the verdict scatter back to caller order.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "batch.hpp"
#include "common.hpp"

using namespace jgk;

namespace {

__global__ void k_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npad) return;
  const int32_t t = perm[p];
  if (t >= 0) verdict[t] = verdict_pad[p];
}

// One thread per job (then one per padding lane).  Slots inside a bucket are
// claimed with one atomic per (wave, bucket): the wave's lanes are grouped by
// bucket with ballots and each group's leader reserves popcount(group) slots.
// The order inside a bucket is arbitrary (perm maps every slot back).
__global__ void __launch_bounds__(256) k_plan_fill(PlanFillArgs a) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = (int)__lane_id();
  if (j < a.n) {
    const jg_tok t = a.toks[j];
    const int alg = t.alg;
    const int c = alg < 16 ? a.cls_tab[(size_t)t.key_idx * 16 + alg] : 0;
    const int b = c == 0 ? a.nkeys : (int)t.key_idx;
    uint64_t pending = __ballot(1);
    int64_t p = 0;
    while (pending) {
      const int leader = __ffsll((unsigned long long)pending) - 1;
      const int lb = __shfl(b, leader);
      const uint64_t grp = __ballot(b == lb) & pending;
      unsigned long long basep = 0;
      if (lane == leader) basep = atomicAdd(&a.cursor[lb], (unsigned long long)__popcll(grp));
      basep = __shfl(basep, leader);
      if (b == lb) p = (int64_t)basep + __popcll(grp & ((1ull << lane) - 1ull));
      pending &= ~grp;
    }
    const uint64_t o = t.off - a.base;
    a.jobs[p] = JobDev{(uint32_t)o, t.sig_in_len, (uint32_t)(o + t.sig_rel_off),
                       job_pack(c == 0 ? 0u : t.key_idx, (uint32_t)alg, t.sig_b64_len)};
    a.perm[p] = (int32_t)j;
  } else {
    const int64_t k = j - a.n;
    const int64_t b = k >> 6;
    if (b > a.nkeys) return;
    const int64_t p = a.pad[2 * b] + (k & 63);
    if (p >= a.pad[2 * b + 1]) return;
    a.jobs[p] = JobDev{0, 0, 0, job_pack(b == a.nkeys ? 0u : (uint32_t)b, JOB_PAD, 0)};
    a.perm[p] = -1;
  }
}

__global__ void __launch_bounds__(256) k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16,
                                              const uint8_t* __restrict__ tsrc, uint8_t* __restrict__ tdst, int tail) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) tdst[threadIdx.x] = tsrc[threadIdx.x];
}

__global__ void __launch_bounds__(256) k_copy1(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

}  // namespace

void launch_copy(const void* src, void* dst, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  const uintptr_t a = (uintptr_t)src | (uintptr_t)dst;
  if (a & 15) {
    const unsigned blocks = (unsigned)std::min<size_t>(4096, (bytes + 255) / 256);
    hipLaunchKernelGGL(k_copy1, dim3(blocks), dim3(256), 0, s, (const uint8_t*)src, (uint8_t*)dst, bytes);
    return;
  }
  const size_t n16 = bytes / 16;
  const int tail = (int)(bytes % 16);
  // ~4 waves per SIMD in flight keeps the PCIe link busy (56 GB/s measured, tools/ubench/zc_read.hip)
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(4096, (n16 + 255) / 256));
  hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16,
                     (const uint8_t*)src + n16 * 16, (uint8_t*)dst + n16 * 16, tail);
}

void launch_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad, hipStream_t s) {
  if (npad <= 0) return;
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, perm, verdict_pad, verdict, npad);
}

void launch_plan_fill(const PlanFillArgs& a, hipStream_t s) {
  const int64_t threads = a.n + (int64_t)(a.nkeys + 1) * 64;
  hipLaunchKernelGGL(k_plan_fill, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a);
}
