// batch.hip -- batch-level helper kernels: the device half of a pipeline
// chunk's dispatch plan, and the verdict scatter back to caller order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

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
    a.vpad[p] = 0;
  } else {
    const int64_t k = j - a.n;
    const int64_t b = k >> 6;
    if (b > a.nkeys) return;
    const int64_t p = a.pad[2 * b] + (k & 63);
    if (p >= a.pad[2 * b + 1]) return;
    a.jobs[p] = JobDev{0, 0, 0, job_pack(b == a.nkeys ? 0u : (uint32_t)b, JOB_PAD, 0)};
    a.perm[p] = -1;
    a.vpad[p] = 0;
  }
}

// Two-level form for chunks of many jobs over few buckets (a mixed JWKS
// stream): a block of 256 threads takes PF_ITEMS jobs per thread, counts its
// jobs per bucket with LDS atomics, reserves each bucket's run with ONE global
// atomic per (block, bucket), and places its jobs there.  The one-level
// kernel above issues one global atomic per (wave, bucket) -- ~25 per wave of
// a 32-kid mixed stream, all on the same 33 cursors: 1.2 ms per 524 k-job
// chunk on the critical path of every chunk (profiles/r04_s3/zc_trace_*).
constexpr int PF_THREADS = 256, PF_ITEMS = 4, PF_MAX_BUCKETS = 2048;
__global__ void __launch_bounds__(PF_THREADS) k_plan_fill_blocked(PlanFillArgs a) {
  __shared__ uint32_t cnt[PF_MAX_BUCKETS];
  __shared__ unsigned long long gbase[PF_MAX_BUCKETS];
  const int nb = a.nkeys + 1;
  for (int b = threadIdx.x; b < nb; b += PF_THREADS) cnt[b] = 0;
  __syncthreads();
  const int64_t j0 = (int64_t)blockIdx.x * PF_THREADS * PF_ITEMS;
  int bk[PF_ITEMS];
  uint32_t loc[PF_ITEMS];
#pragma unroll
  for (int it = 0; it < PF_ITEMS; ++it) {
    const int64_t j = j0 + (int64_t)it * PF_THREADS + threadIdx.x;
    bk[it] = -1;
    if (j < a.n) {
      const jg_tok t = a.toks[j];
      const int alg = t.alg;
      const int c = alg < 16 ? a.cls_tab[(size_t)t.key_idx * 16 + alg] : 0;
      bk[it] = c == 0 ? a.nkeys : (int)t.key_idx;
      loc[it] = atomicAdd(&cnt[bk[it]], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += PF_THREADS)
    if (cnt[b]) gbase[b] = atomicAdd(&a.cursor[b], (unsigned long long)cnt[b]);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < PF_ITEMS; ++it) {
    if (bk[it] < 0) continue;
    const int64_t j = j0 + (int64_t)it * PF_THREADS + threadIdx.x;
    const jg_tok t = a.toks[j];
    const int64_t p = (int64_t)gbase[bk[it]] + loc[it];
    const uint64_t o = t.off - a.base;
    a.jobs[p] = JobDev{(uint32_t)o, t.sig_in_len, (uint32_t)(o + t.sig_rel_off),
                       job_pack(bk[it] == a.nkeys ? 0u : t.key_idx, (uint32_t)t.alg, t.sig_b64_len)};
    a.perm[p] = (int32_t)j;
    a.vpad[p] = 0;
  }
}

// the padding lanes of every bucket (the second half of k_plan_fill)
__global__ void __launch_bounds__(256) k_plan_pad(PlanFillArgs a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = k >> 6;
  if (b > a.nkeys) return;
  const int64_t p = a.pad[2 * b] + (k & 63);
  if (p >= a.pad[2 * b + 1]) return;
  a.jobs[p] = JobDev{0, 0, 0, job_pack(b == a.nkeys ? 0u : (uint32_t)b, JOB_PAD, 0)};
  a.perm[p] = -1;
  a.vpad[p] = 0;
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

// 16 lanes per job, 16 B per lane, grid-stride over the class range: the
// access pattern of tools/ubench/zc_read.hip's gather (56 GB/s from pinned
// memory, the SDMA copy's rate).  A job's bytes [off, end) are copied as the
// 16-byte-aligned span around them (src is 16-byte aligned: submit_to), so
// the copy starts (off & 15) bytes into its slot.  Reads reach at most 15
// bytes past the last token's end (inside the block's ARENA_SLACK).
__global__ void __launch_bounds__(256) k_zc_gather(ZcGatherArgs a) {
  const int sub = threadIdx.x & 15;
  const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int64_t ng = ((int64_t)gridDim.x * blockDim.x) >> 4;
  for (int64_t p = a.begin + g0; p < a.end; p += ng) {
    const JobDev jb = a.jobs[p];
    if (!job_live(jb)) continue;
    const int key = job_key(jb);
    const uint32_t end = max(jb.off + jb.sig_in_len, jb.sig_off + job_siglen(jb));
    const uint32_t lo = jb.off & ~15u, hi = (end + 15u) & ~15u;
    const uint64_t d0 = a.kbase[key] + (uint64_t)(p - a.kstart[key]) * a.kstride[key];
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.src + lo);
    uint4* __restrict__ dst = reinterpret_cast<uint4*>(a.dst + d0);
    const uint32_t n16 = (hi - lo) >> 4;
    for (uint32_t i = (uint32_t)sub; i < n16; i += 16) dst[i] = src[i];
    if (sub == 0) {
      a.jobs[p].off = (uint32_t)(d0 + (jb.off - lo));
      a.jobs[p].sig_off = (uint32_t)(d0 + (jb.sig_off - lo));
    }
  }
}

}  // namespace

void launch_zc_gather(const ZcGatherArgs& a, hipStream_t s) {
  const int64_t n = a.end - a.begin;
  if (n <= 0) return;
  // 2048 waves at most (~2 per SIMD): enough in flight for the link, few
  // enough to leave the arithmetic kernels of earlier classes their slots
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(512, (n * 16 + 255) / 256));
  hipLaunchKernelGGL(k_zc_gather, dim3(blocks), dim3(256), 0, s, a);
}

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
  // two-level fill (LDS bucket counts, one global atomic per block and
  // bucket); the one-level kernel serves key tables past PF_MAX_BUCKETS and
  // small chunks (jobs and padding in one launch: one dependent launch fewer
  // on a coalesced single-token batch's chain)
  if (a.nkeys + 1 <= PF_MAX_BUCKETS && a.n > 4096) {
    constexpr int64_t per = PF_THREADS * PF_ITEMS;
    if (a.n > 0) hipLaunchKernelGGL(k_plan_fill_blocked, dim3((unsigned)((a.n + per - 1) / per)), dim3(PF_THREADS), 0, s, a);
    const int64_t pads = (int64_t)(a.nkeys + 1) * 64;
    hipLaunchKernelGGL(k_plan_pad, dim3((unsigned)((pads + 255) / 256)), dim3(256), 0, s, a);
    return;
  }
  const int64_t threads = a.n + (int64_t)(a.nkeys + 1) * 64;
  hipLaunchKernelGGL(k_plan_fill, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a);
}
