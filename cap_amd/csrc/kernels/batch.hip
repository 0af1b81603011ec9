// batch.hip -- batch-level helper kernels: verdict scatter back to caller order.
#include <hip/hip_runtime.h>

#include "batch.hpp"
#include "common.hpp"

namespace {

__global__ void k_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npad) return;
  const int32_t t = perm[p];
  if (t >= 0) verdict[t] = verdict_pad[p];
}

}  // namespace

void launch_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad, hipStream_t s) {
  if (npad <= 0) return;
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, s, perm, verdict_pad, verdict, npad);
}
