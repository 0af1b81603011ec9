// batch.hpp -- batch-level helper kernels (batch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

void launch_scatter(const int32_t* perm, const uint8_t* verdict_pad, uint8_t* verdict, int64_t npad, hipStream_t s);
