// hash.hpp -- launch interface of the batched SHA-2 kernel (hash.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../../include/jg.h"

// digests as 16 big-endian 32-bit words per job (SHA-256: first 8 used)
void launch_hash(const uint8_t* arena, const jg_hjob* jobs, int64_t n, uint32_t* out, hipStream_t s);
