// prep.hpp -- launch interface of the prep kernel (prep.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"

struct PrepArgs {
  const uint8_t* arena;
  const jgk::JobDev* jobs;    // padded, (class, key)-sorted jobs
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  uint32_t* sigw;             // SIGW_ROWS x npad
  uint32_t* dig;              // DIG_ROWS x npad
  uint8_t* status;            // npad
  uint16_t* siglen;           // npad
  int64_t npad, begin, end;
  int32_t zrows;              // signature rows the class's kernel reads
  int32_t ec_words;           // ECDSA classes: words of r (and of s) the kernels read
};

// hash_mask: bit 0 = some token of the range uses SHA-256, bit 1 = SHA-384/512
void launch_prep(int cls, int hash_mask, const PrepArgs& a, hipStream_t s);
