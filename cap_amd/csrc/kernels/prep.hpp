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
  uint32_t* mid;              // PREP_MID_WORDS per key index, or null: a key run's shared SHA-256
                              // block 0 (words 0-15), its midstate (16-23), valid flag (24)
};
constexpr int PREP_MID_WORDS = 32;

// hash_mask: bit 0 = some token of the range uses SHA-256, bit 1 = SHA-384/512
void launch_prep(int cls, int hash_mask, const PrepArgs& a, hipStream_t s);
