// ed25519.hpp -- launch interface of the Ed25519 kernels (ed25519.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct EdArgs {
  const int32_t* perm;
  const int32_t* wave_key;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // R at rows 0..7, S at rows 8..15 (LE words)
  const uint32_t* dig;        // SHA-512(R || A || M), big-endian words
  uint8_t* status;
  const uint16_t* siglen;
  uint8_t* verdict_pad;
  uint32_t* xyz;              // X, Y, Z of R' (3 x 10 limb rows)
  const uint32_t* btab;       // comb table of the base point B (Niels form)
  int64_t npad, begin, end;
};

constexpr int ED_L = 10;
constexpr int ED_STRIDE = 32;                   // 3 x 10 limbs, padded to 16 B
constexpr int ED_WINDOWS = 33;
constexpr int64_t ED_TABLE_WORDS = (int64_t)ED_WINDOWS * jgk::COMB_ENTRIES * ED_STRIDE;

void launch_ed(const EdArgs& a, hipStream_t s, const jgk::Marker& mk);
// key staging: decode each listed key's 32 public-key bytes (words at aux_off),
// mark validity and build the comb table of -A at tab_off
void launch_ed_keyprep(jgk::DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
void launch_ed_btable(uint32_t* tab, hipStream_t s);
