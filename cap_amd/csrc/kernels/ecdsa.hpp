// ecdsa.hpp -- launch interface of the ECDSA kernels (ecdsa.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct EcArgs {
  const jg_tok_dev* toks;
  const int32_t* perm;
  const int32_t* wave_key;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // r at rows 0.., s at rows EC_S_ROW.. (LE words)
  const uint32_t* dig;        // digest rows (big-endian words)
  uint8_t* status;
  uint8_t* verdict_pad;
  uint32_t* digs;             // per window: packed signed digits (d1 | d2 << 16), int16 each
  uint32_t* u1w;              // u1, u2 canonical 28-bit limb rows (exact path)
  uint32_t* u2w;
  const uint32_t* gtab;       // comb table of the generator for this curve
  int32_t* exc_list;          // padded indices needing the exact path
  uint32_t* exc_count;
  int64_t npad, begin, end;
};

// table geometry per curve: words per entry (x,y Montgomery limbs, 16-B aligned)
constexpr int ec_limbs(int cls) { return cls == jgk::CLS_P256 ? 10 : cls == jgk::CLS_P384 ? 15 : 20; }
constexpr int ec_stride(int cls) { return (2 * ec_limbs(cls) + 3) & ~3; }
constexpr int ec_order_bits(int cls) { return cls == jgk::CLS_P256 ? 256 : cls == jgk::CLS_P384 ? 384 : 521; }
// Fixed-base comb over signed w-bit digits: u = sum_w d_w 2^(W w), d_w in
// [-2^(W-1), 2^(W-1)), so a token costs ceil((bits+1)/W) mixed additions per
// scalar and each (key, window) holds 2^(W-1) affine multiples d 2^(W w) P.
// Wider W trades HBM for fewer additions -- the point kernel is VALU-issue
// bound (SQ counters, profiles/), so additions are the cost that matters:
// P-256 at W = 20 is 13 windows (the top one holds 16 bits of u < n, so its
// digit never carries out), 25 additions per token instead of ~32 at W = 16,
// for 545 MB of table per key (and for G) out of 288 GB of HBM.
constexpr int ec_comb_w(int cls) { return cls == jgk::CLS_P256 ? 20 : 12; }
constexpr int ec_entries(int cls) { return 1 << (ec_comb_w(cls) - 1); }
constexpr int ec_windows(int cls) { return (ec_order_bits(cls) + 1 + ec_comb_w(cls) - 1) / ec_comb_w(cls); }
// digit rows of the scalar -> point hand-off: two int16 per word when W <= 16,
// else one row of u1 digits then one row of u2 digits per window
constexpr bool ec_digits_packed(int cls) { return ec_comb_w(cls) <= 16; }
constexpr int ec_digit_rows(int cls) { return ec_digits_packed(cls) ? ec_windows(cls) : 2 * ec_windows(cls); }
// comb-table budget: at most this many keys of a class per jg_keys_load
constexpr int ec_max_keys(int cls) { return cls == jgk::CLS_P256 ? 256 : 65535; }
constexpr int64_t ec_table_words(int cls) {
  return (int64_t)ec_windows(cls) * ec_entries(cls) * ec_stride(cls);
}

void launch_ec(int cls, const EcArgs& a, hipStream_t s, const jgk::Marker& mk);
// key staging: validate each listed key (plain 28-bit limbs x,y at aux_off), write
// Montgomery affine coordinates back to aux_off and build its comb table.
void launch_ec_keyprep(int cls, jgk::DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
// generator table for a curve into `tab` (ec_table_words(cls) words)
void launch_ec_gtable(int cls, uint32_t* tab, hipStream_t s);
