// ecdsa.hpp -- launch interface of the ECDSA kernels (ecdsa.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct EcArgs {
  const jgk::JobDev* jobs;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // r at rows 0.., s at rows EC_S_ROW.. (LE words)
  const uint32_t* dig;        // digest rows (big-endian words)
  uint8_t* status;
  uint8_t* verdict_pad;
  uint32_t* digs;             // signed digit rows: u1 windows (generator) then u2 windows (key)
  uint32_t* u1w;              // u1, u2 canonical 28-bit limb rows (exact path)
  uint32_t* u2w;
  const uint32_t* gtab;       // comb table of the generator for this curve
  int32_t* exc_list;          // padded indices needing the exact path
  uint32_t* exc_count;
  int64_t npad, begin, end;
  int32_t wq;                 // comb width of the launch's key tables (every key of [begin, end) has it)
  int32_t exc_reset;          // zero *exc_count first (the class's first launch)
  // which kernels launch_ec enqueues: EC_ALL (scalar, point, exact), EC_FAST
  // (scalar, point) or EC_EXACT (exact alone, later, on another stream)
  int32_t part;
};
enum : int32_t { EC_ALL = 0, EC_FAST = 1, EC_EXACT = 2 };

// table geometry per curve: words per entry (x,y Montgomery limbs, 16-B aligned)
constexpr int ec_limbs(int cls) { return cls == jgk::CLS_P256 ? 10 : cls == jgk::CLS_P384 ? 15 : 20; }
// 32-bit words of r (and of s) as prep leaves them: ceil(coordinate bytes / 4)
constexpr int ec_sig_words(int cls) { return cls == jgk::CLS_P256 ? 8 : cls == jgk::CLS_P384 ? 12 : 17; }
// P-256 entries packed to 64 bytes (JG_EC_PACK64, default on): x and y as 8
// 32-bit words each (canonical Montgomery values < p < 2^256), unpacked to
// 28-bit limbs on load (~2 VALU per limb).  A 64-B-aligned entry touches one
// 128-B line where the 80-B limb form touched 1.5 on average, and every P-256
// table is 20 % smaller (generator W = 26: 21.5 GB, a W = 26 key 21.5 GB, W =
// 24 5.9 GB, W = 22 1.6 GB, W = 20 436 MB).  Measured: point kernel -0.6 %
// (profiles/r03_s4_ab.json; the same A/B with every gather confined to 256
// entries bounds what gather traffic costs at all: -7 %).  Other curves keep
// the limb form (P-384's 128-B stride is already line-aligned).
#ifndef JG_EC_PACK64
#define JG_EC_PACK64 1
#endif
constexpr bool ec_packed(int cls) { return JG_EC_PACK64 && cls == jgk::CLS_P256; }
constexpr int ec_stride(int cls) { return ec_packed(cls) ? 16 : (2 * ec_limbs(cls) + 3) & ~3; }
constexpr int ec_order_bits(int cls) { return cls == jgk::CLS_P256 ? 256 : cls == jgk::CLS_P384 ? 384 : 521; }
// Fixed-base comb over signed W-bit digits: u = sum_w d_w 2^(W w), d_w in
// [-2^(W-1), 2^(W-1)), so a token costs ceil((bits+1)/W) mixed additions per
// scalar and each (point, window) holds 2^(W-1) affine multiples d 2^(W w) P.
// Wider W trades HBM for fewer additions -- the point kernel is VALU-issue
// bound (SQ counters, profiles/), so additions are the cost that matters.  The
// generator's table is built once per engine and shared by every key, so it
// gets the wider window (gen = true); per-key tables stay narrower so a JWKS of
// hundreds of keys still fits:
//   P-256: G W=26 (10 windows, 21.5 GB packed), keys W=20 (13 windows, 436 MB each):
//          22 additions per token (23 with G W=24, 25 with W=20/20, ~32 with 16/16)
//   P-384: G W=24 (17 windows, 18.3 GB), keys W=16 (25 windows, 105 MB): 41 (65 at 12/12);
//          round 6 widened G from 20 (20 windows, 1.3 GB): 3 additions fewer per token
//   P-521: G W=20 (27 windows, 2.3 GB), keys W=16 (33 windows, 173 MB): 59 (87 at 12/12)
// The top window of each scalar (u < n) never carries out of the last digit.
// ec_comb_w(cls, false) is the narrowest key window; P-256 keys get a wider
// one when few keys share the context's table budget (ec_key_w below).
constexpr int ec_comb_w(int cls, bool gen) {
  return cls == jgk::CLS_P256 ? (gen ? 26 : 20) : cls == jgk::CLS_P384 ? (gen ? 24 : 16) : (gen ? 20 : 16);
}
// Windows per scalar: ceil((bits + 2) / W).  The signed recoding carries +1
// into the next window whenever a window's value reaches 2^(W-1), so the top
// window must hold at most W - 2 bits of u < n (its value + the incoming carry
// then stays below 2^(W-1) and no carry leaves the last digit).  Round 3 used
// ceil((bits + 1) / W): for P-521 at W = 18 that is 29 windows = 522 bits, the
// top window got 17 = W - 1 bits, and a scalar whose bits 504..520 were all
// ones with a carry in (probability ~2^-18) lost that carry -- a wrong u2 and
// a false reject (tests/golden/edge_digit_tokens.json, "p521_w18_top_carry").
constexpr int ec_windows_w(int cls, int w) { return (ec_order_bits(cls) + 2 + w - 1) / w; }
constexpr int ec_entries(int cls, bool gen) { return 1 << (ec_comb_w(cls, gen) - 1); }
constexpr int ec_windows(int cls, bool gen) { return ec_windows_w(cls, ec_comb_w(cls, gen)); }
// digit rows of the scalar -> point hand-off: one int32 row per window, the
// u1 (generator) digits first, then the u2 (key) digits (rows for the
// narrowest key window, which has the most windows)
constexpr int ec_digit_rows(int cls) { return ec_windows(cls, true) + ec_windows(cls, false); }
// comb-table budget: at most this many keys of a class per jg_keys_load
constexpr int ec_max_keys(int cls) { return 256; }
constexpr int64_t ec_table_words_w(int cls, int w) {
  return (int64_t)ec_windows_w(cls, w) * (1 << (w - 1)) * ec_stride(cls);
}
constexpr int64_t ec_table_words(int cls, bool gen) { return ec_table_words_w(cls, ec_comb_w(cls, gen)); }
// Key-table width tiers (HBM for fewer additions, as the generators' wide
// windows do), widest first.  P-256 (64-B packed entries): W = 26 (10 windows,
// 21.5 GB per key: 20 additions per token with the W = 26 generator), 24 (11
// windows, 5.9 GB), 22 (12, 1.6 GB), 20 (13, 436 MB); P-384: 24 (17 windows, 18.3 GB), 20 (20
// windows, 1.34 GB), 18 (22, 369 MB), 16 (25, 105 MB); P-521: 20 (27, 2.26 GB),
// 18 (30, 629 MB), 16 (33, 173 MB).  The runtime picks one width per curve
// from the context's table budget, a single total over every curve's key
// tables (jg_runtime.cpp key_widths); the narrowest width is always allowed.
constexpr int EC_P256_WQ[4] = {26, 24, 22, 20};
constexpr int EC_P384_WQ[4] = {24, 20, 18, 16};
constexpr int EC_P521_WQ[3] = {20, 18, 16};
// every tier leaves the top window at most W - 2 bits (see ec_windows_w)
constexpr bool ec_top_window_ok(int cls, int w) { return ec_order_bits(cls) - w * (ec_windows_w(cls, w) - 1) <= w - 2; }
static_assert(ec_top_window_ok(jgk::CLS_P256, 26) && ec_top_window_ok(jgk::CLS_P256, 24) &&
              ec_top_window_ok(jgk::CLS_P256, 22) && ec_top_window_ok(jgk::CLS_P256, 20) &&
              ec_top_window_ok(jgk::CLS_P384, 24) && ec_top_window_ok(jgk::CLS_P384, 20) &&
              ec_top_window_ok(jgk::CLS_P384, 18) && ec_top_window_ok(jgk::CLS_P384, 16) &&
              ec_top_window_ok(jgk::CLS_P521, 20) && ec_top_window_ok(jgk::CLS_P521, 18) &&
              ec_top_window_ok(jgk::CLS_P521, 16), "comb window count leaves no room for the top carry");

void launch_ec(int cls, const EcArgs& a, hipStream_t s, const jgk::Marker& mk);

// One-launch verification of a small batch (ec_small.hpp): one two-wave block
// per token runs the whole chain -- signing input and signature read straight
// from the (pinned host or device) arena, hash, scalar stage, comb sum, x(R)
// check -- and writes the verdict byte to verdict[out[i]] (pinned host memory).
// The jobs travel in the kernel arguments.  Every token of a launch has a key
// of class `cls` whose comb table has width `wq`, a signing input of at most
// EC_SMALL_IN_MAX bytes, and its alg in the key's family (the host plan).
constexpr int EC_SMALL_MAX = jgk::SMALL_MAX;              // tokens per launch
constexpr uint32_t EC_SMALL_IN_MAX = jgk::SMALL_IN_MAX;   // signing-input bytes staged in LDS
struct EcSmallArgs {
  const uint8_t* arena;                     // JobDev offsets are relative to it
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* gtab;
  uint8_t* verdict;
  uint32_t n;
  jgk::JobDev jobs[EC_SMALL_MAX];
  uint16_t out[EC_SMALL_MAX];
};
void launch_ec_small(int cls, int wq, const EcSmallArgs& a, hipStream_t s);
// key staging: validate each listed key (plain 28-bit limbs x,y at aux_off:
// coordinates < p, on the curve) and write its Montgomery affine coordinates
// back to aux_off
void launch_ec_keyprep(int cls, jgk::DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
// comb tables (width wq) of the valid keys tidx[0..tn), written at each key's
// `tab` (ec_table_words_w(cls, wq) words); after launch_ec_keyprep
void launch_ec_keytables(int cls, int wq, jgk::DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn,
                         hipStream_t s, bool sliced = false);
// generator table for a curve into `tab` (ec_table_words(cls) words)
void launch_ec_gtable(int cls, uint32_t* tab, hipStream_t s);
