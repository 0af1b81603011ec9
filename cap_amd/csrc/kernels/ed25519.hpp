// ed25519.hpp -- launch interface of the Ed25519 kernels (ed25519.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct EdArgs {
  const jgk::JobDev* jobs;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // R at rows 0..7, S at rows 8..15 (LE words)
  const uint32_t* dig;        // SHA-512(R || A || M), big-endian words
  uint8_t* status;
  const uint16_t* siglen;
  uint8_t* verdict_pad;
  uint32_t* xyz;              // X, Y, Z of R' (3 x 10 limb rows), then 10 rows of
                              // k_ed_finish's prefix products
  const uint32_t* btab;       // comb table of the base point B (Niels form)
  int64_t npad, begin, end;
  int32_t wa;                 // comb width of the launch's key tables (ED_WA)
};

constexpr int ED_L = 10;
constexpr int ED_STRIDE = 32;                   // 3 x 10 limbs, padded to 16 B
// Signed-digit comb geometry (as ecdsa.hpp): scalars S, k < L < 2^253, so
// ceil(254 / W) windows.  The base point's table is shared by all keys and gets
// the widest window: B W = 24 (11 windows, 11.8 GB).  Key tables take the
// widest tier the context's table budget allows (ED_WA, picked with the EC
// tiers of ecdsa.hpp, jg_runtime.cpp key_widths): W = 24 (11 windows, 11.8 GB
// per key: 22 additions per token), 22 (12, 3.2 GB), 20 (13, 872 MB), 18 (15,
// 252 MB), 16 (16, 67 MB).  Round 2 stopped at W = 20 for both (26 additions).
constexpr int ed_comb_w(bool base) { return base ? 24 : 16; }
constexpr int ed_windows_w(int w) { return (253 + 1 + w - 1) / w; }
constexpr int ed_entries(bool base) { return 1 << (ed_comb_w(base) - 1); }
constexpr int ed_windows(bool base) { return ed_windows_w(ed_comb_w(base)); }
constexpr int64_t ed_table_words_w(int w) { return (int64_t)ed_windows_w(w) * (1 << (w - 1)) * ED_STRIDE; }
constexpr int64_t ed_table_words(bool base) { return ed_table_words_w(ed_comb_w(base)); }
constexpr int ED_WA[5] = {24, 22, 20, 18, 16};   // key-table width tiers, widest first
// recode (ed25519.hip) carries out of a window when its value exceeds 2^(W-1):
// the top window must hold at most W - 1 bits of a scalar < 2^253 (its value
// + the incoming carry then stays <= 2^(W-1) and no carry leaves the last digit)
constexpr bool ed_top_window_ok(int w) { return 253 - w * (ed_windows_w(w) - 1) <= w - 1; }
static_assert(ed_top_window_ok(ed_comb_w(true)) && ed_top_window_ok(24) && ed_top_window_ok(22) &&
              ed_top_window_ok(20) && ed_top_window_ok(18) && ed_top_window_ok(16),
              "Ed25519 comb window count leaves no room for the top carry");
constexpr int ED_MAX_KEYS = 256;

void launch_ed(const EdArgs& a, hipStream_t s, const jgk::Marker& mk);
// key staging: decode each listed key's 32 public-key bytes (words at
// aux_off) and mark validity
void launch_ed_keyprep(jgk::DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s);
// comb tables of -A (width wa) of the valid keys tidx[0..tn), at each key's `tab`
void launch_ed_keytables(int wa, jgk::DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s,
                         bool sliced = false);
void launch_ed_btable(uint32_t* tab, hipStream_t s);

// One-launch verification of a small batch of EdDSA tokens (k_ed_small,
// ed25519.hip): one two-wave block per token -- SHA-512(R || A || M) on one
// lane, the comb sum over 16 lanes with pairwise complete additions, Z^-1 by
// the variable-time safegcd on four lanes, encode(R') == R -- writing
// verdict[out[i]] (pinned host memory).  Every key of a launch has key-table
// width `wa`.  Jobs in the arguments, arena read in place (as EcSmallArgs).
struct EdSmallArgs {
  const uint8_t* arena;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* btab;
  uint8_t* verdict;
  uint32_t n;
  jgk::JobDev jobs[jgk::SMALL_MAX];
  uint16_t out[jgk::SMALL_MAX];
};
void launch_ed_small(int wa, const EdSmallArgs& a, hipStream_t s);
