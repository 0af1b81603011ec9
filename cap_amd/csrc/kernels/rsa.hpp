// rsa.hpp -- launch interface of the RSA kernels (rsa.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "prep.hpp"

struct RsaArgs {
  const jgk::JobDev* jobs;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  const uint32_t* sigw;       // decoded signature integer, LE words, SoA rows
  const uint32_t* dig;        // digest rows
  uint32_t* xmw;              // x*R mod n, limb rows (generic-e path)
  uint32_t* xlr;              // x, limb rows
  uint32_t* yw;               // s^e mod n rows (LE words)
  uint8_t* status;
  const uint16_t* siglen;
  uint8_t* verdict_pad;
  uint8_t* pss_scratch;       // 2 KiB per token of the class range
  int32_t has_pss;            // the range holds PS* tokens (else the PKCS#1-only pad kernel)
  int32_t layouts;            // RSA-4K+ class: bit i = keys of rsa4k_layout_limbs(i) limbs are loaded
  int64_t npad, begin, end;
};

// RSA-2048 layout: JG_RSA2K_G lanes per token, H limbs per lane
#ifndef JG_RSA2K_G
#define JG_RSA2K_G 2
#endif
constexpr int RSA2K_G = JG_RSA2K_G;
constexpr int RSA2K_H = RSA2K_G == 2 ? 37 : 19;
// RSA-3072 layout (112 limbs): JG_RSA3K_G lanes per token, 112 / G limbs per
// lane, JG_RSA3K_U CIOS rows per unrolled block (compile-time A/B knobs).
// Two lanes of 56 limbs (round 4) against four of 28: the class's modexp
// 16.2 -> 14.8 ns per token alone (tools/class_costs.py), 1.97 -> 1.81 ms in
// configs[4] (profiles/r04_s3/rsa3k_*), although the 56-limb accumulator
// windows spill ~140 VGPRs at two waves per SIMD -- the 4-lane rows pay more
// in cross-lane broadcasts and limb hand-offs per MAD than the spills cost.
// U (4 / 8 / 14 / 16) measured within 1.5 %.  Keeping the modulus limbs in
// LDS instead of VGPRs (re-read every CIOS row, a broadcast read) freed 20-30
// VGPRs per layout but made every modexp 2-6x slower
// (profiles/r04_s6/class_costs_nlds*.json): not kept.
#ifndef JG_RSA3K_G
#define JG_RSA3K_G 2
#endif
#ifndef JG_RSA3K_U
#define JG_RSA3K_U 8
#endif
constexpr int RSA3K_G = JG_RSA3K_G;
constexpr int RSA3K_H = 112 / RSA3K_G;
constexpr int RSA3K_U = JG_RSA3K_U;
static_assert(RSA3K_G * RSA3K_H == 112, "RSA-3K layouts hold 112 limbs");
// limbs of the class's (smallest) layout: 74 / 112 / 148
constexpr int rsa_limbs(int cls) {
  return cls == jgk::CLS_RSA2K ? RSA2K_G * RSA2K_H : cls == jgk::CLS_RSA3K ? 112 : 148;
}
// The RSA-4K+ class (moduli of 3135 bits and up) has three layouts of H = 37
// limbs per lane, picked per key by its size: G = 4, 8 or 16 lanes per token
// (148, 296, 592 limbs: up to 4142, 8286 and 16574 bits).  Each layout's
// kernel runs over the class range and serves the waves of its own keys.
constexpr int RSA4K_H = 37;
constexpr int RSA4K_NLAYOUT = 3;
constexpr int rsa4k_layout_limbs(int i) { return RSA4K_H * (4 << i); }
constexpr int rsa4k_limbs_for_bits(int bits) {
  return bits <= 148 * 28 - 2 ? 148 : bits <= 296 * 28 - 2 ? 296 : bits <= 592 * 28 - 2 ? 592 : 0;
}
// rows of the signature scratch an L-limb modexp reads: its limb loads touch
// words up to (28 L - 1) / 32 + 1 (load_limbs_from_words), so those rows must
// be zeroed by prep; the result y takes as many rows
constexpr int rsa_sig_rows_l(int L) { return (28 * L - 1) / 32 + 2; }
constexpr int rsa_sig_rows(int cls) { return rsa_sig_rows_l(rsa_limbs(cls)); }
static_assert(rsa_sig_rows_l(rsa4k_layout_limbs(RSA4K_NLAYOUT - 1)) <= jgk::SIGW_ROWS,
              "RSA-16K signature rows exceed the scratch");

void launch_rsa(int cls, const RsaArgs& a, hipStream_t s, const jgk::Marker& mk);

// One-launch verification of a small batch of PKCS#1 v1.5 tokens (RS256 /
// RS384 / RS512) on RSA-2K-class keys (k_rsa_small, rsa.hip): one two-wave
// block per token -- the signing input hashed on one lane while the other
// wave decodes the signature and runs s^e mod n on 16 lanes of 5 limbs
// (RSA_SMALL_L = 80 limbs, R = 2^2240: each key carries R^2 mod n for that R
// at rr2_off), then the EM compare -- writing verdict[out[i]] (pinned host
// memory).  Jobs in the arguments, arena read in place (as EcSmallArgs).
constexpr int RSA_SMALL_H = 5, RSA_SMALL_G = 16, RSA_SMALL_L = RSA_SMALL_H * RSA_SMALL_G;
static_assert(RSA_SMALL_L * 28 - 2 >= 74 * 28 - 2, "the small layout holds every RSA-2K modulus");
struct RsaSmallArgs {
  const uint8_t* arena;
  const jgk::DevKey* keys;
  const uint32_t* keyblob;
  uint8_t* verdict;
  uint32_t n;
  jgk::JobDev jobs[jgk::SMALL_MAX];
  uint16_t out[jgk::SMALL_MAX];
};
void launch_rsa_small(const RsaSmallArgs& a, hipStream_t s);
