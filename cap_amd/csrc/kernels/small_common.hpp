// small_common.hpp -- the pieces every one-launch small-batch kernel shares
// (ec_small.hpp k_ec_small, rsa.hip k_rsa_small): one 128-thread block (two
// waves) per token, inputs read in place from the arena (pinned host memory
// over PCIe, or a device copy), staged in LDS with bounded dword loads.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "common.hpp"
#include "mp.hpp"
#include "sha2.hpp"

namespace {

constexpr int SM_THREADS = 128;
constexpr uint32_t SM_IN_DW = jgk::SMALL_IN_MAX / 4 + 72;         // staged signing input + SHA padding blocks

// JG_SMALL_PROF=1 (A/B builds only, tools/small_prof.sh): lane 0 of each wave
// stamps s_memrealtime (100 MHz) at the phase boundaries and the block prints
// one line per token -- where a lone token's time goes.
#ifndef JG_SMALL_PROF
#define JG_SMALL_PROF 0
#endif
#if JG_SMALL_PROF
#define SM_STAMP(i) do { if (lane == 0) stamp[wave][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define SM_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ int sm_b64val(uint32_t c) {
  if (c - 'A' < 26u) return (int)(c - 'A');
  if (c - 'a' < 26u) return (int)(c - 'a' + 26);
  if (c - '0' < 10u) return (int)(c - '0' + 52);
  if (c == '-') return 62;
  if (c == '_') return 63;
  return -1;
}

// N big-endian words of the SHA-padded message from word w0 (length words
// are the caller's), the message staged in LDS as aligned dwords starting
// `shift` bytes before it (sha2::MemString::padded_words on an LDS array)
template <int N>
__device__ __forceinline__ void sm_words(const uint32_t* lds, uint32_t w0, uint32_t shift, uint32_t len,
                                         uint32_t* out) {
  uint32_t u[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) u[k] = mp::lane_value(lds[w0 + k]);   // keep the SHA on VALU (mp::lane_value)
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint32_t raw = sha2::bswap32(__builtin_amdgcn_alignbyte(u[k + 1], u[k], shift));
    const int rem = (int)len - (int)(4u * (w0 + k));
    const uint32_t keep = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (0xffffffffu << (32 - 8 * rem)));
    const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80u << (24 - 8 * rem)) : 0u;
    out[k] = (raw & keep) | pad;
  }
}

// One wave stages the signing input (len bytes at g + shift, g 4-byte aligned)
// into LDS: the dwords holding message bytes, zeros up to the SHA stream of
// hb bits (+ the alignbyte dword).  Only dwords that hold message bytes are
// read (no load leaves the message's pages).  Eight loads in flight per lane.
// `prefix`: bytes hashed before the message (Ed25519's R || A: 64), which
// shift the stream's blocks.
__device__ __forceinline__ void sm_stage_input(uint32_t* in_w, const uint32_t* g, uint32_t shift, uint32_t len,
                                               int hb, int lane, uint32_t prefix = 0) {
  const uint32_t ndw = (shift + len + 3) / 4;
  const uint32_t tot = len + prefix;
  const uint32_t nblk = hb == 256 ? (tot + 9 + 63) / 64 : (tot + 17 + 127) / 128;
  const uint32_t need = nblk * (hb == 256 ? 16u : 32u) - prefix / 4 + 1u;
  for (uint32_t base = 0; base < need; base += 64 * 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t i = base + (uint32_t)lane + 64u * k;
      v[k] = i < ndw ? g[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t i = base + (uint32_t)lane + 64u * k;
      if (i < need) in_w[i] = v[k];
    }
  }
}

// SHA-256 / -384 / -512 (hb) of the staged message on ONE lane; the digest as
// big-endian words into dig_w (8 or 16)
__device__ __forceinline__ void sm_hash(const uint32_t* in_w, uint32_t shift, uint32_t len, int hb, uint32_t* dig_w) {
  if (hb == 256) {
    uint32_t h[8];
    sha2::sha256_init(h);
    const uint32_t nblk = (len + 9 + 63) / 64;
#pragma unroll 1
    for (uint32_t blk = 0; blk < nblk; ++blk) {
      uint32_t w[16];
      sm_words<16>(in_w, blk * 16, shift, len, w);
      if (blk == nblk - 1) { w[14] = len >> 29; w[15] = len << 3; }
      sha2::sha256_compress(h, w);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) dig_w[k] = h[k];
  } else {
    uint64_t h[8];
    sha2::sha512_init(h, hb == 384);
    const uint32_t nblk = (len + 17 + 127) / 128;
#pragma unroll 1
    for (uint32_t blk = 0; blk < nblk; ++blk) {
      uint32_t v[32];
      sm_words<32>(in_w, blk * 32, shift, len, v);
      if (blk == nblk - 1) { v[30] = len >> 29; v[31] = len << 3; }
      uint64_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = ((uint64_t)v[2 * k] << 32) | v[2 * k + 1];
      sha2::sha512_compress(h, w);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { dig_w[2 * k] = (uint32_t)(h[k] >> 32); dig_w[2 * k + 1] = (uint32_t)h[k]; }
  }
}

// base64url characters -> bytes (go-jose base64URLDecode, R3; no padding,
// trailing bits ignored as Go's non-strict decoder does): the nch characters
// staged as dwords in chars_w from byte `shift` on, one quad of 4 characters
// per lane and round; bytes to out[0 .. D).  Returns true on the wave if any
// character is outside the alphabet.
__device__ __forceinline__ bool sm_b64_decode(const uint32_t* chars_w, uint32_t shift, uint32_t nch, uint8_t* out,
                                              int lane) {
  bool bad = false;
  for (uint32_t c0 = 4u * (uint32_t)lane; c0 < nch; c0 += 256u) {
    uint32_t acc = 0;
    const uint32_t cnt = nch - c0 < 4u ? nch - c0 : 4u;
    for (uint32_t k = 0; k < 4; ++k) {
      int v = 0;
      if (k < cnt) {
        const uint32_t b = shift + c0 + k;
        v = sm_b64val((chars_w[b >> 2] >> (8u * (b & 3u))) & 0xffu);
        bad |= v < 0;
      }
      acc = (acc << 6) | (uint32_t)(v < 0 ? 0 : v);
    }
    // cnt characters carry 6 cnt bits: 3 bytes from 4, 2 from 3, 1 from 2
    const uint32_t nb = cnt == 4 ? 3u : cnt - 1u;
    const uint32_t o = 3u * (c0 >> 2);
    for (uint32_t k = 0; k < nb; ++k) out[o + k] = (uint8_t)(acc >> (16u - 8u * k));
  }
  return __ballot(bad) != 0ull;
}

// decoded length of nch base64url characters (0 for the impossible nch % 4 == 1)
__device__ __forceinline__ uint32_t sm_b64_len(uint32_t nch) {
  return (nch & 3u) == 1u ? 0u : (nch >> 2) * 3u + ((nch & 3u) == 2u ? 1u : (nch & 3u) == 3u ? 2u : 0u);
}

}  // namespace
