// sha2.hpp -- thread-per-message SHA-256 / SHA-384 / SHA-512 (FIPS 180-4) over
// byte strings at arbitrary offsets of the token arena in HBM.
//
// Message bytes are fetched as aligned 32-bit words (global_load_dword) and
// realigned with v_alignbyte_b32 + v_perm_b32 byte swaps, so a 255-byte
// signing input costs ~65 dword loads instead of 255 byte loads.  Padding is
// synthesised in registers.  A message may carry a 64-byte register prefix
// (Ed25519 hashes R || A || M, with R || A already in registers).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define SHD __device__ __forceinline__

namespace sha2 {

__constant__ static const uint32_t K256[64] = {
  0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
  0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
  0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
  0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
  0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
  0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
  0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
  0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};

__constant__ static const uint64_t K512[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,0x3956c25bf348b538ULL,
  0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,0xd807aa98a3030242ULL,0x12835b0145706fbeULL,
  0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,
  0xc19bf174cf692694ULL,0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,0x983e5152ee66dfabULL,
  0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,
  0x06ca6351e003826fULL,0x142929670a0e6e70ULL,0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,
  0x53380d139d95b3dfULL,0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,0xd192e819d6ef5218ULL,
  0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,
  0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,
  0x682e6ff3d6b2b8a3ULL,0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,0xca273eceea26619cULL,
  0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,
  0x113f9804bef90daeULL,0x1b710b35131c471bULL,0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,
  0x431d67c49c100d4cULL,0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL};

SHD uint32_t rotr32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// a ^ b ^ c as one gfx950 v_bitop3_b32 (truth table 0x96); LLVM emits two
// v_xor_b32 for the plain expression
SHD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
SHD uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return ((uint64_t)xor3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
         xor3((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
// 64-bit rotate as two v_alignbit_b32 on the halves (n is a compile-time
// constant at every call site): 2 VALU instead of two 64-bit shifts + 2 ors
SHD uint64_t rotr64(uint64_t x, int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (n < 32)
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
  return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, n - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, n - 32);
}
SHD uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

// Big-endian 32-bit word i of the byte string m[0..len) followed by SHA
// padding, where the string lives at byte offset `off` of `base` (only the
// bytes before `len` are taken from memory; the caller guarantees the aligned
// words around the string are readable -- the arena is allocated with slack).
struct MemString {
  const uint32_t* aligned;   // base + (off & ~3)
  uint32_t shift;            // off & 3
  uint32_t len;

  SHD uint32_t raw_be(uint32_t i) const {        // bytes [4i, 4i+4) of m, big-endian
    const uint32_t lo = aligned[i];
    const uint32_t hi = aligned[i + 1];
    return bswap32(__builtin_amdgcn_alignbyte(hi, lo, shift));
  }

  // N consecutive big-endian words starting at word w0, padded (SHA padding
  // 0x80 / zeros; the length words are the caller's).  All N+1 aligned loads
  // are issued unconditionally, back to back: reads may run past the string
  // (the arena carries slack), bytes at or beyond len are masked.
  template <int N>
  SHD void padded_words(uint32_t w0, uint32_t* out) const {
    uint32_t u[N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k) u[k] = aligned[w0 + k];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const uint32_t raw = bswap32(__builtin_amdgcn_alignbyte(u[k + 1], u[k], shift));
      const int rem = (int)len - (int)(4u * (w0 + k));
      const uint32_t keep = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (0xffffffffu << (32 - 8 * rem)));
      const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80u << (24 - 8 * rem)) : 0u;
      out[k] = (raw & keep) | pad;
    }
  }
};

// word i of the padded stream given the big-endian raw word for bytes [4i,4i+4)
SHD uint32_t pad_word(uint32_t raw, uint32_t i, uint32_t len) {
  const int rem = (int)len - (int)(4u * i);       // message bytes present in this word
  if (rem >= 4) return raw;
  if (rem <= -1) return 0u;
  const uint32_t keep = rem == 0 ? 0u : (0xffffffffu << (32 - 8 * rem));
  return (raw & keep) | (0x80u << (24 - 8 * rem));
}

// ---------------------------------------------------------------- SHA-256
SHD void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + K256[i] + wi;
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

SHD void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
}

// SHA-256 of a string in memory; digest as 8 big-endian words
SHD void sha256_mem(uint32_t h[8], const MemString& m) {
  sha256_init(h);
  const uint32_t nblk = (m.len + 9 + 63) / 64;
  const uint32_t nwords = nblk * 16;
  for (uint32_t blk = 0; blk < nblk; ++blk) {
    uint32_t w[16];
    m.padded_words<16>(blk * 16, w);
    if (blk == nblk - 1) {
      w[14] = m.len >> 29;
      w[15] = m.len << 3;
    }
    sha256_compress(h, w);
  }
  (void)nwords;
}

// ---------------------------------------------------------------- SHA-512/384
// One SHA-512 round on the state held in named registers (the caller rotates
// the names, so no moves between rounds).
#define SHA512_ROUND(a, b, c, d, e, f, g, h, k, wi)                                                    \
  do {                                                                                                  \
    const uint64_t t1_ = (h) + xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41)) +                   \
                         (((e) & (f)) ^ (~(e) & (g))) + (k) + (wi);                                         \
    (d) += t1_;                                                                                         \
    (h) = t1_ + xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39)) + (((a) & (b)) ^ ((a) & (c)) ^ ((b) & (c)));       \
  } while (0)

// 8 rounds starting at round i0 (a multiple of 8) with message words w[j0..j0+8)
#define SHA512_8ROUNDS(i0, j0)                                                                   \
  do {                                                                                          \
    SHA512_ROUND(A, B, C, D, E, F, G, H, K512[(i0) + 0], w[(j0) + 0]);                          \
    SHA512_ROUND(H, A, B, C, D, E, F, G, K512[(i0) + 1], w[(j0) + 1]);                          \
    SHA512_ROUND(G, H, A, B, C, D, E, F, K512[(i0) + 2], w[(j0) + 2]);                          \
    SHA512_ROUND(F, G, H, A, B, C, D, E, K512[(i0) + 3], w[(j0) + 3]);                          \
    SHA512_ROUND(E, F, G, H, A, B, C, D, K512[(i0) + 4], w[(j0) + 4]);                          \
    SHA512_ROUND(D, E, F, G, H, A, B, C, K512[(i0) + 5], w[(j0) + 5]);                          \
    SHA512_ROUND(C, D, E, F, G, H, A, B, K512[(i0) + 6], w[(j0) + 6]);                          \
    SHA512_ROUND(B, C, D, E, F, G, H, A, K512[(i0) + 7], w[(j0) + 7]);                          \
  } while (0)

// Rounds 16..79 run as four 16-round blocks of a rolled loop whose body is
// fully unrolled: the schedule index (i & 15) is then static, so w[] stays in
// registers.  (An 80-round #pragma unroll is past LLVM's unroll budget; it
// unrolled partially and indexed w[] with s_set_gpr_idx moves on every access.)
SHD void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t A = h[0], B = h[1], C = h[2], D = h[3], E = h[4], F = h[5], G = h[6], H = h[7];
  SHA512_8ROUNDS(0, 0);
  SHA512_8ROUNDS(8, 8);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), w15 >> 7);
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), w2 >> 6);
      w[j] += s0 + w[(j + 9) & 15] + s1;
    }
    SHA512_8ROUNDS(r, 0);
    SHA512_8ROUNDS(r + 8, 8);
  }
  h[0] += A; h[1] += B; h[2] += C; h[3] += D; h[4] += E; h[5] += F; h[6] += G; h[7] += H;
}
#undef SHA512_8ROUNDS
#undef SHA512_ROUND

SHD void sha512_init(uint64_t h[8], bool is384) {
  if (is384) {
    h[0] = 0xcbbb9d5dc1059ed8ULL; h[1] = 0x629a292a367cd507ULL; h[2] = 0x9159015a3070dd17ULL;
    h[3] = 0x152fecd8f70e5939ULL; h[4] = 0x67332667ffc00b31ULL; h[5] = 0x8eb44a8768581511ULL;
    h[6] = 0xdb0c2e0d64f98fa7ULL; h[7] = 0x47b5481dbefa4fa4ULL;
  } else {
    h[0] = 0x6a09e667f3bcc908ULL; h[1] = 0xbb67ae8584caa73bULL; h[2] = 0x3c6ef372fe94f82bULL;
    h[3] = 0xa54ff53a5f1d36f1ULL; h[4] = 0x510e527fade682d1ULL; h[5] = 0x9b05688c2b3e6c1fULL;
    h[6] = 0x1f83d9abfb41bd6bULL; h[7] = 0x5be0cd19137e2179ULL;
  }
}

// SHA-512 (or -384) of  prefix[0..plen) || m  where plen is 0 or 64 and the
// prefix is given as 16 big-endian 32-bit words.  Digest as 8 64-bit words.
SHD void sha512_mem(uint64_t h[8], bool is384, const MemString& m, const uint32_t* prefix, uint32_t plen) {
  sha512_init(h, is384);
  const uint32_t tot = plen + m.len;                 // bytes hashed
  const uint32_t nblk = (tot + 17 + 127) / 128;
  const uint32_t nw32 = nblk * 32;                   // 32-bit words in the padded stream
  const uint32_t pw = plen / 4;                      // prefix words (0 or 16)
  for (uint32_t blk = 0; blk < nblk; ++blk) {
    uint32_t v[32];
    if (pw != 0 && blk == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = prefix[k];
      m.padded_words<16>(0, v + 16);
    } else {
      m.padded_words<32>(blk * 32 - pw, v);
    }
    if (blk == nblk - 1) {                           // 128-bit length, high 64 bits zero
      v[30] = tot >> 29;
      v[31] = tot << 3;
    }
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = ((uint64_t)v[2 * k] << 32) | v[2 * k + 1];
    sha512_compress(h, w);
  }
  (void)nw32;
}

}  // namespace sha2
