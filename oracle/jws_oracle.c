/*
 * jws_oracle.c -- CPU restatement of the JWS verify arithmetic (TEST
 * INFRASTRUCTURE ONLY; see jws_oracle.h for provenance and scope).
 *
 * Written for clarity, not speed: generic little-endian 32-bit-limb bignums,
 * CIOS Montgomery multiplication, bitwise long division, double-and-add
 * scalar multiplication with every exceptional case of the group law handled
 * explicitly.  Every public function cites the Go semantics it restates
 * (SURVEY.md Appendix A rule numbers).
 */
#include "jws_oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* SHA-2 (FIPS 180-4)                                                       */
/* ======================================================================= */
static const uint32_t K256[64] = {
  0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
  0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
  0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
  0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
  0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
  0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
  0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
  0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};

#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
#define ROR64(x, n) (((x) >> (n)) | ((x) << (64 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)p[4*i] << 24 | (uint32_t)p[4*i+1] << 16 | (uint32_t)p[4*i+2] << 8 | p[4*i+3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR32(w[i-15], 7) ^ ROR32(w[i-15], 18) ^ (w[i-15] >> 3);
    uint32_t s1 = ROR32(w[i-2], 17) ^ ROR32(w[i-2], 19) ^ (w[i-2] >> 10);
    w[i] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void or_sha256(const uint8_t* m, size_t n, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= n; i += 64) sha256_block(h, m + i);
  uint8_t buf[128] = {0};
  size_t r = n - i;
  memcpy(buf, m + i, r);
  buf[r] = 0x80;
  size_t tot = (r + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)n * 8;
  for (int j = 0; j < 8; ++j) buf[tot - 1 - j] = (uint8_t)(bits >> (8 * j));
  for (size_t j = 0; j < tot; j += 64) sha256_block(h, buf + j);
  for (int j = 0; j < 8; ++j) {
    out[4*j] = h[j] >> 24; out[4*j+1] = h[j] >> 16; out[4*j+2] = h[j] >> 8; out[4*j+3] = h[j];
  }
}

static const uint64_t K512[80] = {
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

static void sha512_block(uint64_t h[8], const uint8_t* p) {
  uint64_t w[80];
  for (int i = 0; i < 16; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = v << 8 | p[8*i + j];
    w[i] = v;
  }
  for (int i = 16; i < 80; ++i) {
    uint64_t s0 = ROR64(w[i-15], 1) ^ ROR64(w[i-15], 8) ^ (w[i-15] >> 7);
    uint64_t s1 = ROR64(w[i-2], 19) ^ ROR64(w[i-2], 61) ^ (w[i-2] >> 6);
    w[i] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 80; ++i) {
    uint64_t S1 = ROR64(e, 14) ^ ROR64(e, 18) ^ ROR64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K512[i] + w[i];
    uint64_t S0 = ROR64(a, 28) ^ ROR64(a, 34) ^ ROR64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512_core(const uint64_t iv[8], const uint8_t* m, size_t n, uint8_t* out, int outlen) {
  uint64_t h[8];
  memcpy(h, iv, sizeof h);
  size_t i = 0;
  for (; i + 128 <= n; i += 128) sha512_block(h, m + i);
  uint8_t buf[256] = {0};
  size_t r = n - i;
  memcpy(buf, m + i, r);
  buf[r] = 0x80;
  size_t tot = (r + 17 <= 128) ? 128 : 256;
  uint64_t bits = (uint64_t)n * 8;      /* high 64 bits of the 128-bit length are 0 */
  for (int j = 0; j < 8; ++j) buf[tot - 1 - j] = (uint8_t)(bits >> (8 * j));
  for (size_t j = 0; j < tot; j += 128) sha512_block(h, buf + j);
  for (int j = 0; j < outlen; ++j) out[j] = (uint8_t)(h[j / 8] >> (56 - 8 * (j % 8)));
}

void or_sha512(const uint8_t* m, size_t n, uint8_t out[64]) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL,0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL};
  sha512_core(iv, m, n, out, 64);
}

void or_sha384(const uint8_t* m, size_t n, uint8_t out[48]) {
  static const uint64_t iv[8] = {0xcbbb9d5dc1059ed8ULL,0x629a292a367cd507ULL,0x9159015a3070dd17ULL,
    0x152fecd8f70e5939ULL,0x67332667ffc00b31ULL,0x8eb44a8768581511ULL,0xdb0c2e0d64f98fa7ULL,0x47b5481dbefa4fa4ULL};
  sha512_core(iv, m, n, out, 48);
}

static int hash_len(int hbits) { return hbits / 8; }
static void hash_any(int hbits, const uint8_t* m, size_t n, uint8_t* out) {
  if (hbits == 256) or_sha256(m, n, out);
  else if (hbits == 384) or_sha384(m, n, out);
  else or_sha512(m, n, out);
}

/* ======================================================================= */
/* base64url, go-jose base64URLDecode semantics [R3]                        */
/* ======================================================================= */
long or_b64url_decode(const char* s, size_t n, uint8_t* out, size_t cap) {
  while (n > 0 && s[n - 1] == '=') --n;             /* strings.TrimRight(s, "=") */
  uint32_t acc = 0; int nb = 0; size_t o = 0, nchar = 0;
  for (size_t i = 0; i < n; ++i) {
    char c = s[i];
    int v;
    if (c == '\r' || c == '\n') continue;           /* encoding/base64 skips CR/LF */
    if (c >= 'A' && c <= 'Z') v = c - 'A';
    else if (c >= 'a' && c <= 'z') v = c - 'a' + 26;
    else if (c >= '0' && c <= '9') v = c - '0' + 52;
    else if (c == '-') v = 62;
    else if (c == '_') v = 63;
    else return -1;                                  /* CorruptInputError */
    ++nchar;
    acc = acc << 6 | (uint32_t)v; nb += 6;
    if (nb >= 8) {
      nb -= 8;
      if (o >= cap) return -1;
      out[o++] = (uint8_t)(acc >> nb);
      acc &= (1u << nb) - 1;
    }
  }
  if (nchar % 4 == 1) return -1;                     /* a lone 6-bit group */
  return (long)o;                                    /* non-strict: spare bits ignored */
}

/* ======================================================================= */
/* bignum: little-endian uint32 limbs                                       */
/* ======================================================================= */
#define MAXL 600   /* 19200 bits: RSA moduli up to the GPU path's 16574-bit layout */

static void bn_from_be(uint32_t* r, int L, const uint8_t* b, size_t blen) {
  memset(r, 0, sizeof(uint32_t) * L);
  for (size_t i = 0; i < blen; ++i) {
    size_t bit = (blen - 1 - i) * 8;
    if (bit / 32 < (size_t)L) r[bit / 32] |= (uint32_t)b[i] << (bit % 32);
  }
}
static void bn_to_be(uint8_t* b, size_t blen, const uint32_t* r, int L) {
  for (size_t i = 0; i < blen; ++i) {
    size_t bit = (blen - 1 - i) * 8;
    b[i] = (bit / 32 < (size_t)L) ? (uint8_t)(r[bit / 32] >> (bit % 32)) : 0;
  }
}
static int bn_cmp(const uint32_t* a, const uint32_t* b, int L) {
  for (int i = L - 1; i >= 0; --i) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}
static int bn_is_zero(const uint32_t* a, int L) {
  for (int i = 0; i < L; ++i) if (a[i]) return 0;
  return 1;
}
static uint32_t bn_sub(uint32_t* r, const uint32_t* a, const uint32_t* b, int L) {
  uint64_t br = 0;
  for (int i = 0; i < L; ++i) {
    uint64_t d = (uint64_t)a[i] - b[i] - br;
    r[i] = (uint32_t)d; br = (d >> 63) & 1;
  }
  return (uint32_t)br;
}
static uint32_t bn_add(uint32_t* r, const uint32_t* a, const uint32_t* b, int L) {
  uint64_t c = 0;
  for (int i = 0; i < L; ++i) { c += (uint64_t)a[i] + b[i]; r[i] = (uint32_t)c; c >>= 32; }
  return (uint32_t)c;
}
static int bn_bitlen(const uint32_t* a, int L) {
  for (int i = L - 1; i >= 0; --i)
    if (a[i]) { int b = 32; while (!(a[i] >> (b - 1))) --b; return 32 * i + b; }
  return 0;
}
static int bn_bit(const uint32_t* a, int i) { return (a[i / 32] >> (i % 32)) & 1; }

/* r = x mod m, x has xL limbs, m has L limbs (bitwise long division). */
static void bn_mod(uint32_t* r, const uint32_t* x, int xL, const uint32_t* m, int L) {
  uint32_t t[MAXL + 1];
  memset(t, 0, sizeof(uint32_t) * (L + 1));
  uint32_t mm[MAXL + 1];
  memcpy(mm, m, sizeof(uint32_t) * L); mm[L] = 0;
  for (int i = 32 * xL - 1; i >= 0; --i) {
    uint32_t carry = 0;                               /* t = 2t + bit */
    for (int j = 0; j <= L; ++j) { uint32_t nc = t[j] >> 31; t[j] = t[j] << 1 | carry; carry = nc; }
    t[0] |= (uint32_t)bn_bit(x, i);
    if (bn_cmp(t, mm, L + 1) >= 0) bn_sub(t, t, mm, L + 1);
  }
  memcpy(r, t, sizeof(uint32_t) * L);
}

/* Montgomery context for an odd modulus. */
typedef struct { int L; uint32_t m[MAXL]; uint32_t minv; uint32_t r2[MAXL]; uint32_t one[MAXL]; } mont;

static void mont_init(mont* c, const uint32_t* m, int L) {
  c->L = L;
  memcpy(c->m, m, sizeof(uint32_t) * L);
  uint32_t inv = 1;                                   /* Newton: inv = m0^-1 mod 2^32 */
  for (int i = 0; i < 5; ++i) inv *= 2 - m[0] * inv;
  c->minv = (uint32_t)(0u - inv);
  uint32_t x[2 * MAXL + 1];                           /* R^2 mod m by long division */
  memset(x, 0, sizeof(uint32_t) * (2 * L + 1));
  x[2 * L] = 1;
  bn_mod(c->r2, x, 2 * L + 1, m, L);
  memset(x, 0, sizeof(uint32_t) * (L + 1));
  x[L] = 1;
  bn_mod(c->one, x, L + 1, m, L);
}

/* CIOS: r = a*b*R^-1 mod m, for a,b < m. */
static void mont_mul(const mont* c, uint32_t* r, const uint32_t* a, const uint32_t* b) {
  int L = c->L;
  uint32_t t[MAXL + 2];
  memset(t, 0, sizeof(uint32_t) * (L + 2));
  for (int i = 0; i < L; ++i) {
    uint64_t C = 0;
    for (int j = 0; j < L; ++j) {
      uint64_t v = (uint64_t)t[j] + (uint64_t)a[j] * b[i] + C;
      t[j] = (uint32_t)v; C = v >> 32;
    }
    uint64_t v = (uint64_t)t[L] + C; t[L] = (uint32_t)v; t[L + 1] = (uint32_t)(v >> 32);
    uint32_t mq = t[0] * c->minv;
    v = (uint64_t)t[0] + (uint64_t)mq * c->m[0]; C = v >> 32;
    for (int j = 1; j < L; ++j) {
      v = (uint64_t)t[j] + (uint64_t)mq * c->m[j] + C;
      t[j - 1] = (uint32_t)v; C = v >> 32;
    }
    v = (uint64_t)t[L] + C; t[L - 1] = (uint32_t)v; C = v >> 32;
    t[L] = t[L + 1] + (uint32_t)C;
  }
  if (t[L] || bn_cmp(t, c->m, L) >= 0) bn_sub(t, t, c->m, L);
  memcpy(r, t, sizeof(uint32_t) * L);
}
static void to_mont(const mont* c, uint32_t* r, const uint32_t* a) { mont_mul(c, r, a, c->r2); }
static void from_mont(const mont* c, uint32_t* r, const uint32_t* a) {
  uint32_t one[MAXL] = {1};
  mont_mul(c, r, a, one);
}
static void mod_add(const mont* c, uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t cy = bn_add(r, a, b, c->L);
  if (cy || bn_cmp(r, c->m, c->L) >= 0) bn_sub(r, r, c->m, c->L);
}
static void mod_sub(const mont* c, uint32_t* r, const uint32_t* a, const uint32_t* b) {
  if (bn_sub(r, a, b, c->L)) bn_add(r, r, c->m, c->L);
}
/* r = a^e (all in Montgomery form), e as limbs with eL limbs */
static void mont_pow(const mont* c, uint32_t* r, const uint32_t* a, const uint32_t* e, int eL) {
  uint32_t acc[MAXL];
  memcpy(acc, c->one, sizeof(uint32_t) * c->L);
  for (int i = bn_bitlen(e, eL) - 1; i >= 0; --i) {
    mont_mul(c, acc, acc, acc);
    if (bn_bit(e, i)) mont_mul(c, acc, acc, a);
  }
  memcpy(r, acc, sizeof(uint32_t) * c->L);
}
/* Fermat inverse mod a prime (Montgomery form in and out). */
static void mont_inv(const mont* c, uint32_t* r, const uint32_t* a) {
  uint32_t e[MAXL], two[MAXL] = {2};
  bn_sub(e, c->m, two, c->L);
  mont_pow(c, r, a, e, c->L);
}

/* ======================================================================= */
/* RSA: crypto/rsa VerifyPKCS1v15 and VerifyPSS(opts=nil)  [R12-R17]        */
/* ======================================================================= */
static const uint8_t DI256[] = {0x30,0x31,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x01,0x05,0x00,0x04,0x20};
static const uint8_t DI384[] = {0x30,0x41,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x02,0x05,0x00,0x04,0x30};
static const uint8_t DI512[] = {0x30,0x51,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x03,0x05,0x00,0x04,0x40};

/* rsa "encrypt" (public op) as crypto/rsa does it for verification:
 * checkPub [R12], sig must be < N [R14 (Go >= 1.20)]; em is k bytes. */
static int rsa_public(const uint8_t* nb, size_t nlen, uint64_t e, const uint8_t* sig, size_t slen,
                      uint8_t* em, size_t* k_out) {
  while (nlen > 0 && nb[0] == 0) { ++nb; --nlen; }
  if (nlen == 0 || !(nb[nlen - 1] & 1)) return -1;   /* even / empty modulus: unusable */
  if (e < 2 || e > 0x7fffffffULL) return -1;           /* checkPub: E < 2, E > 1<<31-1 */
  int L = (int)((nlen + 3) / 4);
  if (L > MAXL - 1) return -1;
  uint32_t n[MAXL], s[MAXL], x[MAXL], r[MAXL];
  bn_from_be(n, L, nb, nlen);
  size_t k = (size_t)(bn_bitlen(n, L) + 7) / 8;
  *k_out = k;
  if (slen != k) return -1;
  bn_from_be(s, L, sig, slen);
  if (bn_cmp(s, n, L) >= 0) return -1;                 /* sig >= N rejected */
  mont c;
  mont_init(&c, n, L);
  to_mont(&c, x, s);
  uint32_t el[2] = {(uint32_t)e, (uint32_t)(e >> 32)};
  mont_pow(&c, r, x, el, 2);
  from_mont(&c, x, r);
  bn_to_be(em, k, x, L);
  return 0;
}

int or_rsa_public(const uint8_t* n, size_t nlen, uint64_t e, const uint8_t* sig, size_t slen,
                  uint8_t* out) {
  size_t k;
  return rsa_public(n, nlen, e, sig, slen, out, &k);
}

static int pkcs1v15_verify(int hbits, const uint8_t* n, size_t nlen, uint64_t e,
                           const uint8_t* hashed, const uint8_t* sig, size_t slen) {
  const uint8_t* prefix = hbits == 256 ? DI256 : hbits == 384 ? DI384 : DI512;
  size_t hlen = (size_t)hash_len(hbits), tlen = 19 + hlen, k;
  uint8_t em[MAXL * 4];
  if (rsa_public(n, nlen, e, sig, slen, em, &k) != 0) return 0;
  if (k < tlen + 11) return 0;
  int ok = em[0] == 0 && em[1] == 1;
  ok &= memcmp(em + k - hlen, hashed, hlen) == 0;
  ok &= memcmp(em + k - tlen, prefix, 19) == 0;
  ok &= em[k - tlen - 1] == 0;
  for (size_t i = 2; i < k - tlen - 1; ++i) ok &= em[i] == 0xff;
  return ok;
}

static void mgf1_xor(int hbits, uint8_t* out, size_t olen, const uint8_t* seed, size_t slen) {
  uint8_t buf[64 + 4], d[64];
  memcpy(buf, seed, slen);
  size_t hl = (size_t)hash_len(hbits), done = 0;
  for (uint32_t ctr = 0; done < olen; ++ctr) {
    buf[slen] = ctr >> 24; buf[slen + 1] = ctr >> 16; buf[slen + 2] = ctr >> 8; buf[slen + 3] = ctr;
    hash_any(hbits, buf, slen + 4, d);
    for (size_t i = 0; i < hl && done < olen; ++i) out[done++] ^= d[i];
  }
}

static int pss_verify(int hbits, const uint8_t* n, size_t nlen, uint64_t e,
                      const uint8_t* mhash, const uint8_t* sig, size_t slen) {
  uint8_t emk[MAXL * 4];
  size_t k;
  if (rsa_public(n, nlen, e, sig, slen, emk, &k) != 0) return 0;
  while (nlen > 0 && n[0] == 0) { ++n; --nlen; }
  uint32_t nn[MAXL];
  int L = (int)((nlen + 3) / 4);
  bn_from_be(nn, L, n, nlen);
  int embits = bn_bitlen(nn, L) - 1;
  size_t emlen = (size_t)(embits + 7) / 8;
  uint8_t* em = emk;
  size_t have = k;
  while (have > emlen) {                               /* strip leading zero bytes */
    if (em[0] != 0) return 0;
    ++em; --have;
  }
  size_t hlen = (size_t)hash_len(hbits);
  /* emsaPSSVerify with sLen = PSSSaltLengthAuto */
  if (emlen < hlen + 2) return 0;                      /* emLen < hLen + sLen(-1) + 2 + ... */
  if (em[emlen - 1] != 0xbc) return 0;
  size_t dblen = emlen - hlen - 1;
  uint8_t db[MAXL * 4];
  memcpy(db, em, dblen);
  const uint8_t* h = em + dblen;
  uint8_t bitmask = (uint8_t)(0xff >> (8 * emlen - (size_t)embits));
  if (em[0] & ~bitmask) return 0;
  mgf1_xor(hbits, db, dblen, h, hlen);
  db[0] &= bitmask;
  size_t ps = 0;                                       /* bytes.IndexByte(db, 0x01) */
  while (ps < dblen && db[ps] != 0x01) ++ps;
  if (ps == dblen) return 0;
  for (size_t i = 0; i < ps; ++i) if (db[i] != 0) return 0;
  size_t slen_salt = dblen - ps - 1;
  uint8_t mp[8 + 64 + MAXL * 4];
  memset(mp, 0, 8);
  memcpy(mp + 8, mhash, hlen);
  memcpy(mp + 8 + hlen, db + dblen - slen_salt, slen_salt);
  uint8_t h2[64];
  hash_any(hbits, mp, 8 + hlen + slen_salt, h2);
  return memcmp(h2, h, hlen) == 0;
}

static int alg_hbits(int alg) {
  switch (alg) {
    case OR_RS256: case OR_PS256: case OR_ES256: return 256;
    case OR_RS384: case OR_PS384: case OR_ES384: return 384;
    default: return 512;
  }
}

int or_rsa_verify(int alg, const uint8_t* n, size_t nlen, uint64_t e,
                  const uint8_t* msg, size_t mlen, const uint8_t* sig, size_t slen) {
  if (alg < OR_RS256 || alg > OR_PS512) return 0;     /* R10: RSA key verifies RS / PS only */
  int hb = alg_hbits(alg);
  uint8_t d[64];
  hash_any(hb, msg, mlen, d);
  if (alg <= OR_RS512) return pkcs1v15_verify(hb, n, nlen, e, d, sig, slen);
  return pss_verify(hb, n, nlen, e, d, sig, slen);
}

/* ======================================================================= */
/* short-Weierstrass curves, a = -3 (crypto/elliptic params)               */
/* ======================================================================= */
typedef struct {
  int L, bytes;
  mont fp, fn;
  uint32_t a_m[MAXL], b_m[MAXL];                      /* a = -3 and b, Montgomery form */
  uint32_t gx[MAXL], gy[MAXL];                        /* generator, Montgomery form */
  uint32_t n[MAXL];
} curve;

static const char* CURVE_HEX[4][5] = {
  {0},
  {"ffffffff00000001000000000000000000000000ffffffffffffffffffffffff",
   "ffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551",
   "5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b",
   "6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296",
   "4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5"},
  {"fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffeffffffff0000000000000000ffffffff",
   "ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973",
   "b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef",
   "aa87ca22be8b05378eb1c71ef320ad746e1d3b628ba79b9859f741e082542a385502f25dbf55296c3a545e3872760ab7",
   "3617de4a96262c6f5d9e98bf9292dc29f8f41dbd289a147ce9da3113b5f0b8c00a60b1ce1d7e819d7a431d7c90ea0e5f"},
  {"01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
   "01fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409",
   "0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf073573df883d2c34f1ef451fd46b503f00",
   "00c6858e06b70404e9cd9e3ecb662395b4429c648139053fb521f828af606b4d3dbaa14b5e77efe75928fe1dc127a2ffa8de3348b3c1856a429bf97e7e31c2e5bd66",
   "011839296a789a3bc0045c8a5fb42c7d1bd998f54449579b446817afbd17273e662c97ee72995ef42640c550b9013fad0761353c7086a272c24088be94769fd16650"}};

static void hex_to_bn(uint32_t* r, int L, const char* h) {
  uint8_t b[MAXL * 4];
  size_t n = strlen(h) / 2;
  for (size_t i = 0; i < n; ++i) {
    unsigned v; char t[3] = {h[2*i], h[2*i+1], 0};
    v = (unsigned)strtoul(t, NULL, 16); b[i] = (uint8_t)v;
  }
  bn_from_be(r, L, b, n);
}

static void curve_init(curve* cv, int id) {
  cv->L = id == OR_P256 ? 8 : id == OR_P384 ? 12 : 17;
  cv->bytes = id == OR_P256 ? 32 : id == OR_P384 ? 48 : 66;
  uint32_t p[MAXL], t[MAXL], three[MAXL] = {3};
  hex_to_bn(p, cv->L, CURVE_HEX[id][0]);
  hex_to_bn(cv->n, cv->L, CURVE_HEX[id][1]);
  mont_init(&cv->fp, p, cv->L);
  mont_init(&cv->fn, cv->n, cv->L);
  hex_to_bn(t, cv->L, CURVE_HEX[id][2]); to_mont(&cv->fp, cv->b_m, t);
  bn_sub(t, p, three, cv->L); to_mont(&cv->fp, cv->a_m, t);
  hex_to_bn(t, cv->L, CURVE_HEX[id][3]); to_mont(&cv->fp, cv->gx, t);
  hex_to_bn(t, cv->L, CURVE_HEX[id][4]); to_mont(&cv->fp, cv->gy, t);
}

static curve g_curves[4];
static pthread_once_t g_curve_once = PTHREAD_ONCE_INIT;
static void init_all_curves(void) { for (int i = 1; i <= 3; ++i) curve_init(&g_curves[i], i); }

/* Jacobian point; Z = 0 is the point at infinity. */
typedef struct { uint32_t X[MAXL], Y[MAXL], Z[MAXL]; } jpt;

static void jdbl(const curve* cv, jpt* r, const jpt* p) {
  const mont* F = &cv->fp; int L = cv->L;
  if (bn_is_zero(p->Z, L) || bn_is_zero(p->Y, L)) { memset(r, 0, sizeof *r); return; }
  uint32_t zz[MAXL], yy[MAXL], t1[MAXL], t2[MAXL], m[MAXL], s[MAXL], x3[MAXL], y3[MAXL], z3[MAXL];
  mont_mul(F, zz, p->Z, p->Z);
  mont_mul(F, yy, p->Y, p->Y);
  mod_sub(F, t1, p->X, zz); mod_add(F, t2, p->X, zz);
  mont_mul(F, m, t1, t2); mod_add(F, t1, m, m); mod_add(F, m, t1, m);   /* M = 3(X-Z^2)(X+Z^2) */
  mont_mul(F, s, p->X, yy); mod_add(F, s, s, s); mod_add(F, s, s, s);   /* S = 4XY^2 */
  mont_mul(F, x3, m, m); mod_sub(F, x3, x3, s); mod_sub(F, x3, x3, s);  /* X3 = M^2 - 2S */
  mont_mul(F, t1, yy, yy); mod_add(F, t1, t1, t1); mod_add(F, t1, t1, t1); mod_add(F, t1, t1, t1); /* 8Y^4 */
  mod_sub(F, t2, s, x3); mont_mul(F, y3, m, t2); mod_sub(F, y3, y3, t1);
  mont_mul(F, z3, p->Y, p->Z); mod_add(F, z3, z3, z3);
  memcpy(r->X, x3, sizeof x3); memcpy(r->Y, y3, sizeof y3); memcpy(r->Z, z3, sizeof z3);
}

static void jadd(const curve* cv, jpt* r, const jpt* p, const jpt* q) {
  const mont* F = &cv->fp; int L = cv->L;
  if (bn_is_zero(p->Z, L)) { *r = *q; return; }
  if (bn_is_zero(q->Z, L)) { *r = *p; return; }
  uint32_t z1z1[MAXL], z2z2[MAXL], u1[MAXL], u2[MAXL], s1[MAXL], s2[MAXL], h[MAXL], rr[MAXL];
  uint32_t hh[MAXL], hhh[MAXL], v[MAXL], t[MAXL], x3[MAXL], y3[MAXL], z3[MAXL];
  mont_mul(F, z1z1, p->Z, p->Z); mont_mul(F, z2z2, q->Z, q->Z);
  mont_mul(F, u1, p->X, z2z2); mont_mul(F, u2, q->X, z1z1);
  mont_mul(F, t, q->Z, z2z2); mont_mul(F, s1, p->Y, t);
  mont_mul(F, t, p->Z, z1z1); mont_mul(F, s2, q->Y, t);
  mod_sub(F, h, u2, u1); mod_sub(F, rr, s2, s1);
  if (bn_is_zero(h, L)) {
    if (bn_is_zero(rr, L)) { jdbl(cv, r, p); return; }   /* P == Q */
    memset(r, 0, sizeof *r); return;                     /* P == -Q */
  }
  mont_mul(F, hh, h, h); mont_mul(F, hhh, hh, h); mont_mul(F, v, u1, hh);
  mont_mul(F, x3, rr, rr); mod_sub(F, x3, x3, hhh); mod_sub(F, x3, x3, v); mod_sub(F, x3, x3, v);
  mod_sub(F, t, v, x3); mont_mul(F, y3, rr, t); mont_mul(F, t, s1, hhh); mod_sub(F, y3, y3, t);
  mont_mul(F, t, p->Z, q->Z); mont_mul(F, z3, t, h);
  memcpy(r->X, x3, sizeof x3); memcpy(r->Y, y3, sizeof y3); memcpy(r->Z, z3, sizeof z3);
}

/* y^2 == x^3 - 3x + b, coordinates < p (crypto/elliptic IsOnCurve / nistec SetBytes) */
static int ec_on_curve(const curve* cv, const uint32_t* x, const uint32_t* y) {
  const mont* F = &cv->fp; int L = cv->L;
  if (bn_cmp(x, F->m, L) >= 0 || bn_cmp(y, F->m, L) >= 0) return 0;
  uint32_t xm[MAXL], ym[MAXL], l[MAXL], r[MAXL], t[MAXL];
  to_mont(F, xm, x); to_mont(F, ym, y);
  mont_mul(F, l, ym, ym);
  mont_mul(F, t, xm, xm); mod_add(F, t, t, cv->a_m); mont_mul(F, r, t, xm); mod_add(F, r, r, cv->b_m);
  return bn_cmp(l, r, L) == 0;
}

int or_ec_point_valid(int curve_id, const uint8_t* xb, const uint8_t* yb, size_t coord_len) {
  pthread_once(&g_curve_once, init_all_curves);
  if (curve_id < 1 || curve_id > 3) return 0;
  const curve* cv = &g_curves[curve_id];
  if (coord_len != (size_t)cv->bytes) return 0;
  uint32_t x[MAXL], y[MAXL];
  bn_from_be(x, cv->L + 1, xb, coord_len); bn_from_be(y, cv->L + 1, yb, coord_len);
  if (x[cv->L] || y[cv->L]) return 0;
  return ec_on_curve(cv, x, y);
}

int or_ecdsa_verify(int alg, int curve_id, const uint8_t* xb, const uint8_t* yb, size_t coord_len,
                    const uint8_t* msg, size_t mlen, const uint8_t* sig, size_t slen) {
  pthread_once(&g_curve_once, init_all_curves);
  if (alg < OR_ES256 || alg > OR_ES512) return 0;     /* R10: EC key verifies ES* only */
  if (curve_id < 1 || curve_id > 3) return 0;
  const curve* cv = &g_curves[curve_id];
  int L = cv->L;
  size_t ks = alg == OR_ES256 ? 32 : alg == OR_ES384 ? 48 : 66;   /* R18: size from the alg */
  if (slen != 2 * ks) return 0;
  if (!or_ec_point_valid(curve_id, xb, yb, coord_len)) return 0;
  /* r, s as big-endian integers of ks bytes; must be in [1, N-1]  [R20] */
  uint32_t r[MAXL], s[MAXL], tmp[MAXL];
  int LL = (int)((ks + 3) / 4) > L ? (int)((ks + 3) / 4) : L;
  bn_from_be(tmp, LL, sig, ks);
  for (int i = L; i < LL; ++i) if (tmp[i]) return 0;
  memcpy(r, tmp, sizeof(uint32_t) * L);
  bn_from_be(tmp, LL, sig + ks, ks);
  for (int i = L; i < LL; ++i) if (tmp[i]) return 0;
  memcpy(s, tmp, sizeof(uint32_t) * L);
  if (bn_is_zero(r, L) || bn_is_zero(s, L)) return 0;
  if (bn_cmp(r, cv->n, L) >= 0 || bn_cmp(s, cv->n, L) >= 0) return 0;
  /* e = hashToInt(H(msg))  [R21] */
  uint8_t h[64];
  int hb = alg_hbits(alg);
  hash_any(hb, msg, mlen, h);
  size_t hl = (size_t)hash_len(hb);
  int obits = bn_bitlen(cv->n, L);
  size_t obytes = (size_t)(obits + 7) / 8;
  if (hl > obytes) hl = obytes;
  uint32_t e[MAXL];
  bn_from_be(e, L, h, hl);
  int excess = (int)hl * 8 - obits;
  if (excess > 0) {                                   /* right shift by excess bits */
    for (int i = 0; i < L; ++i)
      e[i] = (e[i] >> excess) | (i + 1 < L ? e[i + 1] << (32 - excess) : 0);
  }
  if (bn_cmp(e, cv->n, L) >= 0) bn_sub(e, e, cv->n, L);
  /* w = s^-1, u1 = e w, u2 = r w (mod N)  [R22] */
  const mont* Fn = &cv->fn;
  uint32_t sm[MAXL], wm[MAXL], em[MAXL], rm[MAXL], u1[MAXL], u2[MAXL];
  to_mont(Fn, sm, s); mont_inv(Fn, wm, sm);
  to_mont(Fn, em, e); to_mont(Fn, rm, r);
  mont_mul(Fn, tmp, em, wm); from_mont(Fn, u1, tmp);
  mont_mul(Fn, tmp, rm, wm); from_mont(Fn, u2, tmp);
  /* X = u1 G + u2 Q (joint double-and-add) */
  jpt G, Q, GQ, acc;
  memcpy(G.X, cv->gx, sizeof G.X); memcpy(G.Y, cv->gy, sizeof G.Y); memcpy(G.Z, cv->fp.one, sizeof G.Z);
  uint32_t qx[MAXL], qy[MAXL];
  bn_from_be(qx, L, xb, coord_len); bn_from_be(qy, L, yb, coord_len);
  to_mont(&cv->fp, Q.X, qx); to_mont(&cv->fp, Q.Y, qy); memcpy(Q.Z, cv->fp.one, sizeof Q.Z);
  jadd(cv, &GQ, &G, &Q);
  memset(&acc, 0, sizeof acc);
  int top = bn_bitlen(cv->n, L);
  for (int i = top - 1; i >= 0; --i) {
    jdbl(cv, &acc, &acc);
    int b1 = bn_bit(u1, i), b2 = bn_bit(u2, i);
    if (b1 && b2) jadd(cv, &acc, &acc, &GQ);
    else if (b1) jadd(cv, &acc, &acc, &G);
    else if (b2) jadd(cv, &acc, &acc, &Q);
  }
  if (bn_is_zero(acc.Z, L)) return 0;                 /* point at infinity */
  const mont* F = &cv->fp;
  uint32_t zi[MAXL], zi2[MAXL], xa[MAXL];
  mont_inv(F, zi, acc.Z); mont_mul(F, zi2, zi, zi);
  mont_mul(F, tmp, acc.X, zi2); from_mont(F, xa, tmp);
  /* x mod N == r  (x < p; p < 2N for these curves, so one subtraction) */
  while (bn_cmp(xa, cv->n, L) >= 0) bn_sub(xa, xa, cv->n, L);
  return bn_cmp(xa, r, L) == 0;
}

/* ======================================================================= */
/* Ed25519: crypto/ed25519.Verify (filippo.io/edwards25519 semantics)       */
/* ======================================================================= */
typedef struct { uint32_t X[8], Y[8], Z[8], T[8]; } ept;   /* Montgomery-form coords */
static int ed_decode_y(ept* P, const uint32_t* ym, int sign);
static mont g_fp25519, g_fl25519;
static uint32_t g_ed_d2[8], g_ed_d[8], g_sqrtm1[8];
static ept g_edB;
static pthread_once_t g_ed_once = PTHREAD_ONCE_INIT;

static void ed_add(ept* r, const ept* p, const ept* q) {       /* add-2008-hwcd-3, complete */
  const mont* F = &g_fp25519;
  uint32_t a[8], b[8], c[8], d[8], t1[8], t2[8], e[8], f[8], g[8], h[8];
  mod_sub(F, t1, p->Y, p->X); mod_sub(F, t2, q->Y, q->X); mont_mul(F, a, t1, t2);
  mod_add(F, t1, p->Y, p->X); mod_add(F, t2, q->Y, q->X); mont_mul(F, b, t1, t2);
  mont_mul(F, t1, p->T, g_ed_d2); mont_mul(F, c, t1, q->T);
  mont_mul(F, t1, p->Z, q->Z); mod_add(F, d, t1, t1);
  mod_sub(F, e, b, a); mod_sub(F, f, d, c); mod_add(F, g, d, c); mod_add(F, h, b, a);
  mont_mul(F, r->X, e, f); mont_mul(F, r->Y, g, h); mont_mul(F, r->Z, f, g); mont_mul(F, r->T, e, h);
}

static void ed_init(void) {
  uint32_t p[8], l[8], t[8], u[8];
  hex_to_bn(p, 8, "7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffed");
  hex_to_bn(l, 8, "1000000000000000000000000000000014def9dea2f79cd65812631a5cf5d3ed");
  mont_init(&g_fp25519, p, 8);
  mont_init(&g_fl25519, l, 8);
  const mont* F = &g_fp25519;
  /* d = -121665/121666 */
  uint32_t n1[8] = {121665}, n2[8] = {121666}, zero[8] = {0};
  to_mont(F, t, n1); to_mont(F, u, n2); mont_inv(F, u, u); mont_mul(F, t, t, u);
  mod_sub(F, g_ed_d, zero, t);
  mod_add(F, g_ed_d2, g_ed_d, g_ed_d);
  /* sqrt(-1) = 2^((p-1)/4) */
  uint32_t two[8] = {2}, e[8];
  memcpy(e, p, sizeof e); bn_sub(e, e, (uint32_t[8]){1}, 8);
  for (int i = 0; i < 8; ++i) e[i] = (e[i] >> 2) | (i < 7 ? e[i + 1] << 30 : 0);
  to_mont(F, t, two); mont_pow(F, g_sqrtm1, t, e, 8);
  /* B: y = 4/5, x even */
  uint32_t four[8] = {4}, five[8] = {5}, y[8];
  to_mont(F, t, four); to_mont(F, u, five); mont_inv(F, u, u); mont_mul(F, y, t, u);
  ed_decode_y(&g_edB, y, 0);
}

/* x from y (Montgomery form), per RFC 8032 5.1.3 / edwards25519 SetBytes. */
static int ed_decode_y(ept* P, const uint32_t* ym, int sign) {
  const mont* F = &g_fp25519;
  uint32_t yy[8], u[8], v[8], vinv[8], xx[8], x[8], chk[8], e[8], zero[8] = {0};
  mont_mul(F, yy, ym, ym);
  mod_sub(F, u, yy, F->one);                           /* u = y^2 - 1 */
  mont_mul(F, v, yy, g_ed_d); mod_add(F, v, v, F->one); /* v = d y^2 + 1 */
  mont_inv(F, vinv, v); mont_mul(F, xx, u, vinv);      /* x^2 = u / v */
  /* candidate x = xx^((p+3)/8) */
  memcpy(e, F->m, sizeof e); bn_add(e, e, (uint32_t[8]){3}, 8);
  for (int i = 0; i < 8; ++i) e[i] = (e[i] >> 3) | (i < 7 ? e[i + 1] << 29 : 0);
  mont_pow(F, x, xx, e, 8);
  mont_mul(F, chk, x, x);
  if (bn_cmp(chk, xx, 8) != 0) {
    mont_mul(F, x, x, g_sqrtm1);
    mont_mul(F, chk, x, x);
    if (bn_cmp(chk, xx, 8) != 0) return 0;             /* not a square: invalid point */
  }
  uint32_t xn[8];
  from_mont(F, xn, x);
  if ((xn[0] & 1) != (uint32_t)sign) mod_sub(F, x, zero, x);   /* x = -x (0 stays 0) */
  memcpy(P->X, x, sizeof x); memcpy(P->Y, ym, 32); memcpy(P->Z, F->one, 32);
  mont_mul(F, P->T, x, ym);
  return 1;
}

static void ed_encode(uint8_t out[32], const ept* P) {
  const mont* F = &g_fp25519;
  uint32_t zi[8], x[8], y[8], t[8];
  mont_inv(F, zi, P->Z);
  mont_mul(F, t, P->X, zi); from_mont(F, x, t);
  mont_mul(F, t, P->Y, zi); from_mont(F, y, t);
  for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(y[i / 4] >> (8 * (i % 4)));
  out[31] |= (uint8_t)((x[0] & 1) << 7);
}

static void ed_scalarmul(ept* r, const uint32_t* k, const ept* P) {
  const mont* F = &g_fp25519;
  ept acc;
  memset(&acc, 0, sizeof acc);
  memcpy(acc.Y, F->one, 32); memcpy(acc.Z, F->one, 32);
  for (int i = 255; i >= 0; --i) {
    ed_add(&acc, &acc, &acc);
    if (bn_bit(k, i)) ed_add(&acc, &acc, P);
  }
  *r = acc;
}

int or_ed25519_verify(const uint8_t pub[32], const uint8_t* msg, size_t mlen,
                      const uint8_t* sig, size_t slen) {
  pthread_once(&g_ed_once, ed_init);
  const mont* F = &g_fp25519;
  if (slen != 64 || (sig[63] & 0xE0)) return 0;        /* R23/R25 */
  /* A = SetBytes(pub): y = low 255 bits (non-canonical accepted, reduced mod p) [R24] */
  uint32_t y[9] = {0}, yr[8], ym[8];
  for (int i = 0; i < 32; ++i) y[i / 4] |= (uint32_t)pub[i] << (8 * (i % 4));
  int sign = y[7] >> 31; y[7] &= 0x7fffffff;
  bn_mod(yr, y, 8, F->m, 8);
  to_mont(F, ym, yr);
  ept A;
  if (!ed_decode_y(&A, ym, sign)) return 0;
  /* s canonical (< L) [R25] */
  uint32_t s[8];
  for (int i = 0; i < 8; ++i) s[i] = 0;
  for (int i = 0; i < 32; ++i) s[i / 4] |= (uint32_t)sig[32 + i] << (8 * (i % 4));
  if (bn_cmp(s, g_fl25519.m, 8) >= 0) return 0;
  /* k = SHA-512(R || A || M) mod L, A = the original 32 public-key bytes */
  uint8_t* buf = (uint8_t*)malloc(64 + mlen);
  memcpy(buf, sig, 32); memcpy(buf + 32, pub, 32); memcpy(buf + 64, msg, mlen);
  uint8_t h[64];
  or_sha512(buf, 64 + mlen, h);
  free(buf);
  uint32_t hl[16], k[8];
  for (int i = 0; i < 16; ++i) hl[i] = 0;
  for (int i = 0; i < 64; ++i) hl[i / 4] |= (uint32_t)h[i] << (8 * (i % 4));
  bn_mod(k, hl, 16, g_fl25519.m, 8);
  /* R' = [s]B - [k]A  (cofactorless)  [R26] */
  ept sB, kA, negkA, Rp;
  ed_scalarmul(&sB, s, &g_edB);
  ed_scalarmul(&kA, k, &A);
  uint32_t zero[8] = {0};
  negkA = kA;
  mod_sub(F, negkA.X, zero, kA.X); mod_sub(F, negkA.T, zero, kA.T);
  ed_add(&Rp, &sB, &negkA);
  uint8_t enc[32];
  ed_encode(enc, &Rp);
  return memcmp(enc, sig, 32) == 0;                    /* byte compare: non-canonical R rejects */
}

/* ======================================================================= */
/* multithreaded batch (bench CPU leg)                                      */
/* ======================================================================= */
typedef struct { const or_job* jobs; size_t count; uint8_t* out; size_t next; pthread_mutex_t mu; } pool;

static int run_job(const or_job* j) {
  if (j->key_kind == 0) return or_rsa_verify(j->alg, j->n, j->nlen, j->e, j->msg, j->mlen, j->sig, j->slen);
  if (j->key_kind == 1) return or_ecdsa_verify(j->alg, j->curve, j->x, j->y, j->coord_len, j->msg, j->mlen, j->sig, j->slen);
  if (j->alg != OR_EDDSA) return 0;
  return or_ed25519_verify(j->x, j->msg, j->mlen, j->sig, j->slen);
}

static void* worker(void* arg) {
  pool* p = (pool*)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    size_t i = p->next; p->next += 64;
    pthread_mutex_unlock(&p->mu);
    if (i >= p->count) return NULL;
    size_t e = i + 64 < p->count ? i + 64 : p->count;
    for (; i < e; ++i) p->out[i] = (uint8_t)run_job(&p->jobs[i]);
  }
}

void or_verify_many(const or_job* jobs, size_t count, int threads, uint8_t* verdicts) {
  pthread_once(&g_curve_once, init_all_curves);
  pthread_once(&g_ed_once, ed_init);
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pool p = {jobs, count, verdicts, 0, PTHREAD_MUTEX_INITIALIZER};
  pthread_t th[256];
  for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, &p);
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
}
