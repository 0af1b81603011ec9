// fe25519.hpp -- GF(2^255 - 19) in radix 2^25.5 for the Ed25519 point loop
// (k_ed_point's Niels additions; ed25519.hip).
//
// Ten unsigned limbs of alternating 26 and 25 bits: limb i sits at bit
// s_i = ceil(25.5 i), so s_i + s_j = s_(i+j) except for two odd indices
// (+1 bit: the product doubles) and 2^(s_10) = 2^255 = 19 mod p (a column
// past the top wraps with a factor 19).  A product is therefore 100 partial
// products (v_mad_u64_u32 into ten 64-bit columns; the factor 2 rides on the
// odd limbs of one operand, the factor 19 on the other operand's limbs) and ONE
// carry chain with a 19-fold -- no reduction rows at all, where the Montgomery
// form of mp.hpp spends 2 signed MADs, a digit computation and a 64-bit carry
// per row (ED25519P: ~200 VALU per product, this form ~160).
//
// Bounds (checked exhaustively by tools/fe25519_bounds.py, which the CPU
// suite runs):
//   "normalized" (mul output): limbs < 2^w_i, limb 1 < 2^25 + 2^13;
//   add(a, b)   : limbs add;
//   sub(a, b)   : a + 2p - b limb by limb (2p's limbs are >= any normalized
//                 or canonical limb, so no limb goes negative);
//   mul(f, g)   : every 64-bit column must stay below 2^64 and 19 g_j below
//                 2^32 -- the Niels addition's operands (at most ~4x a
//                 normalized limb on the f side, ~3x on the g side) fit, with
//                 the g side the smaller operand.
// Canonical values (table entries, encodings) are fully reduced: [0, p).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#define FE_D __device__ __forceinline__

namespace fe {

constexpr int L = 10;
constexpr int wid(int i) { return (i & 1) ? 25 : 26; }
constexpr int off(int i) { return (51 * i + 1) / 2; }          // s_i = ceil(25.5 i)
constexpr uint32_t lmask(int i) { return (1u << wid(i)) - 1u; }
// limbs of 2p = 2^256 - 38: every one >= the largest normalized / canonical limb
constexpr uint32_t p2(int i) { return i == 0 ? (1u << 27) - 38u : (1u << (wid(i) + 1)) - 2u; }

FE_D void add(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = a[i] + b[i];
}
FE_D void sub(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = a[i] + p2(i) - b[i];
}
// r = 2 a + b and r = 2 a - b (+ 2p): one v_lshl_add per limb for the doubling
FE_D void add_dbl(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = (a[i] << 1) + b[i];
}
FE_D void sub_dbl(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = (a[i] << 1) + p2(i) - b[i];
}
FE_D void neg(uint32_t* r, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = p2(i) - b[i];
}
FE_D void copy(uint32_t* r, const uint32_t* a) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = a[i];
}
FE_D void set_small(uint32_t* r, uint32_t v) {
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = i == 0 ? v : 0u;
}

// 19 x (two full-rate adds: v_mul_lo_u32 is a quarter-rate instruction)
FE_D uint32_t x19(uint32_t g) { return (g << 4) + (g << 1) + g; }

// The operand forms of a product: g19_j = 19 g_j (j >= 1; the columns past
// the top), f2_i = 2 f_i (odd i; the odd x odd products).  An operand used by
// several products (the Niels addition's E, F, G, H) is prepared once.
FE_D void pre_g(uint32_t* g19, const uint32_t* g) {
#pragma unroll
  for (int j = 1; j < L; ++j) g19[j] = x19(g[j]);
}
FE_D void pre_f(uint32_t* f2, const uint32_t* f) {
#pragma unroll
  for (int i = 1; i < L; i += 2) f2[i] = f[i] << 1;
}

// r = f g mod p, normalized, from prepared operands.  Product scanning: column
// k is summed in full, starting from the carry out of column k - 1 (the first
// v_mad_u64_u32 of a column takes the carry as its addend, so a carry costs
// one 64-bit shift and one mask -- no 64-bit add).  Column values, and so the
// output, are bit-identical to summing every column first and carrying after
// (tools/fe25519_bounds.py model_mul).
// One product column as ONE asm statement: ten v_mad_u64_u32 in a chain whose
// first addend is the carry in; the limb is the column's low bits (one mask),
// the carry out its high part (one 64-bit shift).  Written as asm because LLVM reassociates a C++ sum so that the carry
// is added last, with a separate 64-bit add per column; one statement per
// column also keeps the hazard padding after inline asm to one s_nop.
#define FE_COL_TAIL                                                                                  \
  "v_mad_u64_u32 %[c], s[94:95], %[a1], %[b1], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[92:93], %[a2], %[b2], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[94:95], %[a3], %[b3], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[92:93], %[a4], %[b4], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[94:95], %[a5], %[b5], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[92:93], %[a6], %[b6], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[94:95], %[a7], %[b7], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[92:93], %[a8], %[b8], %[c]\n\t"                                            \
  "v_mad_u64_u32 %[c], s[94:95], %[a9], %[b9], %[c]"
#define FE_COL_IN                                                                                    \
  [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [a4] "v"(a[4]), [a5] "v"(a[5]),      \
      [a6] "v"(a[6]), [a7] "v"(a[7]), [a8] "v"(a[8]), [a9] "v"(a[9]), [b0] "v"(b[0]), [b1] "v"(b[1]),  \
      [b2] "v"(b[2]), [b3] "v"(b[3]), [b4] "v"(b[4]), [b5] "v"(b[5]), [b6] "v"(b[6]), [b7] "v"(b[7]),  \
      [b8] "v"(b[8]), [b9] "v"(b[9])
// column sum into c (in place: c enters as the carry in, leaves as the column)
template <bool FIRST>
FE_D void column(uint64_t& c, const uint32_t (&a)[L], const uint32_t (&b)[L]) {
  if constexpr (FIRST) {
    // column 0 has no carry in: its first addend is the literal 0 (no register to clear)
    asm("v_mad_u64_u32 %[c], s[92:93], %[a0], %[b0], 0\n\t" FE_COL_TAIL
        : [c] "=&v"(c)
        : FE_COL_IN
        : "s92", "s93", "s94", "s95");
  } else {
    asm("v_mad_u64_u32 %[c], s[92:93], %[a0], %[b0], %[c]\n\t" FE_COL_TAIL
        : [c] "+v"(c)
        : FE_COL_IN
        : "s92", "s93", "s94", "s95");
  }
}
#undef FE_COL_TAIL
#undef FE_COL_IN

#ifndef JG_FE_ASM
#define JG_FE_ASM 1
#endif
FE_D void mul_pre(uint32_t* r, const uint32_t* f, const uint32_t* f2, const uint32_t* g, const uint32_t* g19) {
#if !JG_FE_ASM
  // (A/B: the C++ form, which LLVM schedules as operand-scanning columns + a carry chain)
  uint64_t h[L];
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint32_t a = ((i & 1) && (j & 1)) ? f2[i] : f[i];
      const uint32_t b = (i + j >= L) ? g19[j] : g[j];
      const int k = (i + j) % L;
      if (i == 0) h[k] = (uint64_t)a * b;
      else h[k] += (uint64_t)a * b;
    }
#pragma unroll
  for (int i = 0; i < L - 1; ++i) {
    h[i + 1] += h[i] >> wid(i);
    r[i] = (uint32_t)h[i] & lmask(i);
  }
  const uint64_t c = h[L - 1] >> 25;
  r[L - 1] = (uint32_t)h[L - 1] & lmask(L - 1);
#else
  uint64_t c;                     // column 0 writes it
#pragma unroll
  for (int k = 0; k < L; ++k) {
    uint32_t a[L], b[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int j = (k - i + L) % L;
      a[i] = ((i & 1) && (j & 1)) ? f2[i] : f[i];
      b[i] = (i > k) ? g19[j] : g[j];
    }
    if (k == 0) column<true>(c, a, b);
    else column<false>(c, a, b);
    r[k] = (uint32_t)c & lmask(k);
    c >>= wid(k);
  }
#endif
  // the carry out of limb 9 folded into limb 0 (x19), and one more step 0 -> 1
  const uint64_t t = (uint64_t)r[0] + c * 19ull;
  r[0] = (uint32_t)t & lmask(0);
  r[1] += (uint32_t)(t >> 26);
}

// r = f g mod p, normalized.  g is the operand whose limbs carry the factor 19
// (keep it the smaller one: 19 g_j < 2^32).
FE_D void mul(uint32_t* r, const uint32_t* f, const uint32_t* g) {
  uint32_t g19[L], f2[L];
  pre_g(g19, g);
  pre_f(f2, f);
  mul_pre(r, f, f2, g, g19);
}

// any value with limbs < 2^31 -> canonical [0, p)
FE_D void canon(uint32_t* r) {
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const uint32_t v = r[i] + c;
      r[i] = v & lmask(i);
      c = v >> wid(i);
    }
    r[0] += 19u * c;
  }
  // now limbs < 2^w_i except limb 0 < 2^26 + 19 * 2: one more carry step
  {
    const uint32_t c0 = r[0] >> 26;
    r[0] &= lmask(0);
    r[1] += c0;
  }
  // value < 2^255 + small; subtract p iff value + 19 >= 2^255
  uint32_t q = (r[0] + 19u) >> 26;
#pragma unroll
  for (int i = 1; i < L; ++i) q = (r[i] + q) >> wid(i);
  r[0] += 19u * q;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t v = r[i] + c;
    r[i] = v & lmask(i);
    c = v >> wid(i);
  }
  // c == q: the 2^255 carried out is dropped (value - p)
}

// 8 little-endian 32-bit words of a value < 2^255 -> limbs (canonical in, canonical out)
FE_D void from_words(uint32_t* r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int s = off(i), q = s / 32, b = s % 32;
    uint32_t v = w[q] >> b;
    if (b + wid(i) > 32 && q + 1 < 8) v |= w[q + 1] << (32 - b);
    r[i] = v & lmask(i);
  }
}

// canonical limbs -> 8 little-endian 32-bit words
FE_D void to_words(uint32_t* w, const uint32_t* r) {
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int s = off(i), q = s / 32, b = s % 32;
    w[q] |= r[i] << b;
    if (b + wid(i) > 32 && q + 1 < 8) w[q + 1] |= r[i] >> (32 - b);
  }
}

}  // namespace fe
