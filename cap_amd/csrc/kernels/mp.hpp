// mp.hpp -- fixed-modulus multi-precision arithmetic for the EC / Ed25519
// verify kernels on gfx950.
//
// Representation: L limbs of 28 bits held in 32-bit VGPRs ("lazy"): limbs may
// temporarily exceed 28 bits and values may exceed the modulus by a small
// multiple.  Products accumulate in 64-bit VGPR pairs with v_mad_u64_u32
// (one instruction per 28x28 partial product, no carry chains: on gfx950 a
// v_mad_u64_u32 issues at the rate of a plain add, profiles/r01_int_rates.json,
// so eliminating carry instructions halves the instruction count).
//
// Bounds (checked in tools/gen_field_consts.py, R = 2^(28L) > 4096 m):
//   mul/sqr inputs : limbs < 3*2^28, value(a)*value(b) < R*m
//   mul/sqr output : limbs < 2^28, value < 2m          ("normalized")
//   sub(a, b)      : b limbs < 2^28 and value(b) < 2m; result = a + KSUB - b,
//                    KSUB = 4m limb-padded so no limb goes negative
//   freduce        : any non-negative value < 2^(FOLD_S+32) -> normalized, < 2m
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "field_consts.hpp"
#include "mad.hpp"
#include "mad_blocks.hpp"
#include "col_chains.hpp"

#define MP_W 28
#define MP_MASK 0x0fffffffu
#define MPD __device__ __forceinline__
#ifndef JG_P384_COLS
#define JG_P384_COLS 1
#endif

namespace mp {

// Limb indices j of the reduction row's non-zero constants: m+1 (j >= 1) when
// m = -1 mod 2^28 (NP1), else m.  One reduction row = one mad_blocks.hpp asm
// statement per 8 of them (the constants are wave-uniform SGPR operands).
struct NzIdx {
  int n;
  int j[32];
};
template <class F>
constexpr uint32_t red_const(int j) { return F::NP1 ? (j == 0 ? 0u : F::M1[j]) : F::M[j]; }
template <class F>
constexpr NzIdx red_idx() {
  NzIdx r{0, {}};
  for (int j = 0; j < F::L; ++j)
    if (red_const<F>(j) != 0) r.j[r.n++] = j;
  return r;
}

// t[j] += q * c_j over the non-zero reduction constants, from the S-th on
template <class F, int S>
MPD void red_row(uint64_t* t, uint32_t q) {
  constexpr NzIdx z = red_idx<F>();
  constexpr int n = z.n - S;
#define RJ(k) z.j[S + (k)]
#define RT(k) t[RJ(k)]
#define RC(k) red_const<F>(RJ(k))
  if constexpr (n >= 8) {
    mb::mads8(RT(0), RT(1), RT(2), RT(3), RT(4), RT(5), RT(6), RT(7), q,
              RC(0), RC(1), RC(2), RC(3), RC(4), RC(5), RC(6), RC(7));
    red_row<F, S + 8>(t, q);
  } else if constexpr (n == 7) {
    mb::mads7(RT(0), RT(1), RT(2), RT(3), RT(4), RT(5), RT(6), q, RC(0), RC(1), RC(2), RC(3), RC(4), RC(5), RC(6));
  } else if constexpr (n == 6) {
    mb::mads6(RT(0), RT(1), RT(2), RT(3), RT(4), RT(5), q, RC(0), RC(1), RC(2), RC(3), RC(4), RC(5));
  } else if constexpr (n == 5) {
    mb::mads5(RT(0), RT(1), RT(2), RT(3), RT(4), q, RC(0), RC(1), RC(2), RC(3), RC(4));
  } else if constexpr (n == 4) {
    mb::mads4(RT(0), RT(1), RT(2), RT(3), q, RC(0), RC(1), RC(2), RC(3));
  } else if constexpr (n == 3) {
    mb::mads3(RT(0), RT(1), RT(2), q, RC(0), RC(1), RC(2));
  } else if constexpr (n == 2) {
    mb::mads2(RT(0), RT(1), q, RC(0), RC(1));
  } else if constexpr (n == 1) {
    mb::mads1(RT(0), q, RC(0));
  }
#undef RJ
#undef RT
#undef RC
}

MPD int32_t opaque_sgpr(int32_t v) {      // a constant the compiler cannot strength-reduce
  int32_t r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(v));
  return r;
}

// Ed25519's p = 2^255 - 19: q*p = +8q at limb i+9 (255 = 9*28 + 3) and -19q at
// limb i -- two MADs per row instead of ten.  Columns read as int64: with
// operand limbs < 3*2^28 (mp.hpp bounds) a column stays below 10*9*2^56 < 2^63.
MPD void mont_reduce_25519(uint32_t* r, uint64_t* t) {
  constexpr int L = ED25519P::L;
  int64_t* s = reinterpret_cast<int64_t*>(t);
  const int32_t c19 = opaque_sgpr(-19), c8 = opaque_sgpr(8);
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t q = (int32_t)(((uint32_t)s[i] * ED25519P::NP) & MP_MASK);
    s[i] += (int64_t)q * (int64_t)c19;        // low 28 bits of s[i] become zero
    s[i + 9] += (int64_t)q * (int64_t)c8;
    s[i + 1] += s[i] >> MP_W;
  }
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int64_t v = s[L + j] + c;
    r[j] = (uint32_t)v & MP_MASK;
    c = v >> MP_W;
  }
}

// Unmasked Montgomery digits (NP1 fields whose columns have the headroom):
// rows 0..L-2 take q = the low 32 bits of t[i] instead of its low 28.  Then
// t[i] + q m = (t[i] - q) + q (m+1) leaves hi32(t[i]) 2^32 = 16 hi32(t[i]) 2^28
// in column i, so the carry into column i+1 is ONE mad (hi * 16) -- no mask,
// no 64-bit shift, no 64-bit add.  The top row keeps a 28-bit digit, so
// Q = sum q_i 2^(28 i) < (1 + 2^-24) R and the output stays below
// T/R + (1 + 2^-24) m (was T/R + m); every caller's T/R is far below m/2.
// Column headroom, in units of 2^56: L * 9 for a product of limbs < 3*2^28
// (mp.hpp bounds; 2 L * 9 for the two-product sums of prod_acc callers is
// checked there) plus sum_j M1[j] 2^32 / 2^56 from the reduction rows.
template <class F>
constexpr bool unmasked_rows() {
  if constexpr (!F::NP1) {
    return false;
  } else {
    double red = 0;
    for (int j = 1; j < F::L; ++j) red += (double)F::M1[j] / 16777216.0;
    return 9.0 * F::L + red + 1.0 < 256.0;
  }
}

// SEMI: the output keeps 32-bit limbs ("semi-normalized": value as usual,
// limbs < 2^32): the final chain moves only hi32 of each column up (one mad
// per limb instead of add + mask + 64-bit shift).  Only valid as an operand of
// a product whose other operand has limbs < 2^28 and only where L 2^60 plus
// the reduction rows fits a column (see semi_ok); the top column's hi32 is 0
// because the value is < 2^(28(L-1)+32).
template <class F>
constexpr bool semi_ok() {
  if constexpr (!F::NP1) {
    return false;
  } else {
    double red = 0;
    for (int j = 1; j < F::L; ++j) red += (double)F::M1[j] / 16777216.0;
    return 16.0 * F::L + red + 1.0 < 256.0;
  }
}

template <class F, bool SEMI = false>
MPD void mont_reduce(uint32_t* r, uint64_t* t) {
  constexpr int L = F::L;
  if constexpr (std::is_same<F, ED25519P>::value) {
    mont_reduce_25519(r, t);
    return;
  }
  if constexpr (unmasked_rows<F>()) {
    const uint32_t c16 = (uint32_t)opaque_sgpr(16);
#pragma unroll
    for (int i = 0; i < L - 1; ++i) {
      red_row<F, 0>(t + i, (uint32_t)t[i]);
      t[i + 1] += (uint64_t)(uint32_t)(t[i] >> 32) * c16;
    }
    red_row<F, 0>(t + L - 1, (uint32_t)t[L - 1] & MP_MASK);
    t[L] += t[L - 1] >> MP_W;
    if constexpr (SEMI) {
      static_assert(semi_ok<F>(), "semi-normalized output needs column headroom");
#pragma unroll
      for (int j = 0; j < L - 1; ++j) {
        r[j] = (uint32_t)t[L + j];
        t[L + j + 1] += (uint64_t)(uint32_t)(t[L + j] >> 32) * c16;
      }
      r[L - 1] = (uint32_t)t[2 * L - 1];
      return;
    }
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t v = t[L + j] + c;
      r[j] = (uint32_t)v & MP_MASK;
      c = v >> MP_W;
    }
    return;
  }
  static_assert(!SEMI || unmasked_rows<F>(), "semi-normalized output needs unmasked rows");
#pragma unroll
  for (int i = 0; i < L; ++i) {
    // NP1: m = -1 mod 2^28 => NP = 1, q = t[i] mod 2^28 and q*m = q*(m+1) - q:
    // the "- q" is exactly the low limb the carry shift drops, and m+1 is
    // sparse (P-256: 4 non-zero limbs of 10, P-521: 1 of 20).
    const uint32_t q = F::NP1 ? ((uint32_t)t[i] & MP_MASK) : (((uint32_t)t[i] * F::NP) & MP_MASK);
    red_row<F, 0>(t + i, q);
    t[i + 1] += t[i] >> MP_W;
  }
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const uint64_t v = t[L + j] + c;
    r[j] = (uint32_t)v & MP_MASK;
    c = v >> MP_W;
  }
}

// ---- product scanning for the unmasked-row fields (P-256, P-521) --------------
// The product and its Montgomery reduction column by column, each column ONE
// asm MAD chain (col_chains.hpp UChain): the carry in, the reduction terms
// q_j (m+1)_{k-j} of the digits already known, then the partial products.  A
// low column k <= L-2 yields the unmasked digit q_k = lo32 and carries
// hi32 * 16 (one MAD at the head of the next chain, on the literal 0); column
// L-1 yields a 28-bit digit and carries >> 28; a high column yields an output
// limb (mask) and carries >> 28 -- or, semi-normalized, lo32 and hi32 * 16.
// Every term lands in the column mont_reduce's row order puts it in, so the
// value, the column bounds and the output are mont_reduce's bit for bit; the
// row form pays a 64-bit add per carry of its final chain, which this saves
// (and it keeps one column live instead of 2L).
// OP: 0 = a*b, 1 = a^2, 2 = a*b + c*d, 3 = a^2 + e*R (e added to the high
// columns: x3_from's column subtraction).
#ifndef JG_PS_ASM
#define JG_PS_ASM 1
#endif
template <class F>
constexpr int ps_nmul(int k) {
  const int lo = k - F::L + 1 > 0 ? k - F::L + 1 : 0, hi = k < F::L - 1 ? k : F::L - 1;
  return hi >= lo ? hi - lo + 1 : 0;
}
template <class F>
constexpr int ps_nsqr(int k) {
  const int lo = k - F::L + 1 > 0 ? k - F::L + 1 : 0, hi = k / 2;
  return hi >= lo ? hi - lo + 1 : 0;
}
template <class F>
constexpr int ps_nprod(int op, int k) {
  return op == 0 ? ps_nmul<F>(k) : op == 2 ? 2 * ps_nmul<F>(k) : ps_nsqr<F>(k);
}
template <class F>
constexpr int ps_nred(int k) {        // digits q_j (j < L, j < k) whose constant (m+1)_{k-j} is non-zero
  int n = 0;
  for (int j = (k - F::L + 1 > 0 ? k - F::L + 1 : 0); j < k && j < F::L; ++j)
    if (red_const<F>(k - j) != 0) ++n;
  return n;
}
template <class F, bool SEMI>
constexpr bool ps_carry_term(int k) {  // the carry into column k is hi32(column k-1) * 16
  return (k >= 1 && k - 1 <= F::L - 2) || (SEMI && k - 1 >= F::L);
}
template <class F>
constexpr bool ps_ok(int op) {         // every column fits a generated chain
  for (int k = 0; k < 2 * F::L - 1; ++k)
    if (ps_nprod<F>(op, k) > 20 || ps_nred<F>(k) + 2 > 6) return false;
  return true;
}

template <class F, int OP, bool SEMI, int K>
MPD void ps_col(uint32_t* r, const uint32_t* a, const uint32_t* a2, const uint32_t* b, const uint32_t* c,
                const uint32_t* d, const uint32_t* e, uint32_t* q, uint64_t& carry, uint32_t& hi, uint32_t c16,
                uint32_t c1) {
  constexpr int L = F::L;
  constexpr int N = ps_nprod<F>(OP, K);
  constexpr bool CT = ps_carry_term<F, SEMI>(K);
  constexpr bool EX = OP == 3 && K >= L;
  constexpr int R = (CT ? 1 : 0) + ps_nred<F>(K) + (EX ? 1 : 0);
  constexpr bool Z = K == 0 || CT;
  uint32_t x[N > 0 ? N : 1], y[N > 0 ? N : 1], u[R > 0 ? R : 1], kc[R > 0 ? R : 1];
  int n = 0, m = 0;
  if constexpr (CT) { u[m] = hi; kc[m++] = c16; }
  constexpr int jlo = K - L + 1 > 0 ? K - L + 1 : 0;
#pragma unroll
  for (int j = jlo; j < K && j < L; ++j)
    if (red_const<F>(K - j) != 0) { u[m] = q[j]; kc[m++] = red_const<F>(K - j); }
  if constexpr (EX) { u[m] = e[K - L]; kc[m++] = c1; }
  constexpr int ilo = K - L + 1 > 0 ? K - L + 1 : 0;
  if constexpr (OP == 1 || OP == 3) {
#pragma unroll
    for (int i = ilo; i <= K / 2; ++i) { x[n] = i == K - i ? a[i] : a2[i]; y[n++] = a[K - i]; }
  } else {
#pragma unroll
    for (int i = ilo; i <= K && i < L; ++i) { x[n] = a[i]; y[n++] = b[K - i]; }
    if constexpr (OP == 2) {
#pragma unroll
      for (int i = ilo; i <= K && i < L; ++i) { x[n] = c[i]; y[n++] = d[K - i]; }
    }
  }
  uint64_t s = carry;
  cc::UChain<N, R, Z>::run(s, x, y, u, kc);
  if constexpr (K <= L - 2) {
    q[K] = (uint32_t)s;
    hi = (uint32_t)(s >> 32);
  } else if constexpr (K == L - 1) {
    q[K] = (uint32_t)s & MP_MASK;
    carry = s >> MP_W;
  } else if constexpr (SEMI) {
    r[K - L] = (uint32_t)s;
    hi = (uint32_t)(s >> 32);
  } else {
    r[K - L] = (uint32_t)s & MP_MASK;
    carry = s >> MP_W;
  }
  if constexpr (K + 1 < 2 * L - 1) ps_col<F, OP, SEMI, K + 1>(r, a, a2, b, c, d, e, q, carry, hi, c16, c1);
}

template <class F, int OP, bool SEMI = false>
MPD void mont_ps(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* c = nullptr,
                 const uint32_t* d = nullptr, const uint32_t* e = nullptr) {
  constexpr int L = F::L;
  static_assert(unmasked_rows<F>() && ps_ok<F>(OP), "product scanning: unmasked-row fields whose columns fit a chain");
  uint32_t a2[L];
  if constexpr (OP == 1 || OP == 3) {
#pragma unroll
    for (int i = 0; i < L; ++i) a2[i] = a[i] << 1;
  }
  uint32_t q[L];
  uint64_t carry = 0;
  uint32_t hi = 0;
  const uint32_t c16 = (uint32_t)opaque_sgpr(16), c1 = (uint32_t)opaque_sgpr(1);
  ps_col<F, OP, SEMI, 0>(r, a, a2, b, c, d, e, q, carry, hi, c16, c1);
  // column 2L-1: no products, the carry (and OP 3's top term e_{L-1})
  if constexpr (SEMI) r[L - 1] = hi * 16u;
  else if constexpr (OP == 3) r[L - 1] = ((uint32_t)carry + e[L - 1]) & MP_MASK;
  else r[L - 1] = (uint32_t)carry & MP_MASK;
}
template <class F>
constexpr bool use_ps(int op) {
  if constexpr (!F::NP1) {
    return false;
  } else {
    return JG_PS_ASM && unmasked_rows<F>() && ps_ok<F>(op);
  }
}

// t = a*b (2L 64-bit columns, t[2L-1] = 0)
template <class F>
MPD void prod(uint64_t* t, const uint32_t* a, const uint32_t* b) {
  constexpr int L = F::L;
  t[2 * L - 1] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int j = 0; j < L; ++j) {
      // first product of column i+j in this loop order writes, not accumulates
      if (i == 0 || j == L - 1) mul64c(t[i + j], a[i], b[j]);
      else mad64c(t[i + j], a[i], b[j]);
    }
}

// t += a*b (all 2L-1 columns accumulate; for sums of products under ONE reduction)
template <class F>
MPD void prod_acc(uint64_t* t, const uint32_t* a, const uint32_t* b) {
  constexpr int L = F::L;
#pragma unroll
  for (int i = 0; i < L; ++i)
#pragma unroll
    for (int j = 0; j < L; ++j) mad64c(t[i + j], a[i], b[j]);
}

// t = a^2  (cross products once, doubled operand)
template <class F>
MPD void sqprod(uint64_t* t, const uint32_t* a) {
  constexpr int L = F::L;
  uint32_t a2[L];
#pragma unroll
  for (int i = 0; i < L; ++i) a2[i] = a[i] << 1;
  t[2 * L - 1] = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    if (i == 0 || i == L - 1) mul64c(t[2 * i], a[i], a[i]);
    else mad64c(t[2 * i], a[i], a[i]);
#pragma unroll
    for (int j = i + 1; j < L; ++j) {
      if (i == 0 || j == L - 1) mul64c(t[i + j], a2[i], a[j]);
      else mad64c(t[i + j], a2[i], a[j]);
    }
  }
}

// r = a*b/R mod m
template <class F>
MPD void mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  if constexpr (use_ps<F>(0)) {
    mont_ps<F, 0>(r, a, b);
  } else {
    uint64_t t[2 * F::L];
    prod<F>(t, a, b);
    mont_reduce<F>(r, t);
  }
}

// r = a^2/R mod m
template <class F>
MPD void sqr(uint32_t* r, const uint32_t* a) {
  if constexpr (use_ps<F>(1)) {
    mont_ps<F, 1>(r, a, a);
  } else {
    uint64_t t[2 * F::L];
    sqprod<F>(t, a);
    mont_reduce<F>(r, t);
  }
}



// P-384's special form: p + 1 = 2^384 - 2^128 - 2^96 + 2^32, i.e. per
// reduction row +q*2^4 at limb i+1, -q*2^12 at i+3, -q*2^16 at i+4 and
// +q*2^20 at i+13 -- four signed MADs where m+1's dense limbs cost 13.  The
// columns are read as int64 (arithmetic carries; the low limb's "- q" is the
// dropped low 28 bits as for every NP1 field), so every product column must
// stay below 2^63: the caller guarantees 15 * max(a_i) * max(b_j) < 2^62.9,
// e.g. one operand with limbs < 2^28 and the other < 2^31.  Output as
// mont_reduce: limbs < 2^28, value < 2m.
MPD void mont_reduce_p384(uint32_t* r, uint64_t* t) {
  constexpr int L = P384P::L;
  int64_t* s = reinterpret_cast<int64_t*>(t);
  // as SGPR operands of v_mad_i64_i32 (a multiply by a visible power of two
  // becomes a 64-bit shift + add/sub pair: 2-3 instructions instead of 1)
  const int32_t c4 = opaque_sgpr(16), c12 = opaque_sgpr(-4096), c16 = opaque_sgpr(-65536),
                c20 = opaque_sgpr(1048576);
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int32_t q = (int32_t)((uint32_t)s[i] & MP_MASK);
    s[i + 1] += (int64_t)q * (int64_t)c4;
    s[i + 3] += (int64_t)q * (int64_t)c12;
    s[i + 4] += (int64_t)q * (int64_t)c16;
    s[i + 13] += (int64_t)q * (int64_t)c20;
    s[i + 1] += s[i] >> MP_W;
  }
  int64_t c = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int64_t v = s[L + j] + c;
    r[j] = (uint32_t)v & MP_MASK;
    c = v >> MP_W;
  }
}

// The same product and reduction column by column (product scanning): column
// k gets its partial products, the reduction terms of the rows that reach it
// (q_{k-1} 2^4, q_{k-3} (-2^12), q_{k-4} (-2^16), q_{k-13} 2^20) and the carry
// of column k-1, then yields q_k (k < L) or output limb k - L.  Every term
// lands in the same column as in mont_reduce_p384's row order, so the value and
// the column bounds are the same; but only the current column, the 13 pending
// q's and the output are live instead of 2L 64-bit columns (P-384 point kernel:
// the register pressure that held it at three waves per SIMD).
template <bool SQR>
MPD void mont_mul_p384_cols(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr int L = P384P::L;
  const int32_t c4 = opaque_sgpr(16), c12 = opaque_sgpr(-4096), c16 = opaque_sgpr(-65536),
                c20 = opaque_sgpr(1048576);
  uint32_t a2[L];
  if constexpr (SQR) {
#pragma unroll
    for (int i = 0; i < L; ++i) a2[i] = a[i] << 1;
  }
  int32_t q[L];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; ++k) {
    uint64_t col = 0;
    bool first = true;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int j = k - i;
      if (j < 0 || j >= L) continue;
      if constexpr (SQR) {
        if (j < i) continue;
        const uint32_t x = i == j ? a[i] : a2[i];
        if (first) mul64c(col, x, a[j]); else mad64c(col, x, a[j]);
      } else {
        if (first) mul64c(col, a[i], b[j]); else mad64c(col, a[i], b[j]);
      }
      first = false;
    }
    int64_t s = (int64_t)col + carry;
    if (k >= 1 && k - 1 < L) s += (int64_t)q[k - 1] * (int64_t)c4;
    if (k >= 3 && k - 3 < L) s += (int64_t)q[k - 3] * (int64_t)c12;
    if (k >= 4 && k - 4 < L) s += (int64_t)q[k - 4] * (int64_t)c16;
    if (k >= 13 && k - 13 < L) s += (int64_t)q[k - 13] * (int64_t)c20;
    if (k < L) q[k] = (int32_t)((uint32_t)s & MP_MASK);
    else r[k - L] = (uint32_t)s & MP_MASK;
    carry = s >> MP_W;
  }
  r[L - 1] = (uint32_t)carry & MP_MASK;    // column 2L-1: no products, only the carries
}

// mont_mul_p384_cols with every column as ONE asm MAD chain (col_chains.hpp):
// the carry of column k-1 is the first addend, then the partial products
// (v_mad_u64_u32) and the reduction terms (v_mad_i64_i32 with the SGPR
// constants).  The same terms land in the same columns, so the value and the
// column bounds are mont_mul_p384_cols'; LLVM's form adds each carry with a
// separate 64-bit add (it reassociates the C++ sum), which this saves: one
// instruction per column, 27 per product.
#ifndef JG_P384_ASM
#define JG_P384_ASM 1
#endif
template <bool SQR, int K>
MPD void p384_col(uint32_t* r, const uint32_t* a, const uint32_t* a2, const uint32_t* b, int32_t* q, int64_t& carry,
                  const int32_t* cs) {
  constexpr int L = P384P::L;
  constexpr int lo = K < L ? 0 : K - L + 1;
  constexpr int hi = SQR ? K / 2 : (K < L ? K : L - 1);
  constexpr int N = hi >= lo ? hi - lo + 1 : 0;
  uint32_t x[N > 0 ? N : 1], y[N > 0 ? N : 1];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const int i = lo + n, j = K - i;
    if constexpr (SQR) {
      x[n] = i == j ? a[i] : a2[i];
      y[n] = a[j];
    } else {
      x[n] = a[i];
      y[n] = b[j];
    }
  }
  constexpr bool t4 = K >= 1 && K - 1 < L, t12 = K >= 3 && K - 3 < L, t16 = K >= 4 && K - 4 < L,
                 t20 = K >= 13 && K - 13 < L;
  constexpr int M = (int)t4 + (int)t12 + (int)t16 + (int)t20;
  int32_t qq[M > 0 ? M : 1], cc_[M > 0 ? M : 1];
  int m = 0;
  if constexpr (t4) { qq[m] = q[K - 1]; cc_[m++] = cs[0]; }
  if constexpr (t12) { qq[m] = q[K - 3]; cc_[m++] = cs[1]; }
  if constexpr (t16) { qq[m] = q[K - 4]; cc_[m++] = cs[2]; }
  if constexpr (t20) { qq[m] = q[K - 13]; cc_[m++] = cs[3]; }
  uint64_t acc = (uint64_t)carry;
  cc::Chain<N, M, K == 0>::run(acc, x, y, qq, cc_);
  const int64_t sv = (int64_t)acc;
  if constexpr (K < L) q[K] = (int32_t)((uint32_t)sv & MP_MASK);
  else r[K - L] = (uint32_t)sv & MP_MASK;
  carry = sv >> MP_W;
  if constexpr (K + 1 < 2 * L - 1) p384_col<SQR, K + 1>(r, a, a2, b, q, carry, cs);
}

template <bool SQR>
MPD void mont_mul_p384_asm(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  constexpr int L = P384P::L;
  const int32_t cs[4] = {opaque_sgpr(16), opaque_sgpr(-4096), opaque_sgpr(-65536), opaque_sgpr(1048576)};
  uint32_t a2[L];
  if constexpr (SQR) {
#pragma unroll
    for (int i = 0; i < L; ++i) a2[i] = a[i] << 1;
  }
  int32_t q[L];
  int64_t carry = 0;
  p384_col<SQR, 0>(r, a, a2, b, q, carry, cs);
  r[L - 1] = (uint32_t)carry & MP_MASK;    // column 2L-1: no products, only the carries
}

// Products for the point-addition hot loop: the field's special-form
// reduction where it has one (P-384), else mul / sqr.  Precondition (P-384):
// at least one operand has limbs < 2^28 (squares: the operand itself).
template <class F>
MPD void mulf(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  if constexpr (std::is_same<F, P384P>::value) {
#if JG_P384_COLS && JG_P384_ASM
    mont_mul_p384_asm<false>(r, a, b);
#elif JG_P384_COLS
    mont_mul_p384_cols<false>(r, a, b);
#else
    uint64_t t[2 * F::L];
    prod<F>(t, a, b);
    mont_reduce_p384(r, t);
#endif
  } else {
    mul<F>(r, a, b);
  }
}
template <class F>
MPD void sqrf(uint32_t* r, const uint32_t* a) {
  if constexpr (std::is_same<F, P384P>::value) {
#if JG_P384_COLS && JG_P384_ASM
    mont_mul_p384_asm<true>(r, a, a);
#elif JG_P384_COLS
    mont_mul_p384_cols<true>(r, a, a);
#else
    uint64_t t[2 * F::L];
    sqprod<F>(t, a);
    mont_reduce_p384(r, t);
#endif
  } else {
    sqr<F>(r, a);
  }
}

// r = a^2/R mod m with a semi-normalized result (limbs < 2^32) where the field
// allows it (semi_ok), else sqrf's normalized result
template <class F>
MPD void sqr_semi(uint32_t* r, const uint32_t* a) {
  if constexpr (semi_ok<F>() && use_ps<F>(1)) {
    mont_ps<F, 1, true>(r, a, a);
  } else if constexpr (semi_ok<F>()) {
    uint64_t t[2 * F::L];
    sqprod<F>(t, a);
    mont_reduce<F, true>(r, t);
  } else {
    sqrf<F>(r, a);
  }
}

template <class F>
MPD void add(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = a[j] + b[j];
}

template <class F>
MPD void sub(uint32_t* r, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = a[j] + F::KSUB[j] - b[j];
}

// m - b (negation of a normalized value), result limbs < 2^29 + 2^28
template <class F>
MPD void neg(uint32_t* r, const uint32_t* b) {
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = F::KSUB[j] - b[j];
}

template <class F>
MPD void copy(uint32_t* r, const uint32_t* a) {
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = a[j];
}

// carry-propagate: limbs < 2^28, value unchanged (value must be < 2^(28L))
template <class F>
MPD void norm(uint32_t* r) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < F::L; ++j) {
    const uint32_t v = r[j] + c;
    r[j] = v & MP_MASK;
    c = v >> MP_W;
  }
}

// lazy operands of sqrf / mulf pairs on P-384 are carry-normalised first
template <class F>
MPD void norm_for_mulf(uint32_t* r) {
  if constexpr (std::is_same<F, P384P>::value) norm<F>(r);
}

// value reduction for pseudo-Mersenne-shaped primes: fold bits >= FOLD_S by 2^FOLD_S mod m
template <class F>
MPD void freduce(uint32_t* r) {
  constexpr int L = F::L;
  constexpr int q = F::FOLD_S / MP_W, s = F::FOLD_S % MP_W;
  norm<F>(r);
  uint32_t h = r[q] >> s;
  if constexpr (q + 1 < L) h |= r[q + 1] << (MP_W - s);
  r[q] &= (1u << s) - 1u;
#pragma unroll
  for (int j = q + 1; j < L; ++j) r[j] = 0;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    uint64_t v = (uint64_t)r[j] + c;
    if (F::FOLDC[j] != 0) mad64c(v, h, F::FOLDC[j]);
    r[j] = (uint32_t)v & MP_MASK;
    c = v >> MP_W;
  }
}

// One-chain value fold for the madd outputs of P-256 (FOLD_S in the top limb):
// input limbs < 2^31 with the top limb < 2^29, i.e. a normalized value plus at
// most three lazy subtractions.  Only the top limb's bits >= FOLD_S are folded
// (the lower limbs' pending carries stay put), then ONE carry chain: the lower
// limbs sum to < 2^31 * 2^(28(L-2)) * (1 + 2^-27) < 2^(FOLD_S-1), so the result
// is < 2^FOLD_S + 2^(FOLD_S-1) + h * 2^(FOLD_S-32) < 2m -- freduce's output
// invariant at one chain instead of two.  Other fields: freduce.
template <class F>
MPD void freduce_lazy(uint32_t* r) {
  constexpr int L = F::L;
  constexpr int q = F::FOLD_S / MP_W, s = F::FOLD_S % MP_W;
  if constexpr (q != L - 1 || 31 + MP_W * (L - 2) + 1 > F::FOLD_S) {
    freduce<F>(r);
  } else {
    const uint32_t h = r[q] >> s;
    r[q] &= (1u << s) - 1u;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      uint64_t v = (uint64_t)r[j] + c;
      if (F::FOLDC[j] != 0) mad64c(v, h, F::FOLDC[j]);
      r[j] = (uint32_t)v & MP_MASK;
      c = v >> MP_W;
    }
  }
}

// normalized value < 2m  ->  canonical [0, m)
template <class F>
MPD void csub(uint32_t* r) {
  uint32_t d[F::L];
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < F::L; ++j) {
    const int32_t v = (int32_t)r[j] - (int32_t)F::M[j] + br;
    d[j] = (uint32_t)v & MP_MASK;
    br = v >> MP_W;                       // arithmetic shift: 0 or -1
  }
  const bool keep = br < 0;
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = keep ? r[j] : d[j];
}

template <class F>
MPD void canon(uint32_t* r) {
  freduce<F>(r);
  csub<F>(r);
}

template <class F>
MPD bool is_zero_canon(const uint32_t* r) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < F::L; ++j) o |= r[j];
  return o == 0;
}

template <class F>
MPD void set_const(uint32_t* r, const uint32_t* c) {
#pragma unroll
  for (int j = 0; j < F::L; ++j) r[j] = c[j];
}

// plain integer (28-bit limbs, value < m) -> Montgomery form
template <class F>
MPD void to_mont(uint32_t* r, const uint32_t* a) {
  uint32_t rr[F::L];
  set_const<F>(rr, F::RR);
  mul<F>(r, a, rr);
}

// Montgomery form -> canonical plain integer in [0, m)
template <class F>
MPD void from_mont(uint32_t* r, const uint32_t* a) {
  constexpr int L = F::L;
  uint64_t t[2 * L];
#pragma unroll
  for (int k = 0; k < 2 * L; ++k) t[k] = k < L ? a[k] : 0;
  mont_reduce<F>(r, t);
  csub<F>(r);
}

// r = x^E for an exponent held in a constexpr array of 28-bit limbs (read with
// wave-uniform indices -> scalar loads); used for the Ed25519 square root at
// key staging.  `minus2` subtracts 2 from limb 0 (E = m - 2, a Fermat
// exponent).  Left-to-right fixed window of WB bits (3 for 10-limb fields, 2
// above, so the 2^WB-entry table fits the register file); the window value is
// uniform across the wave, so the table select is a uniform compare chain.
template <class F>
MPD void pow_e(uint32_t* r, const uint32_t* x, const uint32_t* E, int ebits, bool minus2) {
  constexpr int L = F::L;
  constexpr int WB = L <= 10 ? 3 : 2, NT = 1 << WB;
  uint32_t tab[NT][L];
  set_const<F>(tab[0], F::ONE);
  copy<F>(tab[1], x);
#pragma unroll
  for (int i = 2; i < NT; ++i) mul<F>(tab[i], tab[i - 1], x);
  uint32_t acc[L];
  set_const<F>(acc, F::ONE);
  const int top = (ebits + WB - 1) / WB * WB;
  for (int b = top - WB; b >= 0; b -= WB) {
#pragma unroll
    for (int k = 0; k < WB; ++k) sqr<F>(acc, acc);
    const int w = b / MP_W, o = b % MP_W;
    const uint32_t lo = E[w] - ((minus2 && w == 0) ? 2u : 0u);
    uint32_t nib = lo >> o;
    if (o > MP_W - WB && w + 1 < L) nib |= E[w + 1] << (MP_W - o);
    nib &= (uint32_t)(NT - 1);
    uint32_t sel[L];
#pragma unroll
    for (int j = 0; j < L; ++j) sel[j] = tab[0][j];
#pragma unroll
    for (int i = 1; i < NT; ++i)
      if (nib == (uint32_t)i) {
#pragma unroll
        for (int j = 0; j < L; ++j) sel[j] = tab[i][j];
      }
    mul<F>(acc, acc, sel);
  }
  copy<F>(r, acc);
}

// ---- constant-time modular inversion by Bernstein-Yang "safegcd" ----------
// (half-delta divsteps, the variant of Bernstein & Yang 2019 as refined by
// Wuille).  Numbers are in signed radix 2^28: limbs 0..L-2 in [0, 2^28), the
// top limb signed.  Each batch runs 28 divsteps on the low 32 bits of f, g with
// 32-bit masks only, producing a 2x2 matrix with entries in [-2^28, 2^28]; the
// matrix is then applied to the full-width f, g (an exact shift by one limb)
// and to d, e modulo m (a Montgomery-style correction so the shift is exact).
// The divstep bound floor((45907 b + 26313) / 19929) for a b-bit modulus gives
// 22 batches for 256-bit moduli, 32 for 384 and 43 for 521.  Cost ~0.75k VALU
// per batch for L=10, about 4x below the Fermat ladder.

template <class F>
struct Sg {
  static constexpr int DIVSTEPS = (45907 * F::BITS + 26313) / 19929 + 1;
  static constexpr int BATCHES = (DIVSTEPS + 27) / 28;
  static constexpr uint32_t INV28 = (0u - F::NP) & MP_MASK;  // m^-1 mod 2^28
};

// 28 divsteps on the low bits; returns the new zeta (= -(delta + 1/2)).
MPD int32_t sg_divsteps28(int32_t zeta, uint32_t f, uint32_t g, int32_t* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 28; ++i) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);     // zeta < 0
    const uint32_t c2 = 0u - (g & 1u);              // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    const uint32_t c3 = c1 & c2;                    // swap step
    zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
    f += g & c3;
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return zeta;
}

MPD int64_t smul(int32_t a, int32_t b) { return (int64_t)a * (int64_t)b; }

// [f, g] <- t [f, g] / 2^28 (exact)
template <int L>
MPD void sg_update_fg(int32_t* f, int32_t* g, const int32_t* t) {
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  int64_t cf = smul(u, f[0]) + smul(v, g[0]);
  int64_t cg = smul(q, f[0]) + smul(r, g[0]);
  cf >>= MP_W;
  cg >>= MP_W;
#pragma unroll
  for (int i = 1; i < L; ++i) {
    cf += smul(u, f[i]) + smul(v, g[i]);
    cg += smul(q, f[i]) + smul(r, g[i]);
    f[i - 1] = (int32_t)cf & (int32_t)MP_MASK;
    g[i - 1] = (int32_t)cg & (int32_t)MP_MASK;
    cf >>= MP_W;
    cg >>= MP_W;
  }
  f[L - 1] = (int32_t)cf;
  g[L - 1] = (int32_t)cg;
}

// [d, e] <- (t [d, e] + m [md, me]) / 2^28, keeping d, e in (-2m, m)
template <class F>
MPD void sg_update_de(int32_t* d, int32_t* e, const int32_t* t) {
  constexpr int L = F::L;
  const int32_t u = t[0], v = t[1], q = t[2], r = t[3];
  const int32_t sd = d[L - 1] >> 31, se = e[L - 1] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = smul(u, d[0]) + smul(v, e[0]);
  int64_t ce = smul(q, d[0]) + smul(r, e[0]);
  md -= (int32_t)((Sg<F>::INV28 * (uint32_t)cd + (uint32_t)md) & MP_MASK);
  me -= (int32_t)((Sg<F>::INV28 * (uint32_t)ce + (uint32_t)me) & MP_MASK);
  cd += smul((int32_t)F::M[0], md);
  ce += smul((int32_t)F::M[0], me);
  cd >>= MP_W;
  ce >>= MP_W;
#pragma unroll
  for (int i = 1; i < L; ++i) {
    cd += smul(u, d[i]) + smul(v, e[i]);
    ce += smul(q, d[i]) + smul(r, e[i]);
    if (F::M[i] != 0) {
      cd += smul((int32_t)F::M[i], md);
      ce += smul((int32_t)F::M[i], me);
    }
    d[i - 1] = (int32_t)cd & (int32_t)MP_MASK;
    e[i - 1] = (int32_t)ce & (int32_t)MP_MASK;
    cd >>= MP_W;
    ce >>= MP_W;
  }
  d[L - 1] = (int32_t)cd;
  e[L - 1] = (int32_t)ce;
}

// d in (-2m, m), negated when sign < 0, to canonical [0, m)
template <class F>
MPD void sg_normalize(uint32_t* out, int32_t* d, int32_t sign) {
  constexpr int L = F::L;
  int32_t ca = d[L - 1] >> 31;
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] += (int32_t)F::M[i] & ca;
  const int32_t cn = sign >> 31;
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] = (d[i] ^ cn) - cn;
#pragma unroll
  for (int i = 0; i < L - 1; ++i) {
    d[i + 1] += d[i] >> MP_W;
    d[i] &= (int32_t)MP_MASK;
  }
  ca = d[L - 1] >> 31;
#pragma unroll
  for (int i = 0; i < L; ++i) d[i] += (int32_t)F::M[i] & ca;
#pragma unroll
  for (int i = 0; i < L - 1; ++i) {
    d[i + 1] += d[i] >> MP_W;
    d[i] &= (int32_t)MP_MASK;
  }
#pragma unroll
  for (int i = 0; i < L; ++i) out[i] = (uint32_t)d[i];
}

// plain canonical a in [0, m) -> a^-1 mod m (0 -> 0)
template <class F>
MPD void inv_plain(uint32_t* r, const uint32_t* a) {
  constexpr int L = F::L;
  int32_t d[L], e[L], f[L], g[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    d[i] = 0;
    e[i] = i == 0 ? 1 : 0;
    f[i] = (int32_t)F::M[i];
    g[i] = (int32_t)a[i];
  }
  int32_t zeta = -1;
  for (int b = 0; b < Sg<F>::BATCHES; ++b) {
    int32_t t[4];
    zeta = sg_divsteps28(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    sg_update_de<F>(d, e, t);
    sg_update_fg<L>(f, g, t);
  }
  sg_normalize<F>(r, d, f[L - 1]);
}

// ---- variable-time safegcd (public inputs only) -----------------------------
// Wuille's var-time divsteps (original divstep, eta = -delta): the trailing
// zeros of g go in one step, and each odd step cancels up to 6 (after a swap)
// or 4 low bits of g with one multiple of f.  A 28-divstep batch produces the
// same transition matrix meaning as sg_divsteps28 (f 2^28 = u f0 + v g0,
// g 2^28 = q f0 + r g0), so sg_update_fg / sg_update_de apply unchanged; the
// loop stops once g == 0.  For 256-bit moduli that is ~19.4 batches of ~7
// odd steps each instead of 22 batches of 28 masked steps (tools/safegcd_var_sim.py).
// Used where the value is public and one lane works alone (the one-launch
// small-batch path: a signature's s), so its branches cost nothing.
MPD int32_t sg_divsteps28_var(int32_t eta, uint32_t f, uint32_t g, int32_t* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 28;
  for (;;) {
    const int zeros = (int)__builtin_ctz(g | (0xffffffffu << i));   // the sentinel stops at i
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    uint32_t w;
    if (eta < 0) {
      eta = -eta;
      uint32_t x = f;
      f = g; g = 0u - x;
      x = u; u = q; q = 0u - x;
      x = v; v = r; r = 0u - x;
      const int limit = eta + 1 < i ? eta + 1 : i;
      const uint32_t m = (0xffffffffu >> (32 - limit)) & 63u;
      w = (f * g * (f * f - 2u)) & m;                 // g + w f == 0 mod 2^min(limit, 6)
    } else {
      const int limit = eta + 1 < i ? eta + 1 : i;
      const uint32_t m = (0xffffffffu >> (32 - limit)) & 15u;
      w = f + (((f + 1u) & 4u) << 1);                 // -f^-1 mod 16
      w = (0u - w * g) & m;
    }
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t[0] = (int32_t)u;
  t[1] = (int32_t)v;
  t[2] = (int32_t)q;
  t[3] = (int32_t)r;
  return eta;
}

// A value the compiler must treat as per-lane (divergent): code that runs on
// one active lane with inputs it can prove wave-uniform (LDS reads at uniform
// addresses, constants) is otherwise scalarised -- 64-bit products as 4-5
// SALU instructions each, VALU-only ops (v_alignbit) bracketed by
// v_readfirstlane -- measured 2-3x slower than the same code on VGPRs.
MPD uint32_t lane_value(uint32_t v) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// plain canonical a in [1, m) -> a^-1 mod m, variable time (a is public).
// For ONE active lane: the divsteps run on the wave-uniform copies of f[0],
// g[0] (readfirstlane), so they are scalar code -- SGPRs, s_ff1 for the
// trailing zeros, branches on SCC -- and the matrix reaches the limb updates
// as SGPR operands; with several active lanes every lane would get the first
// one's inverse.
template <class F>
MPD void inv_plain_var(uint32_t* r, const uint32_t* a) {
  constexpr int L = F::L;
  int32_t d[L], e[L], f[L], g[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {     // the limbs on VGPRs, the divsteps scalar
    d[i] = (int32_t)lane_value(0u);
    e[i] = (int32_t)lane_value(i == 0 ? 1u : 0u);
    f[i] = (int32_t)lane_value(F::M[i]);
    g[i] = (int32_t)lane_value(a[i]);
  }
  int32_t eta = -1;
  // every input reaches g == 0 well inside the constant-time bound; the cap
  // only guarantees that the loop ends
#pragma unroll 1
  for (int b = 0; b < 2 * Sg<F>::BATCHES; ++b) {
    int32_t t[4];
    eta = sg_divsteps28_var(eta, __builtin_amdgcn_readfirstlane((uint32_t)f[0]),
                            __builtin_amdgcn_readfirstlane((uint32_t)g[0]), t);
    sg_update_de<F>(d, e, t);
    sg_update_fg<L>(f, g, t);
    int32_t o = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) o |= g[i];
    if (__builtin_amdgcn_readfirstlane(o) == 0) break;
  }
  sg_normalize<F>(r, d, f[L - 1]);
}

// inv_plain_var with its four limb rows on four lanes: lanes 0..3 of the wave
// (all four active, the same `a` on each) hold f, g, d, e's update rows --
// lane 0 computes f' = (u f + v g) / 2^28, lane 1 g' = (q f + r g) / 2^28,
// lane 2 d', lane 3 e' (with the Montgomery-style correction) -- each one
// carry chain instead of four in a row, then the pairs swap rows so lanes
// 0, 1 hold (f, g) and lanes 2, 3 hold (d, e) again.  The divsteps stay
// scalar, on lane 0's f[0], g[0].  The inverse lands in every one of the four
// lanes.
template <class F>
MPD void inv_plain_var4(uint32_t* r, const uint32_t* a) {
  constexpr int L = F::L;
  const int l = (int)(threadIdx.x & 3);
  const bool de = l >= 2, second = (l & 1) != 0;
  int32_t X[L], Y[L];                 // lanes 0, 1: (f, g); lanes 2, 3: (d, e)
#pragma unroll
  for (int i = 0; i < L; ++i) {
    X[i] = (int32_t)lane_value(de ? 0u : F::M[i]);
    Y[i] = (int32_t)lane_value(de ? (i == 0 ? 1u : 0u) : a[i]);
  }
  int32_t eta = -1;
#pragma unroll 1
  for (int b = 0; b < 2 * Sg<F>::BATCHES; ++b) {
    int32_t t[4];
    eta = sg_divsteps28_var(eta, (uint32_t)__builtin_amdgcn_readlane(X[0], 0),
                            (uint32_t)__builtin_amdgcn_readlane(Y[0], 0), t);
    const int32_t ca = second ? t[2] : t[0], cb = second ? t[3] : t[1];
    // d, e rows: the multiple of m that makes the division by 2^28 exact and
    // keeps the row in (-2m, m) (sg_update_de, one row); f, g rows add none
    const int32_t sx = X[L - 1] >> 31, sy = Y[L - 1] >> 31;
    int32_t mm = (ca & sx) + (cb & sy);
    int64_t c = smul(ca, X[0]) + smul(cb, Y[0]);
    mm -= (int32_t)((Sg<F>::INV28 * (uint32_t)c + (uint32_t)mm) & MP_MASK);
    if (!de) mm = 0;
    c += smul((int32_t)F::M[0], mm);
    c >>= MP_W;
    int32_t nw[L];
#pragma unroll
    for (int i = 1; i < L; ++i) {
      c += smul(ca, X[i]) + smul(cb, Y[i]);
      if (F::M[i] != 0) c += smul((int32_t)F::M[i], mm);
      nw[i - 1] = (int32_t)c & (int32_t)MP_MASK;
      c >>= MP_W;
    }
    nw[L - 1] = (int32_t)c;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int32_t o = __shfl_xor(nw[i], 1);
      X[i] = second ? o : nw[i];
      Y[i] = second ? nw[i] : o;
    }
    int32_t o = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) o |= Y[i];
    if (__builtin_amdgcn_readlane(o, 0) == 0) break;      // g == 0
  }
  const int32_t fsign = __builtin_amdgcn_readlane(X[L - 1], 0);
  uint32_t out[L];
  sg_normalize<F>(out, X, fsign);                          // lanes 2, 3: d
#pragma unroll
  for (int i = 0; i < L; ++i) r[i] = (uint32_t)__builtin_amdgcn_readlane((int32_t)out[i], 2);
}

// inverse in Montgomery form: x = aR  ->  a^-1 R  (lazy input accepted)
template <class F>
MPD void inv(uint32_t* r, const uint32_t* x) {
  uint32_t a[F::L];
  from_mont<F>(a, x);      // a (plain, canonical)
  inv_plain<F>(a, a);      // a^-1
  to_mont<F>(r, a);        // a^-1 R
}

// Batched inversion shared by the WPB waves of a block (Montgomery's trick
// through LDS).  A wave computes one inversion however many lanes use it, so
// per-thread batching (k_ec_scalar_batch, k_ed_finish: B tokens per thread)
// pays one inversion per wave; here the block's waves hand their per-lane
// products to wave 0, which inverts ONE product per lane for all WPB waves
// (WPB - 1 products forward, 2 (WPB - 1) back) while the other waves wait at
// the barrier.  In: x = aR (Montgomery, nonzero); out: a^-1 R.  Every thread
// of the block must call it (two __syncthreads).
template <class F, int WPB>
MPD void block_inv(uint32_t* r, const uint32_t* x) {
  constexpr int L = F::L;
  __shared__ uint32_t sh_x[WPB * L * 64];           // per wave: its lanes' x, then their inverses
  __shared__ uint32_t sh_p[(WPB > 1 ? WPB - 1 : 1) * L * 64];   // prefix products x_0 ... x_j
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if constexpr (WPB == 1) {
    inv<F>(r, x);
    return;
  }
#pragma unroll
  for (int k = 0; k < L; ++k) sh_x[(w * L + k) * 64 + lane] = x[k];
  __syncthreads();
  if (w == 0) {                                     // wave-uniform
    uint32_t acc[L], t[L];
    copy<F>(acc, x);
#pragma unroll 1
    for (int j = 1; j < WPB; ++j) {
#pragma unroll
      for (int k = 0; k < L; ++k) sh_p[((j - 1) * L + k) * 64 + lane] = acc[k];
#pragma unroll
      for (int k = 0; k < L; ++k) t[k] = sh_x[(j * L + k) * 64 + lane];
      mul<F>(acc, acc, t);
    }
    uint32_t iv[L];
    inv<F>(iv, acc);                                // (x_0 ... x_{WPB-1})^-1
#pragma unroll 1
    for (int j = WPB - 1; j >= 1; --j) {
      uint32_t xj[L], pj[L], out[L];
#pragma unroll
      for (int k = 0; k < L; ++k) {
        xj[k] = sh_x[(j * L + k) * 64 + lane];
        pj[k] = sh_p[((j - 1) * L + k) * 64 + lane];
      }
      mul<F>(out, iv, pj);                          // x_j^-1
      mul<F>(iv, iv, xj);                           // (x_0 ... x_{j-1})^-1
#pragma unroll
      for (int k = 0; k < L; ++k) sh_x[(j * L + k) * 64 + lane] = out[k];
    }
#pragma unroll
    for (int k = 0; k < L; ++k) sh_x[k * 64 + lane] = iv[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < L; ++k) r[k] = sh_x[(w * L + k) * 64 + lane];
}

// canonical equality of two normalized values < 2m (reduces both)
template <class F>
MPD bool eq_mod(const uint32_t* a, const uint32_t* b) {
  uint32_t d[F::L];
  sub<F>(d, a, b);
  canon<F>(d);
  return is_zero_canon<F>(d);
}

// load a big-endian byte string's integer (given as little-endian 32-bit words
// w[0..nw)) into 28-bit limbs (truncating to L limbs)
template <int L, int NW>
MPD void words_to_limbs(uint32_t* r, const uint32_t* w) {
  constexpr int nw = NW;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int bit = MP_W * j, q = bit / 32, s = bit % 32;
    uint32_t v = q < nw ? (w[q] >> s) : 0u;
    if (s > 32 - MP_W && q + 1 < nw) v |= w[q + 1] << (32 - s);
    r[j] = v & MP_MASK;
  }
}

template <int L, int NW>
MPD void limbs_to_words(uint32_t* w, const uint32_t* r) {
  constexpr int nw = NW;
#pragma unroll
  for (int q = 0; q < nw; ++q) w[q] = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int bit = MP_W * j, q = bit / 32, s = bit % 32;
    if (q < nw) w[q] |= r[j] << s;
    if (s > 32 - MP_W && q + 1 < nw) w[q + 1] |= r[j] >> (32 - s);
  }
}

}  // namespace mp
