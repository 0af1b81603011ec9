// ecdsa_impl.hpp -- ECDSA P-256 / P-384 / P-521 verification on gfx950: the
// device code, included by one translation unit per curve (ecdsa_p256.hip,
// ecdsa_p384.hip, ecdsa_p521.hip: each instantiates its curve's kernels for
// every key-table width, compiled in parallel) and by the test kernels.
//
// Replaces go-jose ecEncrypterVerifier.verifyPayload -> crypto/ecdsa.Verify
// (rules R18-R22).  Per token:
//   k_ec_scalar_batch : r, s in [1, n-1] (sizes from the alg, curve from the
//                 key), e = leftmost bits of H, w = s^-1 (one inversion per B
//                 tokens), u1 = e w, u2 = r w (mod n), recoded to signed W-bit
//                 digits (W = ec_comb_w: generator 24 / key 20 for P-256, 20 / 16 above)
//   k_ec_point  : R = u1 G + u2 Q as a sum of one precomputed affine multiple of
//                 G and one of Q per window (comb tables in HBM: entries
//                 d * 2^(W w) * P, d = 1..2^(W-1)), mixed Jacobian+affine
//                 additions, no doublings; accept iff X == r Z^2 or (r+n) Z^2
//   k_ec_exact  : tokens whose fast sum hit an exceptional case of the group
//                 law (Z == 0: a doubling, an inverse pair, or R = infinity) --
//                 recomputed with complete case handling; rare
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "ecdsa.hpp"
#include "mp.hpp"
#include "tables.hpp"

using namespace jgk;

namespace {

// WQ: comb width of the key tables (ecdsa.hpp ec_key_w: P-256 keys 20 / 22 / 24,
// P-384 / P-521 keys 16 / 18 / 20 by the context's table budget; one kernel
// instantiation per width)
template <int WQ_>
struct CurveP256W { using Fp = P256P; using Fn = P256N; using C = P256C; static constexpr int CLS = CLS_P256, WQ = WQ_; };
using CurveP256 = CurveP256W<20>;
template <int WQ_>
struct CurveP384W { using Fp = P384P; using Fn = P384N; using C = P384C; static constexpr int CLS = CLS_P384, WQ = WQ_; };
using CurveP384 = CurveP384W<16>;
template <int WQ_>
struct CurveP521W { using Fp = P521P; using Fn = P521N; using C = P521C; static constexpr int CLS = CLS_P521, WQ = WQ_; };
using CurveP521 = CurveP521W<16>;

__device__ __forceinline__ int es_size(int alg) { return alg == 7 ? 32 : alg == 8 ? 48 : 66; }
__device__ __forceinline__ int es_hash_bytes(int alg) { return alg == 7 ? 32 : alg == 8 ? 48 : 64; }

// plain-integer compare of normalized limbs: a < b
template <int L>
__device__ __forceinline__ bool lt_limbs(const uint32_t* a, const uint32_t* b) {
  int lt = 0, gt = 0;
#pragma unroll
  for (int j = L - 1; j >= 0; --j) {
    const int und = !(lt | gt);
    lt |= und & (a[j] < b[j]);
    gt |= und & (a[j] > b[j]);
  }
  return lt;
}
template <int L>
__device__ __forceinline__ bool zero_limbs(const uint32_t* a) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) o |= a[j];
  return o == 0;
}

// ------------------------------------------------------------------ scalar
// Per-token inputs of the scalar stage, in two halves so the batched kernel
// can issue one token's loads while it computes the previous one:
// ec_scalar_load reads the raw words (job, status, key validity, r / s words,
// digest words), ec_scalar_finish checks them and returns ok with r, s, e as
// plain 28-bit limbs (s replaced by 1 when the token is rejected, so the batch
// product stays invertible).
template <class CV>
struct ScalarRaw {
  static constexpr int CW = ec_sig_words(CV::CLS);
  static constexpr int EW = (CV::C::BYTES + 3) / 4 < 16 ? (CV::C::BYTES + 3) / 4 : 16;   // digest words used
  JobDev jb;
  uint32_t ok;                // status OK and the key valid
  uint32_t rw[CW], sw[CW];
  uint32_t ew[EW];            // e as little-endian words (digest words reversed), zero past the hash
};

template <class CV>
__device__ __forceinline__ int ec_hash_words(int alg) {
  constexpr int CB = CV::C::BYTES;
  return (es_hash_bytes(alg) < CB ? es_hash_bytes(alg) : CB) / 4;   // hl / 4 (hl a multiple of 4)
}

template <class CV>
__device__ __forceinline__ void ec_scalar_load(const EcArgs& a, int64_t p, ScalarRaw<CV>& R) {
  constexpr int CW = ScalarRaw<CV>::CW, EW = ScalarRaw<CV>::EW;
  const int64_t np = a.npad;
  R.jb = a.jobs[p];
  if (!job_live(R.jb)) return;
  const int kidx = job_key(R.jb);
  const int hw = ec_hash_words<CV>(job_alg(R.jb));
  R.ok = a.status[p] == ST_OK && a.keys[kidx].valid;
#pragma unroll
  for (int q = 0; q < CW; ++q) {
    R.rw[q] = a.sigw[(int64_t)q * np + p];
    R.sw[q] = a.sigw[(int64_t)(EC_S_ROW + q) * np + p];
  }
#pragma unroll
  for (int q = 0; q < EW; ++q) {
    const int src = hw - 1 - q;
    R.ew[q] = src >= 0 ? a.dig[(int64_t)(src < 0 ? 0 : src) * np + p] : 0u;
  }
}

template <class CV>
__device__ __forceinline__ bool ec_scalar_finish(const EcArgs& a, int64_t p, const ScalarRaw<CV>& R, uint32_t* r,
                                                 uint32_t* s, uint32_t* e) {
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L;
  constexpr int CB = CV::C::BYTES;
  constexpr int CW = ScalarRaw<CV>::CW, EW = ScalarRaw<CV>::EW;
  const int64_t np = a.npad;
  if (!job_live(R.jb)) {
#pragma unroll
    for (int j = 0; j < L; ++j) { r[j] = 0; e[j] = 0; s[j] = j == 0 ? 1u : 0u; }
    return false;
  }
  const int alg = job_alg(R.jb);
  // R18/R21: the signature size comes from the alg, the curve from the key
  // (go-jose ecEncrypterVerifier: keySize by alg, no curve check), so r and s
  // are es_size(alg)-byte integers that must be < n of the key's curve.  Prep
  // leaves them in rows [0, ..) and [EC_S_ROW, ..), zero above what it wrote
  // up to this curve's CW words; an alg whose r/s are longer than the curve's
  // (ES512 on a P-256 key) must have zero words past CB as well.
  bool ok = R.ok != 0;
  if constexpr (4 * CW > CB) {
    const uint32_t hi = ~0u << (8 * (CB - 4 * (CW - 1)));
    ok = ok && (R.rw[CW - 1] & hi) == 0 && (R.sw[CW - 1] & hi) == 0;
  }
  if (es_size(alg) > CB) {
    const int aw = (es_size(alg) + 3) / 4;      // words prep wrote for this alg
    for (int q = CW; q < aw; ++q)
      ok = ok && a.sigw[(int64_t)q * np + p] == 0 && a.sigw[(int64_t)(EC_S_ROW + q) * np + p] == 0;
  }
  mp::words_to_limbs<L, CW>(r, R.rw);
  mp::words_to_limbs<L, CW>(s, R.sw);
  uint32_t nl[L];
  mp::set_const<Fn>(nl, Fn::M);
  ok = ok && !zero_limbs<L>(r) && !zero_limbs<L>(s) && lt_limbs<L>(r, nl) && lt_limbs<L>(s, nl);
  mp::words_to_limbs<L, EW>(e, R.ew);
  mp::csub<Fn>(e);
  if (!ok) {
#pragma unroll
    for (int j = 0; j < L; ++j) s[j] = j == 0 ? 1u : 0u;
  }
  return ok;
}

template <class CV>
__device__ __forceinline__ bool ec_scalar_inputs(const EcArgs& a, int64_t p, uint32_t* r, uint32_t* s, uint32_t* e) {
  ScalarRaw<CV> R;
  ec_scalar_load<CV>(a, p, R);
  return ec_scalar_finish<CV>(a, p, R, r, s, e);
}

// Pass 2 of the batched scalar stage (the checks are done): the prefix product
// c_{j-1}, s_j (Montgomery) and the raw r / e words of token j, loaded one
// token ahead like pass 1's inputs.
template <class CV>
struct ScalarRaw2 {
  static constexpr int L = CV::Fn::L;
  uint32_t cprev[L], sm[L];
  uint32_t rw[ScalarRaw<CV>::CW], ew[ScalarRaw<CV>::EW];
};

template <class CV>
__device__ __forceinline__ void ec_scalar_load2(const EcArgs& a, int64_t p, int64_t pprev, ScalarRaw2<CV>& R) {
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L, CW = ScalarRaw<CV>::CW, EW = ScalarRaw<CV>::EW;
  const int64_t np = a.npad;
  if (pprev >= 0) {
#pragma unroll
    for (int k = 0; k < L; ++k) R.cprev[k] = a.u1w[(int64_t)k * np + pprev];
  } else {
    mp::set_const<Fn>(R.cprev, Fn::ONE);
  }
#pragma unroll
  for (int k = 0; k < L; ++k) R.sm[k] = a.u2w[(int64_t)k * np + p];
#pragma unroll
  for (int q = 0; q < CW; ++q) R.rw[q] = a.sigw[(int64_t)q * np + p];
  const int hw = ec_hash_words<CV>(job_alg(a.jobs[p]));
#pragma unroll
  for (int q = 0; q < EW; ++q) {
    const int src = hw - 1 - q;
    R.ew[q] = src >= 0 ? a.dig[(int64_t)(src < 0 ? 0 : src) * np + p] : 0u;
  }
}

// r and e of a token that passed ec_scalar_inputs (pass 2 of the batched
// scalar stage: the checks are done, only the values are needed)
template <class CV>
__device__ __forceinline__ void ec_scalar_re(const EcArgs& a, int64_t p, uint32_t* r, uint32_t* e) {
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L;
  ScalarRaw2<CV> R;
  ec_scalar_load2<CV>(a, p, -1, R);
  mp::words_to_limbs<L, ScalarRaw<CV>::CW>(r, R.rw);
  mp::words_to_limbs<L, ScalarRaw<CV>::EW>(e, R.ew);
  mp::csub<Fn>(e);
}

// Signed W-bit recoding: u = sum_w d_w 2^(W w), d_w in [-2^(W-1), 2^(W-1)),
// one int32 row per window starting at digit row `row0`.
template <class CV, int W, int NWIN>
__device__ __forceinline__ void store_digit_rows(const EcArgs& a, int64_t p, const uint32_t* u, int row0) {
  constexpr int L = CV::Fn::L;
  constexpr uint32_t DM = (1u << W) - 1u;
  int c = 0;
#pragma unroll
  for (int w = 0; w < NWIN; ++w) {
    const int bit = W * w, q = bit / MP_W, sh = bit % MP_W;
    uint32_t b = q < L ? (u[q] >> sh) : 0u;
    if (sh > MP_W - W && q + 1 < L) b |= u[q + 1] << (MP_W - sh);
    int v = (int)(b & DM) + c;
    c = v >= (1 << (W - 1));
    v -= c << W;
    a.digs[(int64_t)(row0 + w) * a.npad + p] = (uint32_t)v;
  }
}

// Batched scalar stage (Montgomery's trick): thread i owns the B tokens
// p_j = begin + i + j*S and pays ONE (safegcd) inversion for all of them:
//   pass 1: c_j = s_0 ... s_j (Montgomery), c_j and s_j parked in the u1/u2 rows
//   inv = c_{B-1}^-1
//   pass 2 (j descending): w_j = inv * c_{j-1}, inv *= s_j;
//           u1 = e w_j, u2 = r w_j (mod n), signed W-bit digits
// The inversion is shared by the EC_SCALAR_WPB waves of a block
// (mp::block_inv); JG_EC_SCALAR_WPB = 1 is the round-3 kernel (one inversion
// per wave).
#ifndef JG_EC_SCALAR_WPB
#define JG_EC_SCALAR_WPB 4
#endif
// JG_EC_SCALAR_PF=1: both passes load the next token's words before computing
// the current one.  Measured no faster for P-256 (0.189-0.190 vs 0.192 ms per
// 1 M, profiles/r04_s4/scalar_pf_ab.json) and it costs registers (P-256 138 ->
// 203 VGPRs, P-384 past 256, P-521 spills), so it is off (A/B knob).
#ifndef JG_EC_SCALAR_PF
#define JG_EC_SCALAR_PF 0
#endif
constexpr int EC_SCALAR_WPB = JG_EC_SCALAR_WPB;
// WPB: waves per block sharing one inversion (small launches: 1, launch_chain)
template <class CV, int WPB = EC_SCALAR_WPB>
// JG_EC_SCALAR_ATTR: per translation unit.  ecdsa_p521.hip caps the kernel at
// two waves per SIMD: left alone the compiler gives the P-521 instantiation
// 295 VGPRs (+18 spilled), one wave per SIMD; capped it needs 198 and spills
// nothing (scalar 0.172 -> 0.162 ms in configs[4]).  The same cap on P-384
// squeezes 241 -> 139 VGPRs and runs 37 % slower, so the others keep the
// compiler's choice.
#ifndef JG_EC_SCALAR_ATTR
#define JG_EC_SCALAR_ATTR
#endif
__global__ void __launch_bounds__(64 * WPB) JG_EC_SCALAR_ATTR k_ec_scalar_batch(EcArgs a, int B) {
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L;
  const int64_t np = a.npad;
  const int64_t n = a.end - a.begin;
  const int64_t S = (n + B - 1) / B;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the class's first width run empties its exception list (k_ec_point appends
  // to it after this kernel; a separate memset would be one more dependent
  // launch on the lane, waiting for a free wave slot behind the modexps)
  if (a.exc_reset && i == 0) *a.exc_count = 0u;
  if (WPB == 1 && i >= S) return;                  // (blocks of several waves keep every thread for the barriers)
  uint32_t acc[L];
  mp::set_const<Fn>(acc, Fn::ONE);
  int nb = 0;
  constexpr int WG = ec_comb_w(CV::CLS, true), NG = ec_windows(CV::CLS, true);
  constexpr int WQ = CV::WQ, NQ = ec_windows_w(CV::CLS, CV::WQ);
#if JG_EC_SCALAR_PF
  // Both passes load token j+1's (pass 2: j-1's) words before computing token j.
  {
    ScalarRaw<CV> cur, nxt;
    int64_t p = a.begin + i;
    bool have = B > 0 && i < S && p < a.end;
    if (have) ec_scalar_load<CV>(a, p, cur);
    for (int j = 0; have; ++j) {
      const int64_t pn = p + S;
      const bool more = j + 1 < B && pn < a.end;
      if (more) ec_scalar_load<CV>(a, pn, nxt);
      uint32_t r[L], s[L], e[L], sm[L];
      const bool ok = ec_scalar_finish<CV>(a, p, cur, r, s, e);
      if (!ok && job_live(cur.jb)) a.status[p] = ST_REJECT;
      mp::to_mont<Fn>(sm, s);
      mp::mul<Fn>(acc, acc, sm);
#pragma unroll
      for (int k = 0; k < L; ++k) {
        a.u1w[(int64_t)k * np + p] = acc[k];
        a.u2w[(int64_t)k * np + p] = sm[k];
      }
      ++nb;
      if (!more) break;
      cur = nxt;
      p = pn;
    }
  }
  uint32_t inv[L];
  mp::block_inv<Fn, WPB>(inv, acc);
  if (nb > 0) {
    ScalarRaw2<CV> cur, nxt;
    int64_t p = a.begin + i + (int64_t)(nb - 1) * S;
    ec_scalar_load2<CV>(a, p, nb > 1 ? p - S : -1, cur);
    for (int j = nb - 1; j >= 0; --j) {
      if (j > 0) ec_scalar_load2<CV>(a, p - S, j > 1 ? p - 2 * S : -1, nxt);
      uint32_t w[L], r[L], e[L], u1[L], u2[L];
      mp::mul<Fn>(w, inv, cur.cprev);              // s_j^-1 R
      mp::mul<Fn>(inv, inv, cur.sm);
      mp::words_to_limbs<L, ScalarRaw<CV>::CW>(r, cur.rw);
      mp::words_to_limbs<L, ScalarRaw<CV>::EW>(e, cur.ew);
      mp::csub<Fn>(e);
      mp::mul<Fn>(u1, e, w); mp::csub<Fn>(u1);
      mp::mul<Fn>(u2, r, w); mp::csub<Fn>(u2);
      store_digit_rows<CV, WG, NG>(a, p, u1, 0);  // (the rare exact path recomputes u1, u2 itself)
      store_digit_rows<CV, WQ, NQ>(a, p, u2, NG);
      if (j == 0) break;
      cur = nxt;
      p -= S;
    }
  }
#else
  for (int j = 0; j < B && i < S; ++j) {
    const int64_t p = a.begin + i + (int64_t)j * S;
    if (p >= a.end) break;
    uint32_t r[L], s[L], e[L], sm[L];
    const bool ok = ec_scalar_inputs<CV>(a, p, r, s, e);
    if (!ok && job_live(a.jobs[p])) a.status[p] = ST_REJECT;
    mp::to_mont<Fn>(sm, s);
    mp::mul<Fn>(acc, acc, sm);
#pragma unroll
    for (int k = 0; k < L; ++k) {
      a.u1w[(int64_t)k * np + p] = acc[k];
      a.u2w[(int64_t)k * np + p] = sm[k];
    }
    ++nb;
  }
  uint32_t inv[L];
  mp::block_inv<Fn, WPB>(inv, acc);
  for (int j = nb - 1; j >= 0; --j) {
    const int64_t p = a.begin + i + (int64_t)j * S;
    uint32_t cprev[L], sm[L], w[L];
    if (j > 0) {
      const int64_t pp = p - S;
#pragma unroll
      for (int k = 0; k < L; ++k) cprev[k] = a.u1w[(int64_t)k * np + pp];
    } else {
      mp::set_const<Fn>(cprev, Fn::ONE);
    }
#pragma unroll
    for (int k = 0; k < L; ++k) sm[k] = a.u2w[(int64_t)k * np + p];
    mp::mul<Fn>(w, inv, cprev);                  // s_j^-1 R
    mp::mul<Fn>(inv, inv, sm);
    uint32_t r[L], e[L], u1[L], u2[L];
    ec_scalar_re<CV>(a, p, r, e);
    mp::mul<Fn>(u1, e, w); mp::csub<Fn>(u1);
    mp::mul<Fn>(u2, r, w); mp::csub<Fn>(u2);
    store_digit_rows<CV, WG, NG>(a, p, u1, 0);  // (the rare exact path recomputes u1, u2 itself)
    store_digit_rows<CV, WQ, NQ>(a, p, u2, NG);
  }
#endif
}

// ------------------------------------------------------------------ point ops
// Y3 = r t - Y1 hhh.  Fields with the column headroom (sum_ok) take both
// products under ONE Montgomery reduction: (r t + (KSUB - Y1) hhh) / R, with
// r, t < 3*2^28 limbs and KSUB - Y1 < 2^29, hhh < 2^28 (values < 6m, 6m, 4m,
// 2m: the sum is < 44 m^2, far below R m), so Y3 comes out normalized with no
// subtraction and no value fold.  P-384 keeps two special-form products.
template <class Fp>
constexpr bool sum_ok() {
  if constexpr (std::is_same<Fp, P384P>::value) {
    return false;
  } else {
    uint32_t kmax = 0;
    for (int j = 0; j < Fp::L; ++j) kmax = Fp::KSUB[j] > kmax ? Fp::KSUB[j] : kmax;
    double red = 0;
    if constexpr (Fp::NP1)
      for (int j = 1; j < Fp::L; ++j) red += (double)Fp::M1[j] / 16777216.0;
    else
      red = 16.0 * Fp::L;
    return 9.0 * Fp::L + Fp::L * (double)kmax / 268435456.0 + red + 1.0 < 256.0;
  }
}

template <class Fp>
__device__ __forceinline__ void y3_from(uint32_t* Y, const uint32_t* r, const uint32_t* t, const uint32_t* y1,
                                        const uint32_t* hhh) {
  constexpr int L = Fp::L;
  if constexpr (sum_ok<Fp>() && mp::use_ps<Fp>(2)) {
    uint32_t ny1[L];
    mp::neg<Fp>(ny1, y1);
    mp::mont_ps<Fp, 2>(Y, r, t, ny1, hhh);
  } else if constexpr (sum_ok<Fp>()) {
    uint32_t ny1[L];
    mp::neg<Fp>(ny1, y1);
    uint64_t T[2 * L];
    mp::prod<Fp>(T, r, t);
    mp::prod_acc<Fp>(T, ny1, hhh);
    mp::mont_reduce<Fp>(Y, T);
  } else {
    uint32_t u[L];
    mp::mulf<Fp>(Y, r, t);
    mp::mulf<Fp>(u, y1, hhh);
    mp::sub<Fp>(Y, Y, u); mp::freduce_lazy<Fp>(Y);
  }
}

// X3 = r^2 - hhh - 2v.  Fields with a column constant KX3 (P-256,
// tools/gen_field_consts.py XCOL) subtract inside r^2's high columns:
// (r^2 + (KX3 - hhh - 2v) R) / R, where KX3 = 8m has every limb >= 3(2^28-1),
// so KX3 - hhh - 2v >= 0 limb by limb.  X3 then comes out of the reduction
// with 28-bit limbs and value < 8m + r^2/R + (1 + 2^-24) m < 10m: no value
// fold.  Subtractions with X as the subtrahend use KSUBX (16m, covers < 10m).
template <class Fp, class = void>
struct has_kx3 : std::false_type {};
template <class Fp>
struct has_kx3<Fp, std::void_t<decltype(Fp::KX3)>> : std::true_type {};

template <class Fp>
__device__ __forceinline__ void x3_from(uint32_t* X, const uint32_t* r, const uint32_t* hhh, const uint32_t* v) {
  constexpr int L = Fp::L;
  if constexpr (has_kx3<Fp>::value && mp::use_ps<Fp>(3)) {
    uint32_t e[L];
#pragma unroll
    for (int j = 0; j < L; ++j) e[j] = Fp::KX3[j] - (hhh[j] + 2 * v[j]);
    mp::mont_ps<Fp, 3>(X, r, r, nullptr, nullptr, e);
  } else if constexpr (has_kx3<Fp>::value) {
    uint64_t T[2 * L];
    mp::sqprod<Fp>(T, r);
    const uint32_t c1 = (uint32_t)mp::opaque_sgpr(1);
#pragma unroll
    for (int j = 0; j < L; ++j) T[L + j] += (uint64_t)(Fp::KX3[j] - (hhh[j] + 2 * v[j])) * c1;
    mp::mont_reduce<Fp>(X, T);
  } else {
    uint32_t r2[L];
    mp::sqrf<Fp>(r2, r);
    mp::sub<Fp>(X, r2, hhh); mp::sub<Fp>(X, X, v); mp::sub<Fp>(X, X, v); mp::freduce_lazy<Fp>(X);
  }
}

// a - X for an X produced by x3_from (value < 10m on KX3 fields)
template <class Fp>
__device__ __forceinline__ void sub_x(uint32_t* r, const uint32_t* a, const uint32_t* x) {
  if constexpr (has_kx3<Fp>::value) {
#pragma unroll
    for (int j = 0; j < Fp::L; ++j) r[j] = a[j] + Fp::KSUBX[j] - x[j];
  } else {
    mp::sub<Fp>(r, a, x);
  }
}

// Mixed addition P1 (Jacobian; X < 10m on KX3 fields, else < 2m; Y, Z < 2m,
// 28-bit limbs) += P2 (affine x2, y2).
// 8M + 3S, lazy; X3, Y3 value-reduced so they can be subtrahends.
// Products go through mulf / sqrf (P-384: special-form reduction, which needs
// one operand with 28-bit limbs per product -- h and r are normalised for it).
// Z1Z1 is semi-normalized where the field allows (mp::sqr_semi): both its
// consumers multiply it by an operand with 28-bit limbs (x2, Z).
// An exceptional pair (P1 == +-P2) yields H == 0 and so Z3 == 0, which is
// absorbing in later additions and is detected at the end.
template <class Fp>
__device__ __forceinline__ void madd(uint32_t* X, uint32_t* Y, uint32_t* Z, const uint32_t* x2, const uint32_t* y2) {
  constexpr int L = Fp::L;
  uint32_t z1z1[L], u2[L], t[L], s2[L], h[L], r[L], hh[L], hhh[L], v[L];
  mp::sqr_semi<Fp>(z1z1, Z);
  mp::mulf<Fp>(u2, x2, z1z1);
  mp::mulf<Fp>(t, Z, z1z1);
  mp::mulf<Fp>(s2, y2, t);
  sub_x<Fp>(h, u2, X);
  mp::sub<Fp>(r, s2, Y);
  mp::norm_for_mulf<Fp>(h);                  // P-384: h, r are squared (mulf precondition)
  mp::norm_for_mulf<Fp>(r);
  mp::sqrf<Fp>(hh, h);
  mp::mulf<Fp>(Z, Z, h);                     // Z3 before hhh and v: h dies at hhh, hh at v
  mp::mulf<Fp>(hhh, h, hh);
  mp::mulf<Fp>(v, X, hh);
  uint32_t y1[L];
  mp::copy<Fp>(y1, Y);
  x3_from<Fp>(X, r, hhh, v);
  // Y3 = r (v - X3) - Y1 hhh
  sub_x<Fp>(t, v, X);
  y3_from<Fp>(Y, r, t, y1, hhh);
}

// madd with Z1 == 1 (P1 affine: the accumulator after its first assignment):
// u2 = x2, s2 = y2, Z3 = h -- 4M + 2S instead of 8M + 3S.
template <class Fp>
__device__ __forceinline__ void madd_z1(uint32_t* X, uint32_t* Y, uint32_t* Z, const uint32_t* x2, const uint32_t* y2) {
  constexpr int L = Fp::L;
  uint32_t h[L], r[L], hh[L], hhh[L], v[L], t[L], y1[L];
  mp::sub<Fp>(h, x2, X);
  mp::sub<Fp>(r, y2, Y);
  mp::norm<Fp>(h);                           // Z3 = h: 28-bit limbs (mulf operand), value < 6m
  mp::norm<Fp>(r);                           // y2 may be negated (limbs < 2^29): keep r^2's columns in range
  mp::sqrf<Fp>(hh, h);
  mp::mulf<Fp>(hhh, h, hh);
  mp::mulf<Fp>(v, X, hh);
  mp::copy<Fp>(Z, h);
  mp::copy<Fp>(y1, Y);
  x3_from<Fp>(X, r, hhh, v);
  sub_x<Fp>(t, v, X);
  y3_from<Fp>(Y, r, t, y1, hhh);
}

// A table entry (affine x, y; canonical Montgomery form): 2L limbs, or 16
// packed words for P-256 (ecdsa.hpp ec_packed)
template <class CV>
__device__ __forceinline__ void load_entry(const uint32_t* __restrict__ ent, uint32_t* x, uint32_t* y) {
  constexpr int L = CV::Fp::L;
  if constexpr (ec_packed(CV::CLS)) {
    const uint4* e4 = reinterpret_cast<const uint4*>(ent);
    const uint4 a = e4[0], b = e4[1], c = e4[2], d = e4[3];
    const uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t wy[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    mp::words_to_limbs<L, 8>(x, wx);
    mp::words_to_limbs<L, 8>(y, wy);
  } else {
#pragma unroll
    for (int j = 0; j < L; ++j) { x[j] = ent[j]; y[j] = ent[L + j]; }
  }
}

template <class CV>
__device__ __forceinline__ void store_entry(uint32_t* out, const uint32_t* x, const uint32_t* y) {
  constexpr int L = CV::Fp::L;
  if constexpr (ec_packed(CV::CLS)) {
    uint32_t w[16];
    mp::limbs_to_words<L, 8>(w, x);
    mp::limbs_to_words<L, 8>(w + 8, y);
#pragma unroll
    for (int j = 0; j < 16; ++j) out[j] = w[j];
  } else {
#pragma unroll
    for (int j = 0; j < L; ++j) { out[j] = x[j]; out[L + j] = y[j]; }
  }
}

// Z1ONE: the accumulator, if not empty, holds exactly one table entry (Z == 1)
template <class CV, bool GEN, bool Z1ONE = false>
__device__ __forceinline__ void add_window(uint32_t* X, uint32_t* Y, uint32_t* Z, bool& empty,
                                           const uint32_t* __restrict__ tab, int w, int d) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L, STRIDE = ec_stride(CV::CLS), NE = GEN ? ec_entries(CV::CLS, true) : 1 << (CV::WQ - 1);
  if (d == 0) return;
  const int ad = d < 0 ? -d : d;
  const uint32_t* ent = tab + ((int64_t)w * NE + (ad - 1)) * STRIDE;
  uint32_t x2[L], y2[L];
  load_entry<CV>(ent, x2, y2);
  if (d < 0) mp::neg<Fp>(y2, y2);
  if (empty) {
    mp::copy<Fp>(X, x2);
    mp::copy<Fp>(Y, y2); mp::freduce<Fp>(Y);
    mp::set_const<Fp>(Z, Fp::ONE);
    empty = false;
  } else if constexpr (Z1ONE) {
    madd_z1<Fp>(X, Y, Z, x2, y2);
  } else {
    madd<Fp>(X, Y, Z, x2, y2);
  }
}

// Packed (P-256) entries as raw words, for the one-entry-ahead loop of
// k_ec_point (JG_EC_POINT_PF): the loads of the next addition's entry are in
// flight while the current addition computes.
template <class CV>
__device__ __forceinline__ void load_raw(const uint32_t* __restrict__ ent, uint4* r) {
  const uint4* e4 = reinterpret_cast<const uint4*>(ent);
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = e4[i];
}
template <class CV, bool Z1ONE = false>
__device__ __forceinline__ void add_raw(uint32_t* X, uint32_t* Y, uint32_t* Z, bool& empty, const uint4* r, int d) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  if (d == 0) return;
  const uint32_t wx[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
  const uint32_t wy[8] = {r[2].x, r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
  uint32_t x2[L], y2[L];
  mp::words_to_limbs<L, 8>(x2, wx);
  mp::words_to_limbs<L, 8>(y2, wy);
  if (d < 0) mp::neg<Fp>(y2, y2);
  if (empty) {
    mp::copy<Fp>(X, x2);
    mp::copy<Fp>(Y, y2); mp::freduce<Fp>(Y);
    mp::set_const<Fp>(Z, Fp::ONE);
    empty = false;
  } else if constexpr (Z1ONE) {
    madd_z1<Fp>(X, Y, Z, x2, y2);
  } else {
    madd<Fp>(X, Y, Z, x2, y2);
  }
}
// JG_EC_POINT_PF=1 (P-256 at equal G / key widths): 128 VGPRs, still 4 waves
// per SIMD, point kernel 1.282-1.288 -> 1.270-1.284 ms per 1 M tokens
// (profiles/r04_s6/point_pf_ab.json) -- within noise, so off (A/B knob)
#ifndef JG_EC_POINT_PF
#define JG_EC_POINT_PF 0
#endif

// JG_EC_POINT_ATTR: per translation unit, as JG_EC_SCALAR_ATTR (occupancy A/Bs)
#ifndef JG_EC_POINT_ATTR
#define JG_EC_POINT_ATTR
#endif
template <class CV>
__global__ void __launch_bounds__(64) JG_EC_POINT_ATTR k_ec_point(EcArgs a) {
  using Fp = typename CV::Fp;
  using Fn = typename CV::Fn;
  constexpr int L = Fp::L;
  constexpr int NG = ec_windows(CV::CLS, true), NQ = ec_windows_w(CV::CLS, CV::WQ);
  constexpr int NWIN = NG > NQ ? NG : NQ;
  const int64_t p = a.begin + (int64_t)blockIdx.x * WAVE + threadIdx.x;
  const int64_t np = a.npad;
  const JobDev jb = a.jobs[p];
  if (!job_live(jb)) return;
  if (a.status[p] != ST_OK) { a.verdict_pad[p] = 0; return; }
  const int kidx = __builtin_amdgcn_readfirstlane(job_key(jb));
  const uint32_t* __restrict__ qtab = key_table(a.keys[kidx]);
  const uint32_t* __restrict__ gtab = a.gtab;

  uint32_t X[L], Y[L], Z[L];
  bool empty = true;
#if JG_EC_POINT_PF
  if constexpr (ec_packed(CV::CLS) && NG == NQ) {
    // additions k = 0 .. 2 NG - 1 alternate G window k/2 and Q window k/2;
    // digit k+2 and entry k+1 are loaded while addition k computes
    constexpr int NS = 2 * NG, STRIDE = ec_stride(CV::CLS);
    constexpr int NEG = ec_entries(CV::CLS, true), NEQ = 1 << (CV::WQ - 1);
    auto dig = [&](int k) { return (int)a.digs[(int64_t)((k & 1) ? NG + (k >> 1) : (k >> 1)) * np + p]; };
    auto ent = [&](int k, int d) {
      const int ad = d < 0 ? -d : d;
      const int64_t idx = ad == 0 ? 0 : ad - 1;          // a zero digit adds nothing (its load is harmless)
      return (k & 1) ? qtab + ((int64_t)(k >> 1) * NEQ + idx) * STRIDE : gtab + ((int64_t)(k >> 1) * NEG + idx) * STRIDE;
    };
    uint4 rc[4], rn[4];
    int dc = dig(0), dn = dig(1);
    load_raw<CV>(ent(0, dc), rc);
    load_raw<CV>(ent(1, dn), rn);
    int dnn = dig(2);
    add_raw<CV>(X, Y, Z, empty, rc, dc);                 // window 0: G is an assignment,
#pragma unroll
    for (int i = 0; i < 4; ++i) rc[i] = rn[i];
    dc = dn; dn = dnn;
    load_raw<CV>(ent(2, dn), rn);
    dnn = dig(3);
    add_raw<CV, true>(X, Y, Z, empty, rc, dc);           // so Q adds onto Z == 1
    for (int k = 2; k < NS; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i) rc[i] = rn[i];
      dc = dn; dn = dnn;
      if (k + 1 < NS) load_raw<CV>(ent(k + 1, dn), rn);
      if (k + 2 < NS) dnn = dig(k + 2);
      add_raw<CV>(X, Y, Z, empty, rc, dc);
    }
  } else
#endif
  {
  // window 0 peeled: its G entry is an assignment, so its Q entry adds onto Z == 1
  add_window<CV, true>(X, Y, Z, empty, gtab, 0, (int)a.digs[p]);
  add_window<CV, false, true>(X, Y, Z, empty, qtab, 0, (int)a.digs[(int64_t)NG * np + p]);
  for (int w = 1; w < NWIN; ++w) {
    if (w < NG) add_window<CV, true>(X, Y, Z, empty, gtab, w, (int)a.digs[(int64_t)w * np + p]);
    if (w < NQ) add_window<CV, false>(X, Y, Z, empty, qtab, w, (int)a.digs[(int64_t)(NG + w) * np + p]);
  }
  }
  if (empty) { a.verdict_pad[p] = 0; return; }           // R = infinity (unreachable: u2 != 0)
  uint32_t zc[L];
  mp::copy<Fp>(zc, Z);
  mp::canon<Fp>(zc);
  if (mp::is_zero_canon<Fp>(zc)) {                        // exceptional case: exact recompute
    const uint32_t idx = atomicAdd(a.exc_count, 1u);
    a.exc_list[idx] = (int32_t)p;
    a.status[p] = ST_EXCEPTIONAL;
    return;
  }
  // x(R) mod n == r  <=>  X == r Z^2  or  (r + n < p and X == (r + n) Z^2)
  constexpr int CW = ec_sig_words(CV::CLS);
  uint32_t rw[CW], r[L];
#pragma unroll
  for (int q = 0; q < CW; ++q) rw[q] = a.sigw[(int64_t)q * np + p];
  mp::words_to_limbs<L, CW>(r, rw);
  uint32_t zz[L], rm[L], tt[L];
  mp::sqr<Fp>(zz, Z);
  mp::to_mont<Fp>(rm, r);
  mp::mul<Fp>(tt, rm, zz);
  bool ok = mp::eq_mod<Fp>(X, tt);
  if (!ok) {
    uint32_t rn[L], pl[L];
    mp::add<Fp>(rn, r, Fn::M);
    mp::norm<Fp>(rn);
    mp::set_const<Fp>(pl, Fp::M);
    if (lt_limbs<L>(rn, pl)) {
      mp::to_mont<Fp>(rm, rn);
      mp::mul<Fp>(tt, rm, zz);
      ok = mp::eq_mod<Fp>(X, tt);
    }
  }
  a.verdict_pad[p] = ok;
}

// ------------------------------------------------------------------ exact path
// Jacobian points with an explicit infinity flag; every coordinate kept
// normalized (< 2p) so any of them can be a subtrahend.
template <class Fp>
struct JPt { uint32_t X[Fp::L], Y[Fp::L], Z[Fp::L]; bool inf; };

template <class Fp>
__device__ bool is_zero_mod(const uint32_t* a) {
  uint32_t c[Fp::L];
  mp::copy<Fp>(c, a);
  mp::canon<Fp>(c);
  return mp::is_zero_canon<Fp>(c);
}

template <class Fp>
__device__ void times2(uint32_t* r, const uint32_t* a) {     // r = 2a, normalized
  mp::add<Fp>(r, a, a);
  mp::freduce<Fp>(r);
}

template <class CV>
__device__ void jdbl(JPt<typename CV::Fp>& R, const JPt<typename CV::Fp>& P) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  if (P.inf || is_zero_mod<Fp>(P.Y)) { R.inf = true; return; }
  uint32_t delta[L], gamma[L], beta[L], t1[L], t2[L], alpha[L], b2[L], b4[L], b8[L], x3[L], y3[L], z3[L];
  mp::sqr<Fp>(delta, P.Z);
  mp::sqr<Fp>(gamma, P.Y);
  mp::mul<Fp>(beta, P.X, gamma);
  mp::sub<Fp>(t1, P.X, delta);
  mp::add<Fp>(t2, P.X, delta);
  mp::mul<Fp>(alpha, t1, t2);
  uint32_t three[L];
  mp::set_const<Fp>(three, CV::C::THREE_M);
  mp::mul<Fp>(alpha, alpha, three);                 // 3 (X - delta)(X + delta)
  times2<Fp>(b2, beta); times2<Fp>(b4, b2); times2<Fp>(b8, b4);
  mp::sqr<Fp>(x3, alpha);
  mp::sub<Fp>(x3, x3, b8); mp::freduce<Fp>(x3);     // X3 = alpha^2 - 8 beta
  mp::mul<Fp>(z3, P.Y, P.Z);
  times2<Fp>(z3, z3);                               // Z3 = 2 Y Z
  mp::sub<Fp>(t1, b4, x3);
  mp::mul<Fp>(y3, alpha, t1);
  mp::sqr<Fp>(t2, gamma);
  times2<Fp>(t2, t2); times2<Fp>(t2, t2); times2<Fp>(t2, t2);
  mp::sub<Fp>(y3, y3, t2); mp::freduce<Fp>(y3);     // Y3 = alpha (4 beta - X3) - 8 gamma^2
  mp::copy<Fp>(R.X, x3); mp::copy<Fp>(R.Y, y3); mp::copy<Fp>(R.Z, z3);
  R.inf = false;
}

template <class CV>
__device__ void jadd(JPt<typename CV::Fp>& R, const JPt<typename CV::Fp>& P, const JPt<typename CV::Fp>& Q) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  if (P.inf) { R = Q; return; }
  if (Q.inf) { R = P; return; }
  uint32_t z1z1[L], z2z2[L], u1[L], u2[L], s1[L], s2[L], t[L], h[L], rr[L];
  mp::sqr<Fp>(z1z1, P.Z); mp::sqr<Fp>(z2z2, Q.Z);
  mp::mul<Fp>(u1, P.X, z2z2); mp::mul<Fp>(u2, Q.X, z1z1);
  mp::mul<Fp>(t, Q.Z, z2z2); mp::mul<Fp>(s1, P.Y, t);
  mp::mul<Fp>(t, P.Z, z1z1); mp::mul<Fp>(s2, Q.Y, t);
  mp::sub<Fp>(h, u2, u1); mp::freduce<Fp>(h);
  mp::sub<Fp>(rr, s2, s1); mp::freduce<Fp>(rr);
  if (is_zero_mod<Fp>(h)) {
    if (is_zero_mod<Fp>(rr)) { jdbl<CV>(R, P); return; }
    R.inf = true;
    return;
  }
  uint32_t hh[L], hhh[L], v[L], x3[L], y3[L], z3[L];
  mp::sqr<Fp>(hh, h); mp::mul<Fp>(hhh, h, hh); mp::mul<Fp>(v, u1, hh);
  mp::add<Fp>(t, hhh, v); mp::add<Fp>(t, t, v); mp::freduce<Fp>(t);
  mp::sqr<Fp>(x3, rr); mp::sub<Fp>(x3, x3, t); mp::freduce<Fp>(x3);
  mp::sub<Fp>(t, v, x3); mp::mul<Fp>(y3, rr, t);
  mp::mul<Fp>(t, s1, hhh); mp::sub<Fp>(y3, y3, t); mp::freduce<Fp>(y3);
  mp::mul<Fp>(t, P.Z, Q.Z); mp::mul<Fp>(z3, t, h);
  mp::copy<Fp>(R.X, x3); mp::copy<Fp>(R.Y, y3); mp::copy<Fp>(R.Z, z3);
  R.inf = false;
}

template <class CV>
__device__ void affine_point(JPt<typename CV::Fp>& P, const uint32_t* xm, const uint32_t* ym) {
  using Fp = typename CV::Fp;
  mp::copy<Fp>(P.X, xm); mp::copy<Fp>(P.Y, ym); mp::set_const<Fp>(P.Z, Fp::ONE);
  P.inf = false;
}

// x(u1 G + u2 Q) mod n == r by double-and-add with complete case handling
// (the exceptional tokens of the fast sums; Q's affine Montgomery coordinates
// at aux; u1, u2, r canonical plain limbs)
template <class CV>
__device__ bool ec_exact_ok(const uint32_t* aux, const uint32_t* r, const uint32_t* u1, const uint32_t* u2) {
  using Fp = typename CV::Fp;
  using Fn = typename CV::Fn;
  constexpr int L = Fp::L;
  {
    JPt<Fp> G, Q, GQ, R;
    uint32_t gx[L], gy[L];
    mp::set_const<Fp>(gx, CV::C::GX_M); mp::set_const<Fp>(gy, CV::C::GY_M);
    affine_point<CV>(G, gx, gy);
    affine_point<CV>(Q, aux, aux + L);
    jadd<CV>(GQ, G, Q);
    R.inf = true;
    for (int b = Fn::BITS - 1; b >= 0; --b) {
      jdbl<CV>(R, R);
      const int q = b / MP_W, sh = b % MP_W;
      const bool b1 = (u1[q] >> sh) & 1u, b2 = (u2[q] >> sh) & 1u;
      if (b1 && b2) jadd<CV>(R, R, GQ);
      else if (b1) jadd<CV>(R, R, G);
      else if (b2) jadd<CV>(R, R, Q);
    }
    bool ok = false;
    if (!R.inf) {
      uint32_t zi[L], zi2[L], xa[L], x[L];
      mp::inv<Fp>(zi, R.Z);
      mp::sqr<Fp>(zi2, zi);
      mp::mul<Fp>(xa, R.X, zi2);
      mp::from_mont<Fp>(x, xa);                  // canonical x < p
      // x mod n (x < p < 2n)
      uint32_t nl[L], d[L];
      mp::set_const<Fp>(nl, Fn::M);
      if (!lt_limbs<L>(x, nl)) {
        int32_t br = 0;
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int32_t tt = (int32_t)x[j] - (int32_t)nl[j] + br;
          d[j] = (uint32_t)tt & MP_MASK;
          br = tt >> MP_W;
        }
        mp::copy<Fp>(x, d);
      }
      uint32_t o = 0;
#pragma unroll
      for (int j = 0; j < L; ++j) o |= x[j] ^ r[j];
      ok = o == 0;
    }
    return ok;
  }
}

template <class CV>
__global__ void __launch_bounds__(64) k_ec_exact(EcArgs a) {
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L;
  const uint32_t cnt = *a.exc_count;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const int64_t p = a.exc_list[i];
    const int kidx = job_key(a.jobs[p]);
    const uint32_t* aux = a.keyblob + a.keys[kidx].aux_off;
    // u1 = e / s, u2 = r / s (mod n), recomputed with one inversion per token
    // (the status goes back to OK first: ec_scalar_inputs checks it)
    a.status[p] = ST_OK;
    uint32_t r[L], s[L], e[L], sm[L], w[L], u1[L], u2[L];
    (void)ec_scalar_inputs<CV>(a, p, r, s, e);
    mp::to_mont<Fn>(sm, s);
    mp::inv<Fn>(w, sm);                          // s^-1 R
    mp::mul<Fn>(u1, e, w); mp::csub<Fn>(u1);
    mp::mul<Fn>(u2, r, w); mp::csub<Fn>(u2);
    a.verdict_pad[p] = ec_exact_ok<CV>(aux, r, u1, u2);
    a.status[p] = ST_OK;
  }
}

// ------------------------------------------------------------------ split point (small launches)
// k_ec_point with S lanes per token, for launches that fill the GPU poorly
// (a coalesced single-token batch, a mixed batch's small EC classes): lane s
// of a token sums the comb windows w = s, s + S, ... of both scalars into its
// own Jacobian partial (the fast madd chain; a partial with Z == 0 is
// exceptional, as in k_ec_point), and the partials are combined pairwise
// across lanes with the exact addition (jadd: doubling and infinity handled).
// S partial chains of NWIN / S additions run side by side, so a token's
// latency is ~1/S of k_ec_point's plus log2(S) additions; the work per token
// grows by those additions and the conversions to normalized form.
// Raw table entry for the prefetching chain: the packed words (P-256) or the
// 2L limbs, converted at use
template <class CV>
struct RawEnt {
  static constexpr int NW = ec_packed(CV::CLS) ? 16 : 2 * CV::Fp::L;
  uint32_t w[NW];
};
template <class CV>
__device__ __forceinline__ void load_ent(RawEnt<CV>& r, const uint32_t* __restrict__ ent) {
  if constexpr (RawEnt<CV>::NW % 4 == 0) {
    const uint4* e4 = reinterpret_cast<const uint4*>(ent);
#pragma unroll
    for (int i = 0; i < RawEnt<CV>::NW / 4; ++i) {
      const uint4 q = e4[i];
      r.w[4 * i] = q.x; r.w[4 * i + 1] = q.y; r.w[4 * i + 2] = q.z; r.w[4 * i + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < RawEnt<CV>::NW; ++i) r.w[i] = ent[i];
  }
}
template <class CV>
__device__ __forceinline__ void add_ent(uint32_t* X, uint32_t* Y, uint32_t* Z, bool& empty, const RawEnt<CV>& r, int d) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  if (d == 0) return;
  uint32_t x2[L], y2[L];
  if constexpr (ec_packed(CV::CLS)) {
    mp::words_to_limbs<L, 8>(x2, r.w);
    mp::words_to_limbs<L, 8>(y2, r.w + 8);
  } else {
#pragma unroll
    for (int j = 0; j < L; ++j) { x2[j] = r.w[j]; y2[j] = r.w[L + j]; }
  }
  if (d < 0) mp::neg<Fp>(y2, y2);
  if (empty) {
    mp::copy<Fp>(X, x2);
    mp::copy<Fp>(Y, y2); mp::freduce<Fp>(Y);
    mp::set_const<Fp>(Z, Fp::ONE);
    empty = false;
  } else {
    madd<Fp>(X, Y, Z, x2, y2);
  }
}

// PF (launches of about one wave per SIMD, JG_EC_PF_MAX): the lane's chain
// of additions runs one table entry and two digits ahead -- addition j
// computes while entry j + 1 and digit j + 2 load.  With no other wave on the
// SIMD to switch to, each addition otherwise waited on a digit load and then
// on the dependent entry gather.
template <class CV, int S, bool PF = false>
__global__ void __launch_bounds__(64) k_ec_point_split(EcArgs a) {
  using Fp = typename CV::Fp;
  using Fn = typename CV::Fn;
  constexpr int L = Fp::L;
  constexpr int NG = ec_windows(CV::CLS, true), NQ = ec_windows_w(CV::CLS, CV::WQ);
  constexpr int NWIN = NG > NQ ? NG : NQ;
  const int lane = threadIdx.x, sub = lane % S;
  const int64_t p = a.begin + (int64_t)blockIdx.x * (WAVE / S) + lane / S;
  const int64_t np = a.npad;
  bool live = p < a.end;
  JobDev jb{};
  if (live) jb = a.jobs[p];
  live = live && job_live(jb);
  const bool ok_status = live && a.status[p] == ST_OK;
  if (live && !ok_status && sub == 0) a.verdict_pad[p] = 0;
  const bool run = ok_status;                     // the S lanes of a token agree
  // (every lane stays for the cross-lane exchanges below; idle lanes compute nothing)
  JPt<Fp> P;
  bool exc = false;
  P.inf = true;
  if (run) {
    const int kidx = job_key(jb);
    const uint32_t* __restrict__ qtab = key_table(a.keys[kidx]);
    const uint32_t* __restrict__ gtab = a.gtab;
    uint32_t X[L], Y[L], Z[L];
    bool empty = true;
    if constexpr (PF) {
      // step j: window sub + S (j / 2), the G comb (even j) or the Q comb (odd j)
      constexpr int STRIDE = ec_stride(CV::CLS), NEG = ec_entries(CV::CLS, true), NEQ = 1 << (CV::WQ - 1);
      const int nsteps = sub < NWIN ? 2 * ((NWIN - sub + S - 1) / S) : 0;
      auto dig = [&](int j) {
        const int w = sub + S * (j >> 1);
        const bool q = j & 1;
        return w < (q ? NQ : NG) ? (int)a.digs[(int64_t)(q ? NG + w : w) * np + p] : 0;
      };
      auto ent = [&](int j, int d) {
        const int ad = d < 0 ? -d : d;
        const int w = ad ? sub + S * (j >> 1) : 0;      // a zero digit loads window 0's first entry (unused)
        const int64_t i = ad ? ad - 1 : 0;
        return (j & 1) ? qtab + ((int64_t)w * NEQ + i) * STRIDE : gtab + ((int64_t)w * NEG + i) * STRIDE;
      };
      RawEnt<CV> rn;
      int dn = nsteps > 0 ? dig(0) : 0, dnn = nsteps > 1 ? dig(1) : 0;
      if (nsteps > 0) load_ent<CV>(rn, ent(0, dn));
#pragma unroll 1
      for (int j = 0; j < nsteps; ++j) {
        const RawEnt<CV> rc = rn;
        const int dc = dn;
        dn = dnn;
        if (j + 1 < nsteps) load_ent<CV>(rn, ent(j + 1, dn));
        if (j + 2 < nsteps) dnn = dig(j + 2);
        add_ent<CV>(X, Y, Z, empty, rc, dc);
      }
    } else {
    for (int w = sub; w < NWIN; w += S) {
      if (w < NG) add_window<CV, true>(X, Y, Z, empty, gtab, w, (int)a.digs[(int64_t)w * np + p]);
      if (w < NQ) add_window<CV, false>(X, Y, Z, empty, qtab, w, (int)a.digs[(int64_t)(NG + w) * np + p]);
    }
    }
    if (!empty) {
      mp::canon<Fp>(X); mp::canon<Fp>(Y); mp::canon<Fp>(Z);
      exc = mp::is_zero_canon<Fp>(Z);            // an exceptional step in this lane's chain
      mp::copy<Fp>(P.X, X); mp::copy<Fp>(P.Y, Y); mp::copy<Fp>(P.Z, Z);
      P.inf = false;
    }
  }
#pragma unroll 1
  for (int off = 1; off < S; off <<= 1) {
    JPt<Fp> Q;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      Q.X[j] = __shfl_xor(P.X[j], off);
      Q.Y[j] = __shfl_xor(P.Y[j], off);
      Q.Z[j] = __shfl_xor(P.Z[j], off);
    }
    Q.inf = __shfl_xor((int)P.inf, off) != 0;
    const int pexc = __shfl_xor((int)exc, off);    // every lane reads (see ec_small.hpp jadd_pair)
    exc = exc || pexc != 0;
    if (run && (sub & off) == 0 && !exc) jadd<CV>(P, P, Q);
  }
  if (!run || sub != 0) return;
  if (exc) {                                      // exact recompute (k_ec_exact)
    const uint32_t idx = atomicAdd(a.exc_count, 1u);
    a.exc_list[idx] = (int32_t)p;
    a.status[p] = ST_EXCEPTIONAL;
    return;
  }
  if (P.inf) { a.verdict_pad[p] = 0; return; }    // R = infinity: rejected
  // x(R) mod n == r  <=>  X == r Z^2  or  (r + n < p and X == (r + n) Z^2)
  constexpr int CW = ec_sig_words(CV::CLS);
  uint32_t rw[CW], r[L];
#pragma unroll
  for (int q = 0; q < CW; ++q) rw[q] = a.sigw[(int64_t)q * np + p];
  mp::words_to_limbs<L, CW>(r, rw);
  uint32_t zz[L], rm[L], tt[L];
  mp::sqr<Fp>(zz, P.Z);
  mp::to_mont<Fp>(rm, r);
  mp::mul<Fp>(tt, rm, zz);
  bool ok = mp::eq_mod<Fp>(P.X, tt);
  if (!ok) {
    uint32_t rn[L], pl[L];
    mp::add<Fp>(rn, r, Fn::M);
    mp::norm<Fp>(rn);
    mp::set_const<Fp>(pl, Fp::M);
    if (lt_limbs<L>(rn, pl)) {
      mp::to_mont<Fp>(rm, rn);
      mp::mul<Fp>(tt, rm, zz);
      ok = mp::eq_mod<Fp>(P.X, tt);
    }
  }
  a.verdict_pad[p] = ok;
}

// ------------------------------------------------------------------ staging
// thread per key: validate (coordinates < p, on the curve) and convert to Montgomery
template <class CV>
__global__ void k_ec_keyprep(DevKey* keys, uint32_t* blob, const int32_t* idx, int n) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DevKey& K = keys[idx[i]];
  uint32_t* aux = blob + K.aux_off;
  uint32_t x[L], y[L], pl[L];
#pragma unroll
  for (int j = 0; j < L; ++j) { x[j] = aux[j]; y[j] = aux[L + j]; }
  mp::set_const<Fp>(pl, Fp::M);
  bool ok = K.valid && lt_limbs<L>(x, pl) && lt_limbs<L>(y, pl);
  uint32_t xm[L], ym[L], lhs[L], rhs[L], t[L], three[L], b[L];
  mp::to_mont<Fp>(xm, x);
  mp::to_mont<Fp>(ym, y);
  mp::sqr<Fp>(lhs, ym);
  mp::sqr<Fp>(t, xm); mp::mul<Fp>(rhs, t, xm);
  mp::set_const<Fp>(three, CV::C::THREE_M);
  mp::mul<Fp>(t, xm, three);
  mp::sub<Fp>(rhs, rhs, t);
  mp::set_const<Fp>(b, CV::C::B_M);
  mp::add<Fp>(rhs, rhs, b);
  ok = ok && mp::eq_mod<Fp>(rhs, lhs);
  mp::canon<Fp>(xm); mp::canon<Fp>(ym);
#pragma unroll
  for (int j = 0; j < L; ++j) { aux[j] = xm[j]; aux[L + j] = ym[j]; }
  K.valid = ok ? 1 : 0;
}

template <class CV>
__device__ void store_affine(uint32_t* out, const JPt<typename CV::Fp>& P) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  uint32_t zi[L], zi2[L], zi3[L], x[L], y[L];
  mp::inv<Fp>(zi, P.Z);
  mp::sqr<Fp>(zi2, zi);
  mp::mul<Fp>(zi3, zi2, zi);
  mp::mul<Fp>(x, P.X, zi2);
  mp::mul<Fp>(y, P.Y, zi3);
  mp::canon<Fp>(x); mp::canon<Fp>(y);
  store_entry<CV>(out, x, y);
}

// window base 2^(W w) * B (= entry d = 1 of window w), affine Montgomery form
template <class CV, int W>
__device__ void window_base(uint32_t* out, const uint32_t* bx, const uint32_t* by, int w) {
  using Fp = typename CV::Fp;
  JPt<Fp> P;
  affine_point<CV>(P, bx, by);
  for (int i = 0; i < W * w; ++i) jdbl<CV>(P, P);
  store_affine<CV>(out, P);
}

// entry d * base (d < 2^W), affine Montgomery form
template <class CV, int W>
__device__ void table_entry(uint32_t* out, const uint32_t* base, int d) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  JPt<Fp> P, acc;
  uint32_t bx[L], by[L];
  load_entry<CV>(base, bx, by);
  affine_point<CV>(P, bx, by);
  acc.inf = true;
  for (int bit = W - 1; bit >= 0; --bit) {
    jdbl<CV>(acc, acc);
    if ((d >> bit) & 1) jadd<CV>(acc, acc, P);
  }
  store_affine<CV>(out, acc);
}

// Tables are built in two launches: thread per (key, window) for the window
// bases (entry 1), then thread per (key, entry >= 2) from its window's base.
template <class CV>
__global__ void k_ec_table_base_keys(const DevKey* keys, uint32_t* blob, const int32_t* idx, int n) {
  constexpr int W = CV::WQ, NWIN = ec_windows_w(CV::CLS, CV::WQ);
  constexpr int NE = 1 << (CV::WQ - 1), STRIDE = ec_stride(CV::CLS);
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (k >= n || w >= NWIN) return;
  const DevKey& K = keys[idx[k]];
  if (!K.valid) return;
  const uint32_t* aux = blob + K.aux_off;
  window_base<CV, W>((uint32_t*)K.tab + (int64_t)w * NE * STRIDE, aux, aux + CV::Fp::L, w);
}

template <class CV>
__global__ void k_ec_table_keys(const DevKey* keys, uint32_t* blob, const int32_t* idx, int n, int e0, int e1) {
  constexpr int W = CV::WQ, NWIN = ec_windows_w(CV::CLS, CV::WQ);
  constexpr int NE = 1 << (CV::WQ - 1), STRIDE = ec_stride(CV::CLS);
  const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (k >= n || e >= e1 || e >= NWIN * NE || e % NE == 0) return;
  const DevKey& K = keys[idx[k]];
  if (!K.valid) return;
  uint32_t* tab = (uint32_t*)K.tab;
  table_entry<CV, W>(tab + (int64_t)e * STRIDE, tab + (int64_t)(e / NE) * NE * STRIDE, e % NE + 1);
}

template <class CV>
__global__ void k_ec_table_base_g(uint32_t* tab) {
  constexpr int W = ec_comb_w(CV::CLS, true), NWIN = ec_windows(CV::CLS, true);
  constexpr int NE = ec_entries(CV::CLS, true), STRIDE = ec_stride(CV::CLS);
  using Fp = typename CV::Fp;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= NWIN) return;
  uint32_t gx[Fp::L], gy[Fp::L];
  mp::set_const<Fp>(gx, CV::C::GX_M); mp::set_const<Fp>(gy, CV::C::GY_M);
  window_base<CV, W>(tab + (int64_t)w * NE * STRIDE, gx, gy, w);
}

template <class CV>
__global__ void k_ec_table_g(uint32_t* tab) {
  constexpr int W = ec_comb_w(CV::CLS, true), NWIN = ec_windows(CV::CLS, true);
  constexpr int NE = ec_entries(CV::CLS, true), STRIDE = ec_stride(CV::CLS);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= NWIN * NE || e % NE == 0) return;
  table_entry<CV, W>(tab + (int64_t)e * STRIDE, tab + (int64_t)(e / NE) * NE * STRIDE, e % NE + 1);
}

// Launches of up to EC_SPLIT_MAX_TOKENS padded tokens run k_ec_point_split
// with EC_SPLIT lanes per token.  Measured (profiles/r05_s2/split_ab/): a lone
// ES256 batch of 1 ... 4096 tokens 238 -> 183 us (4 lanes; 2 lanes: 198 us),
// 16 coalesced single-token callers 45 k -> 60 k calls/s; but the configs[4]
// classes (62.5 k tokens per launch) ran slower split (P-256 point 0.31 ->
// 0.26 of the MAD roofline at 4 lanes, P-384 0.40 -> 0.31; 2 lanes: P-256 0.34,
// P-384 0.38, the batch 82.1 -> 81.2 M/s), so only small launches split.
#ifndef JG_EC_SPLIT
#define JG_EC_SPLIT 4
#endif
#ifndef JG_EC_SCALAR_SOLO_MAX
#define JG_EC_SCALAR_SOLO_MAX 16384
#endif
constexpr int64_t EC_SCALAR_SOLO_MAX = JG_EC_SCALAR_SOLO_MAX;   // launches up to this size: k_ec_scalar_batch<CV, 1>
#ifndef JG_EC_SPLIT_MAX
#define JG_EC_SPLIT_MAX 16384
#endif
// P-256 launches of 16 k ... JG_EC_SPLIT2_P256 tokens run two lanes per token
// (round 5: point 0.30 -> 0.34-0.35 of the MAD roofline at configs[4],
// profiles/r05_s2/q_ab/), with the prefetch (PF below).  On one key at W = 24
// the one-lane PF chain was faster (62 k tokens 0.1325 -> 0.1046 ms,
// profiles/r06_s16/pf3.txt), but in configs[4] -- four keys at W = 26, 86 GB
// of key tables, so slower gathers -- the class took 0.161 ms one-lane
// against 0.153 two-lane (profiles/r06_s17 vs r06_s16/cfg_head.json): the
// second wave per SIMD hides more of the gather than one entry of prefetch.
#ifndef JG_EC_SPLIT2_P256
#define JG_EC_SPLIT2_P256 131072
#endif
constexpr int64_t EC_SPLIT2_MAX_P256 = JG_EC_SPLIT2_P256;
// Launches above the split sizes and up to JG_EC_PF_MAX padded tokens (a
// mixed batch's EC classes, ~1-4 waves per SIMD) run the prefetching chain:
// k_ec_point_split<CV, 2, true> for P-256 up to EC_SPLIT2_MAX_P256, <CV, 1,
// true> otherwise (one lane per token, as k_ec_point)
// (262 k-token launches: P-256 point 0.3467 -> 0.3428 ms, P-384 1.150 ->
// 1.146 ms with it, profiles/r06_s16/pf4.txt; the 1 M headline launch keeps
// k_ec_point and its four waves per SIMD)
#ifndef JG_EC_PF_MAX
#define JG_EC_PF_MAX 262144
#endif
constexpr int64_t EC_PF_MAX_TOKENS = JG_EC_PF_MAX;
// JG_EC_SPLIT_PF: the prefetching chain in the small-launch split too (lone
// ES256 chain batches of 256 / 2048 / 8000 tokens: p50 163 -> 157, 182 -> 179,
// 269 -> 267 us; profiles/r06_s20/pf5.txt).  Off: the two-slot multi-device
// leg, whose chunk ramp starts with split-size launches, read 105.6 / 98.3 /
// 79.7 M/s with it against 104.5-106.4 without (profiles/r06_s20/md_ab.txt)
#ifndef JG_EC_SPLIT_PF
#define JG_EC_SPLIT_PF 0
#endif
constexpr int EC_SPLIT = JG_EC_SPLIT;                    // lanes per token of k_ec_point_split
constexpr int64_t EC_SPLIT_MAX_TOKENS = JG_EC_SPLIT_MAX;  // launches up to this many padded tokens use it

template <class CV>
void launch_chain(const EcArgs& a, hipStream_t s, const Marker& mk) {
  const int64_t waves = (a.end - a.begin) / WAVE;
  dim3 g((unsigned)waves), b(WAVE);
  if (a.part == EC_EXACT) {
    hipLaunchKernelGGL(k_ec_exact<CV>, dim3(64), b, 0, s, a);
    mk("exact");
    return;
  }
  // tokens per thread for the batched inversion: keep >= ~8 waves per CU
  // (profiles/r04_s3/scalar_occupancy_ab.json: more waves, fewer tokens per
  // inversion, measured 12-26 % slower)
  const int64_t n = a.end - a.begin;
  constexpr int wpc = 8;
  int B = (int)std::min<int64_t>(16, std::max<int64_t>(1, n / (256 * wpc * WAVE)));
  const int64_t S = (n + B - 1) / B;
  if (n <= EC_SCALAR_SOLO_MAX) {
    // a small launch: one inversion per wave, no block barrier (the shared
    // inversion saves inversions only when the chip is full)
    hipLaunchKernelGGL((k_ec_scalar_batch<CV, 1>), dim3((unsigned)((S + WAVE - 1) / WAVE)), dim3(WAVE), 0, s, a, B);
  } else {
    constexpr int TPB = WAVE * EC_SCALAR_WPB;
    hipLaunchKernelGGL(k_ec_scalar_batch<CV>, dim3((unsigned)((S + TPB - 1) / TPB)), dim3(TPB), 0, s, a, B);
  }
  mk("scalar");
  // a launch of fewer waves than ~2 per SIMD runs its tokens S lanes each
  // (k_ec_point_split): one wave per SIMD leaves the madd chain's latency bare
  bool launched = false;
  if (n <= EC_SPLIT_MAX_TOKENS) {
    hipLaunchKernelGGL((k_ec_point_split<CV, EC_SPLIT, JG_EC_SPLIT_PF != 0>),
                       dim3((unsigned)((n * EC_SPLIT + WAVE - 1) / WAVE)), b, 0, s, a);
    launched = true;
  }
  if constexpr (CV::CLS == jgk::CLS_P256 && EC_SPLIT2_MAX_P256 > 0) {
    if (!launched && n <= EC_SPLIT2_MAX_P256) {
      if (n <= EC_PF_MAX_TOKENS)
        hipLaunchKernelGGL((k_ec_point_split<CV, 2, true>), dim3((unsigned)((n * 2 + WAVE - 1) / WAVE)), b, 0, s, a);
      else
        hipLaunchKernelGGL((k_ec_point_split<CV, 2>), dim3((unsigned)((n * 2 + WAVE - 1) / WAVE)), b, 0, s, a);
      launched = true;
    }
  }
  // P-521's chain takes 256 VGPRs with the prefetch (one wave per SIMD, 200
  // without): only launches of under ~one wave per SIMD
  constexpr int64_t pf_max = CV::CLS == jgk::CLS_P521 ? std::min<int64_t>(EC_PF_MAX_TOKENS, 65536) : EC_PF_MAX_TOKENS;
  if (!launched && n <= pf_max) {
    hipLaunchKernelGGL((k_ec_point_split<CV, 1, true>), dim3((unsigned)((n + WAVE - 1) / WAVE)), b, 0, s, a);
    launched = true;
  }
  if (!launched) hipLaunchKernelGGL(k_ec_point<CV>, g, b, 0, s, a);
  mk("point");
  if (a.part == EC_FAST) return;
  hipLaunchKernelGGL(k_ec_exact<CV>, dim3(64), b, 0, s, a);
  mk("exact");
}

// key staging: validate + Montgomery form (width-independent)
template <class CV>
void keyprep_chain(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_ec_keyprep<CV>, dim3((n + 63) / 64), dim3(64), 0, s, keys, blob, idx, n);
}

// comb tables of keys tidx[0..tn) at CV::WQ, written to each key's `tab`;
// `sliced`: the entries in launches of TABLE_SLICE threads, the stream
// synchronised after each (table_slices)
template <class CV>
void keytables_chain(DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s, bool sliced) {
  constexpr int NWIN = ec_windows_w(CV::CLS, CV::WQ), NE = 1 << (CV::WQ - 1);
  if (tn <= 0) return;
  dim3 b(64);
  hipLaunchKernelGGL(k_ec_table_base_keys<CV>, dim3((NWIN + 63) / 64, tn), b, 0, s, keys, blob, tidx, tn);
  table_slices(NWIN * NE, tn, sliced, s, [&](int e0, int e1, dim3 g) {
    hipLaunchKernelGGL(k_ec_table_keys<CV>, g, b, 0, s, keys, blob, tidx, tn, e0, e1);
  });
}

template <class CV>
void gtable_chain(uint32_t* tab, hipStream_t s) {
  constexpr int NWIN = ec_windows(CV::CLS, true), NE = ec_entries(CV::CLS, true);
  hipLaunchKernelGGL(k_ec_table_base_g<CV>, dim3((NWIN + 63) / 64), dim3(64), 0, s, tab);
  hipLaunchKernelGGL(k_ec_table_g<CV>, dim3((NWIN * NE + 63) / 64), dim3(64), 0, s, tab);
}

}  // namespace

