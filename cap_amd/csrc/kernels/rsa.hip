// rsa.hip -- RSA public operation + PKCS#1 v1.5 / PSS checks on gfx950.
//
// Replaces crypto/rsa VerifyPKCS1v15 / VerifyPSS(opts=nil) behind go-jose's
// rsaEncrypterVerifier.verifyPayload (rules R12-R17).
//
// k_rsa_modexp<L,U>: one thread per token, one 64-lane wave per key-uniform
// run of tokens.  s^e mod n by left-to-right square-and-multiply on Montgomery
// products in 28-bit limbs (L limbs, R = 2^(28L) > 4n so no final subtraction
// until the end).  Montgomery product = lazy CIOS:
//   for i: T += a_i * v ; m = T0 * n' mod 2^28 ; T += m * n ; T >>= 28 (limb shift)
// with T in 64-bit VGPR pairs (v_mad_u64_u32, no carry chains), v in VGPRs,
// the per-lane a_i streamed from LDS (lane-contiguous, conflict-free) and the
// modulus limbs n_j wave-uniform (scalar loads / SGPR operands).  The limb
// shift is a register rename inside a U-times unrolled block; one physical
// shift per block (amortised 1/U).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "rsa.hpp"
#include "sha2.hpp"
#include "mad.hpp"
#include "mad_blocks.hpp"
#include "small_common.hpp"

using namespace jgk;

#define W28 28
#define M28 0x0fffffffu
#ifndef SQR_SLOTS
#define SQR_SLOTS 4
#endif
#define SQR_SLOT(k) ((k) % SQR_SLOTS)
#ifndef JG_RSA_SHIFT28
#define JG_RSA_SHIFT28 1
#endif
#ifndef JG_RSA_BLOCKS
#define JG_RSA_BLOCKS 1
#endif

namespace {

// ---------------------------------------------------------------- cross-lane
// Token = group of G consecutive lanes; lane g of the group holds limbs
// [g*H, (g+1)*H) of every multi-limb value.  G = 2 or 4: one DPP quad
// (quad_perm); G = 8 or 16 (the RSA-8K / RSA-16K layouts of the 4K+ class):
// neighbours by DPP row shifts inside a 16-lane row, group-wide broadcasts by
// ds_swizzle in bitmask mode (lane' = lane & and_mask | or_mask inside each
// 32-lane half), one instruction each.
template <int G>
__device__ __forceinline__ uint32_t swz(uint32_t x, int or_mask) {
  static_assert(G == 8 || G == 16, "swizzle broadcasts serve the 8/16-lane groups");
  constexpr int AND = 0x1f & ~(G - 1);
  if (or_mask == 0) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, AND);
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, AND | ((G - 1) << 5));
}
template <int G>
__device__ __forceinline__ uint32_t bcast0(uint32_t x) {        // value of group lane 0
  if constexpr (G > 4) {
    return swz<G>(x, 0);
  } else {
    constexpr int ctrl = G == 2 ? 0xA0 /* quad_perm 0,0,2,2 */ : 0x00 /* 0,0,0,0 */;
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, true);
  }
}
template <int G>
__device__ __forceinline__ uint32_t bcast_last(uint32_t x) {    // value of group lane G-1
  if constexpr (G > 4) {
    return swz<G>(x, G - 1);
  } else {
    constexpr int ctrl = G == 2 ? 0xF5 /* quad_perm 1,1,3,3 */ : 0xFF /* 3,3,3,3 */;
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, true);
  }
}
template <int G>
__device__ __forceinline__ uint32_t from_next(uint32_t x) {     // value of group lane g+1
  constexpr int ctrl = G == 2 ? 0xF5 /* 1,1,3,3 */ : G == 4 ? 0xF9 /* 1,2,3,3 */ : 0x101 /* row_shl:1 */;
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, true);
}
template <int G>
__device__ __forceinline__ uint32_t from_prev(uint32_t x) {     // value of group lane g-1
  constexpr int ctrl = G == 2 ? 0xA0 /* quad_perm 0,0,2,2 */ : G == 4 ? 0x90 /* 0,0,1,2 */ : 0x111 /* row_shr:1 */;
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, true);
}

// T[k] += a * b[k] for k < n (n compile-time after unrolling) as blocks of up
// to JG_RSA_MADBLK MADs per inline-asm statement: LLVM pads a hazard s_nop
// after an asm statement whose results the next instruction touches, so one
// MAD per asm cost ~1 s_nop per 4 MADs here (profiles/r01_int_rates2.json:
// 28.8 T MAD/s with one MAD per asm vs 33.6 T with 8 per asm at 2 waves/SIMD).
// 16-MAD blocks halve the s_nops but measured the same at 2 waves/SIMD and
// spill more (profiles/r02_s11_rsa_occupancy_ab.json).
//
// Occupancy: left alone, the compiler gives k_rsa_modexp 256 VGPRs plus a few
// AGPRs as spill space (RSA-2048: 262 in all), which allows ONE wave per
// SIMD.  Capped at 256 (two waves per SIMD) it spills 5 registers to scratch
// (RSA-4096: 2) and the RSA-2048 modexp runs 13 % faster (7.93 -> 6.91 ms per
// 1M tokens): the second wave covers the CIOS rows' dependent chains.
#ifndef JG_RSA_MODEXP_ATTR
#define JG_RSA_MODEXP_ATTR __attribute__((amdgpu_waves_per_eu(2)))
#endif
#ifndef JG_RSA_PAD_ATTR
#define JG_RSA_PAD_ATTR __attribute__((amdgpu_waves_per_eu(2)))
#endif
#ifndef JG_RSA_MADBLK
#define JG_RSA_MADBLK 8
#endif
__device__ __forceinline__ void madv_run(uint64_t* T, uint32_t a, const uint32_t* b, int n) {
  for (int k = 0; k < n; k += JG_RSA_MADBLK) mb::madv_n(n - k < JG_RSA_MADBLK ? n - k : JG_RSA_MADBLK, T + k, a, b + k);
}

// All-ones in the lanes that keep a cross-lane value, zero in the others, as
// a value the optimizer cannot see through.  Written as `lane0 ? 0 : dpp(x)`
// the select may become a branch, and LLVM then sinks the computation of x --
// and the DPP read of it -- under that branch, where EXEC has switched off the
// very lanes the DPP reads (they read as 0).  That lost lane 0's borrow in the
// final subtraction whenever s^e mod n = n - 1 (tests/test_gpu_rsa.py).  An
// AND with an opaque mask keeps every DPP source computed in every lane.
__device__ __forceinline__ uint32_t opaque_mask(bool keep) {
  uint32_t m = keep ? ~0u : 0u;
  asm volatile("" : "+v"(m));
  return m;
}

// The limb shift that ends a CIOS row: every lane keeps T[0]'s bits above
// 28 in its own T[1] (same weight) and hands the low 28 bits to the lane below,
// which places them in its fresh top slot T[H] (the top lane's fresh slot is
// zero).  In lane 0, T[0] mod 2^28 = 0 after the reduction: the limb that the
// Montgomery division drops.  One 32-bit DPP move per row, no lane-0 select.
template <int H, int G>
__device__ __forceinline__ void limb_shift(uint64_t* T, bool lane0, uint32_t mlast) {
  const uint64_t t0 = T[0];
#if JG_RSA_SHIFT28
  T[1] += t0 >> W28;
  const uint32_t lo = from_next<G>((uint32_t)t0 & M28);
  T[H] = (uint64_t)(lo & mlast);
#else
  T[1] += lane0 ? (t0 >> W28) : 0ull;
  const uint32_t lo = from_next<G>((uint32_t)t0);
  const uint32_t hi = from_next<G>((uint32_t)(t0 >> 32));
  T[H] = ((uint64_t)(hi & mlast) << 32) | (lo & mlast);
#endif
}

// The row's Montgomery digit m from group lane 0 to the group: a DPP / ds_swizzle
// broadcast, or -- ONE: the wave runs a single token (k_rsa_small, every group
// a copy of group 0) -- v_readfirstlane, so m is an SGPR operand and the row's
// dependent chain skips the swizzle's LDS-path latency.
template <int G, bool ONE>
__device__ __forceinline__ uint32_t row_digit(uint32_t x) {
  if constexpr (ONE) return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
  else return bcast0<G>(x);
}

// One CIOS iteration on this lane's window T[0..H) of the token's accumulator.
//   T += a_i * v ; m = T0 * n' (group lane 0, broadcast) ; T += m * n ;
//   lane 0: T1 += T0 >> 28 ; every lane hands T0 to the lane below, which
//   places it in its fresh top slot T[H] (the limb shift across lanes).
template <int H, int G, bool ONE = false>
__device__ __forceinline__ void cios_step(uint64_t* T, uint32_t ai, const uint32_t* v, const uint32_t* n,
                                          uint32_t np, bool lane0, uint32_t mlast) {
#if JG_RSA_BLOCKS
  madv_run(T, ai, v, H);
  const uint32_t m = row_digit<G, ONE>(((uint32_t)T[0] * np) & M28);
  madv_run(T, m, n, H);
#else
#pragma unroll
  for (int j = 0; j < H; ++j) mad64(T[j], ai, v[j], j & 1);
  const uint32_t m = row_digit<G, ONE>(((uint32_t)T[0] * np) & M28);
#pragma unroll
  for (int j = 0; j < H; ++j) mad64(T[j], m, n[j], 2 + (j & 1));
#endif
  limb_shift<H, G>(T, lane0, mlast);
}

// v <- the lane's accumulator window P[0..H), normalised within the lane, then
// the carries rippled up the group: each round moves every pending carry one
// lane up (the top lane's carry-out is zero because the value is
// < 2n < 2^(28L)).
template <int H, int G>
__device__ __forceinline__ void finish_product(uint32_t* v, const uint64_t* P, uint32_t ml0) {
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const uint64_t t = P[j] + c;
    v[j] = (uint32_t)t & M28;
    c = t >> W28;
  }
#pragma unroll
  for (int r = 0; r < G - 1; ++r) {
    const uint32_t clo = from_prev<G>((uint32_t)c), chi = from_prev<G>((uint32_t)(c >> 32));
    uint64_t cin = ((uint64_t)(chi & ml0) << 32) | (clo & ml0);
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const uint64_t t = (uint64_t)v[j] + cin;
      v[j] = (uint32_t)t & M28;
      cin = t >> W28;
    }
    c = cin;
  }
}

// v <- (a * v) / R mod n with a streamed from LDS (la[i * TPW], shared by the
// group's lanes: a broadcast read).  R = 2^(28 H G).  In: v < 2n limb-normalized.
// Out: v < 2n, limbs < 2^28 (carries rippled across the group).
template <int H, int G, int U, int TPW, bool ONE = false>
__device__ __forceinline__ void mont_mul(uint32_t* v, const uint32_t* la, const uint32_t* n, uint32_t np,
                                         bool lane0, uint32_t mlast, uint32_t ml0) {
  constexpr int L = H * G, NB = L / U, REM = L % U;
  uint64_t P[H + U];
#pragma unroll
  for (int j = 0; j < H + U; ++j) P[j] = 0;
  for (int ib = 0; ib < NB; ++ib) {
    uint32_t a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = la[(ib * U + u) * TPW];
#pragma unroll
    for (int u = 0; u < U; ++u) cios_step<H, G, ONE>(P + u, a[u], v, n, np, lane0, mlast);
    if constexpr (2 * L > 250) {
      // keep every 64-bit column < 2^64: a row adds two products of < 2^56 to
      // each column, so normalise within the lane every 80 rows (RSA-4K: once,
      // half-way; the 8K / 16K layouts every 10 blocks)
      if ((ib + 1) % 10 == 0 && ib + 1 < NB) {
#pragma unroll
        for (int j = U; j < U + H - 1; ++j) { P[j + 1] += P[j] >> W28; P[j] &= M28; }
      }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) P[j] = P[j + U];
#pragma unroll
    for (int j = H; j < H + U; ++j) P[j] = 0;
  }
#pragma unroll
  for (int u = 0; u < REM; ++u) cios_step<H, G, ONE>(P + u, la[(NB * U + u) * TPW], v, n, np, lane0, mlast);
  finish_product<H, G>(v, P + REM, ml0);
}

// v <- v^2 / R mod n: the squaring form of mont_mul (16 of the 18 products of
// e = 65537).  Same lazy CIOS rows and the same limb shift, but the multiply
// half adds every product v_i v_j once (doubled when i != j).  Lane g's
// register k is limb gH + k, so row i = rH + x multiplies a_i into registers
// k >= x only, covering the limb pairs {rH + x, gH + k}:
//   k > x   both rows (r,x) and (g,k) could hold the pair; only (r,x) does (x 2)
//   k == x  lane g < r: nothing (row (g,x) had it), g == r: the square v_i^2
//           once, g > r: the cross product (x 2)
// Any row may add a product v_i v_j as long as it runs before column i + j is
// reduced, and rows i and j both do.  Multiply MADs: G*H(H+1)/2 per lane
// instead of G*H^2 (RSA-2048: 1406 + 2738 = 4144 per lane and product instead
// of 5476).  The column bound is unchanged: the doubled products sum to the
// same column totals as the full product.  The x loop is unrolled (the
// triangle needs compile-time register indices), the r loop is not: one
// physical shift of the window per H rows.
template <int H, int G, int TPW, bool ONE = false>
__device__ __forceinline__ void mont_sqr(uint32_t* v, const uint32_t* la, const uint32_t* n, uint32_t np, int g,
                                         bool lane0, uint32_t mlast, uint32_t ml0) {
  constexpr int L = H * G;
  uint64_t P[2 * H];
#pragma unroll
  for (int j = 0; j < H; ++j) P[j] = 0;
#pragma unroll 1
  for (int r = 0; r < G; ++r) {
    const uint32_t sh = g > r ? 1u : 0u;
    const uint32_t msk = g >= r ? ~0u : 0u;
    const uint32_t* lr = la + r * H * TPW;
#pragma unroll
    for (int x = 0; x < H; ++x) {
      const uint32_t ai = lr[x * TPW];
      uint64_t* T = P + x;
      mad64(T[x], (ai << sh) & msk, v[x], SQR_SLOT(x));
      const uint32_t a2 = ai << 1;
#if JG_RSA_BLOCKS
      madv_run(T + x + 1, a2, v + x + 1, H - x - 1);
      const uint32_t m = row_digit<G, ONE>(((uint32_t)T[0] * np) & M28);
      madv_run(T, m, n, H);
#else
#pragma unroll
      for (int k = x + 1; k < H; ++k) mad64(T[k], a2, v[k], SQR_SLOT(k));
      const uint32_t m = row_digit<G, ONE>(((uint32_t)T[0] * np) & M28);
#pragma unroll
      for (int k = 0; k < H; ++k) mad64(T[k], m, n[k], SQR_SLOT(k + 2));
#endif
      limb_shift<H, G>(T, lane0, mlast);
    }
    if constexpr (2 * L > 250) {
      // keep every 64-bit column < 2^64: a squaring row adds at most one doubled
      // product (< 2^57) and one reduction product (< 2^56) to a column, so
      // normalise every two lane blocks (74 rows at H = 37: < 222 * 2^56)
      if (r % 2 == 1 && r < G - 1) {
#pragma unroll
        for (int j = H; j < 2 * H - 1; ++j) { P[j + 1] += P[j] >> W28; P[j] &= M28; }
      }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) P[j] = P[j + H];
  }
  finish_product<H, G>(v, P, ml0);
}

template <int H, int TPW>
__device__ __forceinline__ void lds_store(uint32_t* la, const uint32_t* v, int g) {
#pragma unroll
  for (int j = 0; j < H; ++j) la[(g * H + j) * TPW] = v[j];
}

// limbs [gH, gH+H) of the integer held as LE 32-bit words in SoA rows
template <int H>
__device__ __forceinline__ void load_limbs_from_words(uint32_t* v, const uint32_t* rows, int64_t np, int64_t p,
                                                      int g, int nrows) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const int bit = W28 * (g * H + j), q = bit >> 5, s = bit & 31;
    const uint32_t w0 = rows[(int64_t)q * np + p];       // rows up to (28 L - 1) / 32 + 1
    const uint32_t w1 = rows[(int64_t)(q + 1) * np + p]; // exist and are zeroed (rsa_sig_rows)
    const uint64_t ww = ((uint64_t)w1 << 32) | w0;
    v[j] = (uint32_t)(ww >> s) & M28;
  }
}

// Row-major SoA scratch: limb j of lane segment g of token p lives at
// rows[(g*H + j) * np + p].  Addressed as (rows + j*np) [uniform, SGPR base]
// + loff (one 32-bit VGPR lane offset, loff = g*H*np + p), so the H loads share
// a single address VGPR instead of H 64-bit addresses.
template <int H>
__device__ __forceinline__ void load_limb_rows(uint32_t* v, const uint32_t* rows, int64_t np, uint32_t loff) {
#pragma unroll
  for (int j = 0; j < H; ++j) v[j] = (rows + (int64_t)j * np)[loff];
}
template <int H>
__device__ __forceinline__ void store_limb_rows(uint32_t* rows, int64_t np, uint32_t loff, const uint32_t* v) {
#pragma unroll
  for (int j = 0; j < H; ++j) (rows + (int64_t)j * np)[loff] = v[j];
}

template <int H, int G, int U>
__global__ void __launch_bounds__(64) JG_RSA_MODEXP_ATTR k_rsa_modexp(RsaArgs a) {
  constexpr int L = H * G, TPW = WAVE / G;
  constexpr int NWOUT = (W28 * L + 31) / 32;
  static_assert((W28 * L - 1) / 32 + 2 <= SIGW_ROWS, "limb loads and y words must fit the signature rows");
  __shared__ uint32_t lds[L * TPW];
  const int lane = threadIdx.x;
  const int g = lane % G, tl = lane / G;
  const bool lane0 = g == 0, lastl = g == G - 1;
  const uint32_t ml0 = opaque_mask(!lane0), mlast = opaque_mask(!lastl);
  const int64_t pbase = a.begin + (int64_t)blockIdx.x * TPW;
  const int64_t p = pbase + tl;
  const int64_t np = a.npad;
  const int kidx = __builtin_amdgcn_readfirstlane(job_key(a.jobs[pbase]));
  const DevKey K = a.keys[kidx];
  if (K.nlimbs != (uint32_t)L) return;      // a wave of another layout of the class (wave-uniform)
  const uint32_t* __restrict__ N = a.keyblob + K.n_off;
  const uint32_t* __restrict__ RR = a.keyblob + K.rr_off;
  const uint32_t np28 = K.np;
  const uint64_t e = ((uint64_t)K.e_hi << 32) | K.e_lo;
  uint32_t* la = lds + tl;

  uint32_t n[H];
#pragma unroll
  for (int j = 0; j < H; ++j) n[j] = N[g * H + j];

  bool act = job_live(a.jobs[p]) && a.status[p] == ST_OK && a.siglen[p] == (uint16_t)K.kbytes && K.valid;

  const uint32_t loff = (uint32_t)((int64_t)g * H * np + p);
  uint32_t v[H];
  load_limbs_from_words<H>(v, a.sigw, np, p, g, SIGW_ROWS);
  store_limb_rows<H>(a.xlr, np, loff, v);        // x as limb rows (MULX operand)
  // sig < N (Go >= 1.20, R14): per-lane compare, the highest differing lane decides
  {
    int lt = 0, gt = 0;
#pragma unroll
    for (int j = H - 1; j >= 0; --j) {
      const int und = !(lt | gt);
      lt |= und & (v[j] < n[j]);
      gt |= und & (v[j] > n[j]);
    }
    int code = lt ? 1 : (gt ? 2 : 0);        // 1: x<n here, 2: x>n here, 0: equal
    // walk from the top lane down: the first lane with code != 0 decides
    int dec = code;
#pragma unroll
    for (int r = 0; r < G - 1; ++r) {
      const int up = (int)from_next<G>((uint32_t)dec);
      dec = (up & (int)mlast) != 0 ? (up & (int)mlast) : dec;
    }
    dec = (int)bcast0<G>((uint32_t)dec);
    act = act && dec == 1;
  }

  // Exponentiation as one loop over Montgomery products (one inlined copy of
  // the product body).  Ops, left-to-right over the bits of e:
  //   TOMONT  v = Mont(x, R^2) = xR      SQUARE  v = Mont(v, v)
  //   MULXM   v = Mont(v, xR)            (set bits other than bit 0)
  //   MULX    v = Mont(v, x)             (bit 0 set: leaves the Montgomery domain)
  //   MULONE  v = Mont(v, 1)             (bit 0 clear)
  enum { TOMONT, SQUARE, MULXM, MULX, MULONE };
  const int ebits = 64 - __builtin_clzll(e);
  const bool mid = ((e >> 1) & ((1ull << (ebits - 2)) - 1ull)) != 0;
  int op = TOMONT, bit = ebits - 2;
  for (;;) {
    // opaque zero: stops LICM from hoisting the ~2H per-limb load addresses of
    // the operand loads below out of the loop (they would stay live in VGPRs)
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    lds_store<H, TPW>(la, v, g);
    if (op == TOMONT) {
      const uint32_t* rr = RR + z + g * H;
#pragma unroll
      for (int j = 0; j < H; ++j) v[j] = rr[j];
    } else if (op == MULXM) {
      load_limb_rows<H>(v, a.xmw + z, np, loff);
    } else if (op == MULX) {
      load_limb_rows<H>(v, a.xlr + z, np, loff);
    } else if (op == MULONE) {
#pragma unroll
      for (int j = 0; j < H; ++j) v[j] = (j == 0 && lane0) ? 1u : 0u;
    }
    if (op == SQUARE) mont_sqr<H, G, TPW>(v, la, n, np28, g, lane0, mlast, ml0);
    else mont_mul<H, G, U, TPW>(v, la, n, np28, lane0, mlast, ml0);
    if (op == TOMONT) {
      if (mid) store_limb_rows<H>(a.xmw, np, loff, v);
      op = SQUARE;
    } else if (op == SQUARE) {
      if ((e >> bit) & 1ull) op = bit > 0 ? MULXM : MULX;
      else if (bit == 0) op = MULONE;
      else --bit;
    } else if (op == MULXM) {
      --bit;
      op = SQUARE;
    } else {
      break;
    }
  }

  // canonical: v < 2n -> v mod n.  d = v - n with the borrow rippled up the
  // group (G rounds), then the top lane's final borrow picks v or d.
  {
    uint32_t d[H];
    int32_t bout = 0;
#pragma unroll
    for (int r = 0; r < G; ++r) {
      int32_t br = (int32_t)(from_prev<G>((uint32_t)bout) & ml0);
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const int32_t t = (int32_t)v[j] - (int32_t)n[j] + br;
        d[j] = (uint32_t)t & M28;
        br = t >> W28;
      }
      bout = br;
    }
    const int32_t b_top = (int32_t)bcast_last<G>((uint32_t)bout);
#pragma unroll
    for (int j = 0; j < H; ++j) v[j] = b_top < 0 ? v[j] : d[j];
  }
  // y as LE 32-bit words: stage limbs in LDS, each group lane converts a slice
  lds_store<H, TPW>(la, v, g);
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): own-group LDS writes visible to the group
  __builtin_amdgcn_wave_barrier();
  constexpr int PER = (NWOUT + G - 1) / G;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int q = g * PER + k;
    if (q < NWOUT) {
      const int bit = 32 * q, j0 = bit / W28, s0 = bit % W28;
      uint64_t acc = (uint64_t)la[j0 * TPW] >> s0;
      int have = W28 - s0;
      int j = j0 + 1;
      while (have < 32 && j < L) { acc |= (uint64_t)la[j * TPW] << have; have += W28; ++j; }
      if (act) a.yw[(int64_t)q * np + p] = (uint32_t)acc;
    }
  }
  if (!act && lane0) a.status[p] = ST_REJECT;
}

// ------------------------------------------------------------------ padding
__constant__ uint8_t DI256[19] = {0x30,0x31,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x01,0x05,0x00,0x04,0x20};
__constant__ uint8_t DI384[19] = {0x30,0x41,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x02,0x05,0x00,0x04,0x30};
__constant__ uint8_t DI512[19] = {0x30,0x51,0x30,0x0d,0x06,0x09,0x60,0x86,0x48,0x01,0x65,0x03,0x04,0x02,0x03,0x05,0x00,0x04,0x40};

__device__ __forceinline__ uint32_t ybyte(const uint32_t* yw, int64_t np, int64_t p, int k, int pos) {
  const int j = k - 1 - pos;                 // integer byte index (little-endian)
  return (yw[(int64_t)(j >> 2) * np + p] >> ((j & 3) * 8)) & 0xffu;
}
__device__ __forceinline__ uint32_t dbyte(const uint32_t* dig, int64_t np, int64_t p, int i) {
  return (dig[(int64_t)(i >> 2) * np + p] >> (24 - 8 * (i & 3))) & 0xffu;
}

// big-endian word of I2OSP(y, k) bytes [m, m+4): the little-endian word of
// the integer at byte offset k-4-m (integer bytes below 0 are past EM's end)
__device__ __forceinline__ uint32_t bword(const uint32_t* yw, int64_t np, int64_t p, int k, int m) {
  const int jlo = k - 4 - m;
  const int q = jlo >> 2;                    // floor (arithmetic shift)
  const int nrows = (k + 3) >> 2;
  const uint32_t lo = (q >= 0 && q < nrows) ? yw[(int64_t)q * np + p] : 0u;
  const uint32_t hi = (q + 1 >= 0 && q + 1 < nrows) ? yw[(int64_t)(q + 1) * np + p] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(jlo & 3));
}

// one MGF1 block: Hash(H || BE32(c)), H = hw big-endian words (one SHA block)
__device__ __forceinline__ void mgf1_block(int hb, const uint32_t* Hw, int hw, uint32_t c, uint32_t* out16) {
  const uint32_t len = 4u * (uint32_t)hw + 4u;
  if (hb == 256) {
    uint32_t w[16], h[8];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = t < hw ? Hw[t] : t == hw ? c : t == hw + 1 ? 0x80000000u : 0u;
    w[15] = len << 3;
    sha2::sha256_init(h);
    sha2::sha256_compress(h, w);
#pragma unroll
    for (int t = 0; t < 8; ++t) { out16[t] = h[t]; out16[8 + t] = 0u; }
  } else {
    uint32_t v[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) v[t] = t < hw ? Hw[t] : t == hw ? c : t == hw + 1 ? 0x80000000u : 0u;
    v[31] = len << 3;
    uint64_t w[16], h[8];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = ((uint64_t)v[2 * t] << 32) | v[2 * t + 1];
    sha2::sha512_init(h, hb == 384);
    sha2::sha512_compress(h, w);
#pragma unroll
    for (int t = 0; t < 8; ++t) { out16[2 * t] = (uint32_t)(h[t] >> 32); out16[2 * t + 1] = (uint32_t)h[t]; }
  }
}

template <bool PSS>
__global__ void __launch_bounds__(64) JG_RSA_PAD_ATTR k_rsa_pad(RsaArgs a) {
  const int64_t p = a.begin + (int64_t)blockIdx.x * WAVE + threadIdx.x;
  const int64_t np = a.npad;
  const JobDev jb = a.jobs[p];
  if (!job_live(jb)) return;
  uint8_t verdict = 0;
  if (a.status[p] == ST_OK) {
    const int kidx = job_key(jb);
    const DevKey K = a.keys[kidx];
    const int k = K.kbytes;
    const int alg = job_alg(jb);
    const int hb = (alg == 1 || alg == 4) ? 256 : (alg == 2 || alg == 5) ? 384 : 512;
    const int hlen = hb / 8;
    if (alg <= 3) {
      // PKCS#1 v1.5: EM == 00 01 FF..FF 00 || DigestInfo || H   (R15)
      // Compared word by word on the little-endian integer y: LE byte j holds
      // EM[k-1-j]; H occupies j < hlen (whole words: y word q == digest word
      // hlen/4-1-q), DigestInfo hlen <= j < tlen, then 00, FF.., 01, 00.
      const int tlen = 19 + hlen;
      const uint8_t* DI = hb == 256 ? DI256 : hb == 384 ? DI384 : DI512;
      bool ok = k >= tlen + 11;
      uint32_t diff = 0;
      for (int q = 0; q < hlen / 4; ++q)
        diff |= a.yw[(int64_t)q * np + p] ^ a.dig[(int64_t)(hlen / 4 - 1 - q) * np + p];
      const int nw = (k + 3) / 4;
      for (int q = hlen / 4; q < nw; ++q) {
        const uint32_t yv = a.yw[(int64_t)q * np + p];
        uint32_t ev = 0xffffffffu;          // the FF run: every word but the ~8 at its ends
        if (4 * q <= tlen || 4 * q + 3 >= k - 2) {
          ev = 0;
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) {
            const int j = 4 * q + bb;
            uint32_t ex;
            if (j < tlen) ex = DI[tlen - 1 - j];
            else if (j == tlen) ex = 0;
            else if (j < k - 2) ex = 0xff;
            else if (j == k - 2) ex = 1;
            else ex = 0;                    // j == k-1, and j >= k (y < n < 2^(8k))
            ev |= ex << (8 * bb);
          }
        }
        diff |= yv ^ ev;
      }
      verdict = ok && diff == 0;
    } else if constexpr (PSS) {
      // EMSA-PSS-VERIFY with auto salt length (R16)
      const int embits = K.embits;
      const int emlen = (embits + 7) / 8;
      const int lead = k - emlen;                       // 0 or 1
      bool ok = true;
      for (int i = 0; i < lead; ++i) ok = ok && ybyte(a.yw, np, p, k, i) == 0;
      ok = ok && emlen >= hlen + 2;
      ok = ok && ybyte(a.yw, np, p, k, lead + emlen - 1) == 0xbc;
      const uint32_t bitmask = 0xffu >> (8 * emlen - embits);
      ok = ok && (ybyte(a.yw, np, p, k, lead) & ~bitmask) == 0;
      if (ok) {
        // Word-level EMSA-PSS-VERIFY: EM words come straight from the y rows
        // (bword), DB = maskedDB ^ MGF1(H) is kept as big-endian words in this
        // token's 2 KiB scratch, M' = 0^8 || mHash || salt is fed to SHA-2
        // word by word from the digest rows and the DB words.
        uint32_t* dbw = reinterpret_cast<uint32_t*>(a.pss_scratch + (p - a.begin) * 2048);
        const int dblen = emlen - hlen - 1;
        const int hw = hlen / 4;
        uint32_t Hw[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) Hw[t] = t < hw ? bword(a.yw, np, p, k, lead + dblen + 4 * t) : 0u;
        for (int c = 0; c * hlen < dblen; ++c) {
          uint32_t mask[16];
          mgf1_block(hb, Hw, hw, (uint32_t)c, mask);
#pragma unroll
          for (int t = 0; t < 16; ++t) {
            const int di = c * hlen + 4 * t;
            if (t < hw && di < dblen) dbw[di >> 2] = bword(a.yw, np, p, k, lead + di) ^ mask[t];
          }
        }
        // DB[0] &= bitmask; PS = leading zero bytes, then 0x01
        const int nw = (dblen + 3) / 4;
        int ps = -1;
        for (int q = 0; q < nw && ps < 0; ++q) {
          uint32_t w = dbw[q];
          if (q == 0) w &= (bitmask << 24) | 0x00ffffffu;
          const int live = dblen - 4 * q;                    // bytes of DB in this word
          if (live < 4) w &= 0xffffffffu << (32 - 8 * live);
          if (w != 0) {
            const int b = __builtin_clz(w) >> 3;
            ps = 4 * q + b;
            ok = ((w >> (24 - 8 * b)) & 0xffu) == 0x01u;
          }
        }
        ok = ok && ps >= 0;
        if (ok) {
          const int slen = dblen - ps - 1;
          const uint32_t mlen = (uint32_t)(8 + hlen + slen);
          auto mword = [&](uint32_t w) -> uint32_t {          // big-endian word w of M', padded
            const int o = 4 * (int)w;
            uint32_t raw;
            if (o < 8) raw = 0u;
            else if (o < 8 + hlen) raw = a.dig[(int64_t)((o - 8) >> 2) * np + p];
            else {
              const int st = ps + 1 + (o - 8 - hlen);         // DB byte index of the salt bytes
              const int q = st >> 2, r = st & 3;
              raw = r == 0 ? dbw[q] : (dbw[q] << (8 * r)) | (dbw[q + 1] >> (32 - 8 * r));
            }
            return sha2::pad_word(raw, w, mlen);
          };
          uint32_t h2[16];
          if (hb == 256) {
            uint32_t h[8];
            sha2::sha256_init(h);
            const uint32_t nblk = (mlen + 9 + 63) / 64;
            for (uint32_t blk = 0; blk < nblk; ++blk) {
              uint32_t w[16];
              for (int t = 0; t < 16; ++t) w[t] = mword(16 * blk + t);
              if (blk == nblk - 1) { w[14] = mlen >> 29; w[15] = mlen << 3; }
              sha2::sha256_compress(h, w);
            }
            for (int t = 0; t < 8; ++t) h2[t] = h[t];
          } else {
            uint64_t h[8];
            sha2::sha512_init(h, hb == 384);
            const uint32_t nblk = (mlen + 17 + 127) / 128;
            for (uint32_t blk = 0; blk < nblk; ++blk) {
              uint32_t v[32];
              for (int t = 0; t < 32; ++t) v[t] = mword(32 * blk + t);
              if (blk == nblk - 1) { v[30] = mlen >> 29; v[31] = mlen << 3; }
              uint64_t w[16];
              for (int t = 0; t < 16; ++t) w[t] = ((uint64_t)v[2 * t] << 32) | v[2 * t + 1];
              sha2::sha512_compress(h, w);
            }
            for (int t = 0; t < 8; ++t) { h2[2 * t] = (uint32_t)(h[t] >> 32); h2[2 * t + 1] = (uint32_t)h[t]; }
          }
          uint32_t diff = 0;
          for (int t = 0; t < hw; ++t) diff |= h2[t] ^ Hw[t];
          ok = diff == 0;
        }
      }
      verdict = ok;
    }
  }
  a.verdict_pad[p] = verdict;
}

// ------------------------------------------------------------------ one launch (small batches)
// k_rsa_small: one 128-thread block per RS256 / RS384 / RS512 token on an
// RSA-2K-class key, the whole verification in one launch (the batch chain's
// prep, modexp and pad kernels), for coalesced single-token calls
// (jwt/keyset.go:27-32).  A lone token's modexp is a chain of 17 dependent
// Montgomery products; here each runs on 16 lanes of 5 limbs (R = 2^2240, the
// key's rr2_off constants): 80 CIOS rows of ~10 MADs per lane instead of the
// batch layout's 74 rows of 74 MADs on 2 lanes.  Wave 0 hashes the signing
// input on one lane meanwhile (s^e does not depend on it).  The four 16-lane
// groups of wave 1 run the same token (lanes of groups 1-3 compute copies);
// group 0's result is compared with EM = 00 01 FF..FF 00 || DigestInfo || H
// word by word across the wave (R15).
constexpr uint32_t RS_SIG_CHARS = 352;          // 264 bytes; the RSA-2K class has k <= 259
__global__ void __launch_bounds__(SM_THREADS) k_rsa_small(RsaSmallArgs a) {
  constexpr int H = RSA_SMALL_H, G = RSA_SMALL_G, L = RSA_SMALL_L, TPW = WAVE / G, U = 8;
  constexpr int NWOUT = (W28 * L + 31) / 32;
  __shared__ uint32_t in_w[SM_IN_DW];
  __shared__ uint32_t sig_w[RS_SIG_CHARS / 4 + 2];
  __shared__ uint8_t sig_b[3 * (RS_SIG_CHARS / 4) + 4];
  __shared__ uint32_t dig_w[16];
  __shared__ uint32_t lds[L * TPW];
  __shared__ uint32_t yw[NWOUT];
  __shared__ int32_t flag[2];                   // [0] signature characters bad, [1] the modexp ran
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const JobDev jb = a.jobs[blockIdx.x];
  const int alg = job_alg(jb);
  const DevKey& K = a.keys[job_key(jb)];
  const int k = K.kbytes;
  const uint32_t nch = job_siglen(jb);
  const int hb = alg == 1 ? 256 : alg == 2 ? 384 : 512;
  const bool in_ok = jb.sig_in_len <= SMALL_IN_MAX;
  const uint32_t in_shift = (uint32_t)((uintptr_t)(a.arena + jb.off) & 3u);
  const uint32_t sig_shift = (uint32_t)((uintptr_t)(a.arena + jb.sig_off) & 3u);
  if (tid == 0) { flag[0] = 0; flag[1] = 0; }
  // ---- both streams into LDS
  if (wave == 0 && in_ok) {
    sm_stage_input(in_w, reinterpret_cast<const uint32_t*>(a.arena + jb.off - in_shift), in_shift, jb.sig_in_len, hb,
                   lane);
  } else if (wave == 1) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(a.arena + jb.sig_off - sig_shift);
    const uint32_t nd = nch <= RS_SIG_CHARS ? (sig_shift + nch + 3) / 4 : 0u;
    for (uint32_t i = (uint32_t)lane; i < nd; i += 64) sig_w[i] = g[i];
  }
  __syncthreads();
  // ---- characters -> bytes; len(sig) == k (R13)
  const bool size_ok = nch <= RS_SIG_CHARS && (nch & 3u) != 1u && sm_b64_len(nch) == (uint32_t)k;
  if (wave == 1 && size_ok) {
    if (sm_b64_decode(sig_w, sig_shift, nch, sig_b, lane) && lane == 0) flag[0] = 1;
  }
  __syncthreads();
  const bool ok0 = in_ok && size_ok && flag[0] == 0 && K.valid != 0 && K.rr2_off != 0 && alg >= 1 && alg <= 3;
  // ---- hash (wave 0 lane 0) || s^e mod n (wave 1, 16 lanes per group)
  if (wave == 0 && lane == 0 && in_ok) sm_hash(in_w, in_shift, jb.sig_in_len, hb, dig_w);
  if (wave == 1 && ok0) {
    const int g = lane % G, tl = lane / G;
    const bool lane0 = g == 0, lastl = g == G - 1;
    const uint32_t ml0 = opaque_mask(!lane0), mlast = opaque_mask(!lastl);
    const uint32_t* __restrict__ N = a.keyblob + K.n_off;
    const uint32_t* __restrict__ RR = a.keyblob + K.rr2_off;
    const uint32_t np28 = K.np;
    const uint64_t e = ((uint64_t)K.e_hi << 32) | K.e_lo;
    uint32_t* la = lds + tl;
    uint32_t n[H], v[H], xl[H], xm[H];
#pragma unroll
    for (int j = 0; j < H; ++j) n[j] = N[g * H + j];
    // x: limb j = bits [28 j, 28 j + 28) of the big-endian k-byte signature
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const int bit = W28 * (g * H + j), i0 = bit >> 3, sh = bit & 7;
      uint64_t acc = 0;
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int i = i0 + t;                       // little-endian byte index of the integer
        acc |= (uint64_t)(i < k ? sig_b[k - 1 - i] : 0u) << (8 * t);
      }
      v[j] = (uint32_t)(acc >> sh) & M28;
      xl[j] = v[j];
    }
    // sig < N (Go >= 1.20, R14): the highest differing lane of the group decides
    bool act = true;
    {
      int lt = 0, gt = 0;
#pragma unroll
      for (int j = H - 1; j >= 0; --j) {
        const int und = !(lt | gt);
        lt |= und & (v[j] < n[j]);
        gt |= und & (v[j] > n[j]);
      }
      int dec = lt ? 1 : (gt ? 2 : 0);
#pragma unroll
      for (int r = 0; r < G - 1; ++r) {
        const int up = (int)from_next<G>((uint32_t)dec);
        dec = (up & (int)mlast) != 0 ? (up & (int)mlast) : dec;
      }
      dec = (int)bcast0<G>((uint32_t)dec);
      act = dec == 1;
    }
    enum { TOMONT, SQUARE, MULXM, MULX, MULONE };
    const int ebits = 64 - __builtin_clzll(e);
    int op = TOMONT, bit = ebits - 2;
    for (;;) {
      lds_store<H, TPW>(la, v, g);
      if (op == TOMONT) {
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = RR[g * H + j];
      } else if (op == MULXM) {
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = xm[j];
      } else if (op == MULX) {
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = xl[j];
      } else if (op == MULONE) {
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = (j == 0 && lane0) ? 1u : 0u;
      }
      if (op == SQUARE) mont_sqr<H, G, TPW, true>(v, la, n, np28, g, lane0, mlast, ml0);
      else mont_mul<H, G, U, TPW, true>(v, la, n, np28, lane0, mlast, ml0);
      if (op == TOMONT) {
#pragma unroll
        for (int j = 0; j < H; ++j) xm[j] = v[j];
        op = SQUARE;
      } else if (op == SQUARE) {
        if ((e >> bit) & 1ull) op = bit > 0 ? MULXM : MULX;
        else if (bit == 0) op = MULONE;
        else --bit;
      } else if (op == MULXM) {
        --bit;
        op = SQUARE;
      } else {
        break;
      }
    }
    // canonical: v < 2n -> v mod n (borrow rippled up the group)
    {
      uint32_t d[H];
      int32_t bout = 0;
#pragma unroll
      for (int r = 0; r < G; ++r) {
        int32_t br = (int32_t)(from_prev<G>((uint32_t)bout) & ml0);
#pragma unroll
        for (int j = 0; j < H; ++j) {
          const int32_t t = (int32_t)v[j] - (int32_t)n[j] + br;
          d[j] = (uint32_t)t & M28;
          br = t >> W28;
        }
        bout = br;
      }
      const int32_t b_top = (int32_t)bcast_last<G>((uint32_t)bout);
#pragma unroll
      for (int j = 0; j < H; ++j) v[j] = b_top < 0 ? v[j] : d[j];
    }
    // y as LE 32-bit words (group 0)
    lds_store<H, TPW>(la, v, g);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    constexpr int PER = (NWOUT + G - 1) / G;
#pragma unroll
    for (int kk = 0; kk < PER; ++kk) {
      const int q = g * PER + kk;
      if (q < NWOUT && tl == 0) {
        const int b32 = 32 * q, j0 = b32 / W28, s0 = b32 % W28;
        uint64_t acc = (uint64_t)la[j0 * TPW] >> s0;
        int have = W28 - s0;
        int j = j0 + 1;
        while (have < 32 && j < L) { acc |= (uint64_t)la[j * TPW] << have; have += W28; ++j; }
        yw[q] = (uint32_t)acc;
      }
    }
    if (lane == 0) flag[1] = act ? 1 : 0;
  }
  __syncthreads();
  // ---- PKCS#1 v1.5 (R15): EM == 00 01 FF..FF 00 || DigestInfo || H, word by
  // word on the little-endian y (k_rsa_pad's rule), one word per lane
  if (wave != 1) return;
  const int hlen = hb / 8, tlen = 19 + hlen, nw = (k + 3) / 4;
  const uint8_t* DI = hb == 256 ? DI256 : hb == 384 ? DI384 : DI512;
  uint32_t diff = 0;
  if (ok0 && flag[1] != 0) {
    for (int q = lane; q < nw; q += 64) {
      uint32_t ev;
      if (q < hlen / 4) {
        ev = dig_w[hlen / 4 - 1 - q];
      } else {
        ev = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const int j = 4 * q + bb;
          uint32_t ex;
          if (j < tlen) ex = DI[tlen - 1 - j];
          else if (j == tlen) ex = 0;
          else if (j < k - 2) ex = 0xff;
          else if (j == k - 2) ex = 1;
          else ex = 0;
          ev |= ex << (8 * bb);
        }
      }
      diff |= yw[q] ^ ev;
    }
  }
  const bool any = __ballot(diff != 0) != 0ull;
  if (lane == 0) a.verdict[a.out[blockIdx.x]] = (ok0 && flag[1] != 0 && k >= tlen + 11 && !any) ? 1 : 0;
}

}  // namespace

void launch_rsa_small(const RsaSmallArgs& a, hipStream_t s) {
  if (a.n == 0) return;
  hipLaunchKernelGGL(k_rsa_small, dim3(a.n), dim3(SM_THREADS), 0, s, a);
}

void launch_rsa(int cls, const RsaArgs& a, hipStream_t s, const Marker& mk) {
  const int64_t waves = (a.end - a.begin) / WAVE;
  if (waves <= 0) return;
  dim3 g((unsigned)waves), b(WAVE);
  switch (cls) {
    case CLS_RSA2K: hipLaunchKernelGGL((k_rsa_modexp<RSA2K_H, RSA2K_G, 8>), dim3((unsigned)(waves * RSA2K_G)), b, 0, s, a); break;
    case CLS_RSA3K:
      hipLaunchKernelGGL((k_rsa_modexp<RSA3K_H, RSA3K_G, RSA3K_U>), dim3((unsigned)(waves * RSA3K_G)), b, 0, s, a);
      break;
    case CLS_RSA4K:
      if (a.layouts & 1) hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 4, 8>), dim3((unsigned)(waves * 4)), b, 0, s, a);
      if (a.layouts & 2) hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 8, 8>), dim3((unsigned)(waves * 8)), b, 0, s, a);
      if (a.layouts & 4) hipLaunchKernelGGL((k_rsa_modexp<RSA4K_H, 16, 8>), dim3((unsigned)(waves * 16)), b, 0, s, a);
      break;
    default: return;
  }
  mk("modexp");
  if (a.has_pss) hipLaunchKernelGGL(k_rsa_pad<true>, g, b, 0, s, a);
  else hipLaunchKernelGGL(k_rsa_pad<false>, g, b, 0, s, a);
  mk("pad");
}

