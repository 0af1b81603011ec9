// ec_small.hpp -- ECDSA verification of a small batch in ONE launch (the
// coalesced single-token calls behind jwt/keyset.go:27-32 VerifySignature and
// jwt/jwt.go:95-97 Validate): one 128-thread block (two waves) per token runs
// what the batch chain spreads over plan fill, k_prep, k_ec_scalar_batch,
// k_ec_point_split, k_ec_exact and k_scatter -- same rules, same verdicts.
//
// A lone token is latency-bound: one lane's dependent instruction stream, ~2 ns
// per VALU instruction.  The block overlaps what does not depend on the hash:
//   wave 0: stage the signing input from the arena into LDS (bounded dword
//           loads, every lane), lane 0 hashes it (SHA-256/384/512 by alg, R9)
//   wave 1: stage and base64url-decode the signature (R3, every lane a quad of
//           characters), r / s from the decoded bytes (R18, R20), then lane 0
//           inverts s with the variable-time safegcd (s is public; ~2.5x fewer
//           instructions than the constant-time ladder), u2 = r s^-1
//   then    lane 0 of wave 1: e from the digest (R21), u1 = e s^-1, signed
//           comb digits into LDS
//   wave 0: lanes 0..S-1 each sum every S-th comb window of both scalars
//           (mixed additions, as k_ec_point_split), partials combined across
//           lanes with the exact addition, x(R) == r checked (R22); a partial
//           that hit an exceptional case (Z == 0) sends the token through the
//           complete double-and-add (ec_exact_ok), in the same block.
// Inputs: the jobs in the kernel arguments, the arena read in place (a pinned
// host arena over PCIe: no copy launch), the verdict byte written straight to
// pinned host memory (no scatter or copy launch).
#pragma once
#include "ecdsa_impl.hpp"
#include "small_common.hpp"

namespace {

constexpr int SM_SPLIT = 16;                                      // point lanes per token
constexpr uint32_t SM_SIG_CHARS = 176;                            // ES512's 132 bytes; longer is rejected

__device__ __forceinline__ int sm_hash_bits(int alg) { return alg == 7 ? 256 : alg == 8 ? 384 : 512; }

// x(R) mod n == r for R = (X : Y : Z) Jacobian, Z != 0:
// X == r Z^2, or r + n < p and X == (r + n) Z^2
template <class CV>
__device__ bool ec_x_matches(const uint32_t* X, const uint32_t* Z, const uint32_t* r) {
  using Fp = typename CV::Fp;
  using Fn = typename CV::Fn;
  constexpr int L = Fp::L;
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
  return ok;
}

// One level of the cross-lane combine: lane a (bit `off` clear, "lo") and lane
// a ^ off ("hi") hold Jacobian partials P_lo, P_hi (normalized coordinates)
// and split the products of P_lo + P_hi between them (jadd's arithmetic, same
// operations, same bounds): each lane first brings the OTHER lane's Z into
// its own U and S (lo: U1 = X1 Z2^2, S1 = Y1 Z2^3; hi: U2, S2), then
// lo takes HH, HHH, V while hi takes r^2, Z1 Z2, Z3, and the last pair of
// products (r (V - X3), S1 HHH) runs one per lane: 8 dependent products
// instead of jadd's 16 on one lane.  The sum lands in lo; hi's copy is
// garbage.  H == 0 (P_lo == +-P_hi: a doubling or an inverse pair) is not
// handled here: both lanes set `exc` and the token takes the complete
// double-and-add (ec_exact_ok).  Every lane of the wave must call it (shuffles).
template <class CV>
__device__ __forceinline__ void jadd_pair(JPt<typename CV::Fp>& P, int off, bool& exc) {
  using Fp = typename CV::Fp;
  constexpr int L = Fp::L;
  const bool lo = (threadIdx.x & off) == 0;
  uint32_t oz[L], ox[L], oy[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    ox[j] = __shfl_xor(P.X[j], off);
    oy[j] = __shfl_xor(P.Y[j], off);
    oz[j] = __shfl_xor(P.Z[j], off);
  }
  const bool oinf = __shfl_xor((int)P.inf, off) != 0;
  // the partner's flag is read by every lane: `exc || __shfl_xor(...)` left the
  // shuffle to the lanes whose own flag was clear, and a lane reading from one
  // that had skipped it got 0 -- an exceptional partial lost on its way to lane 0
  // (ec_edge.json exc-p521-G-accept-deq at equal G / key widths)
  const int pexc = __shfl_xor((int)exc, off);
  exc = exc || pexc != 0;
  const bool both = !P.inf && !oinf && !exc;
  // stage 1: own U, S against the other lane's Z
  uint32_t zz[L], u[L], t[L], sv[L], uo[L], so[L];
  mp::sqr<Fp>(zz, oz);
  mp::mul<Fp>(u, P.X, zz);
  mp::mul<Fp>(t, oz, zz);
  mp::mul<Fp>(sv, P.Y, t);
#pragma unroll
  for (int j = 0; j < L; ++j) {
    uo[j] = __shfl_xor(u[j], off);
    so[j] = __shfl_xor(sv[j], off);
  }
  uint32_t u1[L], s1[L], h[L], r[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    u1[j] = lo ? u[j] : uo[j];
    s1[j] = lo ? sv[j] : so[j];
    h[j] = lo ? uo[j] : u[j];            // U2
    r[j] = lo ? so[j] : sv[j];           // S2
  }
  mp::sub<Fp>(h, h, u1); mp::freduce<Fp>(h);
  mp::sub<Fp>(r, r, s1); mp::freduce<Fp>(r);
  const bool hzero = is_zero_mod<Fp>(h);
  // stage 2: lo HH, HHH, V | hi r^2, Z1 Z2, Z3
  uint32_t a[L], b[L], p1[L], p2[L], p3[L];
#pragma unroll
  for (int j = 0; j < L; ++j) a[j] = lo ? h[j] : r[j];
  mp::sqr<Fp>(p1, a);
#pragma unroll
  for (int j = 0; j < L; ++j) { a[j] = lo ? h[j] : P.Z[j]; b[j] = lo ? p1[j] : oz[j]; }
  mp::mul<Fp>(p2, a, b);
#pragma unroll
  for (int j = 0; j < L; ++j) { a[j] = lo ? u1[j] : p2[j]; b[j] = lo ? p1[j] : h[j]; }
  mp::mul<Fp>(p3, a, b);
  uint32_t q1[L], q2[L], q3[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    q1[j] = __shfl_xor(p1[j], off);      // lo: r^2   hi: HH
    q2[j] = __shfl_xor(p2[j], off);      // lo: Z1 Z2 hi: HHH
    q3[j] = __shfl_xor(p3[j], off);      // lo: Z3    hi: V
  }
  // stage 3 (lo): X3 = r^2 - HHH - 2V; then lo r (V - X3) | hi S1 HHH
  uint32_t x3[L], t2[L];
  mp::add<Fp>(t, p2, p3); mp::add<Fp>(t, t, p3); mp::freduce<Fp>(t);
  mp::sub<Fp>(x3, q1, t); mp::freduce<Fp>(x3);
  mp::sub<Fp>(t2, p3, x3);
#pragma unroll
  for (int j = 0; j < L; ++j) { a[j] = lo ? r[j] : s1[j]; b[j] = lo ? t2[j] : q2[j]; }
  uint32_t m[L], mo[L];
  mp::mul<Fp>(m, a, b);
#pragma unroll
  for (int j = 0; j < L; ++j) mo[j] = __shfl_xor(m[j], off);
  if (lo && both && !hzero) {
    mp::sub<Fp>(m, m, mo); mp::freduce<Fp>(m);
    mp::copy<Fp>(P.X, x3); mp::copy<Fp>(P.Y, m); mp::copy<Fp>(P.Z, q3);
  } else if (lo && P.inf && !oinf) {     // an empty partial takes the other one
    mp::copy<Fp>(P.X, ox); mp::copy<Fp>(P.Y, oy); mp::copy<Fp>(P.Z, oz);
    P.inf = false;
  }
  if (both && hzero) exc = true;
}

// signed W-bit recoding of u into digits d[0..NWIN) (store_digit_rows, into LDS)
template <int W, int NWIN, int L>
__device__ __forceinline__ void sm_recode(const uint32_t* u, int32_t* d) {
  constexpr uint32_t DM = (1u << W) - 1u;
  int c = 0;
#pragma unroll
  for (int wi = 0; wi < NWIN; ++wi) {
    const int bit = W * wi, q = bit / MP_W, sh = bit % MP_W;
    uint32_t b = q < L ? (u[q] >> sh) : 0u;
    if (sh > MP_W - W && q + 1 < L) b |= u[q + 1] << (MP_W - sh);
    int v = (int)(b & DM) + c;
    c = v >= (1 << (W - 1));
    v -= c << W;
    d[wi] = v;
  }
}

template <class CV>
__global__ void __launch_bounds__(SM_THREADS) k_ec_small(EcSmallArgs a) {
  using Fp = typename CV::Fp;
  using Fn = typename CV::Fn;
  constexpr int L = Fn::L;
  static_assert((int)Fp::L == (int)Fn::L, "field and order limb counts");
  constexpr int CB = CV::C::BYTES;
  constexpr int CW = ec_sig_words(CV::CLS);
  constexpr int WG = ec_comb_w(CV::CLS, true), NG = ec_windows(CV::CLS, true);
  constexpr int WQ = CV::WQ, NQ = ec_windows_w(CV::CLS, CV::WQ);
  constexpr int NWIN = NG > NQ ? NG : NQ;
  constexpr int S = SM_SPLIT;

  __shared__ uint32_t in_w[SM_IN_DW];           // signing input, aligned dwords (zero past the message)
  __shared__ uint32_t sig_w[SM_SIG_CHARS / 4 + 2];
  __shared__ uint8_t sig_b[3 * (SM_SIG_CHARS / 4) + 4];
  __shared__ uint32_t rs_w[2 * CW];             // r, s as little-endian words
  __shared__ uint32_t dig_w[16];                // digest, big-endian words
  __shared__ uint32_t sc[3 * L];                // r, u1, u2 (canonical plain limbs)
  __shared__ int32_t digs[NG + NQ];
  __shared__ int32_t flag[2];                   // [0] signature decode bad, [1] token runs
#if JG_SMALL_PROF
  __shared__ uint64_t stamp[2][10];
#endif

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const JobDev jb = a.jobs[blockIdx.x];
  const int alg = job_alg(jb);
  const int kidx = job_key(jb);
  const DevKey& K = a.keys[kidx];
  const uint32_t nch = job_siglen(jb);
  const int ks = es_size(alg);                  // bytes of r and of s (R18: from the alg)
  // the host sends only signing inputs that fit the LDS stage (a longer one
  // would never reach this kernel; it is refused here rather than overrun)
  const bool in_ok = jb.sig_in_len <= EC_SMALL_IN_MAX;
  // byte position inside the first aligned dword, from the absolute address
  // (the caller's arena need not be 4-byte aligned)
  const uint32_t in_shift = (uint32_t)((uintptr_t)(a.arena + jb.off) & 3u);
  const uint32_t sig_shift = (uint32_t)((uintptr_t)(a.arena + jb.sig_off) & 3u);
  if (tid == 0) { flag[0] = in_ok ? 0 : 1; flag[1] = 0; }
  SM_STAMP(0);

  // ---- phase 1: both streams into LDS
  if (wave == 0 && in_ok) {
    sm_stage_input(in_w, reinterpret_cast<const uint32_t*>(a.arena + jb.off - in_shift), in_shift, jb.sig_in_len,
                   sm_hash_bits(alg), lane);
  } else if (wave == 1) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(a.arena + jb.sig_off - sig_shift);
    const uint32_t nd = nch <= SM_SIG_CHARS ? (sig_shift + nch + 3) / 4 : 0u;
    if ((uint32_t)lane < nd) sig_w[lane] = g[lane];
  }
  SM_STAMP(1);
  __syncthreads();

  // ---- phase 2: signature characters -> bytes (wave 1, a quad per lane)
  const uint32_t D = sm_b64_len(nch);
  const bool size_ok = nch <= SM_SIG_CHARS && (nch & 3u) != 1u && D == 2u * (uint32_t)ks;
  if (wave == 1 && size_ok) {
    if (sm_b64_decode(sig_w, sig_shift, nch, sig_b, lane) && lane == 0) flag[0] = 1;
  }
  __syncthreads();

  // ---- phase 3: r, s words (wave 1: lane q builds word q of r, lane 32 + q of s)
  if (wave == 1 && size_ok) {
    const int q = lane & 31, half = lane >> 5;
    if (q < CW) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int pos = ks - 1 - (4 * q + b);               // big-endian byte index inside r (or s)
        if (pos >= 0) w |= (uint32_t)sig_b[half * ks + pos] << (8 * b);
      }
      // bytes at or above the curve's size must be zero (r, s < n); the top
      // word keeps only the bits below 8 CB
      if (4 * q + 4 > CB) {
        const uint32_t hi = 4 * q >= CB ? ~0u : ~0u << (8 * (CB - 4 * q));
        if (w & hi) flag[0] = 1;
      }
      rs_w[half * CW + q] = w;
    }
    // an alg whose scalars are longer than the curve's: the leading bytes past CW words
    for (int pos = lane; pos < ks - 4 * CW; pos += 64)
      if (sig_b[pos] != 0 || sig_b[ks + pos] != 0) flag[0] = 1;
  }
  SM_STAMP(2);
  __syncthreads();

  // ---- phase 4: hash (wave 0 lane 0) || checks, s^-1, u2 (wave 1 lane 0)
  if (wave == 0 && lane == 0 && in_ok) {
    // the padded message words straight from the LDS stage (ds_read; through
    // sha2::MemString's generic pointer they were flat loads: ~6.7 us per block)
    sm_hash(in_w, in_shift, jb.sig_in_len, sm_hash_bits(alg), dig_w);
  }
  uint32_t w[L];                                   // s^-1 R (wave 1 lane 0)
  if (wave == 1 && lane < 4) {                     // four lanes: the inversion's limb rows (mp::inv_plain_var4)
    bool ok = size_ok && flag[0] == 0 && K.valid != 0 && (uint32_t)alg - 7u < 3u;
    uint32_t rw[CW], sw[CW], r[L], s[L], nl[L];
#pragma unroll
    for (int q = 0; q < CW; ++q) { rw[q] = rs_w[q]; sw[q] = rs_w[CW + q]; }
    mp::words_to_limbs<L, CW>(r, rw);
    mp::words_to_limbs<L, CW>(s, sw);
    mp::set_const<Fn>(nl, Fn::M);
    ok = ok && !zero_limbs<L>(r) && !zero_limbs<L>(s) && lt_limbs<L>(r, nl) && lt_limbs<L>(s, nl);
    if (ok) {                                      // the same on the four lanes
      uint32_t si[L], u2[L];
      mp::inv_plain_var4<Fn>(si, s);                // s^-1 (plain)
      if (lane == 0) {
        mp::to_mont<Fn>(w, si);                     // s^-1 R
        mp::mul<Fn>(u2, r, w); mp::csub<Fn>(u2);    // r s^-1
#pragma unroll
        for (int j = 0; j < L; ++j) { sc[j] = r[j]; sc[2 * L + j] = u2[j]; }
        flag[1] = 1;
      }
    }
  }
  SM_STAMP(3);
  __syncthreads();
  const bool run = flag[1] != 0;                   // block-uniform

  // ---- phase 5: e (R21), u1, comb digits (wave 1 lane 0)
  if (run && wave == 1 && lane == 0) {
    constexpr int EW = ScalarRaw<CV>::EW;
    const int hw = ec_hash_words<CV>(alg);
    uint32_t ew[EW], e[L], u1[L], u2[L];
#pragma unroll
    for (int q = 0; q < EW; ++q) {
      const int src = hw - 1 - q;
      ew[q] = src >= 0 ? dig_w[src < 0 ? 0 : src] : 0u;
    }
    mp::words_to_limbs<L, EW>(e, ew);
    mp::csub<Fn>(e);
    mp::mul<Fn>(u1, e, w); mp::csub<Fn>(u1);
#pragma unroll
    for (int j = 0; j < L; ++j) { sc[L + j] = u1[j]; u2[j] = sc[2 * L + j]; }
    sm_recode<WG, NG, L>(u1, digs);
    sm_recode<WQ, NQ, L>(u2, digs + NG);
  }
  SM_STAMP(4);
  __syncthreads();

  // ---- phase 6: comb sum over S lanes of wave 0, exact combine, x(R) check
  SM_STAMP(5);
  if (wave != 0) return;
  JPt<Fp> P;
  P.inf = true;
#pragma unroll
  for (int j = 0; j < L; ++j) { P.X[j] = 0; P.Y[j] = 0; P.Z[j] = 0; }
  bool exc = false;
  const int sub = lane;
  if (run && sub < S) {
    const uint32_t* __restrict__ qtab = key_table(K);
    const uint32_t* __restrict__ gtab = a.gtab;
    uint32_t X[L], Y[L], Z[L];
    bool empty = true;
    // the lane's additions k = 0, 1, ...: window sub + S (k / 2) of G (k even)
    // or of Q (k odd); each entry's loads are issued one addition ahead (a
    // lone wave has nothing else to hide their HBM latency behind)
    constexpr int K = 2 * ((NWIN + S - 1) / S);
    constexpr int STRIDE = ec_stride(CV::CLS), NEG = ec_entries(CV::CLS, true), NEQ = 1 << (CV::WQ - 1);
    auto fetch = [&](int k, uint32_t* x, uint32_t* y) -> int {
      const int wi = sub + S * (k >> 1);
      const bool gen = (k & 1) == 0;
      if (wi >= (gen ? NG : NQ)) return 0;
      const int d = digs[gen ? wi : NG + wi];
      if (d == 0) return 0;
      const int ad = d < 0 ? -d : d;
      const uint32_t* ent = gen ? gtab + ((int64_t)wi * NEG + (ad - 1)) * STRIDE
                                : qtab + ((int64_t)wi * NEQ + (ad - 1)) * STRIDE;
      load_entry<CV>(ent, x, y);
      return d;
    };
    uint32_t xc[L], yc[L], xn[L], yn[L];
    int dc = fetch(0, xc, yc);
    int nadd = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int dn = 0;
      if (k + 1 < K) dn = fetch(k + 1, xn, yn);
      if (dc != 0) {
        if (dc < 0) mp::neg<Fp>(yc, yc);
        if (empty) {
          mp::copy<Fp>(X, xc);
          mp::copy<Fp>(Y, yc); mp::freduce<Fp>(Y);
          mp::set_const<Fp>(Z, Fp::ONE);
          empty = false;
        } else if (nadd == 1) {
          madd_z1<Fp>(X, Y, Z, xc, yc);             // the accumulator is one entry (Z == 1)
        } else {
          madd<Fp>(X, Y, Z, xc, yc);
        }
        ++nadd;
      }
      if (k + 1 < K) {
        mp::copy<Fp>(xc, xn);
        mp::copy<Fp>(yc, yn);
        dc = dn;
      }
    }
    if (!empty) {
      mp::canon<Fp>(X); mp::canon<Fp>(Y); mp::canon<Fp>(Z);
      exc = mp::is_zero_canon<Fp>(Z);            // an exceptional step in this lane's chain
      mp::copy<Fp>(P.X, X); mp::copy<Fp>(P.Y, Y); mp::copy<Fp>(P.Z, Z);
      P.inf = false;
    }
  }
  SM_STAMP(6);
  // lanes past S (and every lane of a token that does not run) carry empty
  // partials through the pairwise levels
#pragma unroll 1
  for (int off = 1; off < S; off <<= 1) jadd_pair<CV>(P, off, exc);
  if (lane != 0) return;
  SM_STAMP(7);
  bool ok = false;
  if (run) {
    uint32_t r[L];
#pragma unroll
    for (int j = 0; j < L; ++j) r[j] = sc[j];
    if (exc) {
      uint32_t u1[L], u2[L];
#pragma unroll
      for (int j = 0; j < L; ++j) { u1[j] = sc[L + j]; u2[j] = sc[2 * L + j]; }
      ok = ec_exact_ok<CV>(a.keyblob + K.aux_off, r, u1, u2);
    } else if (!P.inf) {                          // R = infinity: rejected
      ok = ec_x_matches<CV>(P.X, P.Z, r);
    }
  }
  a.verdict[a.out[blockIdx.x]] = ok ? 1 : 0;
#if JG_SMALL_PROF
  SM_STAMP(8);
  const uint64_t t0 = stamp[0][0];
  printf("smallprof w0 %lu %lu %lu %lu %lu %lu %lu %lu w1 %lu %lu %lu %lu %lu\n",
         stamp[0][1] - t0, stamp[0][2] - t0, stamp[0][3] - t0, stamp[0][4] - t0, stamp[0][5] - t0,
         stamp[0][6] - t0, stamp[0][7] - t0, stamp[0][8] - t0, stamp[1][1] - t0, stamp[1][2] - t0,
         stamp[1][3] - t0, stamp[1][4] - t0, stamp[1][5] - t0);
#endif
}

template <class CV>
void small_launch(const EcSmallArgs& a, hipStream_t s) {
  if (a.n == 0) return;
  hipLaunchKernelGGL(k_ec_small<CV>, dim3(a.n), dim3(SM_THREADS), 0, s, a);
}

}  // namespace
