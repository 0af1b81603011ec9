// ed25519.hip -- Ed25519 verification on gfx950.
//
// Replaces go-jose edEncrypterVerifier -> crypto/ed25519.Verify (SURVEY.md a11,
// rules R23-R26): len(sig) == 64, sig[63] & 0xE0 == 0, S < L,
// k = SHA-512(R || A || M) mod L, R' = [S]B + [k](-A) (cofactorless), accept iff
// encode(R') == sig[:32] byte for byte.
//   k_ed_point  : S and k recoded to signed W-bit windows (ed25519.hpp); R' as
//                 a sum of one precomputed multiple of B and one of -A per window
//                 (Niels-form comb tables), extended twisted-Edwards coordinates
//                 with the complete a = -1 addition law (no exceptional cases)
//   k_ed_finish : Z^-1, canonical encoding, byte compare with R
// Key staging decodes A with filippo.io/edwards25519 SetBytes semantics
// (non-canonical y accepted, x = 0 with the sign bit set accepted).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "ed25519.hpp"
#include "fe25519.hpp"
#include "mp.hpp"
#include "tables.hpp"
#include "small_common.hpp"

using namespace jgk;

namespace {

using Fp = ED25519P;
using Fl = ED25519L;
constexpr int L = Fp::L;

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

struct EPt { uint32_t X[L], Y[L], Z[L], T[L]; };

// Hot loop (k_ed_point): points and table entries in the radix-2^25.5 form of
// fe25519.hpp (plain values, no Montgomery factor).  Table building, key
// decoding and the finish stay in ED25519P's Montgomery form (mp.hpp) and
// convert at the boundary (entries are stored canonical in radix 2^25.5).
struct FPt { uint32_t X[fe::L], Y[fe::L], Z[fe::L], T[fe::L]; };

#ifndef JG_ED_SHARE_PRE
#define JG_ED_SHARE_PRE 0
#endif
// extended + Niels (y+x, y-x, 2dxy) affine -> extended (complete, a = -1):
// 7 products.  fe::mul's second operand carries the factor 19 and must be the
// smaller one: the point side for A, B, C, then E and G (tools/fe25519_bounds.py)
__device__ __forceinline__ void add_niels(FPt& P, const uint32_t* ypx, const uint32_t* ymx, const uint32_t* t2d) {
  uint32_t t[fe::L], A[fe::L], B[fe::L], C[fe::L], E[fe::L], F[fe::L], G[fe::L], H[fe::L];
  // ordered so that each input dies as early as it can (P.T and 2dxy first):
  // the live set stays near 4 field elements + one product's columns
  fe::mul(C, t2d, P.T);
  fe::sub_dbl(F, P.Z, C); fe::add_dbl(G, P.Z, C);         // D - C, D + C with D = 2 Z
  fe::sub(t, P.Y, P.X); fe::mul(A, ymx, t);
  fe::add(t, P.Y, P.X); fe::mul(B, ypx, t);
  fe::sub(E, B, A); fe::add(H, B, A);
#if JG_ED_SHARE_PRE
  // E and G are the g side of two products each, F and H the f side: their
  // operand forms are prepared once
  uint32_t e19[fe::L], g19[fe::L], f2[fe::L], h2[fe::L];
  fe::pre_g(e19, E); fe::pre_g(g19, G); fe::pre_f(f2, F); fe::pre_f(h2, H);
  fe::mul_pre(P.X, F, f2, E, e19); fe::mul_pre(P.T, H, h2, E, e19);
  fe::mul_pre(P.Y, H, h2, G, g19); fe::mul_pre(P.Z, F, f2, G, g19);
#else
  fe::mul(P.X, F, E); fe::mul(P.T, H, E); fe::mul(P.Y, H, G); fe::mul(P.Z, F, G);
#endif
}

// extended + extended in radix 2^25.5 (complete, a = -1; add-2008-hwcd-3 with
// k = 2d): 9 products, the operand shapes of add_niels (tools/fe25519_bounds.py)
__device__ __forceinline__ void add_ext(FPt& R, const FPt& P, const FPt& Q) {
  // 2d mod p, canonical radix-2^25.5 limbs
  constexpr uint32_t D2[fe::L] = {0x2b2f159u, 0x1a6e509u, 0x22add7au, 0x0d4141du, 0x0038052u,
                                  0x0f3d130u, 0x3407977u, 0x19ce331u, 0x1c56dffu, 0x0901b67u};
  uint32_t t[fe::L], u[fe::L], A[fe::L], B[fe::L], C[fe::L], E[fe::L], F[fe::L], G[fe::L], H[fe::L];
  fe::mul(t, Q.T, D2);                                    // 2d T2
  fe::mul(C, t, P.T);
  fe::mul(t, P.Z, Q.Z);
  fe::add(t, t, t);                                       // D
  fe::sub(F, t, C); fe::add(G, t, C);
  fe::sub(t, P.Y, P.X); fe::sub(u, Q.Y, Q.X); fe::mul(A, u, t);
  fe::add(t, P.Y, P.X); fe::add(u, Q.Y, Q.X); fe::mul(B, u, t);
  fe::sub(E, B, A); fe::add(H, B, A);
  fe::mul(R.X, F, E); fe::mul(R.T, H, E); fe::mul(R.Y, H, G); fe::mul(R.Z, F, G);
}

// radix-2^25.5 limbs (limbs < 2^31) -> ED25519P Montgomery form
__device__ void fe_to_mont(uint32_t* m, const uint32_t* f) {
  uint32_t c[fe::L], w[8], pl[L];
  fe::copy(c, f);
  fe::canon(c);
  fe::to_words(w, c);
  mp::words_to_limbs<L, 8>(pl, w);
  mp::to_mont<Fp>(m, pl);
}

// ED25519P Montgomery form (normalized) -> canonical radix-2^25.5 limbs
__device__ void mont_to_fe(uint32_t* f, const uint32_t* m) {
  uint32_t pl[L], w[8];
  mp::from_mont<Fp>(pl, m);
  mp::limbs_to_words<L, 8>(w, pl);
  fe::from_words(f, w);
}

// extended + extended (complete)
__device__ void add_full(EPt& R, const EPt& P, const EPt& Q) {
  uint32_t t[L], u[L], A[L], B[L], C[L], D[L], E[L], F[L], G[L], H[L], d2[L];
  mp::sub<Fp>(t, P.Y, P.X); mp::sub<Fp>(u, Q.Y, Q.X); mp::mul<Fp>(A, t, u);
  mp::add<Fp>(t, P.Y, P.X); mp::add<Fp>(u, Q.Y, Q.X); mp::mul<Fp>(B, t, u);
  mp::set_const<Fp>(d2, ED25519C::D2_M);
  mp::mul<Fp>(t, P.T, d2); mp::mul<Fp>(C, t, Q.T);
  mp::mul<Fp>(t, P.Z, Q.Z); mp::add<Fp>(D, t, t); mp::norm<Fp>(D);
  mp::sub<Fp>(E, B, A); mp::sub<Fp>(F, D, C); mp::add<Fp>(G, D, C); mp::add<Fp>(H, B, A);
  mp::mul<Fp>(R.X, E, F); mp::mul<Fp>(R.Y, G, H); mp::mul<Fp>(R.T, E, H); mp::mul<Fp>(R.Z, F, G);
}

template <int NE>
__device__ __forceinline__ void add_window(FPt& P, const uint32_t* __restrict__ tab, int w, int d) {
  if (d == 0) return;
  const int ad = d < 0 ? -d : d;
  const uint32_t* ent = tab + ((int64_t)w * NE + (ad - 1)) * ED_STRIDE;
  uint32_t ypx[fe::L], ymx[fe::L], t2d[fe::L];
#pragma unroll
  for (int j = 0; j < fe::L; ++j) { ypx[j] = ent[j]; ymx[j] = ent[fe::L + j]; t2d[j] = ent[2 * fe::L + j]; }
  // -(x, y) = (-x, y): swap y+x / y-x and negate 2dxy -- selected per lane, so
  // the wave runs ONE addition (a branch on the digit's sign made lanes of
  // both signs execute both inlined copies of add_niels)
  const bool neg = d < 0;
  uint32_t a1[fe::L], a2[fe::L], nt[fe::L];
  fe::neg(nt, t2d);
#pragma unroll
  for (int j = 0; j < fe::L; ++j) {
    a1[j] = neg ? ymx[j] : ypx[j];
    a2[j] = neg ? ypx[j] : ymx[j];
    t2d[j] = neg ? nt[j] : t2d[j];
  }
  add_niels(P, a1, a2, t2d);
}

// signed W-bit digits d_w in [-2^(W-1), 2^(W-1)], s = sum d_w 2^(W w);
// digit w goes to dg[w * stride] (k_ed_point: the wave's LDS digit rows)
template <int W, int NWIN>
__device__ __forceinline__ void recode(int* dg, const uint32_t* s, int stride = 1) {
  constexpr uint32_t DM = (1u << W) - 1u;
  int c = 0;
#pragma unroll
  for (int w = 0; w < NWIN; ++w) {
    const int bit = W * w, q = bit / MP_W, sh = bit % MP_W;
    uint32_t b = q < L ? (s[q] >> sh) : 0u;
    if (sh > MP_W - W && q + 1 < L) b |= s[q + 1] << (MP_W - sh);
    int v = (int)(b & DM) + c;
    c = v > (1 << (W - 1));
    dg[w * stride] = v - (c << W);
  }
}

// JG_ED_POINT_ATTR: occupancy.  With fe::mul's asm columns the compiler takes
// 129-132 VGPRs (3 waves per SIMD); capped at 4 waves it spills 5 registers
// and runs 1 % faster (1 M EdDSA tokens at W = 24: 0.874 -> 0.866 ms, HEAD's
// C++ columns 0.917 ms, profiles/r06_s2/ed_ab.json).  Round 4: with the C++
// columns at ~141 VGPRs the same cap cost 4 % (profiles/r04_s6/).
#ifndef JG_ED_POINT_ATTR
#define JG_ED_POINT_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
// One Niels addition of the table entry at e (30 words: y+x, y-x, 2dxy) for
// digit d, from registers (k_ed_point's prefetching loop)
__device__ __forceinline__ void add_entry(FPt& P, const uint32_t* e, int d) {
  if (d == 0) return;
  const bool neg = d < 0;
  uint32_t a1[fe::L], a2[fe::L], nt[fe::L], t2d[fe::L];
#pragma unroll
  for (int j = 0; j < fe::L; ++j) t2d[j] = e[2 * fe::L + j];
  fe::neg(nt, t2d);
#pragma unroll
  for (int j = 0; j < fe::L; ++j) {
    a1[j] = neg ? e[fe::L + j] : e[j];
    a2[j] = neg ? e[j] : e[fe::L + j];
    t2d[j] = neg ? nt[j] : t2d[j];
  }
  add_niels(P, a1, a2, t2d);
}

// 30 words of a table entry as 7 x 16 B + 8 B loads
struct EdEnt { uint4 q[7]; uint2 t; };
__device__ __forceinline__ void load_ent(EdEnt& r, const uint32_t* __restrict__ ent) {
  const uint4* e4 = reinterpret_cast<const uint4*>(ent);
#pragma unroll
  for (int i = 0; i < 7; ++i) r.q[i] = e4[i];
  r.t = reinterpret_cast<const uint2*>(ent)[14];
}
__device__ __forceinline__ void ent_words(uint32_t* w, const EdEnt& r) {
#pragma unroll
  for (int i = 0; i < 7; ++i) { w[4 * i] = r.q[i].x; w[4 * i + 1] = r.q[i].y; w[4 * i + 2] = r.q[i].z; w[4 * i + 3] = r.q[i].w; }
  w[28] = r.t.x; w[29] = r.t.y;
}

// PF (launches below ~2 waves per SIMD, JG_ED_PF_MAX): the entry of addition
// k + 1 is loaded while addition k computes.  At full occupancy other waves
// hide the gathers' latency; a launch of under one wave per SIMD (configs[4]'s
// Ed25519 class, ~38 k tokens) has no other wave, and its 22 additions each
// waited ~2 us on their entry (k_ed_point ran at 0.20 of the MAD roofline).
template <int WA, bool PF>
__device__ __forceinline__ void ed_point_body(const EdArgs& a) {
  const int64_t p = a.begin + (int64_t)blockIdx.x * WAVE + threadIdx.x;
  const int64_t np = a.npad;
  const JobDev jb = a.jobs[p];
  if (!job_live(jb)) return;
  const int kidx = __builtin_amdgcn_readfirstlane(job_key(jb));
  const DevKey& K = a.keys[kidx];
  bool ok = a.status[p] == ST_OK && K.valid && a.siglen[p] == 64;
  // S: canonical, and sig[63] & 0xE0 == 0
  uint32_t sw[8], s[L];
#pragma unroll
  for (int q = 0; q < 8; ++q) sw[q] = a.sigw[(int64_t)(8 + q) * np + p];
  ok = ok && (sw[7] & 0xE0000000u) == 0;
  mp::words_to_limbs<L, 8>(s, sw);
  uint32_t lord[L];
  mp::set_const<Fl>(lord, Fl::M);
  ok = ok && lt_limbs(s, lord);
  // k = H mod L  (H little-endian, 512 bits)
  uint32_t k[L];
  {
    uint32_t hw[16], hl[2 * L];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t x = a.dig[(int64_t)q * np + p];
      hw[q] = (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
    }
    mp::words_to_limbs<2 * L, 16>(hl, hw);
    uint64_t tt[2 * L];
#pragma unroll
    for (int j = 0; j < 2 * L; ++j) tt[j] = hl[j];
    uint32_t kr[L], rr[L];
    mp::mont_reduce<Fl>(kr, tt);            // H / R mod L
    mp::set_const<Fl>(rr, Fl::RR);
    mp::mul<Fl>(k, kr, rr);                 // H mod L (< 2L)
    mp::csub<Fl>(k);
  }
  constexpr int NB = ed_windows(true), NA = ed_windows_w(WA), NW = NB > NA ? NB : NA;
  // the signed digits of S (B windows) and k (-A windows) wait in LDS, one row
  // per window, lane-contiguous (conflict-free): held in registers they took
  // NB + NA VGPRs through the whole loop and the kernel three waves per SIMD
  __shared__ int dg[(NB + NA) * WAVE];
  const int lane = (int)threadIdx.x;
  recode<ed_comb_w(true), NB>(dg + lane, s, WAVE);
  recode<WA, NA>(dg + NB * WAVE + lane, k, WAVE);
  FPt P;                                      // the neutral element (0, 1, 1, 0)
  fe::set_small(P.X, 0u); fe::set_small(P.Y, 1u); fe::set_small(P.Z, 1u); fe::set_small(P.T, 0u);
  const uint32_t* __restrict__ atab = key_table(K);
  if constexpr (PF) {
    // additions k = 0 .. 2 NW - 1: B window k / 2 (even k), -A window k / 2 (odd)
    constexpr int NEB = ed_entries(true), NEA = 1 << (WA - 1);
    auto digit = [&](int k) {
      const int w = k >> 1;
      return (k & 1) ? (w < NA ? dg[(NB + w) * WAVE + lane] : 0) : (w < NB ? dg[w * WAVE + lane] : 0);
    };
    auto entry = [&](int k, int d) {
      const int ad = d < 0 ? -d : d;
      const int w = ad ? k >> 1 : 0;                 // a zero digit loads window 0's first entry (unused)
      const int64_t i = ad ? ad - 1 : 0;
      return (k & 1) ? atab + ((int64_t)w * NEA + i) * ED_STRIDE : a.btab + ((int64_t)w * NEB + i) * ED_STRIDE;
    };
    EdEnt rn;
    int dn = digit(0);
    load_ent(rn, entry(0, dn));
#pragma unroll 1
    for (int k = 0; k < 2 * NW; ++k) {
      uint32_t e[30];
      ent_words(e, rn);
      const int dc = dn;
      if (k + 1 < 2 * NW) {
        dn = digit(k + 1);
        load_ent(rn, entry(k + 1, dn));
      }
      add_entry(P, e, dc);
    }
  } else {
#pragma unroll 1
  for (int w = 0; w < NW; ++w) {
    // each lane reads back only its own digits: no barrier needed
    const int e1 = w < NB ? dg[w * WAVE + lane] : 0;
    const int e2 = w < NA ? dg[(NB + w) * WAVE + lane] : 0;
    add_window<ed_entries(true)>(P, a.btab, w, e1);
    add_window<(1 << (WA - 1))>(P, atab, w, e2);
  }
  }
#pragma unroll
  for (int j = 0; j < fe::L; ++j) {                // radix-2^25.5 limbs (k_ed_finish converts)
    a.xyz[(int64_t)j * np + p] = P.X[j];
    a.xyz[(int64_t)(L + j) * np + p] = P.Y[j];
    a.xyz[(int64_t)(2 * L + j) * np + p] = P.Z[j];
  }
  if (!ok) a.status[p] = ST_REJECT;
}

template <int WA>
__global__ void __launch_bounds__(64) JG_ED_POINT_ATTR k_ed_point(EdArgs a) {
  ed_point_body<WA, false>(a);
}
#ifndef JG_ED_POINT_PF_ATTR
#define JG_ED_POINT_PF_ATTR __attribute__((amdgpu_waves_per_eu(2)))
#endif
template <int WA>
__global__ void __launch_bounds__(64) JG_ED_POINT_PF_ATTR k_ed_point_pf(EdArgs a) {
  ed_point_body<WA, true>(a);
}

// k_ed_point with S lanes per token (S = 2 or 4), for launches that fill the
// GPU poorly (a coalesced single-token batch, a mixed batch's Ed25519 class):
// the first S/2 lanes sum the [S]B windows, the others the [k](-A) windows,
// each lane every (S/2)-th window into its own extended point; the partials
// are added across lanes with the complete law (add_ext), and lane 0 writes
// the sum.  A token's latency falls to about 2/S of k_ed_point's for
// log2(S) extra additions on its path (S - 1 in all).  The B-side lanes check
// S, the A-side lanes derive k = H mod L.
// PF: the lane's next table entry loads while its current addition computes
// (as k_ed_point_pf)
template <int WA, int S, bool PF = false>
__global__ void __launch_bounds__(64) JG_ED_POINT_ATTR k_ed_point_split(EdArgs a) {
  static_assert(S == 2 || S == 4, "two or four lanes per token");
  constexpr int H = S / 2;                        // lanes per scalar
  const int lane = (int)threadIdx.x, sub = lane % S, side = sub / H, par = sub % H;
  const int64_t p = a.begin + (int64_t)blockIdx.x * (WAVE / S) + lane / S;
  const int64_t np = a.npad;
  bool live = p < a.end;
  JobDev jb{};
  if (live) jb = a.jobs[p];
  live = live && job_live(jb);
  // (every lane stays for the exchange below; dead tokens compute on key 0)
  const int kidx = live ? job_key(jb) : 0;
  const DevKey& K = a.keys[kidx];
  bool ok = live && a.status[p] == ST_OK && K.valid && a.siglen[p] == 64;
  constexpr int NB = ed_windows(true), NA = ed_windows_w(WA), NW = NB > NA ? NB : NA;
  __shared__ int dg[NW * WAVE];
  uint32_t sc[L];                               // B side: S, A side: k
  if (side == 0) {
    // S: canonical, and sig[63] & 0xE0 == 0
    uint32_t sw[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) sw[q] = live ? a.sigw[(int64_t)(8 + q) * np + p] : 0u;
    ok = ok && (sw[7] & 0xE0000000u) == 0;
    mp::words_to_limbs<L, 8>(sc, sw);
    uint32_t lord[L];
    mp::set_const<Fl>(lord, Fl::M);
    ok = ok && lt_limbs(sc, lord);
    recode<ed_comb_w(true), NB>(dg + lane, sc, WAVE);
    for (int w = NB; w < NW; ++w) dg[w * WAVE + lane] = 0;
  } else {
    // k = H mod L  (H little-endian, 512 bits)
    uint32_t hw[16], hl[2 * L];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t x = live ? a.dig[(int64_t)q * np + p] : 0u;
      hw[q] = (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
    }
    mp::words_to_limbs<2 * L, 16>(hl, hw);
    uint64_t tt[2 * L];
#pragma unroll
    for (int j = 0; j < 2 * L; ++j) tt[j] = hl[j];
    uint32_t kr[L], rr[L];
    mp::mont_reduce<Fl>(kr, tt);
    mp::set_const<Fl>(rr, Fl::RR);
    mp::mul<Fl>(sc, kr, rr);
    mp::csub<Fl>(sc);
    recode<WA, NA>(dg + lane, sc, WAVE);
    for (int w = NA; w < NW; ++w) dg[w * WAVE + lane] = 0;
  }
  FPt P;                                        // the neutral element (0, 1, 1, 0)
  fe::set_small(P.X, 0u); fe::set_small(P.Y, 1u); fe::set_small(P.Z, 1u); fe::set_small(P.T, 0u);
  if (live) {
    const uint32_t* __restrict__ tab = side ? key_table(K) : a.btab;
    const int ne = side ? (1 << (WA - 1)) : ed_entries(true);
    if constexpr (PF) {
      // step i: window par + H i (rows past the scalar's windows hold digit 0)
      const int nst = par < NW ? (NW - par + H - 1) / H : 0;
      auto entry = [&](int i, int d) {
        const int ad = d < 0 ? -d : d;
        const int w = ad ? par + H * i : 0;           // a zero digit loads window 0's first entry (unused)
        return tab + ((int64_t)w * ne + (ad ? ad - 1 : 0)) * ED_STRIDE;
      };
      EdEnt rn;
      int dn = nst > 0 ? dg[par * WAVE + lane] : 0;
      if (nst > 0) load_ent(rn, entry(0, dn));
#pragma unroll 1
      for (int i = 0; i < nst; ++i) {
        uint32_t e[30];
        ent_words(e, rn);
        const int dc = dn;
        if (i + 1 < nst) {
          dn = dg[(par + H * (i + 1)) * WAVE + lane];
          load_ent(rn, entry(i + 1, dn));
        }
        add_entry(P, e, dc);
      }
    } else
#pragma unroll 1
    for (int w = par; w < NW; w += H) {
      const int d = dg[w * WAVE + lane];        // this lane's own digit row: no barrier needed
      if (d == 0) continue;
      const int ad = d < 0 ? -d : d;
      const uint32_t* ent = tab + ((int64_t)w * ne + (ad - 1)) * ED_STRIDE;
      uint32_t ypx[fe::L], ymx[fe::L], t2d[fe::L], a1[fe::L], a2[fe::L], nt[fe::L];
#pragma unroll
      for (int j = 0; j < fe::L; ++j) { ypx[j] = ent[j]; ymx[j] = ent[fe::L + j]; t2d[j] = ent[2 * fe::L + j]; }
      const bool neg = d < 0;
      fe::neg(nt, t2d);
#pragma unroll
      for (int j = 0; j < fe::L; ++j) {
        a1[j] = neg ? ymx[j] : ypx[j];
        a2[j] = neg ? ypx[j] : ymx[j];
        t2d[j] = neg ? nt[j] : t2d[j];
      }
      add_niels(P, a1, a2, t2d);
    }
  }
  // the partner lane's partial (and verdict); every lane of the wave joins
  auto partner = [&](FPt& Q, int off) {
#pragma unroll
    for (int j = 0; j < fe::L; ++j) {
      Q.X[j] = __shfl_xor(P.X[j], off);
      Q.Y[j] = __shfl_xor(P.Y[j], off);
      Q.Z[j] = __shfl_xor(P.Z[j], off);
      Q.T[j] = __shfl_xor(P.T[j], off);
    }
    const int pok = __shfl_xor((int)ok, off);      // every lane reads (see ec_small.hpp jadd_pair)
    ok = ok && pok != 0;
  };
  if constexpr (S == 4) {                       // lanes xor 1: the two partials of each scalar
    FPt Q;
    partner(Q, 1);
    add_ext(P, P, Q);                           // (add_ext reads all of P before writing R)
  }
  {                                             // lane 0: [S]B + [k](-A)
    FPt Q;
    partner(Q, H);
    if (!live || sub != 0) return;
    add_ext(P, P, Q);
  }
#pragma unroll
  for (int j = 0; j < fe::L; ++j) {                // radix-2^25.5 limbs (k_ed_finish converts)
    a.xyz[(int64_t)j * np + p] = P.X[j];
    a.xyz[(int64_t)(L + j) * np + p] = P.Y[j];
    a.xyz[(int64_t)(2 * L + j) * np + p] = P.Z[j];
  }
  if (!ok) a.status[p] = ST_REJECT;
}

// Batched finish (Montgomery's trick, as k_ec_scalar_batch): thread i owns the
// B tokens p_j = begin + i + j*S and pays ONE inversion for all their Z:
//   pass 1: c_j = Z_0 ... Z_j, parked in the prefix rows;  inv = c_{B-1}^-1
//   pass 2 (j descending): Z_j^-1 = inv * c_{j-1}, inv *= Z_j; affine x, y,
//           canonical encoding, byte compare with R.
// Z != 0 for every output of the complete addition law; padding and rejected
// tokens contribute Z = 1.
// Waves per block sharing one inversion (mp::block_inv, as k_ec_scalar_batch)
#ifndef JG_ED_FINISH_WPB
#define JG_ED_FINISH_WPB 4
#endif
constexpr int ED_FINISH_WPB = JG_ED_FINISH_WPB;
__global__ void __launch_bounds__(64 * ED_FINISH_WPB) k_ed_finish(EdArgs a, int B) {
  const int64_t np = a.npad;
  const int64_t n = a.end - a.begin;
  const int64_t S = (n + B - 1) / B;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ED_FINISH_WPB == 1 && i >= S) return;       // (blocks of several waves keep every thread for the barriers)
  uint32_t* pre = a.xyz + (int64_t)3 * L * np;
  auto live = [&](int64_t p) { return job_live(a.jobs[p]) && a.status[p] == ST_OK; };
  auto load_z = [&](int64_t p, uint32_t* Z) {
    if (live(p)) {
      uint32_t f[fe::L];
#pragma unroll
      for (int j = 0; j < fe::L; ++j) f[j] = a.xyz[(int64_t)(2 * L + j) * np + p];
      fe_to_mont(Z, f);
    } else {
      mp::set_const<Fp>(Z, Fp::ONE);
    }
  };
  uint32_t acc[L];
  mp::set_const<Fp>(acc, Fp::ONE);
  int nb = 0;
  for (int j = 0; j < B && i < S; ++j) {
    const int64_t p = a.begin + i + (int64_t)j * S;
    if (p >= a.end) break;
    uint32_t Z[L];
    load_z(p, Z);
    mp::mul<Fp>(acc, acc, Z);
#pragma unroll
    for (int k = 0; k < L; ++k) pre[(int64_t)k * np + p] = acc[k];
    ++nb;
  }
  uint32_t inv[L];
  mp::block_inv<Fp, ED_FINISH_WPB>(inv, acc);
  for (int j = nb - 1; j >= 0; --j) {
    const int64_t p = a.begin + i + (int64_t)j * S;
    uint32_t cprev[L], Z[L], zi[L];
    if (j > 0) {
#pragma unroll
      for (int k = 0; k < L; ++k) cprev[k] = pre[(int64_t)k * np + p - S];
    } else {
      mp::set_const<Fp>(cprev, Fp::ONE);
    }
    load_z(p, Z);
    mp::mul<Fp>(zi, inv, cprev);                 // Z_j^-1 (Montgomery)
    mp::mul<Fp>(inv, inv, Z);
    if (!job_live(a.jobs[p])) continue;
    if (a.status[p] != ST_OK) { a.verdict_pad[p] = 0; continue; }
    uint32_t X[L], Y[L], x[L], y[L], tt[L], fx[fe::L], fy[fe::L];
#pragma unroll
    for (int k = 0; k < fe::L; ++k) {
      fx[k] = a.xyz[(int64_t)k * np + p];
      fy[k] = a.xyz[(int64_t)(L + k) * np + p];
    }
    fe_to_mont(X, fx);
    fe_to_mont(Y, fy);
    mp::mul<Fp>(tt, X, zi); mp::from_mont<Fp>(x, tt);
    mp::mul<Fp>(tt, Y, zi); mp::from_mont<Fp>(y, tt);
    uint32_t enc[8];
    mp::limbs_to_words<L, 8>(enc, y);
    enc[7] = (enc[7] & 0x7fffffffu) | ((x[0] & 1u) << 31);
    uint32_t diff = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) diff |= enc[q] ^ a.sigw[(int64_t)q * np + p];
    a.verdict_pad[p] = diff == 0;
  }
}

// ------------------------------------------------------------------ one launch (small batches)
// k_ed_small: one 128-thread block per EdDSA token (jwt/keyset.go:27-32 single
// calls), the work of k_prep_ed, k_ed_point_split and k_ed_finish in one launch:
//   wave 1 decodes the signature (R, S; len 64, S < L, sig[63] & 0xE0 == 0:
//   R24) and recodes S; wave 0 hashes R || A || M on one lane and recodes
//   k = H mod L; 16 lanes of wave 0 each add one or two windows of both combs
//   (complete Niels additions from the neutral point), the partials meet in
//   four levels of complete extended additions across lanes; Z^-1 runs on
//   four lanes (mp::inv_plain_var4: Z is public); encode(R') == R (R26).
constexpr uint32_t ED_SIG_CHARS = 88;
template <int WA>
__global__ void __launch_bounds__(SM_THREADS) k_ed_small(EdSmallArgs a) {
  constexpr int NB = ed_windows(true), NA = ed_windows_w(WA), NW = NB > NA ? NB : NA, S = 16;
  constexpr int K = (NW + S - 1) / S;            // windows per lane
  __shared__ uint32_t in_w[SM_IN_DW];
  __shared__ uint32_t sig_w[ED_SIG_CHARS / 4 + 2];
  __shared__ uint8_t sig_b[3 * (ED_SIG_CHARS / 4) + 4];
  __shared__ int32_t dg[NB + NA];
  __shared__ int32_t flag[2];                    // [0] characters bad, [1] the token runs
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const JobDev jb = a.jobs[blockIdx.x];
  const DevKey& Kk = a.keys[job_key(jb)];
  const uint32_t nch = job_siglen(jb);
  const bool in_ok = jb.sig_in_len <= SMALL_IN_MAX;
  const uint32_t in_shift = (uint32_t)((uintptr_t)(a.arena + jb.off) & 3u);
  const uint32_t sig_shift = (uint32_t)((uintptr_t)(a.arena + jb.sig_off) & 3u);
  if (tid == 0) { flag[0] = 0; flag[1] = 0; }
  if (wave == 0 && in_ok) {
    sm_stage_input(in_w, reinterpret_cast<const uint32_t*>(a.arena + jb.off - in_shift), in_shift, jb.sig_in_len, 512,
                   lane, 64);
  } else if (wave == 1) {
    const uint32_t* g = reinterpret_cast<const uint32_t*>(a.arena + jb.sig_off - sig_shift);
    const uint32_t nd = nch <= ED_SIG_CHARS ? (sig_shift + nch + 3) / 4 : 0u;
    if ((uint32_t)lane < nd) sig_w[lane] = g[lane];
  }
  __syncthreads();
  const bool size_ok = nch <= ED_SIG_CHARS && (nch & 3u) != 1u && sm_b64_len(nch) == 64u;
  if (wave == 1 && size_ok) {
    if (sm_b64_decode(sig_w, sig_shift, nch, sig_b, lane) && lane == 0) flag[0] = 1;
  }
  __syncthreads();
  const bool ok0 = in_ok && size_ok && flag[0] == 0 && Kk.valid != 0 && job_alg(jb) == 10;
  if (ok0 && wave == 0 && lane == 0) {
    // SHA-512(R || A || M): the 64-byte prefix as 16 big-endian words, then M
    const uint32_t* A = a.keyblob + Kk.aux_off;
    uint32_t pre[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      pre[t] = ((uint32_t)sig_b[4 * t] << 24) | ((uint32_t)sig_b[4 * t + 1] << 16) | ((uint32_t)sig_b[4 * t + 2] << 8) |
               sig_b[4 * t + 3];
      pre[8 + t] = sha2::bswap32(A[t]);
    }
    const uint32_t len = jb.sig_in_len, tot = len + 64;
    uint64_t h[8];
    sha2::sha512_init(h, false);
    const uint32_t nblk = (tot + 17 + 127) / 128;
#pragma unroll 1
    for (uint32_t blk = 0; blk < nblk; ++blk) {
      uint32_t v[32];
      if (blk == 0) {
#pragma unroll
        for (int t = 0; t < 16; ++t) v[t] = mp::lane_value(pre[t]);
        sm_words<16>(in_w, 0, in_shift, len, v + 16);
      } else {
        sm_words<32>(in_w, blk * 32 - 16, in_shift, len, v);
      }
      if (blk == nblk - 1) { v[30] = tot >> 29; v[31] = tot << 3; }
      uint64_t w[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) w[t] = ((uint64_t)v[2 * t] << 32) | v[2 * t + 1];
      sha2::sha512_compress(h, w);
    }
    // k = H mod L (H little-endian, 512 bits; k_ed_point's reduction)
    uint32_t hw[16], hl[2 * L];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      hw[2 * q] = sha2::bswap32((uint32_t)(h[q] >> 32));
      hw[2 * q + 1] = sha2::bswap32((uint32_t)h[q]);
    }
    mp::words_to_limbs<2 * L, 16>(hl, hw);
    uint64_t tt[2 * L];
#pragma unroll
    for (int j = 0; j < 2 * L; ++j) tt[j] = hl[j];
    uint32_t kr[L], rr[L], k[L];
    mp::mont_reduce<Fl>(kr, tt);
    mp::set_const<Fl>(rr, Fl::RR);
    mp::mul<Fl>(k, kr, rr);
    mp::csub<Fl>(k);
    recode<WA, NA>(dg + NB, k);
  }
  if (ok0 && wave == 1 && lane == 0) {
    // S: canonical (S < L) and sig[63] & 0xE0 == 0 (R24)
    uint32_t sw[8], sl[L], lord[L];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      sw[q] = (uint32_t)sig_b[32 + 4 * q] | ((uint32_t)sig_b[33 + 4 * q] << 8) | ((uint32_t)sig_b[34 + 4 * q] << 16) |
              ((uint32_t)sig_b[35 + 4 * q] << 24);
    mp::words_to_limbs<L, 8>(sl, sw);
    mp::set_const<Fl>(lord, Fl::M);
    const bool sok = (sw[7] & 0xE0000000u) == 0 && lt_limbs(sl, lord);
    recode<ed_comb_w(true), NB>(dg, sl);
    flag[1] = sok ? 1 : 0;
  }
  __syncthreads();
  if (wave != 0) return;
  const bool run = ok0 && flag[1] != 0;          // block-uniform
  FPt P;                                         // the neutral element (0, 1, 1, 0)
  fe::set_small(P.X, 0u); fe::set_small(P.Y, 1u); fe::set_small(P.Z, 1u); fe::set_small(P.T, 0u);
  if (run && lane < S) {
    const uint32_t* __restrict__ atab = key_table(Kk);
#pragma unroll
    for (int i = 0; i < K; ++i) {
      const int w = lane + S * i;
      if (w < NB) add_window<ed_entries(true)>(P, a.btab, w, dg[w]);
      if (w < NA) add_window<(1 << (WA - 1))>(P, atab, w, dg[NB + w]);
    }
  }
  // partials of lanes 0..15 added pairwise with the complete law (every lane joins the shuffles)
#pragma unroll 1
  for (int off = 1; off < S; off <<= 1) {
    FPt Q;
#pragma unroll
    for (int j = 0; j < fe::L; ++j) {
      Q.X[j] = __shfl_xor(P.X[j], off);
      Q.Y[j] = __shfl_xor(P.Y[j], off);
      Q.Z[j] = __shfl_xor(P.Z[j], off);
      Q.T[j] = __shfl_xor(P.T[j], off);
    }
    add_ext(P, P, Q);
  }
  // Z^-1 on lanes 0..3 (lane 0's Z, plain limbs), then lane 0 encodes R'
  uint32_t zm[L], zp[L], zl[L];
  fe_to_mont(zm, P.Z);
  mp::from_mont<Fp>(zp, zm);
#pragma unroll
  for (int j = 0; j < L; ++j) zl[j] = (uint32_t)__shfl((int)zp[j], 0);
  if (lane >= 4) return;
  uint32_t zi[L];
  mp::inv_plain_var4<Fp>(zi, zl);
  if (lane != 0) return;
  bool ok = false;
  if (run) {
    uint32_t zim[L], X[L], Y[L], tt[L], x[L], y[L], enc[8];
    mp::to_mont<Fp>(zim, zi);
    fe_to_mont(X, P.X);
    fe_to_mont(Y, P.Y);
    mp::mul<Fp>(tt, X, zim); mp::from_mont<Fp>(x, tt);
    mp::mul<Fp>(tt, Y, zim); mp::from_mont<Fp>(y, tt);
    mp::limbs_to_words<L, 8>(enc, y);
    enc[7] = (enc[7] & 0x7fffffffu) | ((x[0] & 1u) << 31);
    uint32_t diff = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      diff |= enc[q] ^ ((uint32_t)sig_b[4 * q] | ((uint32_t)sig_b[4 * q + 1] << 8) | ((uint32_t)sig_b[4 * q + 2] << 16) |
                        ((uint32_t)sig_b[4 * q + 3] << 24));
    ok = diff == 0;
  }
  a.verdict[a.out[blockIdx.x]] = ok ? 1 : 0;
}

// ------------------------------------------------------------------ staging
__device__ void niels_entry(uint32_t* out, const EPt& P) {
  uint32_t zi[L], x[L], y[L], t[L], d2[L];
  mp::inv<Fp>(zi, P.Z);
  mp::mul<Fp>(x, P.X, zi); mp::canon<Fp>(x);
  mp::mul<Fp>(y, P.Y, zi); mp::canon<Fp>(y);
  uint32_t ypx[L], ymx[L], t2d[L];
  mp::add<Fp>(ypx, y, x); mp::canon<Fp>(ypx);
  mp::sub<Fp>(ymx, y, x); mp::canon<Fp>(ymx);
  mp::mul<Fp>(t, x, y);
  mp::set_const<Fp>(d2, ED25519C::D2_M);
  mp::mul<Fp>(t2d, t, d2); mp::canon<Fp>(t2d);
  // stored canonical in k_ed_point's radix-2^25.5 form
  mont_to_fe(out, ypx);
  mont_to_fe(out + fe::L, ymx);
  mont_to_fe(out + 2 * fe::L, t2d);
}

// canonical a -> a / 2 mod p (canonical)
__device__ void half_mod(uint32_t* r, const uint32_t* a) {
  uint32_t v[L];
  const uint32_t odd = 0u - (a[0] & 1u);
#pragma unroll
  for (int j = 0; j < L; ++j) v[j] = a[j] + (Fp::M[j] & odd);
  mp::norm<Fp>(v);                              // a (+ p) < 2p < 2^(28L): even, limbs < 2^28
#pragma unroll
  for (int j = 0; j < L; ++j) r[j] = (v[j] >> 1) | (j + 1 < L ? (v[j + 1] & 1u) << (MP_W - 1) : 0u);
}

// affine (x, y) of a Niels entry (y+x, y-x, 2dxy; stored in radix 2^25.5)
__device__ void niels_affine(uint32_t* x, uint32_t* y, const uint32_t* ent) {
  uint32_t t[L], ypx[L], ymx[L];
  fe_to_mont(ypx, ent);
  fe_to_mont(ymx, ent + fe::L);
  mp::sub<Fp>(t, ypx, ymx); mp::canon<Fp>(t); half_mod(x, t);
  mp::add<Fp>(t, ypx, ymx); mp::canon<Fp>(t); half_mod(y, t);
}

// window base 2^(W w) * P as the Niels entry d = 1 of window w
__device__ void window_base(uint32_t* out, const uint32_t* bx, const uint32_t* by, int shifts) {
  EPt P;
  mp::copy<Fp>(P.X, bx); mp::copy<Fp>(P.Y, by); mp::set_const<Fp>(P.Z, Fp::ONE);
  mp::mul<Fp>(P.T, bx, by);
  for (int i = 0; i < shifts; ++i) add_full(P, P, P);
  niels_entry(out, P);
}

// entry d * base (d <= 2^(W-1)) from the window's d = 1 entry
template <int W>
__device__ void table_entry(uint32_t* out, const uint32_t* base_ent, int d) {
  EPt P, acc;
  uint32_t bx[L], by[L];
  niels_affine(bx, by, base_ent);
  mp::copy<Fp>(P.X, bx); mp::copy<Fp>(P.Y, by); mp::set_const<Fp>(P.Z, Fp::ONE);
  mp::mul<Fp>(P.T, bx, by);
#pragma unroll
  for (int j = 0; j < L; ++j) { acc.X[j] = 0; acc.T[j] = 0; acc.Y[j] = Fp::ONE[j]; acc.Z[j] = Fp::ONE[j]; }
  for (int bit = W - 1; bit >= 0; --bit) {
    add_full(acc, acc, acc);
    if ((d >> bit) & 1) add_full(acc, acc, P);
  }
  niels_entry(out, acc);
}

// Tables in two launches (as ecdsa.hip): thread per window for the bases, then
// thread per entry d >= 2 from its window's base.
__global__ void k_ed_table_base_b(uint32_t* tab) {
  constexpr int W = ed_comb_w(true), NWIN = ed_windows(true), NE = ed_entries(true);
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= NWIN) return;
  uint32_t bx[L], by[L];
  mp::set_const<Fp>(bx, ED25519C::BX_M); mp::set_const<Fp>(by, ED25519C::BY_M);
  window_base(tab + (int64_t)w * NE * ED_STRIDE, bx, by, W * w);
}

__global__ void k_ed_table_b(uint32_t* tab) {
  constexpr int W = ed_comb_w(true), NWIN = ed_windows(true), NE = ed_entries(true);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= NWIN * NE || e % NE == 0) return;
  table_entry<W>(tab + (int64_t)e * ED_STRIDE, tab + (int64_t)(e / NE) * NE * ED_STRIDE, e % NE + 1);
}

// thread per key: decode A (SetBytes semantics), store -A affine at aux + 8
__global__ void k_ed_decode(DevKey* keys, uint32_t* blob, const int32_t* idx, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DevKey& K = keys[idx[i]];
  uint32_t* aux = blob + K.aux_off;
  uint32_t w[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = aux[q];
  const uint32_t sign = w[7] >> 31;
  w[7] &= 0x7fffffffu;
  uint32_t y[L];
  mp::words_to_limbs<L, 8>(y, w);
  mp::csub<Fp>(y);                              // y < 2^255 < 2p: reduce non-canonical y
  uint32_t ym[L], yy[L], u[L], v[L], vi[L], xx[L], x[L], c[L], one[L], dm[L];
  mp::to_mont<Fp>(ym, y);
  mp::sqr<Fp>(yy, ym);
  mp::set_const<Fp>(one, Fp::ONE);
  mp::sub<Fp>(u, yy, one);                      // y^2 - 1
  mp::set_const<Fp>(dm, ED25519C::D_M);
  mp::mul<Fp>(v, yy, dm); mp::add<Fp>(v, v, one);   // d y^2 + 1
  mp::inv<Fp>(vi, v);
  mp::mul<Fp>(xx, u, vi);                       // x^2
  mp::pow_e<Fp>(x, xx, ED25519C::EXP_SQRT, ED25519C::EXP_SQRT_BITS, false);
  mp::sqr<Fp>(c, x);
  bool ok = mp::eq_mod<Fp>(c, xx);
  if (!ok) {
    uint32_t sm[L];
    mp::set_const<Fp>(sm, ED25519C::SQRTM1_M);
    mp::mul<Fp>(x, x, sm);
    mp::sqr<Fp>(c, x);
    ok = mp::eq_mod<Fp>(c, xx);
  }
  uint32_t xp[L];
  mp::from_mont<Fp>(xp, x);
  mp::canon<Fp>(x);
  if ((xp[0] & 1u) != sign) {                   // select the root with the requested sign
    uint32_t nx[L];
    mp::neg<Fp>(nx, x); mp::canon<Fp>(nx);
    mp::copy<Fp>(x, nx);
  }
  // -A = (-x, y)
  uint32_t nx[L];
  mp::neg<Fp>(nx, x); mp::canon<Fp>(nx);
  mp::canon<Fp>(ym);
#pragma unroll
  for (int j = 0; j < L; ++j) { aux[8 + j] = nx[j]; aux[8 + L + j] = ym[j]; }
  K.valid = (K.valid && ok) ? 1 : 0;
}

template <int W>
__global__ void k_ed_table_base_keys(const DevKey* keys, uint32_t* blob, const int32_t* idx, int n) {
  constexpr int NWIN = ed_windows_w(W), NE = 1 << (W - 1);
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (k >= n || w >= NWIN) return;
  const DevKey& K = keys[idx[k]];
  if (!K.valid) return;
  const uint32_t* aux = blob + K.aux_off + 8;
  window_base((uint32_t*)K.tab + (int64_t)w * NE * ED_STRIDE, aux, aux + L, W * w);
}

template <int W>
__global__ void k_ed_table_keys(const DevKey* keys, uint32_t* blob, const int32_t* idx, int n, int e0, int e1) {
  constexpr int NWIN = ed_windows_w(W), NE = 1 << (W - 1);
  const int e = e0 + blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (k >= n || e >= e1 || e >= NWIN * NE || e % NE == 0) return;
  const DevKey& K = keys[idx[k]];
  if (!K.valid) return;
  uint32_t* tab = (uint32_t*)K.tab;
  table_entry<W>(tab + (int64_t)e * ED_STRIDE, tab + (int64_t)(e / NE) * NE * ED_STRIDE, e % NE + 1);
}

}  // namespace

// Measured (profiles/r05_s2/q_ab/, ed_split_ab/, r05_s7/ed4_ab/): a lone
// EdDSA batch of 1 ... 4096 tokens 210-244 -> 182-218 us with two lanes and
// 5-12 us less again with four; configs[4]'s 38 k-token Ed25519 launch
// unchanged with two lanes (0.081 ms either way) and slower with four (0.083
// -> 0.110 ms), so only small launches split (JG_ED_SPLIT4_MAX: A/B knob).
#ifndef JG_ED_SPLIT_MAX
#define JG_ED_SPLIT_MAX 16384
#endif
#ifndef JG_ED_SPLIT_LANES
#define JG_ED_SPLIT_LANES 4
#endif
#ifndef JG_ED_SPLIT4_MAX
#define JG_ED_SPLIT4_MAX 0
#endif
// JG_ED_SPLIT_PF: the prefetching loop in the small-launch split too (lone
// EdDSA chain batches of 256 / 8000 tokens: p50 156 -> 154, 240 -> 229 us;
// 2048: 174 -> 177; profiles/r06_s20/pf5.txt).  Off with JG_EC_SPLIT_PF
// (ecdsa_impl.hpp)
#ifndef JG_ED_SPLIT_PF
#define JG_ED_SPLIT_PF 0
#endif
constexpr int64_t ED_SPLIT_MAX_TOKENS = JG_ED_SPLIT_MAX;  // launches up to this many padded tokens: k_ed_point_split
constexpr int64_t ED_SPLIT4_MAX_TOKENS = JG_ED_SPLIT4_MAX;  // ... with 4 lanes per token above ED_SPLIT_MAX_TOKENS
// launches up to this many padded tokens (above the split sizes): k_ed_point_pf
#ifndef JG_ED_PF_MAX
#define JG_ED_PF_MAX 131072
#endif
constexpr int64_t ED_PF_MAX_TOKENS = JG_ED_PF_MAX;
// ... and up to this many: two lanes per token (k_ed_point_split<2, true>).
// A/B knob, off: at configs[4]'s 38912-token class it ran 0.089 ms against
// k_ed_point_pf's 0.069 (profiles/r06_s16/pf2.txt)
#ifndef JG_ED_SPLIT2_PF_MAX
#define JG_ED_SPLIT2_PF_MAX 0
#endif
constexpr int64_t ED_SPLIT2_PF_MAX_TOKENS = JG_ED_SPLIT2_PF_MAX;

template <int S, bool PF = false>
void launch_ed_split(const EdArgs& a, int64_t waves, hipStream_t s) {
  dim3 g((unsigned)(S * waves)), b(WAVE);
  switch (a.wa) {
    case 24: hipLaunchKernelGGL((k_ed_point_split<24, S, PF>), g, b, 0, s, a); break;
    case 22: hipLaunchKernelGGL((k_ed_point_split<22, S, PF>), g, b, 0, s, a); break;
    case 20: hipLaunchKernelGGL((k_ed_point_split<20, S, PF>), g, b, 0, s, a); break;
    case 18: hipLaunchKernelGGL((k_ed_point_split<18, S, PF>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((k_ed_point_split<16, S, PF>), g, b, 0, s, a); break;
  }
}

void launch_ed(const EdArgs& a, hipStream_t s, const Marker& mk) {
  const int64_t waves = (a.end - a.begin) / WAVE;
  if (waves <= 0) return;
  dim3 g((unsigned)waves), b(WAVE);
  if (a.end - a.begin <= ED_SPLIT_MAX_TOKENS) {
    // a launch of fewer waves than ~2 per SIMD: S lanes per token
    launch_ed_split<JG_ED_SPLIT_LANES, JG_ED_SPLIT_PF != 0>(a, waves, s);
  } else if (a.end - a.begin <= ED_SPLIT4_MAX_TOKENS) {
    launch_ed_split<4>(a, waves, s);
  } else if (a.end - a.begin <= ED_SPLIT2_PF_MAX_TOKENS) {
    launch_ed_split<2, true>(a, waves, s);
  } else if (a.end - a.begin <= ED_PF_MAX_TOKENS) {
    switch (a.wa) {
      case 24: hipLaunchKernelGGL(k_ed_point_pf<24>, g, b, 0, s, a); break;
      case 22: hipLaunchKernelGGL(k_ed_point_pf<22>, g, b, 0, s, a); break;
      case 20: hipLaunchKernelGGL(k_ed_point_pf<20>, g, b, 0, s, a); break;
      case 18: hipLaunchKernelGGL(k_ed_point_pf<18>, g, b, 0, s, a); break;
      default: hipLaunchKernelGGL(k_ed_point_pf<16>, g, b, 0, s, a); break;
    }
  } else {
  switch (a.wa) {
    case 24: hipLaunchKernelGGL(k_ed_point<24>, g, b, 0, s, a); break;
    case 22: hipLaunchKernelGGL(k_ed_point<22>, g, b, 0, s, a); break;
    case 20: hipLaunchKernelGGL(k_ed_point<20>, g, b, 0, s, a); break;
    case 18: hipLaunchKernelGGL(k_ed_point<18>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(k_ed_point<16>, g, b, 0, s, a); break;
  }
  }
  mk("point");
  // tokens per thread for the batched inversion: keep >= ~8 waves per CU
  const int64_t n = a.end - a.begin;
  const int B = (int)std::min<int64_t>(16, std::max<int64_t>(1, n / (256 * 8 * WAVE)));
  const int64_t S = (n + B - 1) / B;
  constexpr int TPB = WAVE * ED_FINISH_WPB;
  hipLaunchKernelGGL(k_ed_finish, dim3((unsigned)((S + TPB - 1) / TPB)), dim3(TPB), 0, s, a, B);
  mk("finish");
}

namespace {
template <int W>
void ed_tables(DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s, bool sliced) {
  constexpr int NWIN = ed_windows_w(W), NE = 1 << (W - 1);
  hipLaunchKernelGGL(k_ed_table_base_keys<W>, dim3((NWIN + 63) / 64, tn), dim3(64), 0, s, keys, blob, tidx, tn);
  table_slices(NWIN * NE, tn, sliced, s, [&](int e0, int e1, dim3 g) {
    hipLaunchKernelGGL(k_ed_table_keys<W>, g, dim3(64), 0, s, keys, blob, tidx, tn, e0, e1);
  });
}
}  // namespace

void launch_ed_keyprep(DevKey* keys, uint32_t* blob, const int32_t* idx, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ed_decode, dim3((n + 63) / 64), dim3(64), 0, s, keys, blob, idx, n);
}

void launch_ed_keytables(int wa, DevKey* keys, uint32_t* blob, const int32_t* tidx, int tn, hipStream_t s, bool sliced) {
  if (tn <= 0) return;
  switch (wa) {
    case 24: ed_tables<24>(keys, blob, tidx, tn, s, sliced); break;
    case 22: ed_tables<22>(keys, blob, tidx, tn, s, sliced); break;
    case 20: ed_tables<20>(keys, blob, tidx, tn, s, sliced); break;
    case 18: ed_tables<18>(keys, blob, tidx, tn, s, sliced); break;
    default: ed_tables<16>(keys, blob, tidx, tn, s, sliced); break;
  }
}

void launch_ed_btable(uint32_t* tab, hipStream_t s) {
  constexpr int NWIN = ed_windows(true), NE = ed_entries(true);
  hipLaunchKernelGGL(k_ed_table_base_b, dim3((NWIN + 63) / 64), dim3(64), 0, s, tab);
  hipLaunchKernelGGL(k_ed_table_b, dim3((NWIN * NE + 63) / 64), dim3(64), 0, s, tab);
}

void launch_ed_small(int wa, const EdSmallArgs& a, hipStream_t s) {
  if (a.n == 0) return;
  dim3 g(a.n), b(SM_THREADS);
  switch (wa) {
    case 24: hipLaunchKernelGGL(k_ed_small<24>, g, b, 0, s, a); break;
    case 22: hipLaunchKernelGGL(k_ed_small<22>, g, b, 0, s, a); break;
    case 20: hipLaunchKernelGGL(k_ed_small<20>, g, b, 0, s, a); break;
    case 18: hipLaunchKernelGGL(k_ed_small<18>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(k_ed_small<16>, g, b, 0, s, a); break;
  }
}
