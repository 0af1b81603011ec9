// prep.hip -- per-token front end of every verify chain:
//   * base64url-decode the signature segment (go-jose base64URLDecode)
//     into the scratch rows in the layout the class's arithmetic kernel wants;
//   * hash the JWS signing input with the alg's SHA-2 (go-jose verifyPayload,
//     R9); EdDSA hashes R || A || M (crypto/ed25519.Verify, R25).
// One 64-thread block = one key-uniform wave of tokens, one token per lane.
//
// Token bytes reach the lanes through LDS, staged with COALESCED loads: for
// each 128-byte window of the strings, the wave copies 33 dwords of every one
// of its 64 tokens (two tokens per load instruction, each half-wave reading
// 128 contiguous bytes) into a per-token LDS slot, then each lane reads its own
// slot.  The loads of window c + 1 are issued before window c is hashed.  A lane-per-token walk over the arena instead makes every load
// instruction touch 64 different cache lines (prep ran at ~0.4 TB/s that way:
// L1 thrash, one L2 request per lane per dword).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "sha2.hpp"
#include "prep.hpp"

using namespace jgk;

namespace {

#ifndef JG_PREP_ED_ATTR
#define JG_PREP_ED_ATTR __attribute__((amdgpu_waves_per_eu(3)))
#endif

constexpr int WIN = 32;         // dwords per window step (128 bytes of string)
// LDS words per token slot (33 used).  JG_PREP_SLOT A/B: the slot stride sets
// the ds_read bank pattern of the per-lane slot reads and the LDS per wave
// (SLOT 36: 11.0 KB per wave, 14 waves per CU)
#ifndef JG_PREP_SLOT
#define JG_PREP_SLOT 36
#endif
constexpr int SLOT = JG_PREP_SLOT;

__device__ __forceinline__ int b64val(uint32_t c) {
  if (c - 'A' < 26u) return (int)(c - 'A');
  if (c - 'a' < 26u) return (int)(c - 'a' + 26);
  if (c - '0' < 10u) return (int)(c - '0' + 52);
  if (c == '-') return 62;
  if (c == '_') return 63;
  return -1;
}

__device__ __forceinline__ int alg_hash_bits(int alg) {
  switch (alg) {
    case 1: case 4: case 7: return 256;
    case 2: case 5: case 8: return 384;
    default: return 512;
  }
}

__device__ __forceinline__ int es_size(int alg) { return alg == 7 ? 32 : alg == 8 ? 48 : 66; }

// layout of the decoded signature in the scratch rows
enum Layout { LAY_BE = 0, LAY_SPLIT_BE = 1, LAY_LE = 2 };

// Window c of token t's stream = arena dwords [base[t] + woff, + 33) with
// woff = WIN c - skip (skip > 0 only past window 0 of Ed25519's hash stream,
// whose first window carries the 16-word register prefix), or woff = 0 once
// the token needs no more windows (nw[t] <= c: it re-reads its first window
// instead of running past the arena).  fetch() loads this lane's share of the
// wave's 64 windows into registers -- dword k = lane % 32 of tokens 2i + lane
// / 32, plus dword 32 of its own -- so that the next window's loads are in
// flight while the current one is hashed (issued one window ahead: prep was
// ~40 % parked on memory with load -> barrier -> compute; prep_body's PF);  put() moves them
// into the LDS slots.  Both in wave-uniform control flow only (one block ==
// one wave; every lane carries words of other lanes' windows).
struct WinRegs { uint32_t v[33]; };

// Without prefetch: every lane names its window start `w`, the wave copies
// dwords [w, w+33) of all 64 windows into the slots (loads and LDS stores
// interleaved, few live registers).
__device__ __forceinline__ void stage(uint32_t* slots, uint32_t* wsh, const uint32_t* arena_w, uint32_t w) {
  const int lane = threadIdx.x;
  wsh[lane] = w;
  __syncthreads();
  const int half = lane >> 5, k = lane & 31;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int tt = 2 * i + half;
    slots[tt * SLOT + k] = arena_w[wsh[tt] + k];
  }
  slots[lane * SLOT + 32] = arena_w[w + 32];
  __syncthreads();
}

__device__ __forceinline__ void fetch(WinRegs& r, const uint32_t* base, const int32_t* nw, const uint32_t* arena_w,
                                      uint32_t c, uint32_t skip) {
  const int lane = threadIdx.x;
  const int half = lane >> 5, k = lane & 31;
  const uint32_t woff = WIN * c - (c ? skip : 0u);
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int tt = 2 * i + half;
    r.v[i] = arena_w[base[tt] + ((int32_t)c < nw[tt] ? woff : 0u) + (uint32_t)k];
  }
  r.v[32] = arena_w[base[lane] + ((int32_t)c < nw[lane] ? woff : 0u) + 32u];
}

__device__ __forceinline__ void put(uint32_t* slots, const WinRegs& r) {
  const int lane = threadIdx.x;
  const int half = lane >> 5, k = lane & 31;
  __syncthreads();                         // the previous window's reads are done
#pragma unroll
  for (int i = 0; i < 32; ++i) slots[(2 * i + half) * SLOT + k] = r.v[i];
  slots[lane * SLOT + 32] = r.v[32];
  __syncthreads();
}

// N big-endian message words i0 .. i0+N-1 (SHA padding applied, length words
// are the caller's) from a staged window whose dword 0 holds aligned message
// word i0 (the message starts `shift` bytes into its first aligned dword).
template <int N>
__device__ __forceinline__ void window_words(const uint32_t* u, uint32_t i0, uint32_t shift, uint32_t len,
                                             uint32_t* out) {
  if (4u * (i0 + N) <= len) {            // all N words inside the message: no length masks
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = sha2::bswap32(__builtin_amdgcn_alignbyte(u[k + 1], u[k], shift));
    return;
  }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint32_t raw = sha2::bswap32(__builtin_amdgcn_alignbyte(u[k + 1], u[k], shift));
    const int rem = (int)len - (int)(4u * (i0 + k));
    const uint32_t keep = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : (0xffffffffu << (32 - 8 * rem)));
    const uint32_t pad = (rem >= 0 && rem < 4) ? (0x80u << (24 - 8 * rem)) : 0u;
    out[k] = (raw & keep) | pad;
  }
}

// Shared block 0 (SHA-256 classes).  Tokens of one issuer usually share their
// first 64 bytes of signing input: the protected header (alg, kid, typ) and the
// start of the payload.  One thread per key run (the first wave of each run in
// the key-sorted plan) hashes its first token's block 0 and records the block
// and the midstate in the key's slot; k_prep then skips block 0 for a wave
// whose every live lane has exactly that block (16-word compare), starting from
// the recorded midstate.  Equal blocks give equal compression outputs, so the
// digest is unchanged.  Runs before k_prep on the same stream; the slots live
// in the batch's own scratch (no sharing between batches in flight).
__global__ void __launch_bounds__(64) k_prep_mid(PrepArgs a) {
  const int64_t w = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (w >= (a.end - a.begin) / WAVE) return;
  const int64_t p0 = a.begin + w * WAVE;
  const JobDev jb = a.jobs[p0];
  if (!job_live(jb)) return;
  const int key = job_key(jb);
  if (w > 0) {
    const JobDev prev = a.jobs[p0 - WAVE];
    if (job_live(prev) && job_key(prev) == key) return;    // not the run's first wave
  }
  uint32_t* slot = a.mid + (size_t)key * PREP_MID_WORDS;
  const uint32_t len = jb.sig_in_len;
  if (alg_hash_bits(job_alg(jb)) != 256 || (len + 9 + 63) / 64 < 2) {   // block 0 is the last block
    slot[24] = 0u;
    return;
  }
  const uint32_t* arena_w = reinterpret_cast<const uint32_t*>(a.arena);
  const uint64_t mw0 = jb.off >> 2;
  uint32_t u[17];
#pragma unroll
  for (int k = 0; k < 17; ++k) u[k] = arena_w[mw0 + k];    // within the arena's slack
  uint32_t blk[16], h[8];
  window_words<16>(u, 0, jb.off & 3u, len, blk);
#pragma unroll
  for (int k = 0; k < 16; ++k) slot[k] = blk[k];
  sha2::sha256_init(h);
  sha2::sha256_compress(h, blk);
#pragma unroll
  for (int k = 0; k < 8; ++k) slot[16 + k] = h[k];
  slot[24] = 1u;
}

// HM: hash families present in the launch range (bit 0 SHA-256, bit 1
// SHA-384/512, from the runtime's dispatch plan).  A single-family variant
// drops the other SHA's code and registers: the SHA-512 path alone raises the
// kernel to ~224 VGPRs (2 waves/SIMD).
template <int CLS, int HM>
__device__ __forceinline__ void prep_body(const PrepArgs& a) {
  __shared__ uint32_t slots[WAVE * SLOT];
  // window streams (signature, signing input): arena dword index of each
  // lane's first window -- 32 bits (JobDev offsets are 32-bit byte offsets)
  __shared__ uint32_t sbase[WAVE], hbase[WAVE];
  __shared__ int32_t snw[WAVE], hnw[WAVE];
  __shared__ uint32_t wsh[WAVE];                  // stage(): this window's start per lane
  __shared__ int8_t b64tab[256];
  const int lane = threadIdx.x;
  const int64_t p = a.begin + (int64_t)blockIdx.x * WAVE + lane;
  const int64_t np = a.npad;
  const JobDev jb = a.jobs[p];
  const bool valid = job_live(jb);
  uint32_t* sigw = a.sigw;
  uint32_t* dig = a.dig;
  const uint32_t* arena_w = reinterpret_cast<const uint32_t*>(a.arena);
  const uint32_t* my = slots + lane * SLOT;
  const int alg = valid ? job_alg(jb) : 0;
  uint8_t st = valid ? ST_OK : ST_REJECT;

  // ---- base64url decode of the signature segment
  const uint32_t n = valid ? job_siglen(jb) : 0u;
  uint32_t D;
  if ((n & 3u) == 1u) { st = ST_REJECT; D = 0; }
  else D = (n >> 2) * 3u + ((n & 3u) == 2u ? 1u : (n & 3u) == 3u ? 2u : 0u);
  // a signature longer than the rows this class reads cannot have the key's
  // length (R13/R18/R23); rejecting it here also keeps every write below in
  // bounds of the zrows x npad scratch the runtime allocated for the batch
  if (D > 4u * (uint32_t)a.zrows) { st = ST_REJECT; D = 0; }
  const int layout = (CLS == CLS_ED25519) ? LAY_LE : (CLS >= CLS_P256 ? LAY_SPLIT_BE : LAY_BE);
  uint32_t ks = 0;
  if (layout == LAY_SPLIT_BE) {
    ks = (alg >= 7 && alg <= 9) ? (uint32_t)es_size(alg) : 0u;
    if (ks == 0 || D != 2 * ks) { st = ST_REJECT; D = 0; }
  }
  // Fast path: whole 32-bit words of decoded bytes (D and, for ECDSA, each of
  // r and s a multiple of 4 bytes -- every standard key size but P-521): 16
  // characters -> 12 bytes -> 3 big-endian words per step, characters mapped
  // through an LDS table, each word stored straight to its row.  Otherwise
  // the byte-serial loop below.
  const bool fast = valid && D != 0 && (D & 3u) == 0 && (layout != LAY_SPLIT_BE || (ks & 3u) == 0);
  const uint32_t DW = D >> 2;                          // decoded words
  if (valid) {
    // zero the rows this token may leave unwritten (scratch is reused across
    // batches); an RSA key reads the rows of its own layout (rsa_sig_rows_l)
    int zr = a.zrows, r0 = 0;
    if (layout == LAY_BE) {
      const int nl = (int)a.keys[__builtin_amdgcn_readfirstlane(job_key(jb))].nlimbs;
      zr = min(zr, (28 * nl - 1) / 32 + 2);
      if (fast) r0 = (int)DW;                          // rows [0, DW) are all written below
    } else if (layout == LAY_SPLIT_BE && fast && (ks >> 2) == (uint32_t)a.ec_words) {
      zr = 0;                                          // r and s fill every row the curve reads
    }
    for (int r = r0; r < zr; ++r) {
      // ECDSA reads r from rows [0, ec_words) and s from [EC_S_ROW, EC_S_ROW + ec_words) only
      if (layout == LAY_SPLIT_BE && ((r >= a.ec_words && r < EC_S_ROW) || r >= EC_S_ROW + a.ec_words)) continue;
      bool written = false;
      if (fast) {
        if (layout == LAY_SPLIT_BE) {
          const uint32_t kw4 = ks >> 2;
          written = (uint32_t)r < kw4 || ((uint32_t)r >= (uint32_t)EC_S_ROW && (uint32_t)r < EC_S_ROW + kw4);
        } else {
          written = (uint32_t)r < DW;
        }
      }
      if (!written) sigw[(int64_t)r * np + p] = 0u;
    }
  }
  b64tab[lane] = (int8_t)b64val((uint32_t)lane);        // table for the fast path (all 256 bytes)
  b64tab[64 + lane] = (int8_t)b64val(64u + lane);
  b64tab[128 + lane] = (int8_t)b64val(128u + lane);
  b64tab[192 + lane] = (int8_t)b64val(192u + lane);    // made visible by the barrier before the first fetch()

  const uint64_t sbyte = valid ? jb.sig_off : 0u;
  const uint64_t sw0 = sbyte >> 2;                     // arena dword of the segment's first char
  const uint32_t first = (uint32_t)(sbyte & 3ull);
  const uint32_t nchars = (valid && D) ? n : 0u;
  const uint32_t span = nchars ? first + nchars : 0u;  // window bytes the chars occupy
  const uint32_t mshift = valid ? jb.off & 3u : 0u;
  const uint32_t len = valid ? jb.sig_in_len : 0u;
  const int hb_alg = alg_hash_bits(alg);
  const int hb = CLS == CLS_ED25519 ? 512
                 : HM == 1          ? 256
                 : HM == 2          ? (hb_alg == 384 ? 384 : 512)
                                    : hb_alg;
  const uint32_t pw = (CLS == CLS_ED25519 && valid) ? 16u : 0u;
  const uint32_t tot = 4 * pw + len;                   // bytes hashed
  uint32_t nblk = 0, nwin = 0;
  if (valid) {
    nblk = hb == 256 ? (len + 9 + 63) / 64 : (tot + 17 + 127) / 128;
    nwin = hb == 256 ? (nblk + 1) / 2 : nblk;
  }
  // both window streams, for fetch(): every lane's base and window count
  sbase[lane] = span ? (uint32_t)sw0 : 0u;
  snw[lane] = (int32_t)((span + 4 * WIN - 1) / (4 * WIN));
  hbase[lane] = valid ? (jb.off >> 2) : 0u;
  hnw[lane] = (int32_t)nwin;
  constexpr uint32_t HSKIP = CLS == CLS_ED25519 ? 16u : 0u;    // window c >= 1 starts at message word 32c - 16
  // Prefetch one window ahead where it measured faster (RSA: 3+ signature
  // windows, -10 %; Ed25519 -3 %); the ECDSA variants lose a wave per SIMD to
  // the 33 extra live registers (96 -> 142 VGPRs) and ran 4-5 % slower
  // (profiles/r03_s7_prep_prefetch_ab.json), so they load each window just
  // before use, as round 2 did.
  constexpr bool PF = CLS == CLS_ED25519 || CLS == CLS_RSA2K;
  __syncthreads();
  WinRegs wr;
  if constexpr (PF) fetch(wr, sbase, snw, arena_w, 0, 0);
  uint32_t acc = 0, bitsn = 0, outi = 0;
  uint32_t cur_row = 0xffffffffu, cur_word = 0;
  uint32_t R_le[8] = {0, 0, 0, 0, 0, 0, 0, 0};          // Ed25519: first 32 bytes (R)
  bool bad = false;
  for (uint32_t c = 0;; ++c) {
    const bool need = !bad && span > 4u * WIN * c;
    if (__ballot(need) == 0ull) break;
    if constexpr (!PF) stage(slots, wsh, arena_w, need ? (uint32_t)sw0 + WIN * c : sbase[lane]);
    else put(slots, wr);
    if (PF && __ballot(span > 4u * WIN * (c + 1)) != 0ull) fetch(wr, sbase, snw, arena_w, c + 1, 0);
    if (!need) continue;
    if (fast) {
      // window c holds characters [128c, 128c + 128) at byte offset `first`
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const uint32_t i0 = 128u * c + 16u * g;         // first character of the step
        if (i0 >= nchars) break;
        uint32_t b24[4];
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const int k = 4 * g + qd;
          const uint32_t q = __builtin_amdgcn_alignbyte(my[k + 1], my[k], first);
          const int cnt = (int)nchars - (int)(i0 + 4u * qd);   // characters of this quad inside the segment
          int t0 = b64tab[q & 0xffu], t1 = b64tab[(q >> 8) & 0xffu];
          int t2 = b64tab[(q >> 16) & 0xffu], t3 = b64tab[q >> 24];
          if (cnt < 4) t3 = 0;
          if (cnt < 3) t2 = 0;
          if (cnt < 2) t1 = 0;
          if (cnt < 1) t0 = 0;
          bad |= (t0 | t1 | t2 | t3) < 0;
          b24[qd] = ((uint32_t)t0 << 18) | ((uint32_t)t1 << 12) | ((uint32_t)t2 << 6) | (uint32_t)t3;
        }
        const uint32_t w3[3] = {(b24[0] << 8) | (b24[1] >> 16), (b24[1] << 16) | (b24[2] >> 8),
                                (b24[2] << 24) | b24[3]};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const uint32_t kw = 24u * c + 3u * g + j;     // big-endian word index in the byte stream
          if (kw >= DW) continue;
          uint32_t row, val = w3[j];
          if (layout == LAY_BE) {
            row = DW - 1u - kw;
          } else if (layout == LAY_SPLIT_BE) {
            const uint32_t kw4 = ks >> 2, h = kw >= kw4 ? 1u : 0u;
            row = h * EC_S_ROW + (kw4 - 1u - (kw - h * kw4));
          } else {
            row = kw;
            val = sha2::bswap32(val);
            if (c == 0 && 3 * g + j < 8) R_le[3 * g + j] = val;
          }
          sigw[(int64_t)row * np + p] = val;
        }
      }
      if (bad) st = ST_REJECT;
      continue;
    }
    const uint32_t lo = 4u * WIN * c;
    const uint32_t beg = lo > first ? lo : first;
    const uint32_t end = span < lo + 4u * WIN ? span : lo + 4u * WIN;
    uint32_t word = my[(beg - lo) >> 2];
    for (uint32_t pos = beg; pos < end; ++pos) {
      if ((pos & 3u) == 0) word = my[(pos - lo) >> 2];
      const int v = b64val((word >> ((pos & 3u) * 8)) & 0xffu);
      if (v < 0) { st = ST_REJECT; bad = true; break; }
      acc = (acc << 6) | (uint32_t)v;
      bitsn += 6;
      if (bitsn >= 8) {
        bitsn -= 8;
        const uint32_t byte = (acc >> bitsn) & 0xffu;
        // map output byte outi -> (row, shift)
        uint32_t row, sh;
        if (layout == LAY_BE) {
          const uint32_t j = D - 1 - outi;
          row = j >> 2; sh = (j & 3u) * 8u;
        } else if (layout == LAY_SPLIT_BE) {
          const uint32_t h = outi >= ks ? 1u : 0u;
          const uint32_t j = ks - 1 - (outi - h * ks);
          row = h * EC_S_ROW + (j >> 2); sh = (j & 3u) * 8u;
        } else {
          row = outi >> 2; sh = (outi & 3u) * 8u;
          if (outi < 32) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if ((outi >> 2) == (uint32_t)k) R_le[k] |= byte << sh;
          }
        }
        if (row != cur_row) {
          if (cur_row != 0xffffffffu) sigw[(int64_t)cur_row * np + p] = cur_word;
          cur_row = row; cur_word = 0;
        }
        cur_word |= byte << sh;
        ++outi;
      }
    }
  }
  if (cur_row != 0xffffffffu && st == ST_OK) sigw[(int64_t)cur_row * np + p] = cur_word;
  if (valid) a.siglen[p] = (uint16_t)D;

  // ---- hash of the signing input.  Tokens of one wave share a key, not
  // necessarily an alg (RS256 and PS512 under one RSA key), so the window loop
  // is uniform and each lane runs its own hash on the staged window:
  //   SHA-256: a 33-dword window holds two 64-byte blocks (message words 32c..);
  //   SHA-512/384: one 128-byte block per window.  Ed25519 hashes R || A || M:
  //   block 0 = the 64-byte register prefix + message words 0..15, block
  //   c >= 1 = message words 32c-16 ..
  uint32_t pre[16];
  if (CLS == CLS_ED25519 && valid) {
    const uint32_t* A = a.keyblob + a.keys[__builtin_amdgcn_readfirstlane(job_key(jb))].aux_off;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pre[k] = sha2::bswap32(R_le[k]);
      pre[8 + k] = sha2::bswap32(A[k]);
    }
  }
  uint32_t h32[8];
  uint64_t h64[8];
  sha2::sha256_init(h32);
  sha2::sha512_init(h64, hb == 384);
  if constexpr (PF) fetch(wr, hbase, hnw, arena_w, 0, HSKIP);
  for (uint32_t c = 0;; ++c) {
    const bool need = c < nwin;
    if (__ballot(need) == 0ull) break;
    const uint32_t i0 = hb == 256 ? 32u * c : (c == 0 ? 0u : 32u * c - pw);   // message word at window dword 0
    if constexpr (!PF) stage(slots, wsh, arena_w, hbase[lane] + (need ? i0 : 0u));
    else put(slots, wr);
    if (PF && __ballot(c + 1 < nwin) != 0ull) fetch(wr, hbase, hnw, arena_w, c + 1, HSKIP);
    if (!need) continue;
    if (hb == 256) {
#pragma unroll 1
      for (uint32_t hf = 0; hf < 2; ++hf) {
        const uint32_t blk = 2 * c + hf;
        if (blk < nblk) {
          uint32_t w[16];
          window_words<16>(my + 16 * hf, 16 * blk, mshift, len, w);
          if (blk == nblk - 1) {
            w[14] = len >> 29;
            w[15] = len << 3;
          }
          if (blk == 0 && a.mid) {
            // the key run's shared block 0 (k_prep_mid): wave-uniform skip
            const uint32_t* ms = a.mid + (size_t)__builtin_amdgcn_readfirstlane(job_key(jb)) * PREP_MID_WORDS;
            bool same = nblk >= 2 && ms[24] != 0u;
#pragma unroll
            for (int k = 0; k < 16; ++k) same = same && w[k] == ms[k];
            if (__ballot(!same) == 0ull) {
#pragma unroll
              for (int k = 0; k < 8; ++k) h32[k] = ms[16 + k];
              continue;
            }
          }
          sha2::sha256_compress(h32, w);
        }
      }
    } else {
      uint32_t v[32];
      if (pw != 0 && c == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = pre[k];
        window_words<16>(my, 0, mshift, len, v + 16);
      } else {
        window_words<32>(my, i0, mshift, len, v);
      }
      if (c == nblk - 1) {                               // 128-bit length, high 64 bits zero
        v[30] = tot >> 29;
        v[31] = tot << 3;
      }
      uint64_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = ((uint64_t)v[2 * k] << 32) | v[2 * k + 1];
      sha2::sha512_compress(h64, w);
    }
  }
  if (valid) {
    uint32_t dout[16];
    if (hb == 256) {
#pragma unroll
      for (int k = 0; k < 16; ++k) dout[k] = k < 8 ? h32[k] : 0u;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { dout[2 * k] = (uint32_t)(h64[k] >> 32); dout[2 * k + 1] = (uint32_t)h64[k]; }
    }
    // digest words only (SHA-256: 8, SHA-384: 12, SHA-512: 16): every consumer
    // reads the alg's hash length, never the rows past it
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < hb / 32) dig[(int64_t)k * np + p] = dout[k];
  }
  a.status[p] = st;
}

template <int CLS, int HM>
__global__ void __launch_bounds__(64) k_prep(PrepArgs a) {
  prep_body<CLS, HM>(a);
}

// Ed25519's prep (SHA-512 of R || A || M) at three waves per SIMD: the
// compiler's own choice is 216 VGPRs, two waves
__global__ void __launch_bounds__(64) JG_PREP_ED_ATTR k_prep_ed(PrepArgs a) {
  prep_body<CLS_ED25519, 2>(a);
}

}  // namespace

template <int CLS>
void launch_hm(int hm, dim3 g, dim3 b, const PrepArgs& a, hipStream_t s) {
  switch (hm) {
    case 1: hipLaunchKernelGGL((k_prep<CLS, 1>), g, b, 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_prep<CLS, 2>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((k_prep<CLS, 3>), g, b, 0, s, a); break;
  }
}

void launch_prep(int cls, int hash_mask, const PrepArgs& a0, hipStream_t s) {
  const int64_t waves = (a0.end - a0.begin) / WAVE;
  if (waves <= 0) return;
  PrepArgs a = a0;
  if (cls == CLS_ED25519 || !(hash_mask & 1)) a.mid = nullptr;      // SHA-256 block 0 only
  // a launch of a few waves (a coalesced single-token batch): one dependent
  // launch fewer on its chain outweighs the shared block 0
  if (waves <= 2) a.mid = nullptr;
  if (a.mid) hipLaunchKernelGGL(k_prep_mid, dim3((unsigned)((waves + 63) / 64)), dim3(64), 0, s, a);
  dim3 g((unsigned)waves), b(WAVE);
  switch (cls) {
    case CLS_RSA2K: case CLS_RSA3K: case CLS_RSA4K:
      launch_hm<CLS_RSA2K>(hash_mask, g, b, a, s); break;
    case CLS_P256: case CLS_P384: case CLS_P521:
      launch_hm<CLS_P256>(hash_mask, g, b, a, s); break;
    case CLS_ED25519:
      hipLaunchKernelGGL(k_prep_ed, g, b, 0, s, a); break;
    default: break;
  }
}
