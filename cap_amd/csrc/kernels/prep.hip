// prep.hip -- per-token front end of every verify chain:
//   * base64url-decode the signature segment (go-jose base64URLDecode)
//     into the scratch rows in the layout the class's arithmetic kernel wants;
//   * hash the JWS signing input with the alg's SHA-2 (go-jose verifyPayload,
//     R9); EdDSA hashes R || A || M (crypto/ed25519.Verify, R25).
// One thread per (padded) token; one 64-thread block = one key-uniform wave.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "sha2.hpp"
#include "prep.hpp"

using namespace jgk;

namespace {

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

template <int CLS>
__global__ void __launch_bounds__(64) k_prep(PrepArgs a) {
  const int64_t p = a.begin + (int64_t)blockIdx.x * WAVE + threadIdx.x;
  const int64_t np = a.npad;
  const int32_t t = a.perm[p];
  uint32_t* sigw = a.sigw;
  uint32_t* dig = a.dig;
  if (t < 0) {
    a.status[p] = ST_REJECT;
    return;
  }
  const jg_tok_dev tk = a.toks[t];
  const int alg = tk.alg;
  uint8_t st = ST_OK;

  // ---- base64url decode of the signature segment
  const uint32_t n = tk.sig_b64_len;
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
  // zero the rows this token may leave partially written
  for (int r = 0; r < a.zrows; ++r) sigw[(int64_t)r * np + p] = 0u;

  // characters are fetched as aligned dwords (4 per load) from the arena
  const uint64_t sbyte = tk.off + tk.sig_rel_off;
  const uint32_t* sw32 = reinterpret_cast<const uint32_t*>(a.arena + (sbyte & ~3ull));
  const uint32_t first = (uint32_t)(sbyte & 3ull);
  uint32_t acc = 0, bitsn = 0, outi = 0;
  uint32_t cur_row = 0xffffffffu, cur_word = 0;
  uint32_t R_le[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // Ed25519: first 32 bytes (R)
  const uint32_t nchars = D ? n : 0u;
  uint32_t word = 0;
  for (uint32_t i = 0; i < nchars; ++i) {
    const uint32_t pos = first + i;
    if (i == 0 || (pos & 3u) == 0) word = sw32[pos >> 2];
    const int v = b64val((word >> ((pos & 3u) * 8)) & 0xffu);
    if (v < 0) { st = ST_REJECT; break; }
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
  if (cur_row != 0xffffffffu && st == ST_OK) sigw[(int64_t)cur_row * np + p] = cur_word;
  a.siglen[p] = (uint16_t)D;

  // ---- hash of the signing input
  sha2::MemString m;
  const uint64_t moff = tk.off;
  m.aligned = reinterpret_cast<const uint32_t*>(a.arena + (moff & ~3ull));
  m.shift = (uint32_t)(moff & 3ull);
  m.len = tk.sig_in_len;
  uint32_t dout[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) dout[k] = 0;
  if (CLS == CLS_ED25519) {
    // SHA-512(R || A || M), A = the key's 32 raw public-key bytes
    const uint32_t* A = a.keyblob + a.keys[a.wave_key[p / WAVE]].aux_off;
    uint32_t pre[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pre[k] = sha2::bswap32(R_le[k]);
      pre[8 + k] = sha2::bswap32(A[k]);
    }
    uint64_t h[8];
    sha2::sha512_mem(h, false, m, pre, 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) { dout[2 * k] = (uint32_t)(h[k] >> 32); dout[2 * k + 1] = (uint32_t)h[k]; }
  } else {
    const int hb = alg_hash_bits(alg);
    if (hb == 256) {
      uint32_t h[8];
      sha2::sha256_mem(h, m);
#pragma unroll
      for (int k = 0; k < 8; ++k) dout[k] = h[k];
    } else {
      uint64_t h[8];
      sha2::sha512_mem(h, hb == 384, m, nullptr, 0);
#pragma unroll
      for (int k = 0; k < 8; ++k) { dout[2 * k] = (uint32_t)(h[k] >> 32); dout[2 * k + 1] = (uint32_t)h[k]; }
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) dig[(int64_t)k * np + p] = dout[k];
  a.status[p] = st;
}

}  // namespace

void launch_prep(int cls, const PrepArgs& a, hipStream_t s) {
  const int64_t waves = (a.end - a.begin) / WAVE;
  if (waves <= 0) return;
  dim3 g((unsigned)waves), b(WAVE);
  switch (cls) {
    case CLS_RSA2K: case CLS_RSA3K: case CLS_RSA4K:
      hipLaunchKernelGGL(k_prep<CLS_RSA2K>, g, b, 0, s, a); break;
    case CLS_P256: case CLS_P384: case CLS_P521:
      hipLaunchKernelGGL(k_prep<CLS_P256>, g, b, 0, s, a); break;
    case CLS_ED25519:
      hipLaunchKernelGGL(k_prep<CLS_ED25519>, g, b, 0, s, a); break;
    default: break;
  }
}
