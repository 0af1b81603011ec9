// hash.hip -- batched SHA-2 of byte strings on gfx950.
//
// The hash half of cap's OIDC hash-claim checks, oidc/id_token.go:92-145
// (IDToken.VerifyAccessToken / VerifyAuthorizationCode -> verifyHashClaim):
// h.Write(token); h.Sum(nil) with sha256 / sha512.New384 / sha512 by the
// id_token's alg.  One thread per string; the SHA-2 rounds are the ones the
// verify path uses (sha2.hpp), reading the arena through aligned word loads.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "hash.hpp"
#include "sha2.hpp"

using namespace jgk;
using namespace sha2;

namespace {

__global__ void __launch_bounds__(64) k_hash(const uint8_t* __restrict__ arena, const jg_hjob* __restrict__ jobs,
                                             int64_t n, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const jg_hjob J = jobs[i];
  MemString m;
  m.aligned = (const uint32_t*)(arena + (J.off & ~(uint64_t)3));
  m.shift = (uint32_t)(J.off & 3);
  m.len = J.len;
  uint32_t* o = out + i * 16;
  if (J.fam == JG_SHA256) {
    uint32_t h[8];
    sha256_mem(h, m);
#pragma unroll
    for (int k = 0; k < 8; ++k) { o[k] = h[k]; o[8 + k] = 0u; }
  } else {
    uint64_t h[8];
    sha512_mem(h, J.fam == JG_SHA384, m, nullptr, 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) { o[2 * k] = (uint32_t)(h[k] >> 32); o[2 * k + 1] = (uint32_t)h[k]; }
  }
}

}  // namespace

void launch_hash(const uint8_t* arena, const jg_hjob* jobs, int64_t n, uint32_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_hash, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, arena, jobs, n, out);
}
