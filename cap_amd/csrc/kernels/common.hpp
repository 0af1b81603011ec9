// common.hpp -- structures shared by the HIP kernels and the host runtime.
#pragma once
#include <cstdint>

namespace jgk {

// Kernel classes a (token, key) pair is bucketed into.  Every token of a class
// runs the same kernel chain; within a class tokens are sorted by key and each
// key's run is padded to a whole wave, so the key is wave-uniform.
enum Cls : int {
  CLS_REJECT = 0,   // alg/key-type mismatch, unsupported alg, invalid key
  CLS_RSA2K = 1,    // RSA, modulus <= 2070 bits  (74 x 28-bit limbs; rsa.hpp rsa_limbs)
  CLS_RSA3K = 2,    // RSA, modulus <= 3134 bits  (112 limbs)
  CLS_RSA4K = 3,    // RSA, modulus >= 3135 bits: 148, 296 or 592 limbs by key (rsa.hpp)
  CLS_P256 = 4,
  CLS_P384 = 5,
  CLS_P521 = 6,
  CLS_ED25519 = 7,
  NCLS = 8
};

constexpr int WAVE = 64;

// One-launch small batches (ec_small.hpp, rsa.hip k_rsa_small): at most
// SMALL_MAX jobs per launch, each signing input at most SMALL_IN_MAX bytes
// (staged in LDS); longer ones take the batch chain.
constexpr int SMALL_MAX = 64;
constexpr uint32_t SMALL_IN_MAX = 8192;

// per-token status codes in the scratch status byte
enum : uint8_t { ST_OK = 0, ST_REJECT = 1, ST_EXCEPTIONAL = 2 };

// scratch rows (each row holds one 32-bit word per padded token, SoA)
constexpr int SIGW_ROWS = 520;      // decoded signature rows, at most (RSA-16574: 2072 bytes)
constexpr int EC_S_ROW = 32;        // ECDSA: s starts at row 32 (r at row 0)
constexpr int DIG_ROWS = 16;        // digest, big-endian 32-bit words

// One (token, key) verification job as the kernels read it: in the padded,
// (class, key)-sorted order of the dispatch plan, so lane p of a launch reads
// jobs[p] (coalesced) and every wave's jobs share one key.  Padding lanes
// carry alg JOB_PAD and the wave's key.  Offsets are byte offsets into the
// device copy of the batch's (or chunk's) arena.
constexpr uint32_t JOB_PAD = 15;      // alg of a padding lane (jg_alg ids are 0..10)
constexpr uint32_t JOB_SIGLEN_MAX = 4095;   // longer signatures are clamped (rejected either way)
struct JobDev {
  uint32_t off;          // signing input
  uint32_t sig_in_len;   // bytes hashed
  uint32_t sig_off;      // base64url signature
  uint32_t meta;         // bits 0-15 key index, 16-19 alg, 20-31 signature length (chars)
};
__host__ __device__ inline uint32_t job_pack(uint32_t key, uint32_t alg, uint32_t siglen) {
  return (key & 0xffffu) | ((alg & 15u) << 16) | ((siglen < JOB_SIGLEN_MAX ? siglen : JOB_SIGLEN_MAX) << 20);
}
__host__ __device__ inline int job_key(const JobDev& j) { return (int)(j.meta & 0xffffu); }
__host__ __device__ inline int job_alg(const JobDev& j) { return (int)((j.meta >> 16) & 15u); }
__host__ __device__ inline uint32_t job_siglen(const JobDev& j) { return j.meta >> 20; }
__host__ __device__ inline bool job_live(const JobDev& j) { return job_alg(j) != (int)JOB_PAD; }

// Device view of one loaded key (arrays live in the key blob, word offsets).
// A key's comb table is its own device allocation, shared by content between
// key loads (a JWKS refresh that keeps a key keeps its table): `tab` is its
// device address and `tab_w` its comb width.
struct DevKey {
  int32_t kind;        // jg_key_kind
  int32_t cls;         // Cls of (this key, a matching alg)
  int32_t valid;       // 0 => every token verifies false
  int32_t kbytes;      // RSA: modulus bytes k; EC: coord bytes; Ed: 32
  uint32_t e_lo, e_hi; // RSA public exponent
  uint32_t np;         // RSA: -n^-1 mod 2^28
  uint32_t nlimbs;     // RSA: limb count used (74/112/148)
  uint64_t n_off;      // RSA: n (28-bit limbs)        -- word offset in blob
  uint64_t rr_off;     // RSA: R^2 mod n (28-bit limbs)
  uint64_t tab;        // EC: comb table of Q / Ed: comb table of -A (device address, 0 = none)
  uint64_t aux_off;    // EC: Q affine Montgomery (x,y) / Ed: raw public key words
  int32_t embits;      // RSA: bitlen(n) - 1
  int32_t tab_w;       // EC / Ed: comb width of `tab`
  uint64_t rr2_off;    // RSA-2K: R^2 mod n for the one-launch layout (RSA_SMALL_L limbs; n_off holds
                       // that many limbs, zero-padded), 0 = none
};
__host__ __device__ inline const uint32_t* key_table(const DevKey& K) { return (const uint32_t*)K.tab; }

// Timing hook: the runtime records a HIP event on the batch's stream after
// each kernel a launcher enqueues (names: "<class>_<kernel>").
struct Marker {
  void* ctx = nullptr;
  void (*fn)(void*, const char*) = nullptr;
  void operator()(const char* name) const {
    if (fn) fn(ctx, name);
  }
};

// Per-class launch range inside a staged batch (padded token index space).
struct ClassRange {
  int64_t begin, end;   // multiples of WAVE
};

}  // namespace jgk
