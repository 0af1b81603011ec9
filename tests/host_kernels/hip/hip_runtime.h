// Host-compile stand-in for <hip/hip_runtime.h> used ONLY by tests/host_kernels
// (CPU checks of the device SHA-2 code, tests/test_sha2_host.py): the AMDGPU
// builtins sha2.hpp uses, emulated with their ISA semantics.
#pragma once
#include <cstdint>
#define __device__
#define __forceinline__ inline
#define __constant__
static inline uint32_t __builtin_amdgcn_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
static inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (s & 3)));
}
// v_perm_b32: byte k of the result = byte sel[k] of {src0 (bytes 4-7), src1 (bytes 0-3)}
static inline uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t c = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t b = (sel >> (8 * k)) & 0xff;
    r |= (b < 8 ? (uint32_t)((c >> (8 * b)) & 0xff) : 0u) << (8 * k);
  }
  return r;
}
// only symmetric truth tables are used on the host path (0x96 = a ^ b ^ c)
static inline uint32_t __builtin_amdgcn_bitop3_b32(uint32_t a, uint32_t b, uint32_t c, unsigned tt) {
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) {
    const unsigned idx = (((a >> i) & 1) << 2) | (((b >> i) & 1) << 1) | ((c >> i) & 1);
    r |= ((tt >> idx) & 1u) << i;
  }
  return r;
}
