// mad.hpp -- 32x32+64 -> 64 multiply-accumulate as one v_mad_u64_u32.
//
// Written as (non-volatile) inline asm because hipcc (ROCm 7.2) lowers
// `acc += (uint64_t)a * b` by zero-extending the 32-bit operands into even-
// aligned 64-bit register pairs, wasting one VGPR per operand: a 37-limb x
// 37-limb CIOS step needed 225 VGPRs that way and 154 with this wrapper
// (gfx950 requires 64-bit VGPR tuples to be even-aligned).  The carry-out
// SGPR pair of the VOP3b encoding is a dead output the allocator may reuse.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ void mad64(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
}

// acc = a * b (first partial product of a column: no zero-initialised accumulator)
__device__ __forceinline__ void mul64(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(acc), "=s"(cc) : "v"(a), "v"(b));
}

// b wave-uniform (SGPR operand)
__device__ __forceinline__ void mad64s(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "s"(b));
}
