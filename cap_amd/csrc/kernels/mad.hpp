// mad.hpp -- 32x32+64 -> 64 multiply-accumulate as one v_mad_u64_u32.
//
// Written as (non-volatile) inline asm because hipcc (ROCm 7.2) lowers
// `acc += (uint64_t)a * b` by zero-extending the 32-bit operands into even-
// aligned 64-bit register pairs, wasting one VGPR per operand: a 37-limb x
// 37-limb CIOS step needed 225 VGPRs that way and 154 with this wrapper
// (gfx950 requires 64-bit VGPR tuples to be even-aligned).  The carry-out
// SGPR pair of the VOP3b encoding is dead.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

// The carry-out goes to a hard-wired SGPR pair chosen by `slot`.  LLVM's
// gfx950 hazard recognizer assumes an inline asm statement may carry a dst-forwarding hazard and pads an s_nop before the next
// instruction that touches any register the asm defined -- with the carry-out
// as an allocated operand every MAD landed on the same dead SGPR pair, so
// every MAD paid an s_nop (4 issue cycles): 36.0 vs 29.1 T MAD/s at 4
// waves/SIMD (profiles/r01_int_rates2.json).  Callers pass a compile-time
// slot (after unrolling) selecting one of 4 pairs: products alternate slots
// 0/1 and reductions 2/3, so interleaved product and reduction streams
// rarely put the same pair back to back.
#define JG_MAD_ACC(PAIR, LO, HI, SRC_B) \
  asm("v_mad_u64_u32 %0, " PAIR ", %1, %2, %0" : "+v"(acc) : "v"(a), SRC_B(b) : LO, HI)
#define JG_MAD_SET(PAIR, LO, HI, SRC_B) \
  asm("v_mad_u64_u32 %0, " PAIR ", %1, %2, 0" : "=v"(acc) : "v"(a), SRC_B(b) : LO, HI)
#define JG_MAD_ASM(ONE, SRC_B)                                  \
  switch (slot & 7) {                                           \
    case 0: ONE("s[88:89]", "s88", "s89", SRC_B); break;        \
    case 1: ONE("s[90:91]", "s90", "s91", SRC_B); break;        \
    case 2: ONE("s[92:93]", "s92", "s93", SRC_B); break;        \
    case 3: ONE("s[94:95]", "s94", "s95", SRC_B); break;        \
    case 4: ONE("s[80:81]", "s80", "s81", SRC_B); break;        \
    case 5: ONE("s[82:83]", "s82", "s83", SRC_B); break;        \
    case 6: ONE("s[84:85]", "s84", "s85", SRC_B); break;        \
    default: ONE("s[86:87]", "s86", "s87", SRC_B); break;       \
  }
#define JG_V(x) "v"(x)
#define JG_S(x) "s"(x)

// acc += a * b
__device__ __forceinline__ void mad64(uint64_t& acc, uint32_t a, uint32_t b, int slot = 0) {
  JG_MAD_ASM(JG_MAD_ACC, JG_V);
}

// acc = a * b (first partial product of a column: no zero-initialised accumulator)
__device__ __forceinline__ void mul64(uint64_t& acc, uint32_t a, uint32_t b, int slot = 0) {
  JG_MAD_ASM(JG_MAD_SET, JG_V);
}

// acc += a * b, b wave-uniform (SGPR operand)
__device__ __forceinline__ void mad64s(uint64_t& acc, uint32_t a, uint32_t b, int slot = 0) {
  JG_MAD_ASM(JG_MAD_ACC, JG_S);
}

// Compiler-scheduled forms for register-resident operand pairs (the fixed-
// modulus field products of mp.hpp).  There the products' 28-bit operands
// need no zero-extension copies, and an inline asm statement costs more than
// it saves: LLVM pads an s_nop 0 after an asm statement before a VALU
// instruction that reads one of its results, which the scheduler's column-
// wise MAD chains hit ~every other MAD (P-256 point kernel: 731 s_nops in 7397
// instructions with asm products, 8 in 6621 with these).  The SGPR-constant
// reduction MADs stay asm, grouped per row (mad_blocks.hpp), where the
// compiler would otherwise strength-reduce power-of-two constants into
// shift + add pairs.
__device__ __forceinline__ void mad64c(uint64_t& acc, uint32_t a, uint32_t b) { acc += (uint64_t)a * b; }
__device__ __forceinline__ void mul64c(uint64_t& acc, uint32_t a, uint32_t b) { acc = (uint64_t)a * b; }
