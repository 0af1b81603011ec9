// hostmem.hpp -- host memory that a batch reuses instead of returning to the OS.
//
// Why (profiles/r05_s1): a 1M-token ValidateBatch builds
// ~1 GB of claims maps.  Built with malloc, glibc's per-thread arenas hand
// whole 64 MiB heaps back to the OS as soon as a batch's maps are freed (its
// trim threshold does not apply to heap deletion), so every batch page-faulted
// the same memory again: 92 k minor faults and 104 ms of payload JSON per pass
// inside the long-running bench process against 9.6 k faults and 25 ms in a
// fresh one, whose malloc state happened to retain it.  Two pools make the
// steady state independent of malloc's history:
//   * blocks of kBlock bytes (mmap'd, MADV_HUGEPAGE) for the bump arenas of
//     claims trees (json::Arena) and decoded payloads;
//   * large blocks (>= 1 MiB) for the per-token record arrays (BatchArray).
// Both keep what a batch returned, up to a retention cap shared by the two
// (CAPJWT_HOST_CACHE_GB, default 4; SetHostMemoryRetention / TrimHostMemory).
#pragma once
#include <cstddef>
#include <cstdint>

namespace capjwt {
namespace hostmem {

constexpr size_t kBlock = size_t(4) << 20;

// one kBlock-byte block (pooled); never null (throws std::bad_alloc)
void* block_get();
void block_put(void* p);

// a block of at least `bytes` for a batch array; *cap receives its capacity
void* big_get(size_t bytes, size_t* cap);
void big_put(void* p, size_t cap);

// bytes of pooled (free, retained) memory; the retention cap
size_t retained();
size_t retention_cap();
void set_retention_cap(size_t bytes);     // also trims down to it
void trim();                              // release every pooled block to the OS

}  // namespace hostmem
}  // namespace capjwt
