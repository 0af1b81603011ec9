// hostmem.cpp -- see hostmem.hpp.
#include "hostmem.hpp"

#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <new>
#include <vector>

// Under AddressSanitizer, pooled memory is poisoned while it sits in a pool:
// a claims tree read after its batch released its arena is reported.
#if defined(__SANITIZE_ADDRESS__)
#include <sanitizer/asan_interface.h>
#define HOSTMEM_POISON(p, n) ASAN_POISON_MEMORY_REGION((p), (n))
#define HOSTMEM_UNPOISON(p, n) ASAN_UNPOISON_MEMORY_REGION((p), (n))
#else
#define HOSTMEM_POISON(p, n) ((void)(p), (void)(n))
#define HOSTMEM_UNPOISON(p, n) ((void)(p), (void)(n))
#endif

namespace capjwt {
namespace hostmem {
namespace {

struct Pools {
  std::mutex mu;
  std::vector<void*> blocks;                      // free kBlock blocks
  std::vector<std::pair<void*, size_t>> bigs;     // free large blocks (base, true capacity)
  size_t bytes = 0;                               // pooled bytes (both kinds)
  size_t cap = [] {
    if (const char* e = std::getenv("CAPJWT_HOST_CACHE_GB")) {
      const double v = std::atof(e);
      if (v >= 0) return (size_t)(v * (double)(size_t(1) << 30));
    }
    return size_t(4) << 30;
  }();
};
Pools& pools() {
  static Pools* p = new Pools();                  // never destroyed: blocks outlive static teardown
  return *p;
}

void* map_bytes(size_t n) {
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  // 2 MiB pages where the kernel allows them (THP "madvise" mode): one fault
  // per 2 MiB the first time a block is touched, fewer TLB misses after
  (void)madvise(p, n, MADV_HUGEPAGE);
  return p;
}
void unmap_bytes(void* p, size_t n) {
  HOSTMEM_UNPOISON(p, n);
  (void)munmap(p, n);
}

// callers hold mu: drop pooled blocks until bytes <= limit (large ones first)
void shrink_locked(Pools& P, size_t limit) {
  while (P.bytes > limit && !P.bigs.empty()) {
    unmap_bytes(P.bigs.back().first, P.bigs.back().second);
    P.bytes -= P.bigs.back().second;
    P.bigs.pop_back();
  }
  while (P.bytes > limit && !P.blocks.empty()) {
    unmap_bytes(P.blocks.back(), kBlock);
    P.bytes -= kBlock;
    P.blocks.pop_back();
  }
}

}  // namespace

void* block_get() {
  Pools& P = pools();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (!P.blocks.empty()) {
      void* p = P.blocks.back();
      P.blocks.pop_back();
      P.bytes -= kBlock;
      HOSTMEM_UNPOISON(p, kBlock);
      return p;
    }
  }
  return map_bytes(kBlock);
}

void block_put(void* p) {
  if (!p) return;
  Pools& P = pools();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (P.bytes + kBlock <= P.cap) {
      HOSTMEM_POISON(p, kBlock);
      P.blocks.push_back(p);
      P.bytes += kBlock;
      return;
    }
  }
  unmap_bytes(p, kBlock);
}

void* big_get(size_t bytes, size_t* cap) {
  bytes = std::max<size_t>(bytes, 1);
  Pools& P = pools();
  {
    std::lock_guard<std::mutex> g(P.mu);
    // the smallest pooled block that holds the request and is at most twice its size
    size_t best = P.bigs.size();
    for (size_t i = 0; i < P.bigs.size(); ++i) {
      const size_t c = P.bigs[i].second;
      if (c >= bytes && c / 2 <= bytes && (best == P.bigs.size() || c < P.bigs[best].second)) best = i;
    }
    if (best < P.bigs.size()) {
      void* p = P.bigs[best].first;
      *cap = P.bigs[best].second;
      P.bytes -= *cap;
      P.bigs.erase(P.bigs.begin() + (std::ptrdiff_t)best);
      HOSTMEM_UNPOISON(p, *cap);
      return p;
    }
  }
  const size_t c = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);   // 2 MiB granules
  *cap = c;
  return map_bytes(c);
}

void big_put(void* p, size_t cap) {
  if (!p) return;
  Pools& P = pools();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (P.bytes + cap <= P.cap) {
      HOSTMEM_POISON(p, cap);
      P.bigs.emplace_back(p, cap);
      P.bytes += cap;
      return;
    }
  }
  unmap_bytes(p, cap);
}

size_t retained() {
  Pools& P = pools();
  std::lock_guard<std::mutex> g(P.mu);
  return P.bytes;
}

size_t retention_cap() {
  Pools& P = pools();
  std::lock_guard<std::mutex> g(P.mu);
  return P.cap;
}

void set_retention_cap(size_t bytes) {
  Pools& P = pools();
  std::lock_guard<std::mutex> g(P.mu);
  P.cap = bytes;
  shrink_locked(P, bytes);
}

void trim() {
  Pools& P = pools();
  std::lock_guard<std::mutex> g(P.mu);
  shrink_locked(P, 0);
}

}  // namespace hostmem
}  // namespace capjwt
