// jg_stub.cpp -- timing stand-in for libcapjwt.so's C ABI, linked ONLY into
// tools/hostprof (the host-phase timing harness).  It verifies nothing: every
// job is reported accepted so the host layer runs its full accept path.  Never
// linked into the product or any test.
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include "../../include/jg.h"

struct jg_ctx {
  int dummy;
};

extern "C" {
jg_ctx* jg_create(const int*, int) { return new jg_ctx{0}; }
void jg_destroy(jg_ctx* c) { delete c; }
const char* jg_last_error(jg_ctx*) { return "stub"; }
int jg_keys_load(jg_ctx*, const jg_key*, int) { return 0; }
int jg_keys_wait_tables(jg_ctx*) { return 0; }
void* jg_host_alloc(size_t n) { return std::malloc(n); }
void jg_host_free(void* p) { std::free(p); }
int jg_verify_batch(jg_ctx*, const uint8_t*, size_t, const jg_tok*, size_t n, uint8_t* verdicts) {
  std::memset(verdicts, JG_ACCEPT, n);
  return 0;
}
int jg_hash_batch(jg_ctx*, const uint8_t*, size_t, const jg_hjob*, size_t, uint8_t*) { return -1; }
struct jg_ticket {
  int rc;
};
int jg_submit(jg_ctx*, const uint8_t*, size_t, const jg_tok*, size_t n, uint8_t* verdicts, jg_ticket** t) {
  std::memset(verdicts, JG_ACCEPT, n);
  *t = new jg_ticket{0};
  return 0;
}
// HOSTPROF_DEVICE_US: simulated device latency of every submission (the
// coalescer's behaviour under many concurrent single-token callers)
int jg_wait(jg_ctx*, jg_ticket* t) {
  delete t;
  static const long us = [] {
    const char* e = std::getenv("HOSTPROF_DEVICE_US");
    return e ? std::atol(e) : 0L;
  }();
  if (us > 0) std::this_thread::sleep_for(std::chrono::microseconds(us));
  return 0;
}
int jg_debug_fail_verify(jg_ctx*, int) { return 0; }
}
