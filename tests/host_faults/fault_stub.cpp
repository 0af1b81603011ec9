// fault_stub.cpp -- a stand-in for libcapjwt.so's C ABI whose verify call
// always fails the way a device fault does (rc != 0, a HIP error in
// jg_last_error).  Linked ONLY into the degraded-path test driver
// (degraded.cpp, tests/test_host_degraded.py); verifies nothing.
#include <cstdlib>

#include "../../include/jg.h"

struct jg_ctx {
  int verify_calls;
};

extern "C" {
jg_ctx* jg_create(const int*, int) { return new jg_ctx{0}; }
void jg_destroy(jg_ctx* c) { delete c; }
const char* jg_last_error(jg_ctx*) { return "hipErrorIllegalAddress (injected)"; }
int jg_keys_load(jg_ctx*, const jg_key*, int) { return 0; }
int jg_keys_wait_tables(jg_ctx*) { return 0; }
void* jg_host_alloc(size_t n) { return std::malloc(n); }
void jg_host_free(void* p) { std::free(p); }
int jg_verify_batch(jg_ctx* c, const uint8_t*, size_t, const jg_tok*, size_t, uint8_t*) {
  ++c->verify_calls;
  return -2;
}
// the host layer submits and waits: the submission is accepted, its wait fails
struct jg_ticket {
  int rc;
};
int jg_submit(jg_ctx* c, const uint8_t*, size_t, const jg_tok*, size_t, uint8_t*, jg_ticket** t) {
  ++c->verify_calls;
  *t = new jg_ticket{-2};
  return 0;
}
int jg_wait(jg_ctx*, jg_ticket* t) {
  const int rc = t->rc;
  delete t;
  return rc;
}
int jg_debug_fail_verify(jg_ctx*, int) { return 0; }
int jg_hash_batch(jg_ctx*, const uint8_t*, size_t, const jg_hjob*, size_t, uint8_t*) { return -2; }
}
