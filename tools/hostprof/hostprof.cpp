// hostprof -- CPU-only timing harness for the host half of Validator.ValidateBatch
// (parse, kid routing, arena packing, payload JSON, claims, frees), the part
// bench.py's `e2e` line found to be the ceiling.  It links the host sources with
// jg_timing_stub.cpp, a STAND-IN for libcapjwt.so that marks every job accepted: the
// signatures are never checked here, so this binary measures host time only and
// is never a verifier.  Not part of the product; not loaded by any test.
//
//   usage: hostprof TOKENS_FILE JWKS_FILE [reps [callers]]   (CAPJWT_TRACE=1 for phases)
//   callers > 0: also time `callers` threads calling Validator::Validate per token
//   (the coalesced single-token path) over the same tokens
#include <sys/resource.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <atomic>
#include <algorithm>
#include <vector>

#include "../../cap_amd/csrc/host/cap_jwt.hpp"

using namespace capjwt;

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s TOKENS JWKS [reps]\n", argv[0]);
    return 2;
  }
  const std::string blob = slurp(argv[1]);
  const std::string jwks = slurp(argv[2]);
  const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
  std::vector<std::string_view> toks;
  for (size_t p = 0; p < blob.size();) {
    size_t e = blob.find('\n', p);
    if (e == std::string::npos) e = blob.size();
    if (e > p) toks.emplace_back(blob.data() + p, e - p);
    p = e + 1;
  }
  std::string err;
  auto ks = NewJSONWebKeySet("https://bench.example/jwks", "", [&](const std::string&, const std::string&) {
    FetchResponse r;
    r.body = jwks;
    r.max_age_s = 3600;
    return r;
  }, &err);
  if (!ks) { std::fprintf(stderr, "keyset: %s\n", err.c_str()); return 1; }
  auto v = NewValidator(ks.get(), &err);
  Expected e;
  e.Issuer = "https://example.com/";
  e.Audiences = {"www.example.com"};
  e.SigningAlgorithms = {"ES256"};
  e.has_now = true;
  e.now_unix_ns = (1611699344LL + 60) * kSecond;
  std::vector<std::string_view> warm(toks.begin(), toks.begin() + std::min<size_t>(4096, toks.size()));
  v->ValidateBatch(warm, e);
  double best = 1e30;
  size_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    rusage ru0, ru1;
    getrusage(RUSAGE_SELF, &ru0);
    const auto t0 = std::chrono::steady_clock::now();
    auto rs = v->ValidateBatch(toks, e);
    acc = 0;
    for (const auto& x : rs) acc += x.ok;
    release_results(rs);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, dt);
    getrusage(RUSAGE_SELF, &ru1);
    const double st = (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) + 1e-6 * (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec);
    std::printf("rep %d: %.1f ms  (%.2f M/s)  accepted %zu/%zu  minflt %ld  stime %.3f s\n", r, dt * 1e3,
                toks.size() / dt / 1e6, acc, toks.size(), ru1.ru_minflt - ru0.ru_minflt, st);
  }
  std::printf("best %.1f ms = %.2f M tokens/s on %d host threads\n", best * 1e3, toks.size() / best / 1e6, host_threads());
  const int callers = argc > 4 ? std::atoi(argv[4]) : 0;
  if (callers > 0) {
    std::atomic<size_t> next{0}, ok{0};
    const size_t total = std::min<size_t>(toks.size(), 200000);
    rusage r0, r1;
    getrusage(RUSAGE_SELF, &r0);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int c = 0; c < callers; ++c)
      th.emplace_back([&] {
        for (size_t i; (i = next.fetch_add(1)) < total;) ok += v->Validate(toks[i], e).ok;
      });
    for (auto& t : th) t.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    getrusage(RUSAGE_SELF, &r1);
    auto secs = [](const timeval& a, const timeval& b) { return (b.tv_sec - a.tv_sec) + 1e-6 * (b.tv_usec - a.tv_usec); };
    std::printf("  cpu: user %.2f s sys %.2f s, vol cs %ld invol cs %ld\n", secs(r0.ru_utime, r1.ru_utime),
                secs(r0.ru_stime, r1.ru_stime), r1.ru_nvcsw - r0.ru_nvcsw, r1.ru_nivcsw - r0.ru_nivcsw);
    const auto st = ks->CoalescingStats();
    std::printf("single-token Validate x %d callers: %zu calls in %.1f ms (%.3f M/s), accepted %zu; %llu batches, max %llu\n",
                callers, total, dt * 1e3, total / dt / 1e6, ok.load(), (unsigned long long)st.batches,
                (unsigned long long)st.max_batch_seen);
  }
  return 0;
}
