// hostprof -- CPU-only timing harness for the host half of Validator.ValidateBatch
// (parse, kid routing, arena packing, payload JSON, claims, frees), the part
// bench.py's `e2e` line found to be the ceiling.  It links the host sources with
// jg_timing_stub.cpp, a STAND-IN for libcapjwt.so that marks every job accepted: the
// signatures are never checked here, so this binary measures host time only and
// is never a verifier.  Not part of the product; not loaded by any test.
//
//   usage: hostprof TOKENS_FILE JWKS_FILE [reps]      (CAPJWT_TRACE=1 for phases)
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
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
    const auto t0 = std::chrono::steady_clock::now();
    auto rs = v->ValidateBatch(toks, e);
    acc = 0;
    for (const auto& x : rs) acc += x.ok;
    release_results(rs);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, dt);
    std::printf("rep %d: %.1f ms  (%.2f M/s)  accepted %zu/%zu\n", r, dt * 1e3, toks.size() / dt / 1e6, acc, toks.size());
  }
  std::printf("best %.1f ms = %.2f M tokens/s on %d host threads\n", best * 1e3, toks.size() / best / 1e6, host_threads());
  return 0;
}
