// Host-plan microbenchmark (no GPU): times make_plan + the chunk's arena-span
// scan on a synthetic ES256 job list, serial and with the helper pool.
// Build: make -C tools/planbench ; run: tools/planbench/plan_bench [ntok] [nkeys]
#include "../../cap_amd/csrc/jg_runtime.cpp"

#include <chrono>

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 32768;
  const int nk = argc > 2 ? atoi(argv[2]) : 4;
  jg_ctx ctx;
  ctx.keys.assign(nk, HostKey{JG_KEY_EC, CLS_P256, 1});
  rebuild_class_tables(&ctx);
  std::vector<jg_tok> toks(n);
  for (size_t i = 0; i < n; ++i)
    toks[i] = jg_tok{i * 342, 255, 256, 86, (uint16_t)(i % nk), JG_ES256, 0};
  std::vector<jg_tok> staging(n);
  PlanScratch X;
  double best = 1e9;
  for (int it = 0; it < 50; ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t amin = UINT64_MAX, amax = 0, need = 0, seen[2];
    jg_tok* ht = staging.data();
    plan_count(&ctx, toks.data(), n, X, false, seen, [&](size_t i) {
      const jg_tok& t = toks[i];
      const uint64_t e = tok_end(t);
      amin = std::min<uint64_t>(amin, t.off);
      amax = std::max<uint64_t>(amax, e);
      need += e - t.off;
      ht[i] = t;
    });
    Plan P;
    plan_layout(&ctx, ht, n, P, X, false, seen);
    const auto t1 = std::chrono::steady_clock::now();
    best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
    if (need == 0 || P.npad < (int64_t)n || amin > amax) return 1;
  }
  std::printf("n=%zu keys=%d: host plan (span + count + job copy + layout) %.1f us -> %.2f ns/job\n", n, nk, best,
              best * 1e3 / n);
  return 0;
}
