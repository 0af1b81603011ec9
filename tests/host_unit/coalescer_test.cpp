// Coalescer (host/cap_jwt.cpp) under many concurrent callers, built with a
// sanitizer by tests/test_coalescer.py: every request is carried by exactly
// one batch, at the index the caller is told; a batch that throws reaches
// exactly its own callers; reconfiguring the dispatcher count while calls are
// in flight loses none; bursts of callers at max_inflight = 1 followed by
// silence all return (no lost wake-up).  The Exec stands in for KeySet::verify_raw (no device).
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../cap_amd/csrc/host/cap_jwt.hpp"

using capjwt::Coalescer;

namespace {
struct Seen {
  uint64_t batch;
  size_t idx;
  bool threw;
};
std::mutex g_mu;
std::unordered_map<std::string, Seen> g_seen;
std::atomic<uint64_t> g_batches{0}, g_dup{0}, g_bad{0};

int fail(const char* what) {
  std::printf("FAIL: %s\n", what);
  return 1;
}
}  // namespace

int main() {
  Coalescer co([](const std::vector<std::string_view>& toks) -> std::shared_ptr<const capjwt::Verified> {
    const uint64_t b = g_batches.fetch_add(1);
    const bool thr = b % 13 == 7;
    {
      std::lock_guard<std::mutex> g(g_mu);
      for (size_t i = 0; i < toks.size(); ++i)
        if (!g_seen.emplace(std::string(toks[i]), Seen{b, i, thr}).second) g_dup.fetch_add(1);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50 + (b * 7919) % 200));
    if (thr) throw std::runtime_error("batch " + std::to_string(b));
    return nullptr;
  });
  const int T = 96, M = 400;
  std::atomic<int> done{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int i = 0; i < M; ++i) {
        const std::string tok = "tok-" + std::to_string(t) + "-" + std::to_string(i);
        Coalescer::Req q;
        q.tok = tok;
        bool threw = false;
        try {
          co.run(&q);
        } catch (const std::runtime_error&) {
          threw = true;
        }
        Seen s;
        {
          std::lock_guard<std::mutex> g(g_mu);
          auto it = g_seen.find(tok);
          if (it == g_seen.end()) {
            g_bad.fetch_add(1);
            continue;
          }
          s = it->second;
        }
        if (s.idx != q.idx || s.threw != threw || q.batch) g_bad.fetch_add(1);
        if (rng() % 8 == 0) std::this_thread::yield();
      }
      done.fetch_add(1);
    });
  // reconfigure while the callers run
  for (int k = 0; done.load() < T; ++k) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    capjwt::CoalesceConfig c;
    c.max_inflight = 1 + k % 6;
    c.max_batch = k % 3 == 0 ? 5 : 65536;
    c.window_us = k % 4 == 0 ? 100 : 0;
    co.configure(c);
  }
  for (auto& x : th) x.join();
  const auto st = co.stats();
  std::printf("calls %llu batches %llu max batch %llu\n", (unsigned long long)st.calls,
              (unsigned long long)st.batches, (unsigned long long)st.max_batch_seen);
  if (g_dup.load()) return fail("a request carried twice");
  if (g_bad.load()) return fail("a caller told a wrong index / outcome, or not carried");
  if (g_seen.size() != (size_t)T * M || st.calls != (uint64_t)T * M) return fail("request count");
  if (st.batches != g_batches.load() || st.max_batch_seen < 2) return fail("batch count");

  // bursts at max_inflight = 1, then silence: every caller must return without
  // a later call arriving to kick the dispatcher (a lost wake-up hangs here)
  {
    capjwt::CoalesceConfig c;
    c.max_inflight = 1;
    c.max_batch = 65536;
    c.window_us = 0;
    co.configure(c);
  }
  for (int round = 0; round < 300; ++round) {
    const int B = 2 + round % 7;
    std::atomic<int> ready{0}, back{0};
    std::vector<std::thread> bt;
    for (int t = 0; t < B; ++t)
      bt.emplace_back([&, t] {
        ready.fetch_add(1);
        while (ready.load() < B) {
        }
        const std::string tok = "burst-" + std::to_string(round) + "-" + std::to_string(t);
        Coalescer::Req q;
        q.tok = tok;
        try {
          co.run(&q);
        } catch (const std::runtime_error&) {
        }
        back.fetch_add(1);
      });
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    while (back.load() < B) {
      if (std::chrono::steady_clock::now() > deadline) {
        std::printf("FAIL: burst %d: %d of %d callers never returned (lost wake-up)\n", round, B - back.load(), B);
        std::fflush(stdout);
        _exit(1);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    for (auto& x : bt) x.join();
  }
  std::printf("coalescer test ok\n");
  return 0;
}
