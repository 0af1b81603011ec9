// jg_runtime.cpp -- host runtime behind include/jg.h.
//
// Owns the per-device state (streams, generator / base-point comb tables, the
// staged key table) and turns a flat job list into a dispatch plan:
//   1. classify every (alg, key) pair into a kernel class (RSA-2K/3K/4K, P-256,
//      P-384, P-521, Ed25519, or reject -- go-jose newVerifier/verifyPayload
//      type dispatch);
//   2. counting-sort the jobs by (class, key) and pad every key's run to a
//      whole 64-lane wave, so each wave's key is uniform (scalar key loads,
//      broadcast modulus limbs);
//   3. launch prep (base64url + SHA-2) and the class's arithmetic kernels over
//      the padded ranges; scatter verdicts back.
//
// Streaming path (jg_submit / jg_wait / jg_verify_batch): a batch
// is split over the devices by the per-alg cost model, and each device's part
// runs in chunks of CHUNK jobs through a ring of NSLOT buffer sets (device
// scratch + pinned host staging).  The H2D copies of all chunks run back to
// back on one copy stream (the link stays busy while the host plans ahead);
// each chunk's kernels run on one of NLANE compute streams (+ per-class
// fan-out streams) once its copy event fires, overlapping the next copies.  One worker thread per device drains a FIFO of submitted
// work, so chunks of consecutive submissions overlap as well.
#include <pthread.h>
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/jg.h"
#include "kernels/batch.hpp"
#include "kernels/common.hpp"
#include "kernels/ecdsa.hpp"
#include "kernels/ed25519.hpp"
#include "kernels/hash.hpp"
#include "kernels/prep.hpp"
#include "host_mont.hpp"
#include "kernels/rsa.hpp"

static_assert(sizeof(jg_tok) == 24 && sizeof(jgk::JobDev) == 16, "job layouts");

using namespace jgk;

namespace {

constexpr size_t ARENA_SLACK = 256;   // aligned SHA word reads may run past the last string
constexpr int NLANE = 3;              // compute streams per device (HW queues 1..3; the copy stream has 0)
constexpr size_t SMALL_SUBMIT = 4096;  // submissions up to this many jobs go whole to one device slot
constexpr int NSLOT = 8;              // chunk buffer sets per device (pipeline depth)
constexpr int NZSLOT = 2;             // buffer sets of zero-copy plans (whole items; after the NSLOT ring)
constexpr int NALG = 16;              // alg ids 0..15 in the class table (jg_alg <= 10)

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

bool pipe_trace() {
  static const bool on = std::getenv("CAPJWT_PIPE_TRACE") != nullptr;
  return on;
}
hipEvent_t g_trace_ref = nullptr;     // first chunk's H2D start (trace only)

// CAPJWT_RELEASE_GTABLES=1: free a device's fixed-base tables when the last
// context using them is destroyed (default: kept for the process, ~54 GB per device)
bool release_gtables() {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_RELEASE_GTABLES");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// CAPJWT_LOAD_TRACE=1: per-phase wall times of jg_keys_load on stderr
bool load_trace() {
  static const bool on = std::getenv("CAPJWT_LOAD_TRACE") != nullptr;
  return on;
}
struct PhaseClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!load_trace()) return;
    std::fprintf(stderr, "[capjwt load] %-28s %8.2f ms\n", what, ms_since(t));
    t = std::chrono::steady_clock::now();
  }
};

// initial zero-copy settings of a context (zc plans: see run_plan's zc_feed)
bool zc_env_enabled() {
  const char* e = std::getenv("CAPJWT_ZC");
  return e && std::atoi(e) != 0;
}
size_t zc_env_max_jobs() {
  const char* e = std::getenv("CAPJWT_ZC_MAX");
  const long long v = e ? std::atoll(e) : 0;
  return v >= 64 ? (size_t)v : (size_t)2 << 20;
}

size_t chunk_jobs() {
  static const size_t n = [] {
    if (const char* e = std::getenv("CAPJWT_CHUNK")) {
      const long v = std::atol(e);
      if (v >= 64) return (size_t)v;
    }
    return (size_t)65536;
  }();
  return n;
}

// HBM a context may spend on P-256 key comb tables (ecdsa.hpp ec_key_w): 32 GiB
// by default (up to 4 keys at W = 24, 17 at W = 22), or CAPJWT_TABLE_BUDGET_GB
uint64_t default_table_budget() {
  static const uint64_t b = [] {
    if (const char* e = std::getenv("CAPJWT_TABLE_BUDGET_GB")) {
      const double v = std::atof(e);
      if (v >= 0) return (uint64_t)(v * (double)(1ull << 30));
    }
    return (uint64_t)32 << 30;
  }();
  return b;
}

// Chunk boundaries of jobs [lo, hi) for a pipeline of C-job chunks: the first
// chunks ramp up from 4096 jobs (the copy engine starts after a short host
// plan) and the tail ends in a quarter-size chunk (little kernel time left
// exposed after the last copy).
// The last chunk is split off at C/4 (`tail`) so an H2D-bound stream exposes
// less compute after its last copy; class-grouped (mixed) streams are
// compute-bound and skip it (tail = false): 524 k chunks of configs[4]
// 25.5-25.9 -> 24.5-25.1 ms per 1.25 M tokens (profiles/r03_s23_c5_tail_ab.txt).
std::vector<size_t> chunk_cuts(size_t lo, size_t hi, size_t C, size_t first = 4096, bool tail_chunk = true) {
  std::vector<size_t> cut{lo};
  for (size_t ramp = std::min<size_t>(C, first); cut.back() < hi; ramp = std::min(C, 2 * ramp))
    cut.push_back(std::min(hi, cut.back() + ramp));
  const size_t tail = C / 4;
  if (tail_chunk && cut.size() > 2 && tail >= 1024 && cut.back() - cut[cut.size() - 2] > tail)
    cut.insert(cut.end() - 1, cut.back() - tail);
  else if (!tail_chunk && cut.size() > 2 && cut.back() - cut[cut.size() - 2] < C / 8)
    // a remainder of a few thousand jobs would end the item with a whole
    // latency-bound kernel chain of its own (configs[4] stream: 4.8 k jobs,
    // +1.5 ms after the last full chunk): the last full chunk takes it
    cut.erase(cut.end() - 2);
  return cut;
}

// l4: limbs of the largest RSA-4K+ layout among the loaded keys (148/296/592)
int cls_rows_sig(int c, int l4) {
  switch (c) {
    case CLS_RSA2K: case CLS_RSA3K: return rsa_sig_rows(c);
    case CLS_RSA4K: return rsa_sig_rows_l(l4);
    case CLS_P256: case CLS_P384: case CLS_P521: return EC_S_ROW + 17;
    case CLS_ED25519: return 16;
    default: return 0;
  }
}
int cls_rows_scratch(int c, int l4) {
  switch (c) {
    case CLS_RSA2K: case CLS_RSA3K: return 2 * rsa_limbs(c) + rsa_sig_rows(c);   // x R, x, y
    case CLS_RSA4K: return 2 * l4 + rsa_sig_rows_l(l4);
    case CLS_P256: case CLS_P384: case CLS_P521: return ec_digit_rows(c) + 2 * ec_limbs(c);
    case CLS_ED25519: return 4 * ED_L;
    default: return 0;
  }
}
// Relative device time per token by kernel class (ES256 = 1): every class
// alone as a resident batch filling one MI355X, summed kernel time per token
// (tools/class_costs.py -> profiles/r03_class_costs.json).  cap_amd/shard.py
// CLASS_COST holds the same numbers (tests/test_shard_dist.py compares them).
// The RSA-4K+ entry is the 148-limb layout; 296- and 592-limb keys scale it
// by (limbs / 148)^2 (the modexp's MADs grow with the square of the width;
// measured 4.1x and 17.5x).  RSA entries average the PKCS#1 and PSS forms
// (RS256 3.94 / PS256 4.50, RS512 15.0 / PS512 16.0).
constexpr double CLS_COST[NCLS] = {0.01, 4.2, 9.0, 15.5, 1.0, 3.4, 6.6, 1.1};

// Grow-only buffers reallocate with 50 % headroom (2 MiB granules): a pipeline
// slot whose chunks vary in size and class mix (scratch rows per class) grows
// a few times, not at every larger chunk -- a reallocation costs a device
// synchronisation (hipFree) or a page-locking pass (hipHostMalloc).
inline size_t grow_size(size_t n, size_t cap) {
  const size_t want = std::max(n, cap + cap / 2);
  return (want + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
}

std::atomic<int> g_grows{0};      // CAPJWT_PIPE_TRACE: Grow / HGrow reallocations so far

struct Grow {                     // grow-only device allocation
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t n) {
    if (n == 0) n = 16;
    if (n > cap) {
      if (p) (void)hipFree(p);
      p = nullptr;
      const size_t c = grow_size(n, cap);
      cap = 0;
      g_grows.fetch_add(1, std::memory_order_relaxed);
      HIPCHK(hipMalloc(&p, c));
      cap = c;
    }
    return p;
  }
  ~Grow() { if (p) (void)hipFree(p); }
};

struct HGrow {                    // grow-only pinned host allocation
  void* p = nullptr;
  void* dp = nullptr;             // the same memory as kernels address it
  size_t cap = 0;
  void* get(size_t n) {
    if (n == 0) n = 16;
    if (n > cap) {
      if (p) (void)hipHostFree(p);
      p = dp = nullptr;
      const size_t want = grow_size(n, cap);
      cap = 0;
      g_grows.fetch_add(1, std::memory_order_relaxed);
      HIPCHK(hipHostMalloc(&p, want, hipHostMallocPortable | hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer(&dp, p, 0));
      cap = want;
    }
    return p;
  }
  ~HGrow() { if (p) (void)hipHostFree(p); }
};

struct HostKey {
  int kind = 0, cls = CLS_REJECT, valid = 0;
  int nlimbs = 0;                 // RSA: limbs of the key's modexp layout
};

// Device memory with shared ownership.  Comb tables are shared by key content
// between key loads (a JWKS refresh that keeps a key keeps its table: no copy,
// no rebuild), and a load's key blob is shared by its later width upgrades.
// A generation is released only once no queued work can reference it
// (pipeline slots hold their key state until their chunk has completed,
// resident batches until the next run or jg_batch_free).  The release must not
// make its caller wait for the device -- hipFree synchronises every stream, so
// dropping an old key table inline would stall a key load behind a background
// comb-table build (~1 s) or the verification pipeline -- so the last holder
// hands the pointer to a reaper thread that calls hipFree.  (Round 3 tried
// stream-ordered hipMallocAsync / hipFreeAsync instead: after a reload that
// re-used freed memory for a new table, a small-order Ed25519 key's table
// gave a wrong verdict and the parity suite hit an illegal address; with
// plain hipMalloc and the reaper the same sequence is exact --
// tools/diag_reload.py, tests/test_gpu_parity.py test_key_reload_reuses_tables.)
class Reaper {
 public:
  void push(int dev, void* p, size_t bytes) {
    std::lock_guard<std::mutex> g(mu_);
    if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    q_.push_back(Item{dev, p, bytes});
    pending_[dev] += bytes;
    cv_.notify_one();
  }
  // bytes handed over on device `dev` and not yet freed
  size_t pending(int dev) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pending_.find(dev);
    return it == pending_.end() ? 0 : it->second;
  }
  // wait until every pointer handed over so far has been freed
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    idle_.wait(lk, [&] { return q_.empty() && !busy_; });
  }
  ~Reaper() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      cv_.notify_one();
    }
    if (th_.joinable()) th_.join();
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) break;                       // stop requested, nothing left
      const auto it = q_.front();
      q_.pop_front();
      busy_ = true;
      lk.unlock();
      if (hipSetDevice(it.dev) == hipSuccess) (void)hipFree(it.p);
      lk.lock();
      pending_[it.dev] -= it.bytes;
      busy_ = false;
      if (q_.empty()) idle_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  struct Item { int dev; void* p; size_t bytes; };
  std::deque<Item> q_;
  std::map<int, size_t> pending_;
  bool stop_ = false, busy_ = false;
  std::thread th_;
};
Reaper& reaper() {
  static Reaper r;
  return r;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int dev = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) reaper().push(dev, p, bytes);
  }
  template <class T>
  T* as() const { return (T*)p; }
};
using DevBufP = std::shared_ptr<DevBuf>;

// hipMalloc into a DevBuf.  `fail` (jg_debug_fail_alloc): a countdown of
// allocations after which one fails as if the device were out of memory.
DevBufP dev_alloc(int dev, size_t bytes, std::atomic<int>* fail = nullptr) {
  if (fail) {
    int f = fail->load();
    while (f > 0 && !fail->compare_exchange_weak(f, f - 1)) {}
    if (f == 1) throw std::runtime_error("hipMalloc: out of memory (jg_debug_fail_alloc)");
  }
  auto b = std::make_shared<DevBuf>();
  b->dev = dev;
  b->bytes = std::max<size_t>(bytes, 16);
  HIPCHK(hipSetDevice(dev));
  hipError_t e = hipMalloc(&b->p, b->bytes);
  if (e == hipErrorOutOfMemory && reaper().pending(dev) > 0) {
    // free_hbm() counts memory the reaper has been handed but not yet freed
    // (its hipFree waits for the whole device): wait for it and try once more
    (void)hipGetLastError();
    b->p = nullptr;
    reaper().drain();
    e = hipMalloc(&b->p, b->bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    b->p = nullptr;
    throw std::runtime_error(std::string("hipMalloc(") + std::to_string(b->bytes >> 20) + " MiB): " +
                             hipGetErrorString(e));
  }
  return b;
}

// Lifetime check (debugging; CAPJWT_CHECK_LIFETIME=1 or jg_debug_lifetime_check).
// The rule the runtime relies on: a key generation's device memory (records,
// blob, comb tables) is released only once every launch that reads it has
// completed -- pipeline slots drop their key state in finish_slot after the
// chunk's `done` event, resident batches after a lane synchronize, loads and
// upgrades synchronise their own streams.  hipFree's implicit device-wide
// synchronisation would hide a violation, so the check does not rely on it:
// every stream that launches against a generation records an event into the
// generation's UseLog, and the generation's destructor (before any of its
// buffers go to the reaper) queries them all; an event still pending is a
// violation, logged with the stream's role and counted.
std::atomic<int> g_lifetime_on{[] {
  const char* e = std::getenv("CAPJWT_CHECK_LIFETIME");
  return e && std::atoi(e) != 0 ? 1 : 0;
}()};
std::atomic<uint64_t> g_lifetime_bad{0}, g_lifetime_checked{0};

struct UseLog {
  std::mutex mu;
  std::vector<std::pair<hipEvent_t, std::string>> ev;
  UseLog() = default;
  UseLog(const UseLog&) {}                         // a copied generation starts with no uses
  UseLog& operator=(const UseLog&) { return *this; }
  void record(hipStream_t s, const char* role, int c = -1) {
    if (!g_lifetime_on.load(std::memory_order_relaxed)) return;
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(e, s));
    char buf[128];
    if (c >= 0) std::snprintf(buf, sizeof buf, "%s of class %d (stream %p)", role, c, (void*)s);
    else std::snprintf(buf, sizeof buf, "%s (stream %p)", role, (void*)s);
    std::lock_guard<std::mutex> g(mu);
    // only pending uses matter: once the log has grown past the last prune,
    // completed events are counted and dropped (a long stream against a
    // stable key set would otherwise keep one event per chunk for ever)
    if (ev.size() >= prune_at) {
      size_t k = 0;
      for (auto& x : ev) {
        if (hipEventQuery(x.first) == hipSuccess) {
          g_lifetime_checked.fetch_add(1, std::memory_order_relaxed);
          (void)hipEventDestroy(x.first);
        } else {
          (void)hipGetLastError();
          ev[k++] = std::move(x);
        }
      }
      ev.resize(k);
      prune_at = std::max<size_t>(64, 2 * k);
    }
    ev.emplace_back(e, buf);
  }
  size_t prune_at = 64;
  ~UseLog() {
    for (auto& x : ev) {
      const hipError_t q = hipEventQuery(x.first);
      g_lifetime_checked.fetch_add(1, std::memory_order_relaxed);
      if (q == hipErrorNotReady) {
        g_lifetime_bad.fetch_add(1, std::memory_order_relaxed);
        std::fprintf(stderr, "[capjwt] lifetime check: a key generation is released while work on %s has not "
                             "completed\n", x.second.c_str());
      }
      (void)hipGetLastError();
      (void)hipEventDestroy(x.first);
    }
  }
};

// One device's copy of a key table generation: the DevKey records, the key
// blob (moduli, R^2, Montgomery coordinates), the class table of k_plan_fill,
// and the comb tables the records point at.  Immutable once published; a
// width upgrade publishes a new generation sharing the blob.
struct DevGen {
  DevBufP dkeys, blob, dcls;
  std::vector<DevBufP> tabs;      // comb tables the keys' `tab` addresses point into
  std::vector<DevKey> mirror;     // host copy of dkeys (after key prep: validity, tables)
  std::vector<uint8_t> kw;        // per key: comb width of its table (0 = none)
  mutable UseLog uses;            // lifetime check; last member, so it is checked before the buffers go
  DevKey* keys() const { return dkeys ? dkeys->as<DevKey>() : nullptr; }
  uint32_t* keyblob() const { return blob ? blob->as<uint32_t>() : nullptr; }
  const uint8_t* cls() const { return dcls ? dcls->as<uint8_t>() : nullptr; }
};
using DevGenP = std::shared_ptr<const DevGen>;

// The key table as every verification sees it: immutable, published whole.
// Submissions capture the state current at submit time and run entirely
// against it, so a key load never drains or blocks queued work; the previous
// state lives until the last chunk using it has completed.
struct KeyState {
  std::vector<HostKey> keys;
  std::vector<uint8_t> cls_tab;          // [key * NALG + alg] -> kernel class of the job
  std::vector<int32_t> cls_keys[NCLS];   // keys of each class, in index order
  int rsa4k_limbs = 148;                 // largest RSA-4K+ layout among the valid keys
  int rsa4k_layouts = 1;                 // RSA-4K+ layouts present (bit i: rsa4k_layout_limbs(i))
  uint64_t epoch = 0;                    // changes with the key list (dispatch plans are per epoch)
  std::string content;                   // the load's key bytes + budget: an identical reload is a no-op
  std::vector<std::string> tab_id;       // per key: content id of its comb table ("" = none)
  std::vector<uint8_t> want_w;           // per key: the comb width the table budget gives it
  std::vector<DevGenP> dev;              // per device slot
};
using KeyStateP = std::shared_ptr<const KeyState>;

// Fixed-base tables of the curve generators / Ed25519 base point depend only
// on (device, curve): every jg_ctx of the process shares one copy per device,
// built on first use and kept for the life of the process (they are constants
// of the curves: ~54 GB per device with all four, the P-256 one 21.5 GB and
// ~1.1 s to build -- a process that opens and closes contexts must not pay
// that again).  Deliberately never freed: the cache outlives static
// destruction, and the driver reclaims device memory at process exit.
struct SharedTable {
  uint32_t* p = nullptr;
};
std::mutex g_tab_mu;
auto& g_tabs = *new std::map<std::pair<int, int>, std::shared_ptr<SharedTable>>();   // (device id, class) -> table

// One in-order stream plus per-class fan-out streams: a mixed batch's classes
// are each too small to fill 256 CUs alone, so untimed runs put every class's
// kernel chain on its own stream, joined back before the scatter.
struct Lane {
  hipStream_t stream = nullptr;
  hipStream_t cstream[NCLS] = {};   // fan-out stream of each class (resident batches; may alias)
  std::vector<hipStream_t> fan;     // the fan-out streams themselves
  hipEvent_t ev_start = nullptr, ev_done[NCLS] = {};
  // Streams are bound to the process's hardware queues round-robin in
  // creation order (GPU_MAX_HW_QUEUES, 4 by default): the device creates
  // every lane's main stream first so the pipeline slots land on distinct
  // queues and really overlap, then the resident lanes' fan-out streams, each
  // lane's back to back (distinct queues while there are no more than the
  // process has).
  void create_main() { HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)); }
  // group[c]: class c's fan-out stream (0 .. ngroups-1)
  void create_fanout(const int* group, int ngroups) {
    fan.assign((size_t)ngroups, nullptr);
    for (auto& f : fan) HIPCHK(hipStreamCreateWithFlags(&f, hipStreamNonBlocking));
    for (int c = 1; c < NCLS; ++c) {
      cstream[c] = fan[(size_t)group[c]];
      HIPCHK(hipEventCreateWithFlags(&ev_done[c], hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&ev_start, hipEventDisableTiming));
  }
  void sync() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (hipStream_t f : fan) (void)hipStreamSynchronize(f);
  }
  void destroy() {
    sync();
    for (hipStream_t f : fan) (void)hipStreamDestroy(f);
    fan.clear();
    for (int c = 1; c < NCLS; ++c) {
      if (ev_done[c]) (void)hipEventDestroy(ev_done[c]);
      cstream[c] = nullptr;
      ev_done[c] = nullptr;
    }
    if (ev_start) (void)hipEventDestroy(ev_start);
    if (stream) (void)hipStreamDestroy(stream);
    ev_start = nullptr;
    stream = nullptr;
  }
};

// Resident batches: one fan-out stream per class.  Sharing one stream among
// the EC / Ed25519 classes (one per RSA class + one for the rest: no class
// chain behind an RSA chain on a shared hardware queue) measured 75.9 vs
// 83.3 M/s on configs[4]: the short, GPU-underfilling EC launches gain more
// from running beside each other (profiles/r05_s2/session_f.log).
constexpr int RES_GROUP[NCLS] = {0, 0, 1, 2, 3, 4, 5, 6};
constexpr int RES_NGROUPS = 7;

struct Bufs {
  // jobs: the plan's padded JobDev array; perm (resident batches only): padded
  // index -> caller index, for the device-side verdict scatter (pipeline
  // chunks scatter on the host from their staged perm instead)
  Grow arena, jobs, perm, meta, sigw, dig, status, siglen, vpad, verdict, rows, pss, exc, exc_cnt;
  Grow mid;                       // per key: shared SHA-256 block 0 and its midstate (k_prep_mid)
};

// Host side of one staged chunk: the counting-sort layout.
struct Plan {
  int64_t ntok = 0, npad = 0;
  ClassRange ranges[NCLS] = {};
  int hash_mask[NCLS] = {};       // per class: bit 0 SHA-256 present, bit 1 SHA-384/512
  int pss_any[NCLS] = {};         // per class: some token uses RSASSA-PSS (PS256/384/512)
  int sig_rows = 1, scratch_rows = 1;
  int rsa4k_limbs = 148, rsa4k_layouts = 1;   // the context's RSA-4K+ layouts at plan time
  int64_t pss_tokens = 0;         // PSS scratch tokens: the RSA classes' ranges back to back
  int64_t pss_off[NCLS] = {};
  int64_t nkeys = 0;              // key table size at plan time (prep midstate slots)
  std::vector<int64_t> kstart;    // per key: first padded slot of its run (runs of one class are contiguous)
};

struct PlanScratch {              // reused across chunks
  std::vector<uint8_t> tcls;      // class per job (host fill only)
  std::vector<int64_t> start, total;   // per bucket [nkeys + 1]
  std::vector<uint64_t> kmax;     // zero-copy plans: per key, the longest job span (bytes)
};

struct Ticket {
  std::mutex m;
  std::condition_variable cv;
  size_t pending = 0;             // chunks not yet complete
  int rc = 0;
  std::string err;
  void fail(int code, const std::string& e) {
    std::lock_guard<std::mutex> g(m);
    if (rc == 0) {
      rc = code;
      err = e;
    }
  }
  void done_chunks(size_t k) {
    std::lock_guard<std::mutex> g(m);
    pending -= std::min(pending, k);
    if (pending == 0) cv.notify_all();
  }
};

// A pipeline slot: the device scratch and pinned host staging of one chunk
// in flight (its kernels run on one of the device's NLANE compute lanes).
struct Slot {
  Bufs bufs;
  HGrow h_arena, h_meta, h_verdict;   // pinned staging: arena repack, plan block (H2D), verdicts (D2H)
  hipEvent_t done = nullptr;       // slot stream: verdicts copied back
  hipEvent_t copied = nullptr;     // copy stream: the chunk's inputs are on the device
  hipEvent_t tr_a = nullptr, tr_b = nullptr, tr_c = nullptr;   // CAPJWT_PIPE_TRACE: H2D start / end, kernels end
  hipEvent_t ev_planned = nullptr, ev_cls[NCLS] = {};            // class-grouped chunks (GroupFan)
  hipEvent_t ev_fed[NCLS] = {};                                  // zero-copy plans: class gathered (GroupFan::fed)
  double host_ms[7] = {};         // wait, plan, enqueue; of enqueue: H2D calls, sizing, before run_plan, run_plan
  int grows = 0;                                                // buffer reallocations while enqueuing (trace)
  int chunk_no = 0;
  size_t reserved = 0;             // chunk capacity (jobs) the buffers were sized for
  uint64_t reserved_epoch = ~0ull; // key table they were sized against
  PlanScratch plan;                // host plan scratch of the chunk being planned into this slot
  bool inflight = false;            // enqueued, not yet completed (Device::cmu)
  std::shared_ptr<Ticket> ticket;
  KeyStateP ks;                    // key state of the chunk in flight (kept alive until it completes)
  uint8_t* out = nullptr;
  size_t n = 0;
};

struct Item {                     // one device's share of a submission
  std::shared_ptr<Ticket> t;
  const uint8_t* arena = nullptr;
  size_t arena_len = 0;
  const jg_tok* toks = nullptr;   // the caller's array, [lo, hi)
  size_t lo = 0, hi = 0;
  uint8_t* out = nullptr;         // the caller's verdicts (index space of toks)
  KeyStateP ks;                   // the key table current at submit time
  const uint8_t* dev_arena = nullptr;   // device view of a page-locked arena (kernels read it over PCIe)
  size_t chunk = 0, nchunks = 0;
  std::vector<size_t> cuts;       // chunk boundaries (chunk_cuts)
  bool grouped = false;           // mixed classes: chunks run class-grouped (plan_chunk / issue_chunk)
  bool zc = false;                // class-major zero-copy plans (zc_enabled): no arena copy
  bool small_ec = true;           // small ECDSA chunks as one launch per (curve, key width) (issue_small_ec)
  std::atomic<uint64_t>* small_launches = nullptr;   // the context's count of them
};

// A thread that runs one job at a time for its owner (the device worker's
// planner: run() hands over a job, wait() returns once it has finished).
class Helper {
 public:
  explicit Helper(int device) : th_([this, device] { loop(device); }) {}
  ~Helper() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void run(std::function<void()> f) {
    std::lock_guard<std::mutex> g(m_);
    job_ = std::move(f);
    busy_ = true;
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return !busy_; });
  }

 private:
  void loop(int device) {
    pthread_setname_np(pthread_self(), "capjwt-plan");
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(m_);
    while (true) {
      cv_.wait(lk, [&] { return stop_ || job_; });
      if (!job_) break;                            // stopping
      auto f = std::move(job_);
      job_ = nullptr;
      lk.unlock();
      f();
      lk.lock();
      busy_ = false;
      cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::function<void()> job_;
  bool busy_ = false, stop_ = false;
  std::thread th_;
};

struct Device {
  int id = 0;
  Lane lane0;                     // resident batches, hashing
  Lane lane1;                     // resident batches staged second, fourth, ...
  hipStream_t kstream = nullptr;  // key loads (staging, narrow tables): beside the verify streams
  hipStream_t ustream = nullptr;  // background width upgrades of key comb tables
  uint32_t* gtab[NCLS] = {};
  uint32_t* btab = nullptr;
  std::shared_ptr<SharedTable> tab_ref[NCLS];   // keeps gtab / btab alive
  std::mutex mu;                  // lane0 + slots
  // streaming pipeline: H2D copies of every chunk back to back on one copy
  // stream (full link bandwidth, no sharing between slots), each slot's
  // kernels on its own stream once its copy event fires
  hipStream_t copy = nullptr;
  Lane lanes[NLANE];
  Slot slots[NSLOT + NZSLOT];      // the chunk ring, then the zero-copy plans' ring
  int next_slot = 0, next_lane = 0, next_zslot = 0;
  double gload[3] = {0, 0, 0};    // class-grouped chunks: class cost queued per group lane (relative)
  int next_res = 0;                // resident batches staged (lane0 / lane1 alternate)
  std::thread worker, completer;
  std::unique_ptr<Helper> planner;  // plans a pipeline item's next chunk (process_item)
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Item> q;
  bool stop = false;
  std::mutex cmu;                  // slots in flight (Slot::inflight, cq)
  std::condition_variable ccv, scv; // completer: a chunk enqueued / worker: a slot freed
  std::deque<Slot*> cq;            // in-flight chunks, enqueue order
  bool cstop = false;
};

}  // namespace

struct jg_batch {
  jg_ctx* ctx = nullptr;
  Device* dev = nullptr;
  Lane* lane = nullptr;
  std::unique_ptr<Bufs> own;
  Bufs* b = nullptr;
  Plan plan;
  size_t arena_len = 0;
  size_t dslot = 0;
  uint64_t epoch = 0;             // key-list epoch the plan was built for
  KeyStateP ks_run;               // key state of the last run (alive while its kernels may run)
  bool timing = true;
  // timing marks of the most recent run: events are created once and
  // re-recorded every run (no per-run event churn)
  std::vector<std::string> mark_names;
  std::vector<hipEvent_t> mark_events;
  size_t marks_used = 0;
  std::vector<std::string> tnames;
  std::vector<float> tms;
  ~jg_batch() {
    for (auto e : mark_events) (void)hipEventDestroy(e);
  }
};

struct jg_ticket {
  std::shared_ptr<Ticket> t;
};

struct jg_ctx {
  std::vector<std::unique_ptr<Device>> devs;
  std::atomic<size_t> chunk{chunk_jobs()};   // jobs per pipeline chunk
  std::atomic<bool> zc{zc_env_enabled()};    // class-major zero-copy plans (jg_set_zero_copy)
  std::atomic<size_t> zc_max{zc_env_max_jobs()};
  std::atomic<uint64_t> table_budget{default_table_budget()};   // HBM for key comb tables, all curves
  std::atomic<int> fail_alloc{0};            // jg_debug_fail_alloc countdown
  std::atomic<uint64_t> tables_built{0};     // comb-table builds launched by this context (jg_debug_tables_built)
  std::atomic<uint64_t> small_rr{0};         // device slot of the next small submission (submit_to)
  std::atomic<bool> small_ec{true};          // one-launch ECDSA small chunks (jg_debug_small_path)
  std::atomic<uint64_t> small_launches{0};   // k_ec_small launches enqueued (jg_debug_small_path)
  // jg_debug_fail_verify: countdown to an injected device failure of a
  // submission; once it fires the context is `poisoned` (every later
  // submission fails, as after a sticky HIP error) until it is destroyed
  std::atomic<int> fail_verify{0};
  std::atomic<bool> poisoned{false};
  // jg_debug_max_upgrades: background table upgrades left before the upgrader
  // stops (-1 = no limit); CAPJWT_DEBUG_MAX_UPGRADES sets the initial value
  std::atomic<int> upgrades_left{[] {
    const char* e = std::getenv("CAPJWT_DEBUG_MAX_UPGRADES");
    return e ? std::atoi(e) : -1;
  }()};
  // the published key table (KeyState): swapped whole under ks_mu
  std::mutex ks_mu;
  KeyStateP ks;
  KeyStateP state() {
    std::lock_guard<std::mutex> g(ks_mu);
    return ks;
  }
  void publish(KeyStateP n) {
    KeyStateP old;
    {
      std::lock_guard<std::mutex> g(ks_mu);
      old = std::move(ks);
      ks = std::move(n);
    }
    // `old` (and, if nothing else holds it, its device memory) dies here, outside the lock
  }
  std::mutex load_mu;             // serialises key loads and upgrade publications
  // background widening of comb tables (narrow table first, wide one swapped in)
  std::thread upgrader;
  std::mutex up_mu;
  std::condition_variable up_cv, up_idle_cv;
  bool up_stop = false, up_pending = false, up_busy = false;
  std::string up_warn;            // a width upgrade that did not fit free HBM
  std::mutex err_mu;
  std::string err;
  void set_err(const std::string& s) {
    std::lock_guard<std::mutex> g(err_mu);
    err = s;
  }
};

namespace {

// big-endian bytes -> 28-bit little-endian limbs; false if the value needs more than L limbs
bool be_to_limbs(const uint8_t* b, size_t n, uint32_t* out, int L) {
  std::memset(out, 0, sizeof(uint32_t) * L);
  for (size_t i = 0; i < n; ++i) {
    const uint8_t v = b[n - 1 - i];
    if (!v) continue;
    for (int k = 0; k < 8; ++k) {
      if (!((v >> k) & 1)) continue;
      const size_t bit = i * 8 + k;
      if (bit / 28 >= (size_t)L) return false;
      out[bit / 28] |= 1u << (bit % 28);
    }
  }
  return true;
}

int bitlen_be(const uint8_t* b, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (b[i]) {
      int k = 8;
      while (!((b[i] >> (k - 1)) & 1)) --k;
      return (int)((n - 1 - i) * 8) + k;
    }
  return 0;
}

int alg_family(int alg) {         // 1 RSA, 2 EC, 3 Ed, 0 none
  if (alg >= JG_RS256 && alg <= JG_PS512) return JG_KEY_RSA;
  if (alg >= JG_ES256 && alg <= JG_ES512) return JG_KEY_EC;
  if (alg == JG_EDDSA) return JG_KEY_ED25519;
  return 0;
}

// kernel class of a job (key_idx already range-checked)
inline int classify(const KeyState& K, const jg_tok& t) {
  return t.alg < NALG ? K.cls_tab[(size_t)t.key_idx * NALG + t.alg] : CLS_REJECT;
}

void rebuild_class_tables(KeyState& K) {
  const size_t nk = K.keys.size();
  K.cls_tab.assign(nk * NALG, (uint8_t)CLS_REJECT);
  for (auto& v : K.cls_keys) v.clear();
  K.rsa4k_limbs = rsa4k_layout_limbs(0);
  K.rsa4k_layouts = 1;
  for (size_t k = 0; k < nk; ++k) {
    const HostKey& hk = K.keys[k];
    if (hk.valid && hk.cls != CLS_REJECT) K.cls_keys[hk.cls].push_back((int32_t)k);
    if (hk.valid && hk.cls == CLS_RSA4K) {
      K.rsa4k_limbs = std::max(K.rsa4k_limbs, hk.nlimbs);
      for (int i = 0; i < RSA4K_NLAYOUT; ++i)
        if (hk.nlimbs == rsa4k_layout_limbs(i)) K.rsa4k_layouts |= 1 << i;
    }
    for (int a = 0; a < NALG; ++a)
      if (hk.valid && alg_family(a) == hk.kind) K.cls_tab[k * NALG + a] = (uint8_t)hk.cls;
  }
}

// Pipeline chunks whose jobs fall into two or more kernel classes run
// class-grouped: the chunk's plan fill on the least-loaded group lane
// (group_ctrl), then each class chain on the lane of its group (cls_group:
// three groups of classes), the exact kernels and the verdict scatter on the
// lane of the chunk's costliest group once every class is done.  A group's launches from consecutive chunks
// queue on one lane (one hardware queue each) while the three groups run side
// by side; lane-per-chunk instead ran each chunk's classes one after another
// (~6 ms of serial latency per 262 k mixed chunk; profiles/r03_s12).
// A class-grouped chunk's plan fill (everything of the chunk waits for it)
// runs on the group lane expected to drain first -- the one with the least
// class cost queued (Device::gload).  On the join lane (round 3) it queued
// behind the previous chunk's whole RSA-4K chain while the other lanes idled
// 2-4 ms; on the copy stream it measured no better (profiles/r04_s3/zc_trace,
// r04_s4/stream_ctrl_*).
// Class -> group lane of a class-grouped chunk: RSA-2K and RSA-4K+ on lane 0,
// RSA-3K and P-384 on lane 1, P-256, P-521 and Ed25519 on lane 2.  In a
// mixed chunk the small EC launches run far below their stand-alone rate
// beside the RSA modexps (the round-3 split, all EC / Ed25519 classes on one
// lane, made that lane the chunk's critical path: 6.8 of ~7 ms per 524 k
// chunk, profiles/r04_s9/stream_trace_timeline.txt); this split measured
// 20.8-21.2 ms per configs[4] stream at 262 k chunks against 22.8-23.2 ms
// (profiles/r04_s10-s12; the round-3 split put every EC / Ed25519 class on
// lane 2 and RSA-3K on lane 0).  Indexed by class 0..7.
constexpr int CLS_GROUP[NCLS] = {0, 0, 1, 0, 2, 1, 2, 2};
inline int cls_group(int c) { return CLS_GROUP[c]; }

// two or more kernel classes among (a sample of) the jobs
bool mixed_classes(const KeyState& K, const jg_tok* toks, size_t n) {
  const size_t step = std::max<size_t>(1, n / 2048), nk = K.keys.size();
  int first = -1;
  for (size_t i = 0; i < n; i += step) {
    if (toks[i].key_idx >= nk) continue;
    const int c = classify(K, toks[i]);
    if (c == CLS_REJECT) continue;
    if (first < 0) first = c;
    else if (c != first) return true;
  }
  return false;
}

// Reject a job list that names a key outside the table or a byte span outside
// the arena (the prep kernel reads the device copy at those offsets).
bool check_jobs(const KeyState& K, size_t arena_len, const jg_tok* toks, size_t ntok, std::string* err,
                size_t base = 0) {
  const size_t nk = K.keys.size();
  for (size_t i = 0; i < ntok; ++i) {
    const jg_tok& t = toks[i];
    if (t.key_idx >= nk) {
      *err = "jg_tok[" + std::to_string(base + i) + "].key_idx " + std::to_string(t.key_idx) +
             " out of range of the loaded key table (" + std::to_string(nk) + " keys)";
      return false;
    }
    if (t.off > arena_len || t.sig_in_len > arena_len - t.off ||
        (uint64_t)t.sig_rel_off + t.sig_b64_len > arena_len - t.off) {
      *err = "jg_tok[" + std::to_string(base + i) + "]: signing input or signature span past the arena (" +
             std::to_string(arena_len) + " bytes)";
      return false;
    }
  }
  return true;
}

inline uint64_t tok_end(const jg_tok& t) {
  return std::max<uint64_t>(t.off + t.sig_in_len, t.off + (uint64_t)t.sig_rel_off + t.sig_b64_len);
}

// The device-visible address of page-locked host memory (hipHostMalloc /
// hipHostRegister), or nullptr for pageable memory.
const uint8_t* device_view(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();      // clear the sticky "invalid value" of pageable memory
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost) return nullptr;
  if (a.devicePointer && a.hostPointer)        // attributes describe the allocation base
    return (const uint8_t*)a.devicePointer + ((const uint8_t*)p - (const uint8_t*)a.hostPointer);
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, const_cast<void*>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return (const uint8_t*)dp;
}

// Blocks from jg_host_alloc: base -> usable size.  Each is allocated with
// ARENA_SLACK more bytes than asked for, so a zero-copy plan's prep kernels
// may read past the last token of an arena held in one (as they do past every
// token of a device arena copy) without leaving the allocation.
std::mutex g_hmu;
std::map<uintptr_t, size_t>& g_hblocks = *new std::map<uintptr_t, size_t>();

// an arena the prep kernels may read in place: inside one jg_host_alloc block
// and under 4 GiB (JobDev offsets are 32-bit)
bool zc_arena_ok(const uint8_t* arena, size_t len) {
  if (!arena || ((uintptr_t)arena & 15) || len + ARENA_SLACK >= (uint64_t(1) << 32)) return false;
  const uintptr_t a = (uintptr_t)arena;
  std::lock_guard<std::mutex> g(g_hmu);
  auto it = g_hblocks.upper_bound(a);
  if (it == g_hblocks.begin()) return false;
  --it;
  return a >= it->first && a + len <= it->first + it->second;
}

// Dispatch plan of toks[0..ntok): a counting sort by (class, key) --
// classes 1..NCLS-1 key by key, then the reject bucket; every bucket padded
// to whole waves.  plan_layout counts (the per-job host work of a pipeline
// chunk) and fills X.start / X.total per bucket; the placement is done either
// on the host (plan_fill_host: resident batches) or on the device
// (k_plan_fill: pipeline chunks).
// per-job part of plan_layout (one pass; `visit(i)` runs on every job too):
// bucket counts into X.total, (class, alg) pairs seen into *seen (bit c*16+alg)
template <class Visit>
void plan_count(const KeyState& K, const jg_tok* toks, size_t ntok, PlanScratch& X, bool keep_cls, uint64_t* seen,
                Visit&& visit) {
  const size_t nk = K.keys.size(), NB = nk + 1, RB = nk;
  X.total.assign(NB, 0);
  if (keep_cls) X.tcls.resize(ntok);
  const uint8_t* ctab = K.cls_tab.data();
  int64_t* tot = X.total.data();
  uint64_t lo = 0, hi = 0;
  for (size_t i = 0; i < ntok; ++i) {
    const jg_tok& tk = toks[i];
    visit(i);
    const unsigned alg = tk.alg;
    const unsigned c = alg < NALG ? ctab[(size_t)tk.key_idx * NALG + alg] : CLS_REJECT;
    if (keep_cls) X.tcls[i] = (uint8_t)c;
    const unsigned combo = c * 16 + (alg & 15u);
    if (combo < 64) lo |= 1ull << combo;
    else hi |= 1ull << (combo - 64);
    tot[c == CLS_REJECT ? RB : tk.key_idx]++;
  }
  seen[0] = lo;
  seen[1] = hi;
}

void plan_layout(const KeyState& K, const jg_tok* toks, size_t ntok, Plan& P, PlanScratch& X, bool keep_cls,
                 const uint64_t* seen_in = nullptr) {
  const size_t nk = K.keys.size();
  const size_t NB = nk + 1, RB = nk;
  uint64_t seen[2];
  if (seen_in) {
    seen[0] = seen_in[0];
    seen[1] = seen_in[1];
  } else {
    plan_count(K, toks, ntok, X, keep_cls, seen, [](size_t) {});
  }
  X.start.assign(NB, 0);
  const int64_t* tot = X.total.data();
  for (int c = 0; c < NCLS; ++c) {
    P.hash_mask[c] = P.pss_any[c] = 0;
    for (int alg = 0; alg < 16; ++alg) {
      const unsigned combo = (unsigned)c * 16 + alg;
      if (!((seen[combo >> 6] >> (combo & 63)) & 1)) continue;
      P.hash_mask[c] |= (alg == JG_RS256 || alg == JG_PS256 || alg == JG_ES256) ? 1 : 2;
      P.pss_any[c] |= alg >= JG_PS256 && alg <= JG_PS512;
    }
  }
  int64_t pos = 0;
  for (int c = 1; c <= NCLS; ++c) {
    const int cc = c % NCLS;
    P.ranges[cc].begin = pos;
    if (cc == CLS_REJECT) {
      X.start[RB] = pos;
      pos += (tot[RB] + WAVE - 1) / WAVE * WAVE;
    } else {
      for (int32_t k : K.cls_keys[cc]) {
        X.start[(size_t)k] = pos;
        pos += (tot[(size_t)k] + WAVE - 1) / WAVE * WAVE;
      }
    }
    P.ranges[cc].end = pos;
  }
  P.kstart.assign(X.start.begin(), X.start.begin() + (int64_t)nk);
  P.npad = pos > 0 ? pos : WAVE;
  P.ntok = (int64_t)ntok;
  P.sig_rows = 1;
  P.scratch_rows = 1;
  P.pss_tokens = 0;
  P.rsa4k_limbs = K.rsa4k_limbs;
  P.rsa4k_layouts = K.rsa4k_layouts;
  P.nkeys = (int64_t)K.keys.size();
  for (int c = 1; c < NCLS; ++c) {
    if (P.ranges[c].end <= P.ranges[c].begin) continue;
    P.sig_rows = std::max(P.sig_rows, cls_rows_sig(c, P.rsa4k_limbs));
    P.scratch_rows = std::max(P.scratch_rows, cls_rows_scratch(c, P.rsa4k_limbs));
    if (c <= CLS_RSA4K) {
      P.pss_off[c] = P.pss_tokens;
      P.pss_tokens += P.ranges[c].end - P.ranges[c].begin;
    }
  }
}

// padding lanes of bucket b: [lo, hi); the empty plan is one wave of padding
inline std::pair<int64_t, int64_t> pad_range(const PlanScratch& X, size_t b, const Plan& P, size_t RB) {
  if (P.npad == WAVE && X.start[RB] == 0 && b == RB) {
    int64_t any = 0;
    for (int64_t t : X.total) any += t;
    if (any == 0) return {0, WAVE};
  }
  return {X.start[b] + X.total[b], X.start[b] + (X.total[b] + WAVE - 1) / WAVE * WAVE};
}

// Host placement (resident batches): JobDev array + perm in padded order.
void plan_fill_host(const KeyState& K, const jg_tok* toks, size_t ntok, const Plan& P, PlanScratch& X, JobDev* jobs,
                    int32_t* perm) {
  const size_t nk = K.keys.size(), NB = nk + 1, RB = nk;
  for (size_t b = 0; b < NB; ++b) {
    const auto r = pad_range(X, b, P, RB);
    const JobDev pad{0, 0, 0, job_pack(b == RB ? 0u : (uint32_t)b, JOB_PAD, 0)};
    for (int64_t p = r.first; p < r.second; ++p) {
      jobs[p] = pad;
      perm[p] = -1;
    }
  }
  std::vector<int64_t> cur = X.start;
  for (size_t i = 0; i < ntok; ++i) {
    const jg_tok& tk = toks[i];
    const int c = X.tcls[i];
    const int64_t p = cur[c == CLS_REJECT ? RB : tk.key_idx]++;
    jobs[p] = JobDev{(uint32_t)tk.off, tk.sig_in_len, (uint32_t)(tk.off + tk.sig_rel_off),
                     job_pack(c == CLS_REJECT ? 0u : tk.key_idx, tk.alg, tk.sig_b64_len)};
    perm[p] = (int32_t)i;
  }
}

// device scratch of a plan (inputs are copied by the caller)
void size_scratch(Bufs* B, const Plan& P, size_t arena_bytes) {
  const int64_t npad = P.npad;
  const size_t ntok = std::max<size_t>((size_t)P.ntok, 1);
  B->arena.get(arena_bytes + ARENA_SLACK);
  B->sigw.get(sizeof(uint32_t) * P.sig_rows * npad);
  B->dig.get(sizeof(uint32_t) * DIG_ROWS * npad);
  B->status.get(npad);
  B->siglen.get(sizeof(uint16_t) * npad);
  B->vpad.get(npad);
  B->verdict.get(ntok);
  B->rows.get(sizeof(uint32_t) * (size_t)P.scratch_rows * npad);
  B->pss.get((size_t)std::max<int64_t>(P.pss_tokens, 1) * 2048);
  B->exc.get(sizeof(int32_t) * npad);
  B->exc_cnt.get(sizeof(uint32_t) * NCLS);
}

// resident batch: arena (slack zeroed), jobs and perm placed by the host
void upload(Bufs* B, hipStream_t s, const Plan& P, const uint8_t* arena, size_t arena_bytes, const JobDev* jobs,
            const int32_t* perm) {
  size_scratch(B, P, arena_bytes);
  B->jobs.get(sizeof(JobDev) * P.npad);
  B->perm.get(sizeof(int32_t) * P.npad);
  uint8_t* da = (uint8_t*)B->arena.p;
  if (arena_bytes && arena) HIPCHK(hipMemcpyAsync(da, arena, arena_bytes, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(da + arena_bytes, 0, ARENA_SLACK, s));
  HIPCHK(hipMemcpyAsync(B->jobs.p, jobs, sizeof(JobDev) * P.npad, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(B->perm.p, perm, sizeof(int32_t) * P.npad, hipMemcpyHostToDevice, s));
}

// Plan block of a pipeline chunk (pinned staging and its device copy alike):
// bucket cursors | padding ranges | the chunk's jg_tok jobs in caller order.
// Zero-copy plans add, per bucket, the base offset, first padded slot and
// slot stride of its region of the device arena (k_zc_gather).
struct PlanBlock {
  size_t cur_off, pad_off, zc_off, toks_off, bytes;
  PlanBlock(size_t nbuckets, size_t n) {
    cur_off = 0;
    pad_off = sizeof(uint64_t) * nbuckets;
    zc_off = pad_off + 2 * sizeof(int64_t) * nbuckets;
    toks_off = (zc_off + 3 * sizeof(uint64_t) * nbuckets + 63) & ~size_t(63);
    bytes = toks_off + sizeof(jg_tok) * std::max<size_t>(n, 1);
  }
};

// ---------------------------------------------------------------- timing marks
void mark(jg_batch* b, const char* name) {
  if (!b || !b->timing) return;
  if (b->marks_used == b->mark_events.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    b->mark_events.push_back(e);
    b->mark_names.emplace_back();
  }
  HIPCHK(hipEventRecord(b->mark_events[b->marks_used], b->lane->stream));
  b->mark_names[b->marks_used] = name;
  ++b->marks_used;
}

const char* cls_name(int c) {
  static const char* n[NCLS] = {"reject", "rsa2048", "rsa3072", "rsa4096", "p256", "p384", "p521", "ed25519"};
  return n[c];
}

struct MarkCtx {
  jg_batch* b;
  int cls;
};
thread_local MarkCtx g_mark_ctx;

void mark_cb(void* p, const char* kname) {
  MarkCtx* m = (MarkCtx*)p;
  mark(m->b, (std::string(cls_name(m->cls)) + "_" + kname).c_str());
}

Marker marker(jg_batch* b, int cls) {
  Marker mk;
  if (!b || !b->timing) return mk;
  g_mark_ctx = MarkCtx{b, cls};
  mk.ctx = &g_mark_ctx;
  mk.fn = mark_cb;
  return mk;
}

// Launch the verify kernels of a staged plan on lane L.  With `marks` (a
// timed resident run) the classes run in sequence on L.stream with a HIP event
// after each kernel; otherwise classes with work run on their own streams.
// fanout: run the classes of a mixed plan on the lane's per-class streams
// (resident batches); pipeline chunks that are not class-grouped keep them in
// order on the lane's own stream (per-class fan-out streams measured 29-31
// against 25.7 ms per configs[4] stream, profiles/r03_s22_c5_stream_fanout_ab.txt)

// Resident batches alternate between two lanes whose main streams sit on
// different hardware queues (lane0, lane1), so runs of two staged batches
// enqueued back to back overlap: one batch's latency-bound front kernels
// (prep, scalar stage) and tails share the CUs with the other's point kernel
// (ES256 +6 %, profiles/r03_s9_altlanes_ab.json).

// Class-major zero-copy streams (round 4).  A mixed (class-grouped)
// submission whose arena lies in memory from jg_host_alloc runs as ONE plan
// over the whole item instead of arrival-order chunks, and its arena is never
// DMAed: per class, a gather kernel (k_zc_gather) copies that class's token
// bytes from the pinned arena over PCIe into the plan's device arena, and the
// class's chain (prep, arithmetic) starts as soon as its own gather is done.
// Every class gets one launch chain over all of its tokens.  Chunked, a mixed
// stream's first chunk copy (~5.7 ms for 524 k tokens) was exposed and each
// chunk's classes were too small to fill the chip
// (profiles/r03_s22_c5_pipe_trace_524k.txt); a zero-copy gather of shuffled
// 640-B records reads at the SDMA copy's rate (profiles/r04_s2_zc_gather.txt).
// (A first form let the prep kernels read the pinned arena directly: their
// 4-byte loads interleaved with SHA rounds drew ~15 GB/s from the link and
// the stream ran at half the chunked rate, profiles/r04_s3/zc_prep_direct_*.)
// Per context (jg_set_zero_copy), OFF by default: the chunked pipeline is
// faster on configs[4] today (profiles/r04_s3/zc_gather_*: 42.6 vs 24.7 ms per
// 1.25 M tokens).  The initial setting is CAPJWT_ZC (1 turns it on) and
// CAPJWT_ZC_MAX, the jobs per zero-copy plan (a
// longer item is cut into equal plans; device scratch grows with it, ~5 KB per
// job with RSA-4K keys).
//
// The gathers of a zero-copy plan all run on one feed stream (the copy
// stream), the costliest class first, so each gather has the link to itself
// and the longest arithmetic chain starts earliest; each class's chain waits
// for its own gather on the lane of its class group.

// Runs of consecutive keys of class c (the plan's key order) whose comb tables
// have one width: fn(begin, end, w) per run, over padded slots.  All of a
// curve's keys share one width except while a background upgrade is widening
// some of them (one launch chain per width then).
template <class Fn>
void width_runs(const KeyState& K, const DevGen& G, const Plan& P, int c, Fn&& fn) {
  const ClassRange r = P.ranges[c];
  int64_t beg = r.begin;
  int w = -1;
  for (int32_t k : K.cls_keys[c]) {
    const int kw = G.kw[(size_t)k];
    // the launch width must be the width of the table the key's record points
    // at: a wider launch would index past the end of a narrower table
    const DevKey& rec = G.mirror[(size_t)k];
    if (kw == 0 || rec.tab == 0 || rec.tab_w != kw)
      throw std::runtime_error("key " + std::to_string(k) + ": comb table record (width " + std::to_string(rec.tab_w) +
                               ", " + (rec.tab ? "set" : "null") + ") does not match its launch width " +
                               std::to_string(kw));
    if (w >= 0 && kw != w) {
      const int64_t kb = P.kstart[(size_t)k];
      if (kb > beg) fn(beg, kb, w);
      beg = kb;
    }
    w = kw;
  }
  if (w >= 0 && r.end > beg) fn(beg, r.end, w);
}

// CAPJWT_CHECK_KEYS=1 (debugging): before each run, read the generation's
// device key records back and compare their comb-table fields with the host mirror
bool check_keys_env() {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_CHECK_KEYS");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

void check_device_records(const DevGen& G) {
  const size_t nk = G.mirror.size();
  if (!nk) return;
  std::vector<DevKey> dev(nk);
  HIPCHK(hipMemcpy(dev.data(), G.keys(), sizeof(DevKey) * nk, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < nk; ++k)
    if (dev[k].tab != G.mirror[k].tab || dev[k].tab_w != G.mirror[k].tab_w || dev[k].valid != G.mirror[k].valid)
      throw std::runtime_error("key " + std::to_string(k) + ": device record (tab_w " + std::to_string(dev[k].tab_w) +
                               ") differs from the host mirror (tab_w " + std::to_string(G.mirror[k].tab_w) + ")");
}

// Explicit streams of a class-grouped pipeline chunk (plan_chunk / issue_chunk): the
// chunk's control work on `ctrl`, each class chain on cls[c], the verdict
// scatter on `join` once every class's `done` event has fired.
struct GroupFan {
  hipStream_t ctrl = nullptr, join = nullptr;
  hipStream_t cls[NCLS] = {};
  hipEvent_t start = nullptr;
  hipEvent_t done[NCLS] = {};
  // zero-copy plans: every class's k_zc_gather on `feed`, costliest class
  // first (zc_feed; else at the head of its own chain); class c's chain on
  // cls[c] waits for fed[c]
  hipStream_t feed = nullptr;
  hipEvent_t fed[NCLS] = {};
  double cost[NCLS] = {};         // class device cost of the plan (feed order)
  bool zc = false;
  ZcGatherArgs gather{};          // begin / end set per class
};

// vpad_zeroed: the device plan fill zeroed every padded slot's verdict (pipeline chunks)
void run_plan(Device* d, const KeyState& K, const DevGen& G, Lane* L, Bufs* B, const Plan& P, jg_batch* marks,
              bool fanout = true, const GroupFan* gf = nullptr, bool vpad_zeroed = false,
              uint8_t* verdict_dst = nullptr) {
  if (check_keys_env()) check_device_records(G);
  const bool timed = marks && marks->timing;
  int nact = 0;
  for (int c = 1; c < NCLS; ++c) nact += P.ranges[c].end > P.ranges[c].begin;
  const bool conc = !timed && !gf && fanout && nact > 1;
  const int64_t np = P.npad;
  const hipStream_t s0 = gf ? gf->join : L->stream;
  mark(marks, "begin");
  if (!vpad_zeroed) HIPCHK(hipMemsetAsync(B->vpad.p, 0, np, gf ? gf->ctrl : s0));
  if (gf) HIPCHK(hipEventRecord(gf->start, gf->ctrl));
  PrepArgs pa{};
  pa.arena = (const uint8_t*)B->arena.p;
  pa.jobs = (const JobDev*)B->jobs.p;
  pa.keys = G.keys();
  pa.keyblob = G.keyblob();
  pa.sigw = (uint32_t*)B->sigw.p;
  pa.dig = (uint32_t*)B->dig.p;
  pa.status = (uint8_t*)B->status.p;
  pa.siglen = (uint16_t*)B->siglen.p;
  pa.npad = np;
  pa.mid = (uint32_t*)B->mid.get(sizeof(uint32_t) * PREP_MID_WORDS * (size_t)std::max<int64_t>(P.nkeys, 1));
  uint32_t* rows = (uint32_t*)B->rows.p;
  if (conc) HIPCHK(hipEventRecord(L->ev_start, s0));
  const bool zc = gf && gf->zc, feed = zc && gf->feed;
  int order[NCLS - 1];
  for (int i = 0; i < NCLS - 1; ++i) order[i] = i + 1;
#ifndef JG_RESIDENT_COST_ORDER
#define JG_RESIDENT_COST_ORDER 0
#endif
  if (JG_RESIDENT_COST_ORDER && conc) {
    // a mixed resident batch's class chains, costliest first: the critical
    // chain (RSA-4K+ in configs[4]) takes the CUs first, the short EC chains
    // fill in beside it
    double cost[NCLS] = {};
    for (int c = 1; c < NCLS; ++c) cost[c] = CLS_COST[c] * (double)(P.ranges[c].end - P.ranges[c].begin);
    std::stable_sort(order, order + NCLS - 1, [&](int x, int y) { return cost[x] > cost[y]; });
  }
  if (feed) {
    std::stable_sort(order, order + NCLS - 1, [&](int x, int y) { return gf->cost[x] > gf->cost[y]; });
    if (gf->feed != gf->ctrl) HIPCHK(hipStreamWaitEvent(gf->feed, gf->start, 0));
  }
  std::vector<std::pair<int, EcArgs>> exact_later;      // class-grouped chunks: k_ec_exact on the join lane
  for (int oi = 0; oi < NCLS - 1; ++oi) {
    const int c = order[oi];
    const ClassRange r = P.ranges[c];
    if (r.end <= r.begin) continue;
    // every class reads and writes only columns [r.begin, r.end) of the shared
    // scratch rows, its own exception counter and its own PSS scratch
    hipStream_t s = s0;
    if (conc) {
      s = L->cstream[c];
      HIPCHK(hipStreamWaitEvent(s, L->ev_start, 0));
    } else if (gf) {
      s = gf->cls[c];
      if (!feed) HIPCHK(hipStreamWaitEvent(s, gf->start, 0));
    }
    if (zc) {
      // the class's token bytes from the caller's pinned arena into HBM
      ZcGatherArgs za = gf->gather;
      za.begin = r.begin;
      za.end = r.end;
      launch_zc_gather(za, feed ? gf->feed : s);
      if (feed) {
        HIPCHK(hipEventRecord(gf->fed[c], gf->feed));
        HIPCHK(hipStreamWaitEvent(s, gf->fed[c], 0));
      }
    }
    pa.begin = r.begin;
    pa.end = r.end;
    pa.zrows = cls_rows_sig(c, P.rsa4k_limbs);
    pa.ec_words = (c >= CLS_P256 && c <= CLS_P521) ? ec_sig_words(c) : 0;
    launch_prep(c, P.hash_mask[c], pa, s);
    mark(marks, (std::string(cls_name(c)) + "_prep").c_str());
    if (c <= CLS_RSA4K) {
      RsaArgs ra{};
      ra.jobs = pa.jobs; ra.keys = pa.keys; ra.keyblob = pa.keyblob;
      ra.sigw = pa.sigw; ra.dig = pa.dig;
      const int Lm = c == CLS_RSA4K ? P.rsa4k_limbs : rsa_limbs(c);
      ra.xmw = rows;
      ra.xlr = rows + (size_t)Lm * np;
      ra.yw = rows + (size_t)2 * Lm * np;
      ra.status = pa.status; ra.siglen = pa.siglen; ra.verdict_pad = (uint8_t*)B->vpad.p;
      ra.pss_scratch = (uint8_t*)B->pss.p + P.pss_off[c] * 2048;
      ra.has_pss = P.pss_any[c];
      ra.layouts = c == CLS_RSA4K ? P.rsa4k_layouts : 1;
      ra.npad = np; ra.begin = r.begin; ra.end = r.end;
      launch_rsa(c, ra, s, marker(marks, c));
    } else if (c <= CLS_P521) {
      if (!d->gtab[c]) throw std::runtime_error("curve table missing");
      EcArgs ea{};
      ea.jobs = pa.jobs; ea.keys = pa.keys; ea.keyblob = pa.keyblob;
      ea.sigw = pa.sigw; ea.dig = pa.dig; ea.status = pa.status; ea.verdict_pad = (uint8_t*)B->vpad.p;
      ea.digs = rows;
      ea.u1w = rows + (size_t)ec_digit_rows(c) * np;
      ea.u2w = rows + (size_t)(ec_digit_rows(c) + ec_limbs(c)) * np;
      ea.gtab = d->gtab[c];
      ea.exc_list = (int32_t*)B->exc.p + r.begin;
      ea.exc_count = (uint32_t*)B->exc_cnt.p + c;
      ea.npad = np;
      ea.exc_reset = 1;
      // class-grouped chunks: the exact kernels wait for the join lane (below).
      // A k_ec_exact launch needs a SIMD with ~290 VGPRs free even when it has
      // no work; behind the RSA modexps (256 VGPRs, 2 waves per SIMD) it waited
      // 0.8-1.4 ms for one, and every later class of the EC group's lane (and
      // the next chunk's) waited behind it (profiles/r04_s3/zc_trace).
      // One exact launch per class, after all of its width runs: k_ec_exact
      // walks the class's whole exception list (every run appends to it)
      ea.part = EC_FAST;
      width_runs(K, G, P, c, [&](int64_t b, int64_t e, int w) {
        ea.begin = b; ea.end = e; ea.wq = w;
        launch_ec(c, ea, s, marker(marks, c));
        ea.exc_reset = 0;          // later runs of the class append to its exception list
      });
      EcArgs x = ea;
      x.begin = r.begin;
      x.end = r.end;
      x.part = EC_EXACT;
      if (gf) exact_later.push_back({c, x});
      else launch_ec(c, x, s, marker(marks, c));
    } else {
      if (!d->btab) throw std::runtime_error("Ed25519 base table missing");
      EdArgs ea{};
      ea.jobs = pa.jobs; ea.keys = pa.keys; ea.keyblob = pa.keyblob;
      ea.sigw = pa.sigw; ea.dig = pa.dig; ea.status = pa.status; ea.siglen = pa.siglen;
      ea.verdict_pad = (uint8_t*)B->vpad.p;
      ea.xyz = rows;
      ea.btab = d->btab;
      ea.npad = np;
      width_runs(K, G, P, c, [&](int64_t b, int64_t e, int w) {
        ea.begin = b; ea.end = e; ea.wa = w;
        launch_ed(ea, s, marker(marks, c));
      });
    }
    // a class stream's key-memory use is logged BEFORE its done event: what the
    // join lane (and so every release of the generation) waits for covers it.
    // Logged after the done event, the use could still be pending behind other
    // work on a shared hardware queue when the join completed (a false
    // lifetime violation, seen once in a full GPU session).
    if (s != s0) G.uses.record(s, conc ? "class stream" : "group lane", c);
    if (conc) {
      HIPCHK(hipEventRecord(L->ev_done[c], s));
      HIPCHK(hipStreamWaitEvent(s0, L->ev_done[c], 0));
    } else if (gf) {
      HIPCHK(hipEventRecord(gf->done[c], s));
      if (s != s0) HIPCHK(hipStreamWaitEvent(s0, gf->done[c], 0));
    }
  }
  for (const auto& [c, x] : exact_later) launch_ec(c, x, s0, Marker{});   // s0 waited for every class
  launch_scatter((const int32_t*)B->perm.p, (const uint8_t*)B->vpad.p,
                 verdict_dst ? verdict_dst : (uint8_t*)B->verdict.p, np, s0);
  mark(marks, "scatter");
  HIPCHK(hipGetLastError());
  // the class streams logged their uses above; the chunk's control stream
  // logged its plan fill (issue_chunk, before `start`); the zero-copy feed's
  // gathers read no key memory
  G.uses.record(s0, gf ? "join lane" : "lane");
}

void collect_times(jg_batch* b) {
  b->tnames.clear();
  b->tms.clear();
  for (size_t i = 1; i < b->marks_used; ++i) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, b->mark_events[i - 1], b->mark_events[i]) == hipSuccess) {
      b->tnames.push_back(b->mark_names[i]);
      b->tms.push_back(ms);
    }
  }
}

// ---------------------------------------------------------------- streaming pipeline
// Complete the chunk held by slot S (its verdicts were copied to pinned
// staging): hand the verdicts to the caller and count the chunk off its ticket.
// Runs on the device's completer thread (completer_loop), S.inflight still
// set: the worker does not touch S until the completer clears it.
void finish_slot(Slot& S) {
  const hipError_t e = hipEventSynchronize(S.done);
  if (e != hipSuccess) S.ticket->fail(-2, std::string("verify chunk: ") + hipGetErrorString(e));
  else if (S.n) std::memcpy(S.out, S.h_verdict.p, S.n);
  if (pipe_trace() && e == hipSuccess && g_trace_ref) {
    float a = 0, b = 0, c = 0, dn = 0;
    (void)hipEventElapsedTime(&a, g_trace_ref, S.tr_a);
    (void)hipEventElapsedTime(&b, g_trace_ref, S.tr_b);
    (void)hipEventElapsedTime(&c, g_trace_ref, S.tr_c);
    (void)hipEventElapsedTime(&dn, g_trace_ref, S.done);
    std::fprintf(stderr, "[pipe] chunk %3d n=%7zu host wait %.3f plan %.3f enq %.3f (h2d calls %.3f, sizing %.3f, pre-launch %.3f, launches %.3f, grows %d) | gpu h2d %.3f-%.3f kern-end %.3f done %.3f ms\n",
                 S.chunk_no, S.n, S.host_ms[0], S.host_ms[1], S.host_ms[2], S.host_ms[3], S.host_ms[4], S.host_ms[5], S.host_ms[6], S.grows, a, b, c, dn);
  }
  auto t = std::move(S.ticket);
  S.ticket.reset();
  S.ks.reset();                    // may free a replaced key state (after this chunk completed)
  t->done_chunks(1);
}


// Plan and enqueue one chunk toks[0..n) of an item on slot S.
// Size a slot's buffers once for the pipeline's chunk capacity C and the
// key table's classes (their largest scratch rows), so chunks of varying size
// and class mix never reallocate in the stream (a hipFree synchronises the
// device, a hipHostMalloc page-locks): ~1 GB of device scratch per slot at
// C = 64 k for a context with RSA-4K keys, far less for ES256 alone.
void reserve_slot(const KeyState& K, Slot& S, size_t C, size_t nbuckets, double bytes_per_job, bool zc) {
  const PlanBlock L(nbuckets, C);
  S.h_meta.get(L.bytes);
  // the plan block's device copy too: grown per chunk size, its hipFree
  // stalled the host 2.5-4.5 ms behind the whole device on each slot's first
  // larger chunk (CAPJWT_PIPE_TRACE "grows")
  S.bufs.meta.get(L.bytes);
  S.h_verdict.get(C);
  int sig_rows = 1, scratch_rows = 1;
  bool rsa = false;
  for (int c = 1; c < NCLS; ++c) {
    if (K.cls_keys[c].empty()) continue;
    sig_rows = std::max(sig_rows, cls_rows_sig(c, K.rsa4k_limbs));
    scratch_rows = std::max(scratch_rows, cls_rows_scratch(c, K.rsa4k_limbs));
    rsa = rsa || c <= CLS_RSA4K;
  }
  const size_t npad = C + (size_t)WAVE * nbuckets;
  Bufs* B = &S.bufs;
  B->arena.get(zc ? ARENA_SLACK : (size_t)(bytes_per_job * 1.25 * (double)C) + ARENA_SLACK);
  B->jobs.get(sizeof(JobDev) * npad);
  B->perm.get(sizeof(int32_t) * npad);
  B->sigw.get(sizeof(uint32_t) * sig_rows * npad);
  B->dig.get(sizeof(uint32_t) * DIG_ROWS * npad);
  B->status.get(npad);
  B->siglen.get(sizeof(uint16_t) * npad);
  B->vpad.get(npad);
  B->verdict.get(C);
  B->rows.get(sizeof(uint32_t) * (size_t)scratch_rows * npad);
  if (rsa) B->pss.get(C * 2048);
  B->exc.get(sizeof(int32_t) * npad);
  B->mid.get(sizeof(uint32_t) * PREP_MID_WORDS * std::max<size_t>(K.keys.size(), 1));
  S.reserved = C;
  S.reserved_epoch = K.epoch;
}

// A job outside the key table or the arena, found by scan_chunk (jg_wait -> -1)
struct BadJob : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// plan_chunk's one host pass over a chunk's jobs: validate each (key_idx in
// the table, spans inside the arena: check_jobs' rule), count the plan's
// buckets and the (class, alg) pairs, find the arena span, and copy the jobs
// into the pinned plan block (ht).  Chunks of 64 k jobs and more are cut over
// four host threads (per-thread counts, merged): a 524 k-job chunk's pass held
// the device worker ~4 ms, during which the next chunk's copy could not start
// (profiles/r04_s9/stream_trace_timeline.txt, the gaps between chunks).
struct ChunkScan {
  uint64_t amin = UINT64_MAX, amax = 0, need = 0, seen[2] = {0, 0};
};
void scan_chunk(const KeyState& K, const jg_tok* toks, size_t n, size_t arena_len, size_t base, jg_tok* ht, bool zc,
                PlanScratch& X, ChunkScan& out) {
  const size_t nk = K.keys.size(), NB = nk + 1, RB = nk;
  const uint8_t* ctab = K.cls_tab.data();
  const int nt = n >= 65536 ? 4 : 1;
  std::vector<std::vector<int64_t>> tot(nt, std::vector<int64_t>(NB, 0));
  std::vector<std::vector<uint64_t>> kmax(zc ? nt : 0, std::vector<uint64_t>(NB, 0));
  std::vector<ChunkScan> part(nt);
  std::vector<size_t> bad(nt, SIZE_MAX);
  auto run = [&](int t) {
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    int64_t* tt = tot[t].data();
    ChunkScan& r = part[t];
    uint64_t sl = 0, sh = 0;
    for (size_t i = lo; i < hi; ++i) {
      const jg_tok& tk = toks[i];
      if (tk.key_idx >= nk || tk.off > arena_len || tk.sig_in_len > arena_len - tk.off ||
          (uint64_t)tk.sig_rel_off + tk.sig_b64_len > arena_len - tk.off) {
        bad[t] = i;
        break;
      }
      const uint64_t e = tok_end(tk);
      r.amin = std::min<uint64_t>(r.amin, tk.off);
      r.amax = std::max<uint64_t>(r.amax, e);
      r.need += e - tk.off;
      ht[i] = tk;
      const unsigned alg = tk.alg;
      const unsigned c = alg < NALG ? ctab[(size_t)tk.key_idx * NALG + alg] : CLS_REJECT;
      const unsigned combo = c * 16 + (alg & 15u);
      if (combo < 64) sl |= 1ull << combo;
      else sh |= 1ull << (combo - 64);
      tt[c == CLS_REJECT ? RB : tk.key_idx]++;
      if (zc && c != CLS_REJECT) kmax[t][tk.key_idx] = std::max<uint64_t>(kmax[t][tk.key_idx], e - tk.off);
    }
    r.seen[0] = sl;
    r.seen[1] = sh;
  };
  if (nt == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
    run(0);
    for (auto& t : th) t.join();
  }
  for (int t = 0; t < nt; ++t)
    if (bad[t] != SIZE_MAX) {
      std::string err;
      check_jobs(K, arena_len, toks + bad[t], 1, &err, base + bad[t]);
      throw BadJob(err);
    }
  X.total.assign(NB, 0);
  if (zc) X.kmax.assign(NB, 0);
  for (int t = 0; t < nt; ++t) {
    for (size_t b = 0; b < NB; ++b) X.total[b] += tot[t][b];
    if (zc)
      for (size_t b = 0; b < NB; ++b) X.kmax[b] = std::max(X.kmax[b], kmax[t][b]);
    out.amin = std::min(out.amin, part[t].amin);
    out.amax = std::max(out.amax, part[t].amax);
    out.need += part[t].need;
    out.seen[0] |= part[t].seen[0];
    out.seen[1] |= part[t].seen[1];
  }
}

// A chunk planned on the host (plan_chunk), ready for issue_chunk.
struct ChunkPlan {
  Plan P;
  size_t n = 0, bytes = 0;
  const uint8_t* src = nullptr;    // arena bytes to DMA (nullptr: none)
  uint64_t base = 0, dbase = 0;
  bool zc = false;
  std::chrono::steady_clock::time_point t_start;
};

// The host half of a chunk: buffers sized, jobs validated and copied into the
// slot's pinned plan block, the arena span staged, the plan laid out.  Touches
// only slot S (free: its previous chunk completed) and read-only key state, so
// the device worker runs it for the next chunk on its planner thread while it
// issues the current one (process_item).
void plan_chunk(Slot& S, const Item& it, const jg_tok* toks, size_t n, size_t job_base, ChunkPlan& CP) {
  CP = ChunkPlan{};
  CP.n = n;
  CP.t_start = std::chrono::steady_clock::now();
  const auto t_start = CP.t_start;
  const KeyState& K = *it.ks;
  if (S.reserved < std::max(it.chunk, n) || S.reserved_epoch != K.epoch) {
    // bytes per job from a sample (jobs are validated by scan_chunk below:
    // a bad span must not size the buffers)
    double bpj = 0;
    for (size_t i = 0; i < std::min<size_t>(n, 256); ++i)
      bpj += (double)std::min<uint64_t>(tok_end(toks[i]) - toks[i].off, it.arena_len);
    reserve_slot(K, S, std::max(it.chunk, n), K.keys.size() + 1, n ? bpj / (double)std::min<size_t>(n, 256) : 512.0,
                 it.zc);
  }
  // One pass over the caller's jobs: the arena span they use, the bucket
  // counts of the plan, and their copy into the pinned plan block.  The span
  // is DMAed straight from a pinned caller arena when it is compact, else
  // repacked job by job into pinned staging.
  const size_t NB = K.keys.size() + 1;
  const PlanBlock L(NB, n);
  uint8_t* hb = (uint8_t*)S.h_meta.get(L.bytes);
  jg_tok* ht = (jg_tok*)(hb + L.toks_off);
  ChunkScan scan;
  scan_chunk(K, toks, n, it.arena_len, job_base, ht, it.zc, S.plan, scan);
  uint64_t amin = scan.amin, amax = scan.amax, need = scan.need, seen[2] = {scan.seen[0], scan.seen[1]};
  std::vector<uint64_t>& kmax = S.plan.kmax;
  if (n == 0) amin = amax = 0;
  const uint64_t base = amin & ~uint64_t(255);
  const uint64_t span = amax - base;
  // JobDev offsets are 32-bit: a span that does not fit is repacked
  const bool compact = span <= 2 * need + 65536 && span < (uint64_t(1) << 32) - ARENA_SLACK;
  const uint8_t* src = nullptr;
  size_t bytes;
  uint64_t dbase;                                  // subtracted from job offsets on the device
  // Zero-copy plan: the device arena holds each key's jobs at a fixed stride
  // (its longest span + 30 bytes of 16-byte alignment, rounded to 16), filled
  // by k_zc_gather from the caller's pinned arena.  A layout of 4 GiB or more
  // (JobDev offsets are 32-bit) takes the DMA path instead.
  bool zc = it.zc;
  uint64_t zbytes = 0;
  uint64_t* zc_tab = (uint64_t*)(hb + L.zc_off);   // [NB] base | [NB] first slot | [NB] stride
  if (zc) {
    const int64_t* tot = S.plan.total.data();
    for (size_t k = 0; k < NB; ++k) {
      const uint64_t slots = k + 1 < NB ? (uint64_t)(tot[k] + WAVE - 1) / WAVE * WAVE : 0;   // the reject bucket is never prepped
      const uint64_t stride = slots ? (kmax[k] + 30 + 15) & ~uint64_t(15) : 0;
      zc_tab[k] = zbytes;
      zc_tab[2 * NB + k] = stride;
      zbytes += slots * stride;
    }
    if (zbytes + ARENA_SLACK >= (uint64_t(1) << 32)) zc = false;
  }
  if (zc) {
    bytes = (size_t)zbytes;                        // arena size; nothing is DMAed
    dbase = base;
  } else if (compact) {
    bytes = (size_t)span;
    dbase = base;
    if (it.dev_arena) {
      src = it.arena + base;                       // page-locked: DMA straight from the caller
    } else {
      uint8_t* h = (uint8_t*)S.h_arena.get(bytes);
      std::memcpy(h, it.arena + base, bytes);
      src = h;
    }
  } else {
    if (need + 4 * n >= (uint64_t(1) << 32) - ARENA_SLACK)
      throw std::runtime_error("a pipeline chunk's jobs span 4 GiB or more of arena: lower jg_set_chunk");
    uint8_t* h = (uint8_t*)S.h_arena.get((size_t)need + 4 * n);
    uint64_t pos = 0;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t len = tok_end(toks[i]) - toks[i].off;
      std::memcpy(h + pos, it.arena + toks[i].off, len);
      ht[i].off = pos;
      pos += (len + 3) & ~uint64_t(3);
    }
    bytes = (size_t)pos;
    dbase = 0;
    src = h;
  }
  Plan& P = CP.P;
  plan_layout(K, ht, n, P, S.plan, false, seen);
  uint64_t* cur = (uint64_t*)(hb + L.cur_off);
  int64_t* pad = (int64_t*)(hb + L.pad_off);
  for (size_t k = 0; k < NB; ++k) {
    const auto r = pad_range(S.plan, k, P, NB - 1);
    cur[k] = (uint64_t)S.plan.start[k];
    pad[2 * k] = r.first;
    pad[2 * k + 1] = r.second;
    if (zc) zc_tab[NB + k] = (uint64_t)S.plan.start[k];
  }
  CP.bytes = bytes;
  CP.src = src;
  CP.base = base;
  CP.dbase = dbase;
  CP.zc = zc;
  if (pipe_trace()) S.host_ms[1] = ms_since(t_start);
}

// A small chunk whose jobs are all ECDSA, EdDSA or RS256/384/512 on RSA-2K-
// class keys (or rejected) -- coalesced single-token calls -- runs as ONE
// launch per (curve, key-table width) and one for the RSA jobs: k_ec_small
// (kernels/ec_small.hpp), k_ed_small (ed25519.hip) and k_rsa_small (rsa.hip)
// read the jobs from their arguments and the
// arena in place (pinned host memory: the caller's, or the slot's staging)
// and writes each verdict byte straight to the slot's pinned verdicts.  No
// arena DMA, plan fill, prep / scalar / point / exact / scatter chain: the
// batch chain paid ~9 dependent launches and ~40 us of launch gaps for a lone
// token (profiles/r06_s9/small_chain).  Rejected jobs (alg / key mismatch, an
// invalid key) get verdict 0 here.  Returns false, having enqueued nothing,
// when the chunk does not qualify: another class, a signing input over
// EC_SMALL_IN_MAX bytes, an arena without a device view, a key whose comb
// table is not in place.
bool issue_small_ec(Device* d, Slot& S, const Item& it, const ChunkPlan& CP, const KeyState& K, const DevGen& G,
                    hipStream_t s) {
  const size_t n = CP.n;
  if (!it.small_ec || n == 0 || n > (size_t)SMALL_MAX || CP.zc || !CP.src) return false;
  const size_t NB = K.keys.size() + 1;
  const jg_tok* ht = (const jg_tok*)((const uint8_t*)S.h_meta.p + PlanBlock(NB, n).toks_off);
  int cls[SMALL_MAX];
  for (size_t i = 0; i < n; ++i) {
    const int c = classify(K, ht[i]);
    cls[i] = c;
    if (c == CLS_REJECT) continue;
    if (ht[i].sig_in_len > SMALL_IN_MAX) return false;
    const int32_t k = ht[i].key_idx;
    const DevKey& rec = G.mirror[(size_t)k];
    if (c == CLS_RSA2K) {                          // k_rsa_small: PKCS#1 v1.5 only
      if (ht[i].alg < JG_RS256 || ht[i].alg > JG_RS512 || rec.rr2_off == 0) return false;
      continue;
    }
    if (c == CLS_ED25519) {
      if (ht[i].alg != JG_EDDSA || !d->btab) return false;
    } else if (c < CLS_P256 || c > CLS_P521 || !d->gtab[c]) {
      return false;
    }
    if (G.kw[(size_t)k] == 0 || rec.tab == 0 || rec.tab_w != G.kw[(size_t)k]) return false;
  }
  // the arena's device view: the caller's page-locked arena, or the staging copy
  const uint8_t* dsrc = nullptr;
  if (CP.src == (const uint8_t*)S.h_arena.p) dsrc = (const uint8_t*)S.h_arena.dp;
  else if (it.dev_arena && CP.src >= it.arena && CP.src < it.arena + it.arena_len) dsrc = it.dev_arena + (CP.src - it.arena);
  if (!dsrc) return false;
  uint8_t* vh = (uint8_t*)S.h_verdict.get(n);
  std::memset(vh, 0, n);
  uint8_t* vd = (uint8_t*)S.h_verdict.dp;
  bool done[SMALL_MAX] = {};
  for (size_t i = 0; i < n; ++i) {
    if (done[i] || cls[i] == CLS_REJECT) continue;
    const int c = cls[i];
    if (c == CLS_RSA2K) {
      RsaSmallArgs A{};
      A.arena = dsrc;
      A.keys = G.keys();
      A.keyblob = G.keyblob();
      A.verdict = vd;
      for (size_t j = i; j < n; ++j) {
        if (done[j] || cls[j] != c) continue;
        const jg_tok& t = ht[j];
        const uint64_t o = t.off - CP.dbase;
        A.jobs[A.n] = JobDev{(uint32_t)o, t.sig_in_len, (uint32_t)(o + t.sig_rel_off),
                             job_pack(t.key_idx, t.alg, t.sig_b64_len)};
        A.out[A.n] = (uint16_t)j;
        ++A.n;
        done[j] = true;
      }
      launch_rsa_small(A, s);
      if (it.small_launches) it.small_launches->fetch_add(1, std::memory_order_relaxed);
      continue;
    }
    const int w = G.kw[ht[i].key_idx];
    if (c == CLS_ED25519) {
      EdSmallArgs A{};
      A.arena = dsrc;
      A.keys = G.keys();
      A.keyblob = G.keyblob();
      A.btab = d->btab;
      A.verdict = vd;
      for (size_t j = i; j < n; ++j) {
        if (done[j] || cls[j] != c || G.kw[ht[j].key_idx] != w) continue;
        const jg_tok& t = ht[j];
        const uint64_t o = t.off - CP.dbase;
        A.jobs[A.n] = JobDev{(uint32_t)o, t.sig_in_len, (uint32_t)(o + t.sig_rel_off),
                             job_pack(t.key_idx, t.alg, t.sig_b64_len)};
        A.out[A.n] = (uint16_t)j;
        ++A.n;
        done[j] = true;
      }
      launch_ed_small(w, A, s);
      if (it.small_launches) it.small_launches->fetch_add(1, std::memory_order_relaxed);
      continue;
    }
    EcSmallArgs A{};
    A.arena = dsrc;
    A.keys = G.keys();
    A.keyblob = G.keyblob();
    A.gtab = d->gtab[c];
    A.verdict = vd;
    for (size_t j = i; j < n; ++j) {
      if (done[j] || cls[j] != c || G.kw[ht[j].key_idx] != w) continue;
      const jg_tok& t = ht[j];
      const uint64_t o = t.off - CP.dbase;
      A.jobs[A.n] = JobDev{(uint32_t)o, t.sig_in_len, (uint32_t)(o + t.sig_rel_off),
                           job_pack(t.key_idx, t.alg, t.sig_b64_len)};
      A.out[A.n] = (uint16_t)j;
      ++A.n;
      done[j] = true;
    }
    launch_ec_small(c, w, A, s);
    if (it.small_launches) it.small_launches->fetch_add(1, std::memory_order_relaxed);
  }
  G.uses.record(s, "small ec");
  return true;
}

// The device half of a chunk planned by plan_chunk: arena DMA, plan fill,
// the class launches and the verdict copy (device worker thread only).
void issue_chunk(Device* d, size_t dslot, Slot& S, const Item& it, const ChunkPlan& CP, uint8_t* out) {
  const int grows0 = g_grows.load(std::memory_order_relaxed);
  const KeyState& K = *it.ks;
  const DevGen& G = *K.dev[dslot];
  const Plan& P = CP.P;
  const size_t n = CP.n, NB = K.keys.size() + 1, bytes = CP.bytes;
  const PlanBlock L(NB, n);
  uint8_t* hb = (uint8_t*)S.h_meta.p;
  const uint8_t* src = CP.src;
  const uint64_t base = CP.base, dbase = CP.dbase;
  const bool zc = CP.zc;
  Lane& LN = d->lanes[d->next_lane];
  d->next_lane = (d->next_lane + 1) % NLANE;
  hipStream_t s = LN.stream;
  const bool tr = pipe_trace();
  const auto t_enq = std::chrono::steady_clock::now();
  // The arena span goes over PCIe on the copy stream's DMA engine (spans of
  // consecutive chunks back to back); the rest of the chunk runs on a compute
  // lane once that copy lands: a copy kernel pulls the plan block's cursors
  // from pinned host memory, k_plan_fill reads the jobs straight from it
  // (zero-copy), and a copy kernel writes the verdicts back to pinned memory.
  size_scratch(&S.bufs, P, bytes);
  S.bufs.jobs.get(sizeof(JobDev) * P.npad);
  S.bufs.perm.get(sizeof(int32_t) * P.npad);
  uint8_t* dm = (uint8_t*)S.bufs.meta.get(L.bytes);
  if (tr) S.host_ms[4] = ms_since(t_enq);
  const uint8_t* hbd = (const uint8_t*)S.h_meta.dp;
  const hipStream_t cs = d->copy;
  int nact = 0, jgrp = 0;
  double gcost[3] = {0, 0, 0};
  for (int c = 1; c < NCLS; ++c) {
    const int64_t m = P.ranges[c].end - P.ranges[c].begin;
    if (m <= 0) continue;
    ++nact;
    gcost[cls_group(c)] += CLS_COST[c] * (double)m;
  }
  for (int g = 1; g < 3; ++g)
    if (gcost[g] > gcost[jgrp]) jgrp = g;
  // a zero-copy plan always runs grouped: its classes' gathers ride on the GroupFan
  const bool grouped = (it.grouped && nact >= 2) || zc;
  // A small ungrouped chunk (coalesced single-token calls) runs its whole
  // chain on its lane: the arena copy on the lane itself (no copy-stream event
  // and wait) and the verdicts scattered straight into pinned memory (no copy
  // kernel) -- 3 of its ~14 HIP calls fewer.  The device's submission thread,
  // which issues them, is what bounds small-batch throughput
  // (profiles/r06_s6/single_probe.log).  (Traced runs keep the copy stream.)
  const bool small = !grouped && n <= SMALL_SUBMIT && !tr;
  if (!tr && issue_small_ec(d, S, it, CP, K, G, s)) {
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(S.done, s));
    S.ticket = it.t;
    S.ks = it.ks;
    S.out = out;
    S.n = n;
    return;
  }
  if (tr) HIPCHK(hipEventRecord(S.tr_a, cs));
  if (bytes && !zc) HIPCHK(hipMemcpyAsync(S.bufs.arena.p, src, bytes, hipMemcpyHostToDevice, small ? s : cs));
  // grouped chunks: the whole plan block goes over by DMA behind the arena
  // (the plan fill then reads device memory); else the header by a copy
  // kernel and the jobs read in place from pinned memory
  if (grouped) HIPCHK(hipMemcpyAsync(dm, hb, L.bytes, hipMemcpyHostToDevice, cs));
  if (!small) HIPCHK(hipEventRecord(S.copied, cs));
  if (tr) HIPCHK(hipEventRecord(S.tr_b, cs));
  if (tr) S.host_ms[3] = ms_since(t_enq);
  GroupFan gf;
  hipStream_t fs = s;                              // the plan fill's stream
  if (zc) {
    gf.zc = true;
    gf.gather.src = it.dev_arena + base;
    gf.gather.jobs = (JobDev*)S.bufs.jobs.p;
    gf.gather.kbase = (const uint64_t*)(dm + L.zc_off);
    gf.gather.kstart = (const int64_t*)(dm + L.zc_off + sizeof(uint64_t) * NB);
    gf.gather.kstride = (const uint64_t*)(dm + L.zc_off + 2 * sizeof(uint64_t) * NB);
    gf.gather.dst = (uint8_t*)S.bufs.arena.p;
    {
      gf.feed = cs;                                // the copy stream carries no arena copies now
      for (int c = 1; c < NCLS; ++c) {
        gf.fed[c] = S.ev_fed[c];
        gf.cost[c] = CLS_COST[c] * (double)(P.ranges[c].end - P.ranges[c].begin);
      }
    }
  }
  if (grouped) {
    gf.join = d->lanes[jgrp].stream;
    int least = 0;
    for (int g = 1; g < 3; ++g)
      if (d->gload[g] < d->gload[least]) least = g;
    gf.ctrl = d->lanes[least].stream;
    // queued class cost per group lane, relative (the smallest kept at 0)
    double lo = 1e300;
    for (int g = 0; g < 3; ++g) lo = std::min(lo, d->gload[g] += gcost[g]);
    for (int g = 0; g < 3; ++g) d->gload[g] -= lo;
    for (int c = 1; c < NCLS; ++c) gf.cls[c] = d->lanes[cls_group(c)].stream;
    gf.start = S.ev_planned;
    for (int c = 0; c < NCLS; ++c) gf.done[c] = S.ev_cls[c];
    fs = gf.ctrl;
  }
  if (fs != cs && !small) HIPCHK(hipStreamWaitEvent(fs, S.copied, 0));
  if (!grouped) launch_copy(hbd, dm, L.toks_off, fs);
  {
    PlanFillArgs fa{};
    fa.toks = (const jg_tok*)((grouped ? (const uint8_t*)dm : hbd) + L.toks_off);
    fa.n = (int64_t)n;
    fa.base = dbase;
    fa.cls_tab = G.cls();
    fa.nkeys = (int32_t)(NB - 1);
    fa.cursor = (unsigned long long*)(dm + L.cur_off);
    fa.pad = (const int64_t*)(dm + L.pad_off);
    fa.jobs = (JobDev*)S.bufs.jobs.p;
    fa.perm = (int32_t*)S.bufs.perm.p;
    fa.vpad = (uint8_t*)S.bufs.vpad.p;
    launch_plan_fill(fa, fs);
    G.uses.record(fs, "plan fill");                // reads the generation's class table
  }
  const auto t_run = std::chrono::steady_clock::now();
  if (tr) S.host_ms[5] = ms_since(t_enq);
  S.h_verdict.get(std::max<size_t>(n, 1));
  if (grouped) {
    run_plan(d, K, G, &LN, &S.bufs, P, nullptr, false, &gf, true);
    s = gf.join;                                   // verdicts leave once every class is done
  } else {
    run_plan(d, K, G, &LN, &S.bufs, P, nullptr, false, nullptr, true, small ? (uint8_t*)S.h_verdict.dp : nullptr);
  }
  if (tr) S.host_ms[6] = ms_since(t_run);
  if (tr) HIPCHK(hipEventRecord(S.tr_c, s));
  if (!small) launch_copy(S.bufs.verdict.p, S.h_verdict.dp, n, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(S.done, s));
  if (tr) S.host_ms[2] = ms_since(t_enq);
  if (tr) S.grows = g_grows.load(std::memory_order_relaxed) - grows0;
  S.ticket = it.t;
  S.ks = it.ks;
  S.out = out;
  S.n = n;
}

// (Issuing the next chunk's arena DMA right after the current chunk's copies
// measured neutral on the configs[4] stream, 20.9-21.6 vs 21.0-21.2 ms at
// 262 k chunks, profiles/r04_s12/; not kept.)
void process_item(Device* d, size_t dslot, Item& it) {
  size_t enq = 0;
  const size_t nch = it.cuts.size() - 1;
  try {
    std::lock_guard<std::mutex> g(d->mu);
    HIPCHK(hipSetDevice(d->id));
    if (pipe_trace()) {
      if (!g_trace_ref) HIPCHK(hipEventCreate(&g_trace_ref));
      HIPCHK(hipEventRecord(g_trace_ref, d->copy));
    }
    auto take_slot = [&]() -> Slot* {
      Slot* Sp;
      if (it.zc) {
        Sp = &d->slots[NSLOT + d->next_zslot];
        d->next_zslot = (d->next_zslot + 1) % NZSLOT;
      } else {
        Sp = &d->slots[d->next_slot];
        d->next_slot = (d->next_slot + 1) % NSLOT;
      }
      const auto tw = std::chrono::steady_clock::now();
      {                               // the slot's previous chunk (a ring length ago) completed
        std::unique_lock<std::mutex> lk(d->cmu);
        d->scv.wait(lk, [&] { return !Sp->inflight; });
      }
      Sp->host_ms[0] = pipe_trace() ? ms_since(tw) : 0.0;
      return Sp;
    };
    auto plan = [&](Slot* S, size_t c, ChunkPlan& cp) {
      const size_t lo = it.cuts[c], hi = it.cuts[c + 1];
      plan_chunk(*S, it, it.toks + lo, hi - lo, lo, cp);
    };
    // Chunk c is issued on this thread while chunk c + 1 is planned on the
    // planner thread (its own slot): the host's per-chunk work is the longer
    // of the two rather than their sum (configs[4] stream: planning ~1.2 ms
    // and issuing ~2 ms per 262 k-job chunk, against ~3.2 ms of device work).
    ChunkPlan cp[2];
    int ci = 0;
    Slot* cur = take_slot();
    bool ok = true;
    try {
      plan(cur, 0, cp[0]);
    } catch (const BadJob& e) {                   // nothing of this chunk was enqueued
      it.t->fail(-1, e.what());
      ok = false;
    }
    for (size_t c = 0; ok && c < nch; ++c) {
      Slot* nxt = nullptr;
      std::exception_ptr nerr;
#ifndef JG_NO_PLANNER
#define JG_NO_PLANNER 0
#endif
      auto plan_next = [&, c] {
        try {
          plan(nxt, c + 1, cp[ci ^ 1]);
        } catch (...) {
          nerr = std::current_exception();
        }
      };
      if (c + 1 < nch) {
        nxt = take_slot();
        if (!JG_NO_PLANNER) d->planner->run(plan_next);
      }
      try {
        issue_chunk(d, dslot, *cur, it, cp[ci], it.out + it.cuts[c]);
      } catch (...) {
        if (nxt) d->planner->wait();
        throw;
      }
      cur->chunk_no = (int)enq;
      {
        std::lock_guard<std::mutex> lk(d->cmu);
        cur->inflight = true;
        d->cq.push_back(cur);
      }
      d->ccv.notify_one();
      ++enq;
      if (nxt) {
        if (JG_NO_PLANNER) plan_next();
        d->planner->wait();
        if (nerr) {
          try {
            std::rethrow_exception(nerr);
          } catch (const BadJob& e) {             // chunk c + 1 and later: not enqueued
            it.t->fail(-1, e.what());
            ok = false;
          }
        }
        cur = nxt;
        ci ^= 1;
      }
    }
    if (enq < nch) it.t->done_chunks(nch - enq);
  } catch (const std::exception& e) {
    it.t->fail(-2, e.what());
    it.t->done_chunks(nch - enq);
  }
}

// The device's submission thread: plans and enqueues each queued item's
// chunks.  Completion runs on a thread of its own (completer_loop), so a
// submission arriving while earlier chunks are on the device is enqueued at
// once rather than after the oldest chunk's event fires (small coalesced
// batches: the device works on several at a time).
void worker_loop(Device* d, size_t dslot) {
  pthread_setname_np(pthread_self(), "capjwt-submit");
  (void)hipSetDevice(d->id);
  std::unique_lock<std::mutex> lk(d->qmu);
  while (true) {
    if (!d->q.empty()) {
      Item it = std::move(d->q.front());
      d->q.pop_front();
      lk.unlock();
      process_item(d, dslot, it);
      lk.lock();
      continue;
    }
    if (d->stop) break;
    d->qcv.wait(lk, [&] { return d->stop || !d->q.empty(); });
  }
}

// Completes the device's in-flight chunks in enqueue order (both slot rings):
// waits for each chunk's verdict copy, hands the verdicts over, frees the slot.
void completer_loop(Device* d) {
  pthread_setname_np(pthread_self(), "capjwt-done");
  (void)hipSetDevice(d->id);
  std::unique_lock<std::mutex> lk(d->cmu);
  while (true) {
    d->ccv.wait(lk, [&] { return d->cstop || !d->cq.empty(); });
    if (d->cq.empty()) break;                    // stopping, nothing in flight
    Slot* S = d->cq.front();
    lk.unlock();
    finish_slot(*S);
    lk.lock();
    d->cq.pop_front();
    S->inflight = false;
    d->scv.notify_all();
  }
}


// ---------------------------------------------------------------- keys
struct StagedKeys {
  std::vector<DevKey> dk;
  std::vector<uint32_t> blob;       // host-initialised key blob (moduli, coordinates)
  std::vector<int32_t> rsa_idx, ec_idx[NCLS], ed_idx;
  std::vector<std::string> tab_id;  // per key: content id of its comb table ("" = none)
  std::vector<uint8_t> want_w;      // per key: comb width the table budget gives it (0 = none)
};

uint64_t blob_alloc(std::vector<uint32_t>& blob, size_t words) {
  const uint64_t off = (blob.size() + 3) & ~size_t(3);          // 16-byte aligned
  blob.resize(off + words, 0);
  return off;
}

// width tiers of a table class, widest first (ecdsa.hpp EC_*_WQ, ed25519.hpp ED_WA)
std::vector<int> width_tiers(int c) {
  switch (c) {
    case CLS_P256: return {std::begin(EC_P256_WQ), std::end(EC_P256_WQ)};
    case CLS_P384: return {std::begin(EC_P384_WQ), std::end(EC_P384_WQ)};
    case CLS_P521: return {std::begin(EC_P521_WQ), std::end(EC_P521_WQ)};
    case CLS_ED25519: return {std::begin(ED_WA), std::end(ED_WA)};
    default: return {};
  }
}
int narrow_w(int c) { return width_tiers(c).back(); }
uint64_t table_bytes(int c, int w) {
  return 4u * (uint64_t)(c == CLS_ED25519 ? ed_table_words_w(w) : ec_table_words_w(c, w));
}

// Key comb widths per class from ONE budget over every curve's key tables:
// each key starts at its class's narrowest width (always allowed, whatever the
// budget); then P-256, P-384, Ed25519 and P-521 in that order (ES256 first:
// BASELINE's headline) each take the widest tier whose extra bytes, for all
// of the class's keys, still fit what is left.
void key_widths(const int count[NCLS], uint64_t budget, int w[NCLS]) {
  uint64_t used = 0;
  for (int c = 0; c < NCLS; ++c) {
    w[c] = 0;
    if (c >= CLS_P256) {
      w[c] = narrow_w(c);
      used += (uint64_t)count[c] * table_bytes(c, w[c]);
    }
  }
  for (int c : {(int)CLS_P256, (int)CLS_P384, (int)CLS_ED25519, (int)CLS_P521}) {
    if (!count[c]) continue;
    for (int t : width_tiers(c)) {
      const uint64_t extra = (uint64_t)count[c] * (table_bytes(c, t) - table_bytes(c, narrow_w(c)));
      if (used + extra <= budget) {
        w[c] = t;
        used += extra;
        break;
      }
    }
  }
}

// The bytes of a key list (plus the budget, which decides table widths): a
// load whose content equals the current table's is a no-op.
std::string key_content(const jg_key* keys, int nkeys, uint64_t budget) {
  std::string s;
  auto put = [&](const void* p, size_t n) { s.append((const char*)p, n); };
  put(&budget, sizeof budget);
  for (int i = 0; i < nkeys; ++i) {
    const jg_key& k = keys[i];
    const uint8_t has = (k.n ? 1 : 0) | (k.x ? 2 : 0) | (k.y ? 4 : 0);
    put(&k.kind, 4); put(&k.curve, 4); put(&k.n_len, 4); put(&k.e, 8); put(&k.coord_len, 4); put(&has, 1);
    if (k.n && k.n_len > 0) put(k.n, (size_t)k.n_len);
    const size_t cl = k.coord_len > 0 ? (size_t)k.coord_len : 0;
    if (k.x) put(k.x, cl);
    if (k.y && k.kind == JG_KEY_EC) put(k.y, cl);
  }
  return s;
}

// Host part of a key load.  Touches no context state; `warn` collects
// informational messages for jg_last_error.
void build_keys(const jg_key* keys, int nkeys, uint64_t table_budget, StagedKeys& S, std::vector<HostKey>& hks,
                std::string* warn) {
  hks.assign((size_t)nkeys, HostKey{});
  S.dk.assign((size_t)nkeys, DevKey{});
  S.tab_id.assign((size_t)nkeys, std::string());
  S.want_w.assign((size_t)nkeys, 0);
  int count[NCLS] = {};
  for (int i = 0; i < nkeys; ++i) {
    const jg_key& k = keys[i];
    if (k.kind == JG_KEY_EC && k.curve >= JG_P256 && k.curve <= JG_P521) ++count[CLS_P256 + k.curve - JG_P256];
    if (k.kind == JG_KEY_ED25519) ++count[CLS_ED25519];
  }
  int wq[NCLS];
  key_widths(count, table_budget, wq);
  for (int i = 0; i < nkeys; ++i) {
    const jg_key& k = keys[i];
    HostKey& hk = hks[i];
    DevKey& K = S.dk[i];
    hk.kind = K.kind = k.kind;
    K.cls = CLS_REJECT;
    if (k.kind == JG_KEY_RSA) {
      const uint8_t* n = k.n;
      size_t nl = k.n_len > 0 && n ? (size_t)k.n_len : 0;
      while (nl > 0 && n[0] == 0) { ++n; --nl; }
      const int bits = bitlen_be(n, nl);
      // crypto/rsa (Go >= 1.24) public-key checks: odd N of >= 1024 bits
      // (rsa1024min), odd E with 2 <= E <= 2^31-1   [SURVEY R12]
      bool ok = nl > 0 && bits >= 1024 && (n[nl - 1] & 1) && k.e >= 2 && k.e <= 0x7fffffffULL && (k.e & 1);
      // layouts: RSA-2K (<= 2070 bits), RSA-3K (<= 3134), RSA-4K+ (148 / 296 /
      // 592 limbs: <= 4142 / 8286 / 16574 bits, rsa.hpp); Go has no upper bound
      const int cls = bits <= rsa_limbs(CLS_RSA2K) * 28 - 2 ? CLS_RSA2K : bits <= 112 * 28 - 2 ? CLS_RSA3K : CLS_RSA4K;
      int L = cls == CLS_RSA4K ? rsa4k_limbs_for_bits(bits) : rsa_limbs(cls);
      if (L == 0) {
        ok = false;
        *warn = "RSA key " + std::to_string(i) + " has " + std::to_string(bits) +
                " bits; the GPU path supports up to 16574-bit moduli (key marked unusable)";
        L = rsa4k_layout_limbs(0);
      }
      K.cls = cls;
      K.valid = ok;
      K.kbytes = (bits + 7) / 8;
      K.embits = bits - 1;
      K.e_lo = (uint32_t)k.e;
      K.e_hi = (uint32_t)(k.e >> 32);
      K.nlimbs = (uint32_t)L;
      // RSA-2K keys also serve the one-launch small path (k_rsa_small): n
      // zero-padded to its RSA_SMALL_L limbs and R'^2 mod n for R' = 2^(28 * 80)
      const int Ln = cls == CLS_RSA2K ? std::max(L, RSA_SMALL_L) : L;
      K.n_off = blob_alloc(S.blob, Ln);
      K.rr_off = blob_alloc(S.blob, L);
      K.rr2_off = 0;
      if (nl > 0) be_to_limbs(n, nl, S.blob.data() + K.n_off, Ln);
      // R^2 mod n (R = 2^(28 L)) and n' on the host: ~0.2 ms for an RSA-4096
      // key (host_mont.hpp; the device's 56 L modular doublings took ~200 ms
      // for the 32-kid bench set, profiles/r04_s1_keyload_trace.log)
      if (ok) hostmont::rsa_key_constants(S.blob.data() + K.n_off, L, S.blob.data() + K.rr_off, &K.np);
      if (ok && cls == CLS_RSA2K) {
        K.rr2_off = blob_alloc(S.blob, RSA_SMALL_L);
        uint32_t np2 = 0;
        hostmont::rsa_key_constants(S.blob.data() + K.n_off, RSA_SMALL_L, S.blob.data() + K.rr2_off, &np2);
      }
      if (ok) S.rsa_idx.push_back(i);
      hk.cls = cls;
      hk.valid = ok;
      hk.nlimbs = L;
    } else if (k.kind == JG_KEY_EC) {
      const int cls = k.curve == JG_P256 ? CLS_P256 : k.curve == JG_P384 ? CLS_P384 : k.curve == JG_P521 ? CLS_P521 : -1;
      if (cls < 0) { hk.valid = 0; continue; }
      const int L = ec_limbs(cls);
      const int cb = cls == CLS_P256 ? 32 : cls == CLS_P384 ? 48 : 66;
      K.cls = cls;
      K.kbytes = cb;
      K.aux_off = blob_alloc(S.blob, 2 * L);
      const size_t cl = k.coord_len > 0 ? (size_t)k.coord_len : 0;
      // crypto/ecdsa pointFromAffine: coordinates must fit the curve's bit size
      bool ok = k.x && k.y && cl > 0 && bitlen_be(k.x, cl) <= (cls == CLS_P521 ? 521 : cb * 8) &&
                bitlen_be(k.y, cl) <= (cls == CLS_P521 ? 521 : cb * 8);
      if (ok) {
        be_to_limbs(k.x, cl, S.blob.data() + K.aux_off, L);
        be_to_limbs(k.y, cl, S.blob.data() + K.aux_off + L, L);
        S.tab_id[i] = std::string("E") + (char)cls + std::string((const char*)S.blob.data() + 4 * K.aux_off, 8 * L);
        S.want_w[i] = (uint8_t)wq[cls];
      }
      K.valid = ok;
      if (ok) S.ec_idx[cls].push_back(i);
      hk.cls = cls;
      hk.valid = ok;              // on-curve check happens on the device
    } else if (k.kind == JG_KEY_ED25519) {
      K.cls = CLS_ED25519;
      K.kbytes = 32;
      K.aux_off = blob_alloc(S.blob, 8 + 2 * ED_L);
      // crypto/ed25519.Verify panics on len(pub) != 32; go-jose never hands it one
      const bool ok = k.x && k.coord_len == 32;
      if (ok) {
        std::memcpy(S.blob.data() + K.aux_off, k.x, 32);
        S.tab_id[i] = std::string("D") + std::string((const char*)k.x, 32);
        S.want_w[i] = (uint8_t)wq[CLS_ED25519];
      }
      K.valid = ok;
      if (ok) S.ed_idx.push_back(i);
      hk.cls = CLS_ED25519;
      hk.valid = ok;
    } else {
      hk.valid = 0;
    }
  }
  for (int c = CLS_P256; c <= CLS_P521; ++c)
    if ((int)S.ec_idx[c].size() > ec_max_keys(c))
      throw std::runtime_error(std::string(cls_name(c)) + ": at most " + std::to_string(ec_max_keys(c)) +
                               " keys per table");
  if ((int)S.ed_idx.size() > ED_MAX_KEYS)
    throw std::runtime_error("Ed25519: at most " + std::to_string(ED_MAX_KEYS) + " keys per table");
  blob_alloc(S.blob, 0);                                      // align the host part
}

// the process-wide table of (device, class), built on stream s and complete
// before any other context can see it
template <class Build>
std::shared_ptr<SharedTable> shared_table(Device* d, int cls, size_t bytes, hipStream_t s, Build&& build) {
  std::lock_guard<std::mutex> g(g_tab_mu);
  const auto key = std::make_pair(d->id, cls);
  if (auto t = g_tabs[key]) return t;
  auto t = std::make_shared<SharedTable>();
  HIPCHK(hipMalloc(&t->p, bytes));
  try {
    build(t->p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
  } catch (...) {
    (void)hipFree(t->p);          // a failed build is not cached
    throw;
  }
  g_tabs[key] = t;
  return t;
}

// Key comb tables by (key content id, width), per physical device: shared by
// every generation, context slot and context on that device.  A reload (JWKS
// refresh) reuses the tables of keys it already had (no copy, no build) and
// builds only new keys' tables; a second slot on the same GPU (Context([0, 0]))
// or a context recreated after a device error finds them built.
struct PhysTables {
  std::mutex mu;
  std::map<std::string, std::weak_ptr<DevBuf>> cache;
};
PhysTables& phys_tables(int dev) {
  static std::mutex m;
  static auto* all = new std::map<int, std::unique_ptr<PhysTables>>();   // never destroyed (static teardown)
  std::lock_guard<std::mutex> g(m);
  auto& p = (*all)[dev];
  if (!p) p = std::make_unique<PhysTables>();
  return *p;
}
DevBufP cached_table(int dev, const std::string& key) {
  PhysTables& T = phys_tables(dev);
  std::lock_guard<std::mutex> g(T.mu);
  auto it = T.cache.find(key);
  return it == T.cache.end() ? nullptr : it->second.lock();
}
void cache_table(int dev, const std::string& key, const DevBufP& t) {
  PhysTables& T = phys_tables(dev);
  std::lock_guard<std::mutex> g(T.mu);
  for (auto it = T.cache.begin(); it != T.cache.end();)
    it = it->second.expired() ? T.cache.erase(it) : std::next(it);
  T.cache[key] = t;
}

// fn(i) for every device slot i of ctx (§8(e): key loads and table widening on
// all GPUs at once, not one after another): one thread per physical device,
// the slots of one physical device in order on its thread (the second finds the
// first one's tables in phys_tables).  The first exception is re-thrown after
// every thread has finished.
template <class Fn>
void per_device(jg_ctx* ctx, Fn&& fn) {
  std::map<int, std::vector<size_t>> by_id;
  for (size_t i = 0; i < ctx->devs.size(); ++i) by_id[ctx->devs[i]->id].push_back(i);
  if (by_id.size() <= 1) {
    for (const auto& kv : by_id)
      for (size_t i : kv.second) fn(i);
    return;
  }
  std::vector<std::exception_ptr> err(by_id.size());
  std::vector<std::thread> th;
  size_t k = 0;
  for (const auto& kv : by_id) {
    th.emplace_back([&fn, &err, k, slots = kv.second] {
      try {
        for (size_t i : slots) fn(i);
      } catch (...) {
        err[k] = std::current_exception();
      }
    });
    ++k;
  }
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

void ensure_tables(Device* d, const StagedKeys& S) {
  HIPCHK(hipSetDevice(d->id));
  const hipStream_t s = d->kstream;
  for (int c = CLS_P256; c <= CLS_P521; ++c) {
    if (S.ec_idx[c].empty() || d->gtab[c]) continue;
    d->tab_ref[c] = shared_table(d, c, sizeof(uint32_t) * ec_table_words(c, true), s,
                                 [&](uint32_t* t) { launch_ec_gtable(c, t, s); });
    d->gtab[c] = d->tab_ref[c]->p;
  }
  if (!S.ed_idx.empty() && !d->btab) {
    d->tab_ref[CLS_ED25519] = shared_table(d, CLS_ED25519, sizeof(uint32_t) * ed_table_words(true), s,
                                           [&](uint32_t* t) { launch_ed_btable(t, s); });
    d->btab = d->tab_ref[CLS_ED25519]->p;
  }
}

// HBM kept free for chunk scratch when key tables are sized against free memory
constexpr uint64_t HBM_RESERVE = uint64_t(2) << 30;

uint64_t free_hbm(int dev) {
  size_t fr = 0, tot = 0;
  HIPCHK(hipSetDevice(dev));
  HIPCHK(hipMemGetInfo(&fr, &tot));
  return fr + reaper().pending(dev);      // released tables the reaper is about to free
}

// CAPJWT_POISON_TABLES=1 (debugging): fill every new key comb table with a
// byte pattern before its build, so an entry the build leaves unwritten cannot
// pass for a stale one
void poison_table(const DevBuf& t, hipStream_t s) {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_POISON_TABLES");
    return e && std::atoi(e) != 0;
  }();
  if (on) HIPCHK(hipMemsetAsync(t.p, 0xA5, t.bytes, s));
}

// jg_debug_table_digest: an order-sensitive 64-bit digest of n words
__global__ void k_digest(const uint32_t* __restrict__ t, uint64_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)t[i] * (2ull * i + 1ull) + (i ^ t[i]);
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}
void launch_digest(const uint32_t* t, uint64_t n, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_digest, dim3(4096), dim3(256), 0, s, t, n, out);
  HIPCHK(hipGetLastError());
}

// Launch the comb-table builds of keys (index list on the device at `didx`,
// grouped by class and width) on stream s.
void build_tables(const std::map<std::pair<int, int>, std::vector<int32_t>>& groups, DevKey* keys, uint32_t* blob,
                  int32_t* didx, hipStream_t s, bool sliced = false) {
  std::vector<int32_t> all;
  std::vector<std::pair<size_t, size_t>> span;
  for (const auto& g : groups) {
    span.emplace_back(all.size(), g.second.size());
    all.insert(all.end(), g.second.begin(), g.second.end());
  }
  if (all.empty()) return;
  HIPCHK(hipMemcpyAsync(didx, all.data(), sizeof(int32_t) * all.size(), hipMemcpyHostToDevice, s));
  size_t i = 0;
  for (const auto& g : groups) {
    const int c = g.first.first, w = g.first.second;
    int32_t* ix = didx + span[i].first;
    const int n = (int)span[i].second;
    if (c == CLS_ED25519) launch_ed_keytables(w, keys, blob, ix, n, s, sliced);
    else launch_ec_keytables(c, w, keys, blob, ix, n, s, sliced);
    ++i;
  }
  HIPCHK(hipGetLastError());
  // the index list is host memory that dies with the caller: wait here
  HIPCHK(hipStreamSynchronize(s));
}

// Stage a key load on one device, beside running verifications (its own
// stream; no drain): upload, key prep (R^2 / n', on-curve checks, Ed25519
// decoding), then a comb table per valid EC / Ed25519 key -- the table of the
// same key content and width when this device already has one (a JWKS
// refresh), else a new one.  With `narrow_first` a key that has no table at
// its budgeted width gets the widest table it already has, or a new table at
// the narrowest width (P-256: 436 MB, ~0.1 s), so it verifies at once; the
// upgrader builds the wide table later (jg_keys_wait_tables).  Throws on any
// failure; the device state and the published key table are then untouched.
std::shared_ptr<DevGen> stage_device(jg_ctx* ctx, Device* d, const StagedKeys& S, bool narrow_first) {
  HIPCHK(hipSetDevice(d->id));
  PhaseClock pc;
  const hipStream_t s = d->kstream;
  const size_t nk = S.dk.size();
  auto g = std::make_shared<DevGen>();
  g->mirror = S.dk;
  g->kw.assign(nk, 0);
  ensure_tables(d, S);
  pc.lap("fixed-base tables");
  g->dkeys = dev_alloc(d->id, sizeof(DevKey) * std::max<size_t>(nk, 1), &ctx->fail_alloc);
  g->blob = dev_alloc(d->id, sizeof(uint32_t) * std::max<size_t>(S.blob.size(), 4), &ctx->fail_alloc);
  // key prep index lists: p256 | p384 | p521 | ed
  std::vector<int32_t> idx;
  size_t at[4];
  for (int c = CLS_P256; c <= CLS_P521; ++c) {
    at[c - CLS_P256] = idx.size();
    idx.insert(idx.end(), S.ec_idx[c].begin(), S.ec_idx[c].end());
  }
  at[3] = idx.size();
  idx.insert(idx.end(), S.ed_idx.begin(), S.ed_idx.end());
  DevBufP didx = dev_alloc(d->id, sizeof(int32_t) * std::max<size_t>(idx.size() + nk, 1), &ctx->fail_alloc);
  int32_t* di = didx->as<int32_t>();
  DevKey* dk = g->keys();
  uint32_t* blob = g->keyblob();
  if (nk) HIPCHK(hipMemcpyAsync(dk, S.dk.data(), sizeof(DevKey) * nk, hipMemcpyHostToDevice, s));
  if (!S.blob.empty()) HIPCHK(hipMemcpyAsync(blob, S.blob.data(), sizeof(uint32_t) * S.blob.size(), hipMemcpyHostToDevice, s));
  if (!idx.empty()) HIPCHK(hipMemcpyAsync(di, idx.data(), sizeof(int32_t) * idx.size(), hipMemcpyHostToDevice, s));
  for (int c = CLS_P256; c <= CLS_P521; ++c)
    launch_ec_keyprep(c, dk, blob, di + at[c - CLS_P256], (int)S.ec_idx[c].size(), s);
  launch_ed_keyprep(dk, blob, di + at[3], (int)S.ed_idx.size(), s);
  HIPCHK(hipGetLastError());
  if (nk) HIPCHK(hipMemcpyAsync(g->mirror.data(), dk, sizeof(DevKey) * nk, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  pc.lap("records + key prep");

  // comb tables of the keys that prepped valid
  struct Req { int cls, w; DevBufP buf; std::string id; };
  std::map<std::string, Req> fresh;               // new tables by id + width
  std::vector<std::pair<size_t, std::string>> use;   // key -> id + width of its table
  {
    auto cached = [&](const std::string& id, int w) -> DevBufP { return cached_table(d->id, id + (char)w); };
    for (size_t i = 0; i < nk; ++i) {
      if (S.tab_id[i].empty() || !g->mirror[i].valid) continue;
      const int c = S.dk[i].cls, wt = S.want_w[i];
      int w = wt;
      DevBufP t = cached(S.tab_id[i], wt);
      if (!t && narrow_first)
        for (int ww : width_tiers(c))
          if (ww < wt && (t = cached(S.tab_id[i], ww))) { w = ww; break; }
      if (t) {
        g->mirror[i].tab = (uint64_t)(uintptr_t)t->p;
        g->mirror[i].tab_w = w;
        g->kw[i] = (uint8_t)w;
        g->tabs.push_back(std::move(t));
        continue;
      }
      if (narrow_first) w = narrow_w(c);
      const std::string key = S.tab_id[i] + (char)w;
      fresh.emplace(key, Req{c, w, nullptr, S.tab_id[i]});
      use.emplace_back(i, key);
    }
  }
  // size the new tables against free HBM (the previous generation stays live
  // until this one is published): narrow widths until they fit
  auto need = [&] {
    uint64_t b = 0;
    for (const auto& f : fresh) b += table_bytes(f.second.cls, f.second.w);
    return b;
  };
  const uint64_t fr = free_hbm(d->id);
  while (!fresh.empty() && need() + HBM_RESERVE > fr) {
    Req* widest = nullptr;
    for (auto& f : fresh)
      if (f.second.w > narrow_w(f.second.cls) && (!widest || table_bytes(f.second.cls, f.second.w) > table_bytes(widest->cls, widest->w)))
        widest = &f.second;
    if (!widest) {
      throw std::runtime_error("key comb tables need " + std::to_string(need() >> 20) + " MiB but only " +
                               std::to_string(fr >> 20) + " MiB of HBM is free on device " + std::to_string(d->id) +
                               " (the previous key table stays in force)");
    }
    const auto tiers = width_tiers(widest->cls);
    for (size_t t = 0; t + 1 < tiers.size(); ++t)
      if (tiers[t] == widest->w) { widest->w = tiers[t + 1]; break; }
  }
  std::map<std::pair<int, int>, std::vector<int32_t>> groups;
  std::map<std::string, int32_t> first;          // one build per distinct (id, width)
  pc.lap("table lookup + free HBM");
  for (auto& f : fresh) {
    f.second.buf = dev_alloc(d->id, table_bytes(f.second.cls, f.second.w), &ctx->fail_alloc);
    poison_table(*f.second.buf, s);
  }
  pc.lap("new table allocations");
  for (const auto& u : use) {
    const Req& r = fresh.at(u.second);
    const size_t i = u.first;
    g->mirror[i].tab = (uint64_t)(uintptr_t)r.buf->p;
    g->mirror[i].tab_w = r.w;
    g->kw[i] = (uint8_t)r.w;
    g->tabs.push_back(r.buf);
    if (first.emplace(u.second, (int32_t)i).second) groups[{r.cls, r.w}].push_back((int32_t)i);
  }
  if (nk) HIPCHK(hipMemcpyAsync(dk, g->mirror.data(), sizeof(DevKey) * nk, hipMemcpyHostToDevice, s));
  build_tables(groups, dk, blob, di, s);          // synchronises s
  ctx->tables_built.fetch_add(first.size());
  pc.lap("new comb tables (kernels)");
  for (const auto& f : fresh) cache_table(d->id, f.second.id + (char)f.second.w, f.second.buf);   // at its final width
  return g;
}

void upload_cls(jg_ctx* ctx, Device* d, DevGen& g, const std::vector<uint8_t>& cls_tab) {
  HIPCHK(hipSetDevice(d->id));
  g.dcls = dev_alloc(d->id, std::max<size_t>(cls_tab.size(), 16), &ctx->fail_alloc);
  if (!cls_tab.empty())
    HIPCHK(hipMemcpyAsync(g.dcls->p, cls_tab.data(), cls_tab.size(), hipMemcpyHostToDevice, d->kstream));
  HIPCHK(hipStreamSynchronize(d->kstream));
}

// CAPJWT_TABLES_SYNC=1: jg_keys_load builds every comb table at its budgeted
// width before returning (A/B of the narrow-first staging)
bool tables_sync() {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_TABLES_SYNC");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

bool needs_upgrade(const KeyState& K) {
  for (size_t k = 0; k < K.keys.size(); ++k)
    if (K.keys[k].valid && !K.tab_id[k].empty() && K.want_w[k] > K.dev[0]->kw[k]) return true;
  return false;
}

// One step of the background upgrader: build the budgeted-width table of ONE
// key that runs on a narrower one, on every device (the upgrade stream, beside
// verification), then publish a generation whose records point at it.  The
// key list is unchanged, so staged batches and queued work stay valid.
// Returns false when nothing is left to widen.
bool upgrade_one(jg_ctx* ctx, std::set<std::string>& skip) {
  KeyStateP cur = ctx->state();
  if (!cur || cur->dev.empty()) return false;
  size_t k = 0;
  for (; k < cur->keys.size(); ++k)
    if (cur->keys[k].valid && !cur->tab_id[k].empty() && cur->want_w[k] > cur->dev[0]->kw[k] &&
        !skip.count(cur->tab_id[k] + (char)cur->want_w[k]))
      break;
  if (k == cur->keys.size()) return false;
  const std::string key = cur->tab_id[k] + (char)cur->want_w[k];
  const int cls = cur->keys[k].cls, w = cur->want_w[k];
  std::vector<DevBufP> built(ctx->devs.size());
  std::mutex nofit_mu;
  std::string nofit;              // a device where the wide table does not fit free HBM
  per_device(ctx, [&](size_t i) {
    Device* d = ctx->devs[i].get();
    if ((built[i] = cached_table(d->id, key))) return;
    {
      std::lock_guard<std::mutex> g(nofit_mu);
      if (!nofit.empty()) return;
    }
    if (table_bytes(cls, w) + HBM_RESERVE > free_hbm(d->id)) {
      std::lock_guard<std::mutex> g(nofit_mu);
      nofit = "a " + std::to_string(table_bytes(cls, w) >> 20) + " MiB comb table (W = " + std::to_string(w) +
              ") does not fit free HBM on device " + std::to_string(d->id) + "; key " + std::to_string(k) +
              " keeps its narrower table";
      return;
    }
    HIPCHK(hipSetDevice(d->id));
    const DevGen& G = *cur->dev[i];
    DevBufP t = dev_alloc(d->id, table_bytes(cls, w));
    poison_table(*t, d->ustream);
    // a one-record key array pointing at the new table (the blob is the generation's)
    DevKey rec = G.mirror[k];
    rec.tab = (uint64_t)(uintptr_t)t->p;
    rec.tab_w = w;
    DevBufP tmp = dev_alloc(d->id, sizeof(DevKey) + 16);
    const int32_t zero = 0;
    HIPCHK(hipMemcpyAsync(tmp->p, &rec, sizeof(DevKey), hipMemcpyHostToDevice, d->ustream));
    HIPCHK(hipMemcpyAsync((char*)tmp->p + sizeof(DevKey), &zero, sizeof zero, hipMemcpyHostToDevice, d->ustream));
    std::map<std::pair<int, int>, std::vector<int32_t>> groups;
    groups[{cls, w}].push_back(0);
    // sliced: the upgrade stream may share a hardware queue with a verify
    // lane, which then waits at most one slice behind it (tables.hpp)
    build_tables(groups, tmp->as<DevKey>(), G.keyblob(), (int32_t*)((char*)tmp->p + sizeof(DevKey)), d->ustream, true);
    ctx->tables_built.fetch_add(1);
    cache_table(d->id, key, t);
    built[i] = t;
  });
  if (!nofit.empty()) {
    skip.insert(key);
    std::lock_guard<std::mutex> g(ctx->up_mu);
    ctx->up_warn = nofit;
    return true;
  }
  // publish against whatever state is current now (a load may have replaced
  // the one the build started from: every key with this content gets the table)
  std::lock_guard<std::mutex> lg(ctx->load_mu);
  KeyStateP now = ctx->state();
  auto ns = std::make_shared<KeyState>(*now);
  bool any = false;
  for (size_t i = 0; i < ctx->devs.size() && i < ns->dev.size(); ++i) {
    Device* d = ctx->devs[i].get();
    auto g = std::make_shared<DevGen>(*ns->dev[i]);
    bool hit = false;
    for (size_t j = 0; j < ns->keys.size(); ++j) {
      if (ns->tab_id[j] + (char)w != key || ns->want_w[j] != w || g->kw[j] >= w || !ns->keys[j].valid) continue;
      g->mirror[j].tab = (uint64_t)(uintptr_t)built[i]->p;
      g->mirror[j].tab_w = w;
      g->kw[j] = (uint8_t)w;
      hit = true;
    }
    if (!hit) continue;
    any = true;
    g->tabs.push_back(built[i]);
    g->dkeys = dev_alloc(d->id, sizeof(DevKey) * std::max<size_t>(g->mirror.size(), 1));
    if (!g->mirror.empty())
      HIPCHK(hipMemcpyAsync(g->dkeys->p, g->mirror.data(), sizeof(DevKey) * g->mirror.size(), hipMemcpyHostToDevice,
                            d->ustream));
    HIPCHK(hipStreamSynchronize(d->ustream));
    ns->dev[i] = g;
  }
  if (any) ctx->publish(ns);
  return true;
}

void upgrade_loop(jg_ctx* ctx) {
  pthread_setname_np(pthread_self(), "capjwt-widen");
  std::set<std::string> skip;     // tables that did not fit (retried after the next key load)
  std::unique_lock<std::mutex> lk(ctx->up_mu);
  while (true) {
    ctx->up_cv.wait(lk, [&] { return ctx->up_stop || ctx->up_pending; });
    if (ctx->up_stop) break;
    ctx->up_pending = false;
    ctx->up_busy = true;
    skip.clear();
    lk.unlock();
    try {
      // jg_debug_max_upgrades (testing): stop after n table upgrades, leaving
      // the rest of the keys on their narrow tables -- a deterministic
      // stand-in for the window in which a class runs mixed widths
      while (ctx->upgrades_left.load() != 0 && upgrade_one(ctx, skip)) {
        int left = ctx->upgrades_left.load();
        while (left > 0 && !ctx->upgrades_left.compare_exchange_weak(left, left - 1)) {}
        std::lock_guard<std::mutex> g(ctx->up_mu);
        if (ctx->up_stop) break;
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(ctx->up_mu);
      ctx->up_warn = std::string("comb table upgrade failed (keys keep their narrower tables): ") + e.what();
    }
    lk.lock();
    ctx->up_busy = false;
    ctx->up_idle_cv.notify_all();
  }
}

thread_local std::string g_tls_err;


// Split jobs [0, ntok) over the context's devices by the cost model and queue
// each device's share, every item running against the key state `ks`.
std::shared_ptr<Ticket> submit_to(jg_ctx* ctx, const KeyStateP& ks, const uint8_t* arena, size_t arena_len,
                                  const jg_tok* toks, size_t ntok, uint8_t* out) {
  auto t = std::make_shared<Ticket>();
  const size_t nd = ctx->devs.size();
  std::vector<size_t> cut(nd + 1, 0);
  cut[nd] = ntok;
  if (nd > 1 && ntok <= SMALL_SUBMIT) {
    // a small submission (coalesced single-token calls) goes whole to one
    // device slot, round robin: split, it would pay one full chain latency on
    // each of several devices and hold each device's submission thread, which
    // is what bounds small-batch throughput (~15 k batches/s per slot: the
    // ~15 HIP calls of a chunk, profiles/r06_s6/single_probe.log)
    const size_t k = (size_t)(ctx->small_rr.fetch_add(1) % nd);
    for (size_t j = 0; j <= nd; ++j) cut[j] = j > k ? ntok : 0;
  } else if (nd > 1) {
    std::vector<double> pre(ntok + 1, 0.0);
    const size_t nk = ks->keys.size();
    for (size_t i = 0; i < ntok; ++i) {
      double w = 0.0;
      if (toks[i].key_idx < nk) {
        const int c = classify(*ks, toks[i]);
        w = CLS_COST[c];
        if (c == CLS_RSA4K) {
          const double r = ks->keys[toks[i].key_idx].nlimbs / 148.0;
          w *= r * r;
        }
      }
      pre[i + 1] = pre[i] + w;
    }
    size_t j = 0;
    for (size_t k = 1; k < nd; ++k) {
      const double target = pre[ntok] * (double)k / (double)nd;
      while (j < ntok && pre[j] < target) ++j;
      cut[k] = j;
    }
  }
  const uint8_t* dview = device_view(arena);
  const bool zc_ok = ctx->zc.load() && dview && zc_arena_ok(arena, arena_len);
  const size_t zmax = ctx->zc_max.load();
  const size_t C = ctx->chunk.load();
  std::vector<Item> items;
  for (size_t k = 0; k < nd; ++k) {
    if (cut[k + 1] <= cut[k]) continue;
    Item it;
    it.t = t;
    it.arena = arena;
    it.arena_len = arena_len;
    it.toks = toks;
    it.lo = cut[k];
    it.hi = cut[k + 1];
    it.out = out;
    it.ks = ks;
    it.dev_arena = dview;
    it.chunk = C;
    it.grouped = mixed_classes(*ks, toks + it.lo, it.hi - it.lo);
    it.small_ec = ctx->small_ec.load();
    it.small_launches = &ctx->small_launches;
    // grouped chunks serialise each class group's launches on one lane, so a
    // long ramp of small chunks would queue latency-bound launches (an
    // RSA-4096 modexp takes ~1.5 ms at any size): start at C / 4
    it.zc = zc_ok && it.grouped;
    if (it.zc) {
      // whole item as one plan (or equal plans of at most zc_max_jobs)
      const size_t n = it.hi - it.lo, parts = (n + zmax - 1) / zmax;
      it.cuts.clear();
      for (size_t k = 0; k <= parts; ++k) it.cuts.push_back(it.lo + n * k / parts);
      it.chunk = (n + parts - 1) / parts;
    } else {
      // (a ramp from C / 2 or from C itself measured slower on the configs[4]
      // stream: 58.4 / 56.7 vs 62-63 M/s, profiles/r05_s2/session_g.log)
      it.cuts = chunk_cuts(it.lo, it.hi, C, it.grouped ? std::max<size_t>(4096, C / 4) : 4096, !it.grouped);
    }
    it.nchunks = it.cuts.size() - 1;
    t->pending += it.nchunks;
    items.push_back(std::move(it));
  }
  for (size_t k = 0, i = 0; k < nd && i < items.size(); ++k) {
    if (cut[k + 1] <= cut[k]) continue;
    Device* d = ctx->devs[k].get();
    Item& it = items[i++];
    // A small submission (coalesced single-token calls) on a device with
    // nothing queued is planned and issued on the calling thread: one thread
    // hand-off fewer on its round trip (the submission thread's wake-up).
    // The device mutex still orders it against the submission thread.
    if (it.nchunks == 1 && it.hi - it.lo <= SMALL_SUBMIT) {
      bool idle;
      {
        std::lock_guard<std::mutex> g(d->qmu);
        idle = d->q.empty();
      }
      if (idle) {
        process_item(d, k, it);
        continue;
      }
    }
    {
      std::lock_guard<std::mutex> g(d->qmu);
      d->q.push_back(std::move(it));
    }
    d->qcv.notify_one();
  }
  return t;
}

int wait_ticket(jg_ctx* ctx, const std::shared_ptr<Ticket>& t) {
  std::unique_lock<std::mutex> lk(t->m);
  t->cv.wait(lk, [&] { return t->pending == 0; });
  if (t->rc) ctx->set_err(t->err);
  return t->rc;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

jg_ctx* jg_create(const int* devices, int ndev) {
  try {
    auto ctx = std::make_unique<jg_ctx>();
    int count = 0;
    HIPCHK(hipGetDeviceCount(&count));
    if (count <= 0) throw std::runtime_error("no HIP device");
    std::vector<int> ids;
    if (!devices || ndev <= 0) ids.push_back(0);
    else ids.assign(devices, devices + ndev);
    for (int id : ids) {
      if (id < 0 || id >= count) throw std::runtime_error("bad device id " + std::to_string(id));
      auto d = std::make_unique<Device>();
      d->id = id;
      HIPCHK(hipSetDevice(id));
      HIPCHK(hipStreamCreateWithFlags(&d->copy, hipStreamNonBlocking));
      for (auto& l : d->lanes) l.create_main();
      d->lane0.create_main();
      d->lane1.create_main();
      // (pipeline lanes run class-grouped on the lanes themselves: no fan-out)
      d->lane0.create_fanout(RES_GROUP, RES_NGROUPS);
      d->lane1.create_fanout(RES_GROUP, RES_NGROUPS);
      for (auto& s : d->slots) {
        // (hipEventBlockingSync here left the completer thread's CPU time and
        // a small batch's round trip unchanged, profiles/r05_s2/session_k.log)
        HIPCHK(hipEventCreateWithFlags(&s.done, pipe_trace() ? hipEventDefault : hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
        HIPCHK(hipEventCreate(&s.tr_a));
        HIPCHK(hipEventCreate(&s.tr_b));
        HIPCHK(hipEventCreate(&s.tr_c));
        HIPCHK(hipEventCreateWithFlags(&s.ev_planned, hipEventDisableTiming));
        for (auto& e : s.ev_cls) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (auto& e : s.ev_fed) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
      HIPCHK(hipStreamCreateWithFlags(&d->kstream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&d->ustream, hipStreamNonBlocking));
      ctx->devs.push_back(std::move(d));
    }
    auto ks = std::make_shared<KeyState>();        // no keys yet: every job is out of range
    for (size_t i = 0; i < ctx->devs.size(); ++i) ks->dev.push_back(std::make_shared<DevGen>());
    ctx->ks = ks;
    jg_ctx* c = ctx.release();
    for (size_t i = 0; i < c->devs.size(); ++i) {
      c->devs[i]->planner = std::make_unique<Helper>(c->devs[i]->id);
      c->devs[i]->worker = std::thread(worker_loop, c->devs[i].get(), i);
      c->devs[i]->completer = std::thread(completer_loop, c->devs[i].get());
    }
    c->upgrader = std::thread(upgrade_loop, c);
    return c;
  } catch (const std::exception& e) {
    g_tls_err = e.what();
    return nullptr;
  }
}

void jg_destroy(jg_ctx* ctx) {
  if (!ctx) return;
  {
    std::lock_guard<std::mutex> g(ctx->up_mu);
    ctx->up_stop = true;
  }
  ctx->up_cv.notify_all();
  if (ctx->upgrader.joinable()) ctx->upgrader.join();
  for (auto& d : ctx->devs) {
    {
      std::lock_guard<std::mutex> g(d->qmu);
      d->stop = true;
    }
    d->qcv.notify_all();
    if (d->worker.joinable()) d->worker.join();
    {
      std::lock_guard<std::mutex> g(d->cmu);
      d->cstop = true;
    }
    d->ccv.notify_all();
    if (d->completer.joinable()) d->completer.join();
    d->planner.reset();
  }
  ctx->publish(nullptr);                           // key generations: handed to the reaper
  reaper().drain();                                // ... and freed before jg_destroy returns
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d->id);
    for (auto& l : d->lanes) l.destroy();
    for (auto& s : d->slots) {
      if (s.done) (void)hipEventDestroy(s.done);
      for (hipEvent_t e : s.ev_cls)
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : s.ev_fed)
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : {s.tr_a, s.tr_b, s.tr_c, s.copied, s.ev_planned})
        if (e) (void)hipEventDestroy(e);
    }
    d->lane0.sync();
    d->lane1.sync();
    if (d->copy) {
      (void)hipStreamSynchronize(d->copy);
      (void)hipStreamDestroy(d->copy);
    }
    for (hipStream_t* st : {&d->kstream, &d->ustream})
      if (*st) {
        (void)hipStreamSynchronize(*st);
        (void)hipStreamDestroy(*st);
        *st = nullptr;
      }
    // this context's hold on the fixed-base tables; the process cache (g_tabs)
    // keeps them for later contexts unless CAPJWT_RELEASE_GTABLES=1
    for (auto& t : d->tab_ref) t.reset();
    if (release_gtables()) {
      std::lock_guard<std::mutex> g(g_tab_mu);
      for (auto it = g_tabs.begin(); it != g_tabs.end();) {
        if (it->first.first == d->id && it->second && it->second.use_count() == 1) {
          (void)hipFree(it->second->p);
          it = g_tabs.erase(it);
        } else {
          ++it;
        }
      }
    }
    d->lane0.destroy();
    d->lane1.destroy();
  }
  delete ctx;
}

int jg_keys_load(jg_ctx* ctx, const jg_key* keys, int nkeys) {
  if (!ctx || nkeys < 0 || (nkeys > 0 && !keys)) return -1;
  if (nkeys > 65535) { ctx->set_err("at most 65535 keys"); return -1; }
  try {
    std::lock_guard<std::mutex> lg(ctx->load_mu);
    PhaseClock pc;
    std::string content = key_content(keys, nkeys, ctx->table_budget.load());
    KeyStateP cur = ctx->state();
    if (cur && cur->epoch > 0 && cur->content == content) return 0;   // unchanged key set: no device work
    StagedKeys S;
    auto ns = std::make_shared<KeyState>();
    std::string warn;
    build_keys(keys, nkeys, ctx->table_budget.load(), S, ns->keys, &warn);   // throws before any device work
    pc.lap("host key staging");
    // stage on every device beside running work; any failure throws and
    // leaves the published table (and what verifies against it) untouched
    std::vector<std::shared_ptr<DevGen>> gens(ctx->devs.size());
    per_device(ctx, [&](size_t i) { gens[i] = stage_device(ctx, ctx->devs[i].get(), S, !tables_sync()); });
    pc.lap("device staging (all devices)");
    // device-side validity (on-curve, Ed25519 decoding) back into the host view
    for (size_t i = 0; i < ns->keys.size(); ++i) ns->keys[i].valid = ns->keys[i].valid && gens[0]->mirror[i].valid;
    rebuild_class_tables(*ns);
    per_device(ctx, [&](size_t i) { upload_cls(ctx, ctx->devs[i].get(), *gens[i], ns->cls_tab); });
    pc.lap("class tables");
    ns->tab_id = std::move(S.tab_id);
    ns->want_w = std::move(S.want_w);
    ns->epoch = (cur ? cur->epoch : 0) + 1;
    ns->content = std::move(content);
    for (auto& g : gens) ns->dev.push_back(std::move(g));
    const bool up = needs_upgrade(*ns);
    ctx->publish(std::move(ns));
    pc.lap("publish (old state released)");
    if (up) {
      std::lock_guard<std::mutex> g(ctx->up_mu);
      ctx->up_pending = true;
      ctx->up_cv.notify_all();
    }
    if (!warn.empty()) ctx->set_err(warn);
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_keys_wait_tables(jg_ctx* ctx) {
  if (!ctx) return -1;
  std::unique_lock<std::mutex> lk(ctx->up_mu);
  ctx->up_idle_cv.wait(lk, [&] { return !ctx->up_pending && !ctx->up_busy; });
  if (!ctx->up_warn.empty()) {
    const std::string w = std::move(ctx->up_warn);
    ctx->up_warn.clear();
    lk.unlock();
    ctx->set_err(w);
    return 1;
  }
  return 0;
}

int jg_keys_table_widths(jg_ctx* ctx, int* widths, int cap) {
  if (!ctx || cap < 0 || (cap > 0 && !widths)) return -1;
  KeyStateP ks = ctx->state();
  const int n = (int)ks->keys.size();
  for (int i = 0; i < n && i < cap; ++i) widths[i] = ks->dev.empty() || ks->dev[0]->kw.empty() ? 0 : ks->dev[0]->kw[(size_t)i];
  return n;
}

int jg_debug_table_digest(jg_ctx* ctx, int key, uint64_t* digest) {
  if (!ctx || !digest || key < 0) return -1;
  try {
    KeyStateP ks = ctx->state();
    if (!ks || key >= (int)ks->keys.size() || ks->dev.empty()) return -1;
    const DevGen& G = *ks->dev[0];
    const int w = G.kw[(size_t)key];
    if (w == 0 || G.mirror[(size_t)key].tab == 0) { *digest = 0; return 0; }
    Device* d = ctx->devs[0].get();
    HIPCHK(hipSetDevice(d->id));
    const uint64_t bytes = table_bytes(ks->keys[(size_t)key].cls, w);
    DevBufP out = dev_alloc(d->id, sizeof(unsigned long long));
    HIPCHK(hipMemsetAsync(out->p, 0, sizeof(unsigned long long), d->kstream));
    launch_digest((const uint32_t*)(uintptr_t)G.mirror[(size_t)key].tab, bytes / 4, out->as<unsigned long long>(),
                  d->kstream);
    HIPCHK(hipMemcpyAsync(digest, out->p, sizeof(uint64_t), hipMemcpyDeviceToHost, d->kstream));
    HIPCHK(hipStreamSynchronize(d->kstream));
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_debug_tables_built(jg_ctx* ctx, uint64_t* built) {
  if (!ctx || !built) return -1;
  *built = ctx->tables_built.load();
  return 0;
}

int jg_debug_small_path(jg_ctx* ctx, int enable, uint64_t* launches) {
  if (!ctx || enable < -1 || enable > 1) return -1;
  if (enable >= 0) ctx->small_ec.store(enable != 0);
  if (launches) *launches = ctx->small_launches.load();
  return 0;
}

int jg_debug_fail_alloc(jg_ctx* ctx, int n) {
  if (!ctx || n < 0) return -1;
  ctx->fail_alloc.store(n);
  return 0;
}

int jg_debug_fail_verify(jg_ctx* ctx, int n) {
  if (!ctx || n < 0) return -1;
  ctx->fail_verify.store(n);
  return 0;
}

int jg_debug_lifetime_check(int enable, uint64_t* violations, uint64_t* checked) {
  if (enable > 0) g_lifetime_on.store(1);
  else if (enable == 0) g_lifetime_on.store(0);
  if (violations) *violations = g_lifetime_bad.load();
  if (checked) *checked = g_lifetime_checked.load();
  return 0;
}

int jg_debug_max_upgrades(jg_ctx* ctx, int n) {
  if (!ctx || n < -1) return -1;
  ctx->upgrades_left.store(n);
  KeyStateP cur = ctx->state();
  if (n != 0 && cur && !cur->dev.empty() && needs_upgrade(*cur)) {   // resume widening
    std::lock_guard<std::mutex> g(ctx->up_mu);
    ctx->up_pending = true;
    ctx->up_cv.notify_all();
  }
  return 0;
}

int jg_submit(jg_ctx* ctx, const uint8_t* arena, size_t arena_len, const jg_tok* toks, size_t ntok,
              uint8_t* verdict_out, jg_ticket** out) {
  if (!ctx || !out || (ntok > 0 && (!toks || !arena || !verdict_out))) return -1;
  *out = nullptr;
  if (ntok > (size_t)INT32_MAX / 2) { ctx->set_err("batch too large"); return -1; }
  try {
    if (ctx->poisoned.load()) {
      ctx->set_err("context unusable after an injected device failure (jg_debug_fail_verify): recreate it");
      return -2;
    }
    if (ctx->fail_verify.load() > 0 && ctx->fail_verify.fetch_sub(1) == 1) {
      // the injected failure surfaces where a kernel fault would: in jg_wait
      ctx->poisoned.store(true);
      auto t = std::make_shared<Ticket>();
      t->fail(-2, "injected device failure (jg_debug_fail_verify)");
      *out = new jg_ticket{std::move(t)};
      return 0;
    }
    if (ntok == 0) {                       // nothing to verify
      *out = new jg_ticket{std::make_shared<Ticket>()};
      return 0;
    }
    // jobs are validated chunk by chunk by the device workers, ahead of each
    // chunk's upload (a bad job fails the ticket with -1 from jg_wait; jg.h)
    auto t = submit_to(ctx, ctx->state(), arena, arena_len, toks, ntok, verdict_out);
    *out = new jg_ticket{std::move(t)};
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_wait(jg_ctx* ctx, jg_ticket* t) {
  if (!ctx || !t) return -1;
  const int rc = wait_ticket(ctx, t->t);
  delete t;
  return rc;
}

int jg_set_chunk(jg_ctx* ctx, size_t jobs) {
  if (!ctx || jobs < 64) return -1;
  ctx->chunk.store(jobs);
  return 0;
}

int jg_set_zero_copy(jg_ctx* ctx, int enable, size_t max_jobs) {
  if (!ctx || (max_jobs != 0 && max_jobs < 64)) return -1;
  ctx->zc.store(enable != 0);
  if (max_jobs) ctx->zc_max.store(max_jobs);
  return 0;
}

int jg_set_table_budget(jg_ctx* ctx, uint64_t bytes) {
  if (!ctx) return -1;
  ctx->table_budget.store(bytes);
  return 0;
}

int jg_verify_batch(jg_ctx* ctx, const uint8_t* arena, size_t arena_len,
                    const jg_tok* toks, size_t ntok, uint8_t* verdict_out) {
  jg_ticket* t = nullptr;
  const int rc = jg_submit(ctx, arena, arena_len, toks, ntok, verdict_out, &t);
  if (rc != 0) return rc;
  return jg_wait(ctx, t);
}

int jg_batch_stage(jg_ctx* ctx, int device_slot, const uint8_t* arena, size_t arena_len,
                   const jg_tok* toks, size_t ntok, jg_batch** out) {
  if (!ctx || !out || (ntok > 0 && (!toks || !arena))) return -1;
  if (device_slot < 0 || device_slot >= (int)ctx->devs.size()) return -1;
  if (ntok > (size_t)INT32_MAX / 2) { ctx->set_err("batch too large"); return -1; }
  try {
    KeyStateP ks = ctx->state();
    std::string err;
    if (!check_jobs(*ks, arena_len, toks, ntok, &err)) { ctx->set_err(err); return -1; }
    auto b = std::make_unique<jg_batch>();
    b->ctx = ctx;
    b->dslot = (size_t)device_slot;
    b->dev = ctx->devs[device_slot].get();
    b->own = std::make_unique<Bufs>();
    b->b = b->own.get();
    std::lock_guard<std::mutex> g(b->dev->mu);
    b->lane = (b->dev->next_res++ & 1) ? &b->dev->lane1 : &b->dev->lane0;
    HIPCHK(hipSetDevice(b->dev->id));
    PlanScratch X;
    if (arena_len >= (uint64_t(1) << 32) - ARENA_SLACK) {
      ctx->set_err("a resident batch's arena must be smaller than 4 GiB");
      return -1;
    }
    std::vector<JobDev> jobs;
    std::vector<int32_t> perm;
    plan_layout(*ks, toks, ntok, b->plan, X, true);
    jobs.resize(b->plan.npad);
    perm.resize(b->plan.npad);
    plan_fill_host(*ks, toks, ntok, b->plan, X, jobs.data(), perm.data());
    upload(b->b, b->lane->stream, b->plan, arena, arena_len, jobs.data(), perm.data());
    // the host vectors die here: the copies above must complete first
    HIPCHK(hipStreamSynchronize(b->lane->stream));
    b->arena_len = arena_len;
    b->epoch = ks->epoch;
    *out = b.release();
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

namespace {
// A resident batch runs against the current key state when its key list is
// the one it was planned for (a comb-width upgrade since staging is fine: the
// run picks up the wider tables); a reload with another key list invalidates it.
// (One stream per class on the batch's lane: running mixed resident batches
// on the pipeline's three group lanes measured 80.0-80.2 against 81.6-82.3
// M/s on configs[4], profiles/r04_s14.)
void run_resident(jg_ctx* ctx, jg_batch* b, bool timed) {
  HIPCHK(hipSetDevice(b->dev->id));
  KeyStateP ks = ctx->state();
  if (b->epoch != ks->epoch) throw std::runtime_error("key table reloaded since this batch was staged");
  b->timing = timed;
  b->marks_used = 0;
  run_plan(b->dev, *ks, *ks->dev[b->dslot], b->lane, b->b, b->plan, b);
  if (b->ks_run && b->ks_run != ks) HIPCHK(hipStreamSynchronize(b->lane->stream));   // its kernels may read the old state
  b->ks_run = std::move(ks);
}
}  // namespace

int jg_batch_run(jg_ctx* ctx, jg_batch* b, uint8_t* verdict_out) {
  if (!ctx || !b) return -1;
  try {
    std::lock_guard<std::mutex> g(b->dev->mu);
    run_resident(ctx, b, true);
    if (verdict_out) {
      if (b->plan.ntok > 0)
        HIPCHK(hipMemcpyAsync(verdict_out, b->b->verdict.p, (size_t)b->plan.ntok, hipMemcpyDeviceToHost,
                              b->lane->stream));
      HIPCHK(hipStreamSynchronize(b->lane->stream));
      collect_times(b);
    }
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_batch_enqueue(jg_ctx* ctx, jg_batch* b, uint8_t* verdict_out) {
  if (!ctx || !b) return -1;
  try {
    std::lock_guard<std::mutex> g(b->dev->mu);
    run_resident(ctx, b, false);
    if (verdict_out && b->plan.ntok > 0)
      HIPCHK(hipMemcpyAsync(verdict_out, b->b->verdict.p, (size_t)b->plan.ntok, hipMemcpyDeviceToHost,
                            b->lane->stream));
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_batch_sync(jg_ctx* ctx, jg_batch* b) {
  if (!ctx || !b) return -1;
  try {
    HIPCHK(hipSetDevice(b->dev->id));
    HIPCHK(hipStreamSynchronize(b->lane->stream));
    collect_times(b);
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

void jg_batch_free(jg_ctx* ctx, jg_batch* b) {
  (void)ctx;
  if (!b) return;
  (void)hipSetDevice(b->dev->id);
  (void)hipStreamSynchronize(b->lane->stream);
  delete b;
}

int jg_batch_kernel_times(jg_batch* b, const char** names, float* ms, int cap) {
  if (!b) return 0;
  const int n = (int)b->tms.size();
  for (int i = 0; i < n && i < cap; ++i) {
    if (names) names[i] = b->tnames[i].c_str();
    if (ms) ms[i] = b->tms[i];
  }
  return n;
}

int jg_batch_exceptions(jg_batch* b, uint32_t* counts, int cap) {
  if (!b || !counts || cap < 0) return -1;
  try {
    HIPCHK(hipSetDevice(b->dev->id));
    uint32_t c[NCLS] = {};
    if (b->b->exc_cnt.p) {
      HIPCHK(hipMemcpyAsync(c, b->b->exc_cnt.p, sizeof(c), hipMemcpyDeviceToHost, b->lane->stream));
      HIPCHK(hipStreamSynchronize(b->lane->stream));
    }
    for (int k = 0; k < cap && k < NCLS; ++k) {
      // a class's counter is only meaningful when the batch has work of that class
      const bool act = b->plan.ranges[k].end > b->plan.ranges[k].begin && k >= CLS_P256 && k <= CLS_P521;
      counts[k] = act ? c[k] : 0u;
    }
    return NCLS;
  } catch (const std::exception& e) {
    b->ctx->set_err(e.what());
    return -2;
  }
}

int jg_hash_batch(jg_ctx* ctx, const uint8_t* arena, size_t arena_len,
                  const jg_hjob* jobs, size_t njobs, uint8_t* digest_out) {
  if (!ctx || (njobs > 0 && (!jobs || !digest_out)) || (arena_len > 0 && !arena)) return -1;
  if (njobs == 0) return 0;
  if (ctx->poisoned.load()) {
    ctx->set_err("context unusable after an injected device failure (jg_debug_fail_verify): recreate it");
    return -2;
  }
  for (size_t i = 0; i < njobs; ++i) {
    const jg_hjob& J = jobs[i];
    if (J.fam < JG_SHA256 || J.fam > JG_SHA512 || J.off > arena_len || J.len > arena_len - J.off) {
      ctx->set_err("jg_hash_batch: job " + std::to_string(i) + " has an unknown hash or a span past the arena");
      return -1;
    }
  }
  try {
    Device* d = ctx->devs[0].get();
    std::lock_guard<std::mutex> g(d->mu);
    HIPCHK(hipSetDevice(d->id));
    const hipStream_t s = d->lane0.stream;
    Grow da, dj, dout;
    uint8_t* a = (uint8_t*)da.get(arena_len + ARENA_SLACK);
    HIPCHK(hipMemsetAsync(a + arena_len, 0, ARENA_SLACK, s));
    if (arena_len) HIPCHK(hipMemcpyAsync(a, arena, arena_len, hipMemcpyHostToDevice, s));
    jg_hjob* j = (jg_hjob*)dj.get(sizeof(jg_hjob) * njobs);
    HIPCHK(hipMemcpyAsync(j, jobs, sizeof(jg_hjob) * njobs, hipMemcpyHostToDevice, s));
    uint32_t* o = (uint32_t*)dout.get(64 * njobs);
    launch_hash(a, j, (int64_t)njobs, o, s);
    HIPCHK(hipGetLastError());
    std::vector<uint32_t> w(16 * njobs);
    HIPCHK(hipMemcpyAsync(w.data(), o, 64 * njobs, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (size_t k = 0; k < w.size(); ++k) {              // big-endian words -> digest bytes
      digest_out[4 * k] = (uint8_t)(w[k] >> 24);
      digest_out[4 * k + 1] = (uint8_t)(w[k] >> 16);
      digest_out[4 * k + 2] = (uint8_t)(w[k] >> 8);
      digest_out[4 * k + 3] = (uint8_t)w[k];
    }
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

const char* jg_last_error(jg_ctx* ctx) {
  if (!ctx) return g_tls_err.c_str();
  std::lock_guard<std::mutex> g(ctx->err_mu);
  g_tls_err = ctx->err;
  return g_tls_err.c_str();
}

void* jg_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (bytes == 0) bytes = 1;
  if (hipHostMalloc(&p, bytes + ARENA_SLACK, hipHostMallocPortable) != hipSuccess) return nullptr;
  std::memset((uint8_t*)p + bytes, 0, ARENA_SLACK);
  std::lock_guard<std::mutex> g(g_hmu);
  g_hblocks[(uintptr_t)p] = bytes;
  return p;
}

void jg_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> g(g_hmu);
    g_hblocks.erase((uintptr_t)p);
  }
  (void)hipHostFree(p);
}

const char* jg_version(void) { return "capjwt 0.2 (gfx950, HIP)"; }

}  // extern "C"
