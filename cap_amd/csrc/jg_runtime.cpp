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
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
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
#include "kernels/rsa.hpp"

static_assert(sizeof(jg_tok) == 24 && sizeof(jgk::JobDev) == 16, "job layouts");

using namespace jgk;

namespace {

constexpr size_t ARENA_SLACK = 256;   // aligned SHA word reads may run past the last string
constexpr int NLANE = 3;              // compute streams per device (HW queues 1..3; the copy stream has 0)
constexpr int NSLOT = 8;              // chunk buffer sets per device (pipeline depth)
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

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
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
std::vector<size_t> chunk_cuts(size_t lo, size_t hi, size_t C) {
  std::vector<size_t> cut{lo};
  for (size_t ramp = std::min<size_t>(C, 4096); cut.back() < hi; ramp = std::min(C, 2 * ramp))
    cut.push_back(std::min(hi, cut.back() + ramp));
  const size_t tail = C / 4;
  if (cut.size() > 2 && tail >= 1024 && cut.back() - cut[cut.size() - 2] > tail)
    cut.insert(cut.end() - 1, cut.back() - tail);
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
// relative device time per token (1 x MI355X kernel times, profiles/r01_s4_*),
// for splitting a batch over devices
double cls_cost(int c) {
  switch (c) {
    case CLS_RSA2K: return 3.6;
    case CLS_RSA3K: return 8.0;
    case CLS_RSA4K: return 16.0;
    case CLS_P256: return 1.0;
    case CLS_P384: return 3.6;
    case CLS_P521: return 8.4;
    case CLS_ED25519: return 1.9;
    default: return 0.01;
  }
}

// Grow-only buffers reallocate with 50 % headroom (2 MiB granules): a pipeline
// slot whose chunks vary in size and class mix (scratch rows per class) grows
// a few times, not at every larger chunk -- a reallocation costs a device
// synchronisation (hipFree) or a page-locking pass (hipHostMalloc).
inline size_t grow_size(size_t n, size_t cap) {
  const size_t want = std::max(n, cap + cap / 2);
  return (want + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
}

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

// Fixed-base tables of the curve generators / Ed25519 base point depend only
// on (device, curve): every jg_ctx of the process shares one copy per device,
// built on first use and kept for the life of the process (they are constants
// of the curves: ~31 GB per device with all four, the P-256 one 26.8 GB and
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
  hipStream_t cstream[NCLS] = {};
  hipEvent_t ev_start = nullptr, ev_done[NCLS] = {};
  // Streams are bound to the process's hardware queues round-robin in
  // creation order (GPU_MAX_HW_QUEUES, 4 by default): the device creates
  // every lane's main stream first so the pipeline slots land on distinct
  // queues and really overlap, then the per-class fan-out streams.
  void create_main() { HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)); }
  void create_fanout() {
    for (int c = 1; c < NCLS; ++c) {
      HIPCHK(hipStreamCreateWithFlags(&cstream[c], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&ev_done[c], hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&ev_start, hipEventDisableTiming));
  }
  void sync() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (int c = 1; c < NCLS; ++c)
      if (cstream[c]) (void)hipStreamSynchronize(cstream[c]);
  }
  void destroy() {
    sync();
    for (int c = 1; c < NCLS; ++c) {
      if (cstream[c]) (void)hipStreamDestroy(cstream[c]);
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
};

struct PlanScratch {              // reused across chunks
  std::vector<uint8_t> tcls;      // class per job (host fill only)
  std::vector<int64_t> start, total;   // per bucket [nkeys + 1]
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
  double host_ms[4] = {};                                       // wait, plan, enqueue, of which H2D calls
  int chunk_no = 0;
  size_t reserved = 0;             // chunk capacity (jobs) the buffers were sized for
  uint64_t reserved_epoch = ~0ull; // key table they were sized against
  bool inflight = false;
  std::shared_ptr<Ticket> ticket;
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
  uint64_t epoch = 0;
  const uint8_t* dev_arena = nullptr;   // device view of a page-locked arena (kernels read it over PCIe)
  size_t chunk = 0, nchunks = 0;
  std::vector<size_t> cuts;       // chunk boundaries (chunk_cuts)
};

struct Device {
  int id = 0;
  int ec_wq[NCLS] = {};           // comb width of the loaded EC key tables per curve
  int ed_wa = 16;                 // comb width of the loaded Ed25519 key tables
  Lane lane0;                     // resident batches, key loads, hashing
  uint32_t* gtab[NCLS] = {};
  uint32_t* btab = nullptr;
  std::shared_ptr<SharedTable> tab_ref[NCLS];   // keeps gtab / btab alive
  // comb tables of the current key blob by key content (class, coordinates):
  // a reload (JWKS refresh) copies the tables of keys it already had instead
  // of rebuilding them (D2D copy ~0.2 ms vs ~80 ms per P-256 key)
  std::unordered_map<std::string, std::pair<uint64_t, uint64_t>> tab_cache;   // id -> (word offset, words)
  DevKey* dkeys = nullptr;
  uint32_t* dblob = nullptr;
  int32_t* didx = nullptr;
  std::mutex mu;                  // device state + lane0 + slots
  // streaming pipeline: H2D copies of every chunk back to back on one copy
  // stream (full link bandwidth, no sharing between slots), each slot's
  // kernels on its own stream once its copy event fires
  hipStream_t copy = nullptr;
  Lane lanes[NLANE];
  Slot slots[NSLOT];
  int next_slot = 0, next_lane = 0;
  std::thread worker;
  std::mutex qmu;
  std::condition_variable qcv, idle_cv;
  std::deque<Item> q;
  bool stop = false, busy = false;
  PlanScratch plan;               // worker scratch of the host plan
  uint8_t* dcls = nullptr;        // device copy of the context's class table (k_plan_fill)
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
  uint64_t epoch = 0;
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
  std::vector<HostKey> keys;
  std::vector<uint8_t> cls_tab;   // [key * NALG + alg] -> kernel class of the job
  std::vector<int32_t> cls_keys[NCLS];   // keys of each class, in index order
  int rsa4k_limbs = 148;          // largest RSA-4K+ layout among the valid keys
  int rsa4k_layouts = 1;          // RSA-4K+ layouts present (bit i: rsa4k_layout_limbs(i))
  bool failed = false;            // the last key load failed half-way: nothing verifies
  std::atomic<size_t> chunk{chunk_jobs()};   // jobs per pipeline chunk
  std::atomic<uint64_t> table_budget{default_table_budget()};   // HBM for P-256 key comb tables
  uint64_t epoch = 0;
  std::shared_mutex key_mu;       // key table: exclusive in jg_keys_load, shared by submitters
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
inline int classify(const jg_ctx* ctx, const jg_tok& t) {
  return t.alg < NALG ? ctx->cls_tab[(size_t)t.key_idx * NALG + t.alg] : CLS_REJECT;
}

void rebuild_class_tables(jg_ctx* ctx) {
  const size_t nk = ctx->keys.size();
  ctx->cls_tab.assign(nk * NALG, (uint8_t)CLS_REJECT);
  for (auto& v : ctx->cls_keys) v.clear();
  ctx->rsa4k_limbs = rsa4k_layout_limbs(0);
  ctx->rsa4k_layouts = 1;
  for (size_t k = 0; k < nk; ++k) {
    const HostKey& hk = ctx->keys[k];
    if (hk.valid && hk.cls != CLS_REJECT) ctx->cls_keys[hk.cls].push_back((int32_t)k);
    if (hk.valid && hk.cls == CLS_RSA4K) {
      ctx->rsa4k_limbs = std::max(ctx->rsa4k_limbs, hk.nlimbs);
      for (int i = 0; i < RSA4K_NLAYOUT; ++i)
        if (hk.nlimbs == rsa4k_layout_limbs(i)) ctx->rsa4k_layouts |= 1 << i;
    }
    for (int a = 0; a < NALG; ++a)
      if (hk.valid && alg_family(a) == hk.kind) ctx->cls_tab[k * NALG + a] = (uint8_t)hk.cls;
  }
}

// Reject a job list that names a key outside the table or a byte span outside
// the arena (the prep kernel reads the device copy at those offsets).
bool check_jobs(const jg_ctx* ctx, size_t arena_len, const jg_tok* toks, size_t ntok, std::string* err,
                size_t base = 0) {
  const size_t nk = ctx->keys.size();
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

// Dispatch plan of toks[0..ntok): a counting sort by (class, key) --
// classes 1..NCLS-1 key by key, then the reject bucket; every bucket padded
// to whole waves.  plan_layout counts (the per-job host work of a pipeline
// chunk) and fills X.start / X.total per bucket; the placement is done either
// on the host (plan_fill_host: resident batches) or on the device
// (k_plan_fill: pipeline chunks).
// per-job part of plan_layout (one pass; `visit(i)` runs on every job too):
// bucket counts into X.total, (class, alg) pairs seen into *seen (bit c*16+alg)
template <class Visit>
void plan_count(const jg_ctx* ctx, const jg_tok* toks, size_t ntok, PlanScratch& X, bool keep_cls, uint64_t* seen,
                Visit&& visit) {
  const size_t nk = ctx->keys.size(), NB = nk + 1, RB = nk;
  X.total.assign(NB, 0);
  if (keep_cls) X.tcls.resize(ntok);
  const uint8_t* ctab = ctx->cls_tab.data();
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

void plan_layout(const jg_ctx* ctx, const jg_tok* toks, size_t ntok, Plan& P, PlanScratch& X, bool keep_cls,
                 const uint64_t* seen_in = nullptr) {
  const size_t nk = ctx->keys.size();
  const size_t NB = nk + 1, RB = nk;
  uint64_t seen[2];
  if (seen_in) {
    seen[0] = seen_in[0];
    seen[1] = seen_in[1];
  } else {
    plan_count(ctx, toks, ntok, X, keep_cls, seen, [](size_t) {});
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
      for (int32_t k : ctx->cls_keys[cc]) {
        X.start[(size_t)k] = pos;
        pos += (tot[(size_t)k] + WAVE - 1) / WAVE * WAVE;
      }
    }
    P.ranges[cc].end = pos;
  }
  P.npad = pos > 0 ? pos : WAVE;
  P.ntok = (int64_t)ntok;
  P.sig_rows = 1;
  P.scratch_rows = 1;
  P.pss_tokens = 0;
  P.rsa4k_limbs = ctx->rsa4k_limbs;
  P.rsa4k_layouts = ctx->rsa4k_layouts;
  P.nkeys = (int64_t)ctx->keys.size();
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
void plan_fill_host(const jg_ctx* ctx, const jg_tok* toks, size_t ntok, const Plan& P, PlanScratch& X, JobDev* jobs,
                    int32_t* perm) {
  const size_t nk = ctx->keys.size(), NB = nk + 1, RB = nk;
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
struct PlanBlock {
  size_t cur_off, pad_off, toks_off, bytes;
  PlanBlock(size_t nbuckets, size_t n) {
    cur_off = 0;
    pad_off = sizeof(uint64_t) * nbuckets;
    toks_off = (pad_off + 2 * sizeof(int64_t) * nbuckets + 63) & ~size_t(63);
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
// (resident batches); pipeline chunks keep them in order on the lane's own
// stream unless CAPJWT_FANOUT=1 (measurement A/B)
// CAPJWT_MIDSTATE=0 turns the shared block-0 midstate of the prep kernel off (A/B)
bool prep_midstate() {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_MIDSTATE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

bool pipeline_fanout() {
  static const bool on = [] {
    const char* e = std::getenv("CAPJWT_FANOUT");
    return e && std::atoi(e) != 0;
  }();
  return on;
}

void run_plan(Device* d, Lane* L, Bufs* B, const Plan& P, jg_batch* marks, bool fanout = true) {
  const bool timed = marks && marks->timing;
  int nact = 0;
  for (int c = 1; c < NCLS; ++c) nact += P.ranges[c].end > P.ranges[c].begin;
  const bool conc = !timed && fanout && nact > 1;
  const int64_t np = P.npad;
  const hipStream_t s0 = L->stream;
  mark(marks, "begin");
  HIPCHK(hipMemsetAsync(B->vpad.p, 0, np, s0));
  PrepArgs pa{};
  pa.arena = (const uint8_t*)B->arena.p;
  pa.jobs = (const JobDev*)B->jobs.p;
  pa.keys = d->dkeys;
  pa.keyblob = d->dblob;
  pa.sigw = (uint32_t*)B->sigw.p;
  pa.dig = (uint32_t*)B->dig.p;
  pa.status = (uint8_t*)B->status.p;
  pa.siglen = (uint16_t*)B->siglen.p;
  pa.npad = np;
  pa.mid = prep_midstate() ? (uint32_t*)B->mid.get(sizeof(uint32_t) * PREP_MID_WORDS * (size_t)std::max<int64_t>(P.nkeys, 1))
                           : nullptr;
  uint32_t* rows = (uint32_t*)B->rows.p;
  if (conc) HIPCHK(hipEventRecord(L->ev_start, s0));
  for (int c = 1; c < NCLS; ++c) {
    const ClassRange r = P.ranges[c];
    if (r.end <= r.begin) continue;
    // every class reads and writes only columns [r.begin, r.end) of the shared
    // scratch rows, its own exception counter and its own PSS scratch
    hipStream_t s = s0;
    if (conc) {
      s = L->cstream[c];
      HIPCHK(hipStreamWaitEvent(s, L->ev_start, 0));
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
      ea.npad = np; ea.begin = r.begin; ea.end = r.end;
      ea.wq = d->ec_wq[c];
      launch_ec(c, ea, s, marker(marks, c));
    } else {
      if (!d->btab) throw std::runtime_error("Ed25519 base table missing");
      EdArgs ea{};
      ea.jobs = pa.jobs; ea.keys = pa.keys; ea.keyblob = pa.keyblob;
      ea.sigw = pa.sigw; ea.dig = pa.dig; ea.status = pa.status; ea.siglen = pa.siglen;
      ea.verdict_pad = (uint8_t*)B->vpad.p;
      ea.xyz = rows;
      ea.btab = d->btab;
      ea.npad = np; ea.begin = r.begin; ea.end = r.end;
      ea.wa = d->ed_wa;
      launch_ed(ea, s, marker(marks, c));
    }
    if (conc) {
      HIPCHK(hipEventRecord(L->ev_done[c], s));
      HIPCHK(hipStreamWaitEvent(s0, L->ev_done[c], 0));
    }
  }
  launch_scatter((const int32_t*)B->perm.p, (const uint8_t*)B->vpad.p, (uint8_t*)B->verdict.p, np, s0);
  mark(marks, "scatter");
  HIPCHK(hipGetLastError());
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
void finish_slot(Slot& S) {
  if (!S.inflight) return;
  const hipError_t e = hipEventSynchronize(S.done);
  if (e != hipSuccess) S.ticket->fail(-2, std::string("verify chunk: ") + hipGetErrorString(e));
  else if (S.n) std::memcpy(S.out, S.h_verdict.p, S.n);
  if (pipe_trace() && e == hipSuccess && g_trace_ref) {
    float a = 0, b = 0, c = 0, dn = 0;
    (void)hipEventElapsedTime(&a, g_trace_ref, S.tr_a);
    (void)hipEventElapsedTime(&b, g_trace_ref, S.tr_b);
    (void)hipEventElapsedTime(&c, g_trace_ref, S.tr_c);
    (void)hipEventElapsedTime(&dn, g_trace_ref, S.done);
    std::fprintf(stderr, "[pipe] chunk %3d n=%7zu host wait %.3f plan %.3f enq %.3f (h2d calls %.3f) | gpu h2d %.3f-%.3f kern-end %.3f done %.3f ms\n",
                 S.chunk_no, S.n, S.host_ms[0], S.host_ms[1], S.host_ms[2], S.host_ms[3], a, b, c, dn);
  }
  S.inflight = false;
  auto t = std::move(S.ticket);
  S.ticket.reset();
  t->done_chunks(1);
}


// Plan and enqueue one chunk toks[0..n) of an item on slot S.
// Size a slot's buffers once for the pipeline's chunk capacity C and the
// key table's classes (their largest scratch rows), so chunks of varying size
// and class mix never reallocate in the stream (a hipFree synchronises the
// device, a hipHostMalloc page-locks): ~1 GB of device scratch per slot at
// C = 64 k for a context with RSA-4K keys, far less for ES256 alone.
void reserve_slot(const jg_ctx* ctx, Slot& S, size_t C, size_t nbuckets, double bytes_per_job) {
  const PlanBlock L(nbuckets, C);
  S.h_meta.get(L.bytes);
  S.h_verdict.get(C);
  int sig_rows = 1, scratch_rows = 1;
  bool rsa = false;
  for (int c = 1; c < NCLS; ++c) {
    if (ctx->cls_keys[c].empty()) continue;
    sig_rows = std::max(sig_rows, cls_rows_sig(c, ctx->rsa4k_limbs));
    scratch_rows = std::max(scratch_rows, cls_rows_scratch(c, ctx->rsa4k_limbs));
    rsa = rsa || c <= CLS_RSA4K;
  }
  const size_t npad = C + (size_t)WAVE * nbuckets;
  Bufs* B = &S.bufs;
  B->arena.get((size_t)(bytes_per_job * 1.25 * (double)C) + ARENA_SLACK);
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
  B->mid.get(sizeof(uint32_t) * PREP_MID_WORDS * std::max<size_t>(ctx->keys.size(), 1));
  S.reserved = C;
  S.reserved_epoch = ctx->epoch;
}

void enqueue_chunk(jg_ctx* ctx, Device* d, Slot& S, const Item& it, const jg_tok* toks, size_t n, uint8_t* out) {
  const auto t_start = std::chrono::steady_clock::now();
  if (S.reserved != it.chunk || S.reserved_epoch != ctx->epoch) {
    double bpj = 0;
    for (size_t i = 0; i < std::min<size_t>(n, 256); ++i) bpj += (double)(tok_end(toks[i]) - toks[i].off);
    reserve_slot(ctx, S, std::max(it.chunk, n), ctx->keys.size() + 1, n ? bpj / (double)std::min<size_t>(n, 256) : 512.0);
  }
  // One pass over the caller's jobs: the arena span they use, the bucket
  // counts of the plan, and their copy into the pinned plan block.  The span
  // is DMAed straight from a pinned caller arena when it is compact, else
  // repacked job by job into pinned staging.
  const size_t NB = ctx->keys.size() + 1;
  const PlanBlock L(NB, n);
  uint8_t* hb = (uint8_t*)S.h_meta.get(L.bytes);
  jg_tok* ht = (jg_tok*)(hb + L.toks_off);
  uint64_t amin = UINT64_MAX, amax = 0, need = 0, seen[2];
  plan_count(ctx, toks, n, d->plan, false, seen, [&](size_t i) {
    const jg_tok& t = toks[i];
    const uint64_t e = tok_end(t);
    amin = std::min<uint64_t>(amin, t.off);
    amax = std::max<uint64_t>(amax, e);
    need += e - t.off;
    ht[i] = t;
  });
  if (n == 0) amin = amax = 0;
  const uint64_t base = amin & ~uint64_t(255);
  const uint64_t span = amax - base;
  // JobDev offsets are 32-bit: a span that does not fit is repacked
  const bool compact = span <= 2 * need + 65536 && span < (uint64_t(1) << 32) - ARENA_SLACK;
  const uint8_t* src;
  size_t bytes;
  uint64_t dbase;                                  // subtracted from job offsets on the device
  if (compact) {
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
  Plan P;
  plan_layout(ctx, ht, n, P, d->plan, false, seen);
  uint64_t* cur = (uint64_t*)(hb + L.cur_off);
  int64_t* pad = (int64_t*)(hb + L.pad_off);
  for (size_t k = 0; k < NB; ++k) {
    const auto r = pad_range(d->plan, k, P, NB - 1);
    cur[k] = (uint64_t)d->plan.start[k];
    pad[2 * k] = r.first;
    pad[2 * k + 1] = r.second;
  }
  Lane& LN = d->lanes[d->next_lane];
  d->next_lane = (d->next_lane + 1) % NLANE;
  const hipStream_t s = LN.stream;
  const bool tr = pipe_trace();
  S.host_ms[1] = tr ? ms_since(t_start) : 0.0;
  const auto t_enq = std::chrono::steady_clock::now();
  // The arena span goes over PCIe on the copy stream's DMA engine (spans of
  // consecutive chunks back to back); the rest of the chunk runs on a compute
  // lane once that copy lands: a copy kernel pulls the plan block's cursors
  // from pinned host memory, k_plan_fill reads the jobs straight from it
  // (zero-copy), and a copy kernel writes the verdicts back to pinned memory.
  size_scratch(&S.bufs, P, bytes);
  S.bufs.jobs.get(sizeof(JobDev) * P.npad);
  S.bufs.perm.get(sizeof(int32_t) * P.npad);
  uint8_t* dm = (uint8_t*)S.bufs.meta.get(L.toks_off);
  const uint8_t* hbd = (const uint8_t*)S.h_meta.dp;
  const hipStream_t cs = d->copy;
  if (tr) HIPCHK(hipEventRecord(S.tr_a, cs));
  if (bytes) HIPCHK(hipMemcpyAsync(S.bufs.arena.p, src, bytes, hipMemcpyHostToDevice, cs));
  HIPCHK(hipEventRecord(S.copied, cs));
  if (tr) HIPCHK(hipEventRecord(S.tr_b, cs));
  if (tr) S.host_ms[3] = ms_since(t_enq);
  HIPCHK(hipStreamWaitEvent(s, S.copied, 0));
  launch_copy(hbd, dm, L.toks_off, s);
  {
    PlanFillArgs fa{};
    fa.toks = (const jg_tok*)(hbd + L.toks_off);
    fa.n = (int64_t)n;
    fa.base = dbase;
    fa.cls_tab = d->dcls;
    fa.nkeys = (int32_t)(NB - 1);
    fa.cursor = (unsigned long long*)(dm + L.cur_off);
    fa.pad = (const int64_t*)(dm + L.pad_off);
    fa.jobs = (JobDev*)S.bufs.jobs.p;
    fa.perm = (int32_t*)S.bufs.perm.p;
    launch_plan_fill(fa, s);
  }
  run_plan(d, &LN, &S.bufs, P, nullptr, pipeline_fanout());
  if (tr) HIPCHK(hipEventRecord(S.tr_c, s));
  S.h_verdict.get(std::max<size_t>(n, 1));
  launch_copy(S.bufs.verdict.p, S.h_verdict.dp, n, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(S.done, s));
  if (tr) S.host_ms[2] = ms_since(t_enq);
  S.ticket = it.t;
  S.out = out;
  S.n = n;
  S.inflight = true;
}

void process_item(jg_ctx* ctx, Device* d, Item& it) {
  size_t enq = 0;
  try {
    std::lock_guard<std::mutex> g(d->mu);
    HIPCHK(hipSetDevice(d->id));
    if (ctx->failed || ctx->epoch != it.epoch)
      throw std::runtime_error("key table reloaded (or its load failed) while the batch was queued");
    if (pipe_trace()) {
      if (!g_trace_ref) HIPCHK(hipEventCreate(&g_trace_ref));
      HIPCHK(hipEventRecord(g_trace_ref, d->copy));
    }
    for (size_t c = 0; c + 1 < it.cuts.size(); ++c) {
      const size_t lo = it.cuts[c], hi = it.cuts[c + 1];
      std::string bad;
      if (!check_jobs(ctx, it.arena_len, it.toks + lo, hi - lo, &bad, lo)) {
        it.t->fail(-1, bad);
        break;
      }
      Slot& S = d->slots[d->next_slot];
      d->next_slot = (d->next_slot + 1) % NSLOT;
      const auto tw = std::chrono::steady_clock::now();
      finish_slot(S);                 // the slot's previous chunk (NSLOT chunks ago)
      const double wait_ms = pipe_trace() ? ms_since(tw) : 0.0;
      enqueue_chunk(ctx, d, S, it, it.toks + lo, hi - lo, it.out + lo);
      S.host_ms[0] = wait_ms;
      S.chunk_no = (int)enq;
      ++enq;
    }
    if (enq < it.nchunks) it.t->done_chunks(it.nchunks - enq);
  } catch (const std::exception& e) {
    it.t->fail(-2, e.what());
    it.t->done_chunks(it.nchunks - enq);
  }
}

void worker_loop(jg_ctx* ctx, Device* d) {
  (void)hipSetDevice(d->id);
  std::unique_lock<std::mutex> lk(d->qmu);
  while (true) {
    if (!d->q.empty()) {
      Item it = std::move(d->q.front());
      d->q.pop_front();
      d->busy = true;
      lk.unlock();
      process_item(ctx, d, it);
      lk.lock();
      continue;
    }
    // queue empty: complete the in-flight chunks oldest first (blocking on
    // each; a submission arriving meanwhile is picked up after that chunk)
    bool any = false;
    lk.unlock();
    {
      std::lock_guard<std::mutex> g(d->mu);
      for (int k = 0; k < NSLOT; ++k) {
        Slot& S = d->slots[(d->next_slot + k) % NSLOT];    // oldest first
        if (!S.inflight) continue;
        finish_slot(S);
        any = true;
        break;
      }
    }
    lk.lock();
    if (any) continue;
    if (d->q.empty()) {
      d->busy = false;
      d->idle_cv.notify_all();
      if (d->stop) break;
      d->qcv.wait(lk, [&] { return d->stop || !d->q.empty(); });
    }
  }
}

void wait_idle(Device* d) {
  std::unique_lock<std::mutex> lk(d->qmu);
  d->idle_cv.wait(lk, [&] { return d->q.empty() && !d->busy; });
}

// ---------------------------------------------------------------- keys
struct StagedKeys {
  int ec_wq[NCLS] = {};             // comb width of this load's EC key tables per curve (ecdsa.hpp ec_key_w)
  int ed_wa = 16;                  // comb width of this load's Ed25519 key tables (ed25519.hpp ed_key_w)
  std::vector<DevKey> dk;
  std::vector<uint32_t> blob;      // host-initialised part of the device key blob
  uint64_t tab_words = 0;          // device-only tail: comb tables (built on the GPU)
  std::vector<int32_t> rsa_idx, ec_idx[NCLS], ed_idx, tab_keys;
  std::vector<std::string> tab_id;  // per key: content id of its comb table ("" = none)
};

// comb tables never exist on the host: offsets are relative to the device-only
// tail until build_keys rebases them past the host part
uint64_t tab_alloc(StagedKeys& S, int key, uint64_t words) {
  const uint64_t off = S.tab_words;
  S.tab_words += (words + 3) & ~uint64_t(3);
  S.tab_keys.push_back(key);
  return off;
}

uint64_t blob_alloc(std::vector<uint32_t>& blob, size_t words) {
  const uint64_t off = (blob.size() + 3) & ~size_t(3);          // 16-byte aligned
  blob.resize(off + words, 0);
  return off;
}

// Host part of a key load.  Touches no context state (the caller commits `hk`
// only after every device has loaded the new table); `warn` collects
// informational messages for jg_last_error.
void build_keys(const jg_key* keys, int nkeys, uint64_t table_budget, StagedKeys& S, std::vector<HostKey>& hks,
                std::string* warn) {
  hks.assign((size_t)nkeys, HostKey{});
  S.dk.assign((size_t)nkeys, DevKey{});
  S.tab_id.assign((size_t)nkeys, std::string());
  // EC key tables: per curve, the widest comb whose tables for every key of
  // that curve in the load fit the context's table budget (fewer additions)
  int nec[4] = {};
  for (int i = 0; i < nkeys; ++i)
    if (keys[i].kind == JG_KEY_EC && keys[i].curve >= JG_P256 && keys[i].curve <= JG_P521) ++nec[keys[i].curve];
  S.ec_wq[CLS_P256] = ec_key_w(CLS_P256, nec[JG_P256], table_budget);
  S.ec_wq[CLS_P384] = ec_key_w(CLS_P384, nec[JG_P384], table_budget);
  S.ec_wq[CLS_P521] = ec_key_w(CLS_P521, nec[JG_P521], table_budget);
  int ned = 0;
  for (int i = 0; i < nkeys; ++i) ned += keys[i].kind == JG_KEY_ED25519;
  S.ed_wa = ed_key_w(ned, table_budget);
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
      K.n_off = blob_alloc(S.blob, L);
      K.rr_off = blob_alloc(S.blob, L);
      if (nl > 0) be_to_limbs(n, nl, S.blob.data() + K.n_off, L);
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
      K.tab_off = tab_alloc(S, i, (uint64_t)ec_table_words_w(cls, S.ec_wq[cls]));
      const size_t cl = k.coord_len > 0 ? (size_t)k.coord_len : 0;
      // crypto/ecdsa pointFromAffine: coordinates must fit the curve's bit size
      bool ok = k.x && k.y && cl > 0 && bitlen_be(k.x, cl) <= (cls == CLS_P521 ? 521 : cb * 8) &&
                bitlen_be(k.y, cl) <= (cls == CLS_P521 ? 521 : cb * 8);
      if (ok) {
        be_to_limbs(k.x, cl, S.blob.data() + K.aux_off, L);
        be_to_limbs(k.y, cl, S.blob.data() + K.aux_off + L, L);
        S.tab_id[i] = std::string("E") + (char)cls + std::string((const char*)S.blob.data() + 4 * K.aux_off, 8 * L);
      }
      K.valid = ok;
      if (ok) S.ec_idx[cls].push_back(i);
      hk.cls = cls;
      hk.valid = ok;              // on-curve check happens on the device
    } else if (k.kind == JG_KEY_ED25519) {
      K.cls = CLS_ED25519;
      K.kbytes = 32;
      K.aux_off = blob_alloc(S.blob, 8 + 2 * ED_L);
      K.tab_off = tab_alloc(S, i, (uint64_t)ed_table_words_w(S.ed_wa));
      // crypto/ed25519.Verify panics on len(pub) != 32; go-jose never hands it one
      const bool ok = k.x && k.coord_len == 32;
      if (ok) {
        std::memcpy(S.blob.data() + K.aux_off, k.x, 32);
        S.tab_id[i] = std::string("D") + std::string((const char*)k.x, 32);
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
                               " keys per table (comb tables are " +
                               std::to_string(ec_table_words_w(c, S.ec_wq[c]) * 4 >> 20) + " MiB each)");
  if ((int)S.ed_idx.size() > ED_MAX_KEYS)
    throw std::runtime_error("Ed25519: at most " + std::to_string(ED_MAX_KEYS) + " keys per table (comb tables are " +
                             std::to_string(ed_table_words_w(S.ed_wa) * 4 >> 20) + " MiB each)");
  blob_alloc(S.blob, 0);                                      // align the host part
  for (int k : S.tab_keys) S.dk[k].tab_off += S.blob.size();
}

// the process-wide table of (device, class), built on this device's stream
// and complete before any other context can see it
template <class Build>
std::shared_ptr<SharedTable> shared_table(Device* d, int cls, size_t bytes, Build&& build) {
  std::lock_guard<std::mutex> g(g_tab_mu);
  const auto key = std::make_pair(d->id, cls);
  if (auto t = g_tabs[key]) return t;
  auto t = std::make_shared<SharedTable>();
  HIPCHK(hipMalloc(&t->p, bytes));
  try {
    build(t->p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(d->lane0.stream));
  } catch (...) {
    (void)hipFree(t->p);          // a failed build is not cached
    throw;
  }
  g_tabs[key] = t;
  return t;
}

void ensure_tables(Device* d, const StagedKeys& S) {
  HIPCHK(hipSetDevice(d->id));
  for (int c = CLS_P256; c <= CLS_P521; ++c) {
    if (S.ec_idx[c].empty() || d->gtab[c]) continue;
    d->tab_ref[c] = shared_table(d, c, sizeof(uint32_t) * ec_table_words(c, true),
                                 [&](uint32_t* t) { launch_ec_gtable(c, t, d->lane0.stream); });
    d->gtab[c] = d->tab_ref[c]->p;
  }
  if (!S.ed_idx.empty() && !d->btab) {
    d->tab_ref[CLS_ED25519] = shared_table(d, CLS_ED25519, sizeof(uint32_t) * ed_table_words(true),
                                           [&](uint32_t* t) { launch_ed_btable(t, d->lane0.stream); });
    d->btab = d->tab_ref[CLS_ED25519]->p;
  }
}

void load_keys_device(Device* d, const StagedKeys& S) {
  HIPCHK(hipSetDevice(d->id));
  for (int c = 0; c < NCLS; ++c) d->ec_wq[c] = S.ec_wq[c];
  d->ed_wa = S.ed_wa;
  hipStream_t s = d->lane0.stream;
  d->lane0.sync();
  if (d->copy) (void)hipStreamSynchronize(d->copy);
  for (auto& ln : d->lanes) ln.sync();
  if (d->dkeys) (void)hipFree(d->dkeys);
  if (d->didx) (void)hipFree(d->didx);
  d->dkeys = nullptr; d->didx = nullptr;
  uint32_t* old_blob = d->dblob;                   // kept until its reusable tables are copied
  auto old_cache = std::move(d->tab_cache);
  d->tab_cache.clear();
  d->dblob = nullptr;
  try {
    const size_t nk = std::max<size_t>(S.dk.size(), 1);
    HIPCHK(hipMalloc(&d->dkeys, sizeof(DevKey) * nk));
    HIPCHK(hipMalloc(&d->dblob, sizeof(uint32_t) * std::max<uint64_t>(S.blob.size() + S.tab_words, 4)));
    if (!S.dk.empty()) HIPCHK(hipMemcpyAsync(d->dkeys, S.dk.data(), sizeof(DevKey) * S.dk.size(), hipMemcpyHostToDevice, s));
    if (!S.blob.empty())
      HIPCHK(hipMemcpyAsync(d->dblob, S.blob.data(), sizeof(uint32_t) * S.blob.size(), hipMemcpyHostToDevice, s));
    // per table class: keys to stage (all) and keys whose tables must be built
    // (the rest are copied from the previous blob, same key content)
    auto split = [&](const std::vector<int32_t>& keys, uint64_t words, std::vector<int32_t>& build) {
      for (int32_t i : keys) {
        const std::string& id = S.tab_id[(size_t)i];
        const uint64_t off = S.dk[(size_t)i].tab_off;
        auto it = id.empty() ? old_cache.end() : old_cache.find(id);
        if (old_blob && it != old_cache.end() && it->second.second == words) {
          HIPCHK(hipMemcpyAsync(d->dblob + off, old_blob + it->second.first, sizeof(uint32_t) * words,
                                hipMemcpyDeviceToDevice, s));
        } else {
          build.push_back(i);
        }
        if (!id.empty()) d->tab_cache[id] = {off, words};
      }
    };
    std::vector<int32_t> build_ec[NCLS], build_ed;
    for (int c = CLS_P256; c <= CLS_P521; ++c)
      split(S.ec_idx[c], (uint64_t)ec_table_words_w(c, S.ec_wq[c]), build_ec[c]);
    split(S.ed_idx, (uint64_t)ed_table_words_w(S.ed_wa), build_ed);
    // one index array: rsa | p256 | p384 | p521 | ed | builds p256 | p384 | p521 | ed
    std::vector<int32_t> idx;
    std::vector<size_t> at;
    auto push = [&](const std::vector<int32_t>& v) { at.push_back(idx.size()); idx.insert(idx.end(), v.begin(), v.end()); };
    push(S.rsa_idx);
    for (int c = CLS_P256; c <= CLS_P521; ++c) push(S.ec_idx[c]);
    push(S.ed_idx);
    for (int c = CLS_P256; c <= CLS_P521; ++c) push(build_ec[c]);
    push(build_ed);
    HIPCHK(hipMalloc(&d->didx, sizeof(int32_t) * std::max<size_t>(idx.size(), 1)));
    if (!idx.empty()) HIPCHK(hipMemcpyAsync(d->didx, idx.data(), sizeof(int32_t) * idx.size(), hipMemcpyHostToDevice, s));
    ensure_tables(d, S);
    if (!S.dk.empty()) launch_rsa_keyprep(d->dkeys, d->dblob, (int)S.dk.size(), s);
    for (int c = CLS_P256; c <= CLS_P521; ++c)
      launch_ec_keyprep(c, S.ec_wq[c], d->dkeys, d->dblob, d->didx + at[1 + c - CLS_P256], (int)S.ec_idx[c].size(),
                        d->didx + at[5 + c - CLS_P256], (int)build_ec[c].size(), s);
    launch_ed_keyprep(S.ed_wa, d->dkeys, d->dblob, d->didx + at[4], (int)S.ed_idx.size(), d->didx + at[8],
                      (int)build_ed.size(), s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
  } catch (...) {
    (void)hipStreamSynchronize(s);
    if (old_blob) (void)hipFree(old_blob);
    d->tab_cache.clear();
    throw;
  }
  if (old_blob) (void)hipFree(old_blob);
}

thread_local std::string g_tls_err;


// Split jobs [0, ntok) over the context's devices by the cost model and queue
// each device's share.  Caller holds key_mu (shared) and has validated the jobs.
std::shared_ptr<Ticket> submit_locked(jg_ctx* ctx, const uint8_t* arena, size_t arena_len, const jg_tok* toks,
                                      size_t ntok, uint8_t* out) {
  auto t = std::make_shared<Ticket>();
  const size_t nd = ctx->devs.size();
  std::vector<size_t> cut(nd + 1, 0);
  cut[nd] = ntok;
  if (nd > 1) {
    std::vector<double> pre(ntok + 1, 0.0);
    const size_t nk = ctx->keys.size();
    for (size_t i = 0; i < ntok; ++i)
      pre[i + 1] = pre[i] + (toks[i].key_idx < nk ? cls_cost(classify(ctx, toks[i])) : 0.0);
    size_t j = 0;
    for (size_t k = 1; k < nd; ++k) {
      const double target = pre[ntok] * (double)k / (double)nd;
      while (j < ntok && pre[j] < target) ++j;
      cut[k] = j;
    }
  }
  const uint8_t* dview = device_view(arena);
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
    it.epoch = ctx->epoch;
    it.dev_arena = dview;
    it.chunk = C;
    it.cuts = chunk_cuts(it.lo, it.hi, C);
    it.nchunks = it.cuts.size() - 1;
    t->pending += it.nchunks;
    items.push_back(std::move(it));
  }
  for (size_t k = 0, i = 0; k < nd && i < items.size(); ++k) {
    if (cut[k + 1] <= cut[k]) continue;
    Device* d = ctx->devs[k].get();
    {
      std::lock_guard<std::mutex> g(d->qmu);
      d->q.push_back(std::move(items[i++]));
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
      for (auto& l : d->lanes) l.create_fanout();
      d->lane0.create_fanout();
      for (auto& s : d->slots) {
        HIPCHK(hipEventCreateWithFlags(&s.done, pipe_trace() ? hipEventDefault : hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
        HIPCHK(hipEventCreate(&s.tr_a));
        HIPCHK(hipEventCreate(&s.tr_b));
        HIPCHK(hipEventCreate(&s.tr_c));
      }
      ctx->devs.push_back(std::move(d));
    }
    jg_ctx* c = ctx.release();
    for (auto& d : c->devs) d->worker = std::thread(worker_loop, c, d.get());
    return c;
  } catch (const std::exception& e) {
    g_tls_err = e.what();
    return nullptr;
  }
}

void jg_destroy(jg_ctx* ctx) {
  if (!ctx) return;
  for (auto& d : ctx->devs) {
    {
      std::lock_guard<std::mutex> g(d->qmu);
      d->stop = true;
    }
    d->qcv.notify_all();
    if (d->worker.joinable()) d->worker.join();
  }
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d->id);
    for (auto& l : d->lanes) l.destroy();
    for (auto& s : d->slots) {
      if (s.done) (void)hipEventDestroy(s.done);
      for (hipEvent_t e : {s.tr_a, s.tr_b, s.tr_c, s.copied})
        if (e) (void)hipEventDestroy(e);
    }
    d->lane0.sync();
    if (d->copy) {
      (void)hipStreamSynchronize(d->copy);
      (void)hipStreamDestroy(d->copy);
    }
    for (auto& t : d->tab_ref) t.reset();         // shared fixed-base tables: last holder frees
    if (d->dkeys) (void)hipFree(d->dkeys);
    if (d->dblob) (void)hipFree(d->dblob);
    if (d->didx) (void)hipFree(d->didx);
    if (d->dcls) (void)hipFree(d->dcls);
    d->lane0.destroy();
  }
  delete ctx;
}

int jg_keys_load(jg_ctx* ctx, const jg_key* keys, int nkeys) {
  if (!ctx || nkeys < 0 || (nkeys > 0 && !keys)) return -1;
  if (nkeys > 65535) { ctx->set_err("at most 65535 keys"); return -1; }
  try {
    std::unique_lock<std::shared_mutex> kl(ctx->key_mu);    // no new submissions
    for (auto& d : ctx->devs) wait_idle(d.get());            // queued work runs against the old table
    std::vector<std::unique_lock<std::mutex>> dl;
    for (auto& d : ctx->devs) dl.emplace_back(d->mu);
    StagedKeys S;
    std::vector<HostKey> hk;
    std::string warn;
    build_keys(keys, nkeys, ctx->table_budget.load(), S, hk, &warn);   // throws before any device state changes
    try {
      for (auto& d : ctx->devs) load_keys_device(d.get(), S);
      // device-side validity (on-curve, Ed25519 decoding) back into the host view
      Device* d0 = ctx->devs[0].get();
      std::vector<DevKey> back(S.dk.size());
      if (!back.empty()) {
        HIPCHK(hipSetDevice(d0->id));
        HIPCHK(hipMemcpy(back.data(), d0->dkeys, sizeof(DevKey) * back.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < back.size(); ++i) hk[i].valid = hk[i].valid && back[i].valid;
      }
    } catch (...) {
      // some device may hold part of the new table: nothing verifies until a
      // load succeeds, and batches staged before now are stale
      ctx->keys.clear();
      rebuild_class_tables(ctx);
      ctx->failed = true;
      ++ctx->epoch;
      throw;
    }
    ctx->keys = std::move(hk);
    rebuild_class_tables(ctx);
    for (auto& d : ctx->devs) {
      HIPCHK(hipSetDevice(d->id));
      if (d->dcls) (void)hipFree(d->dcls);
      d->dcls = nullptr;
      HIPCHK(hipMalloc(&d->dcls, std::max<size_t>(ctx->cls_tab.size(), 16)));
      if (!ctx->cls_tab.empty())
        HIPCHK(hipMemcpy(d->dcls, ctx->cls_tab.data(), ctx->cls_tab.size(), hipMemcpyHostToDevice));
    }
    ctx->failed = false;
    ++ctx->epoch;
    if (!warn.empty()) ctx->set_err(warn);
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_submit(jg_ctx* ctx, const uint8_t* arena, size_t arena_len, const jg_tok* toks, size_t ntok,
              uint8_t* verdict_out, jg_ticket** out) {
  if (!ctx || !out || (ntok > 0 && (!toks || !arena || !verdict_out))) return -1;
  *out = nullptr;
  if (ntok > (size_t)INT32_MAX / 2) { ctx->set_err("batch too large"); return -1; }
  try {
    if (ntok == 0) {                       // nothing to verify
      *out = new jg_ticket{std::make_shared<Ticket>()};
      return 0;
    }
    std::shared_lock<std::shared_mutex> kl(ctx->key_mu);
    if (ctx->failed) { ctx->set_err("the last jg_keys_load failed; no key table is loaded"); return -2; }
    // jobs are validated chunk by chunk by the device workers, ahead of each
    // chunk's upload (a bad job fails the ticket with -1 from jg_wait)
    auto t = submit_locked(ctx, arena, arena_len, toks, ntok, verdict_out);
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
    std::shared_lock<std::shared_mutex> kl(ctx->key_mu);
    if (ctx->failed) { ctx->set_err("the last jg_keys_load failed; no key table is loaded"); return -2; }
    std::string err;
    if (!check_jobs(ctx, arena_len, toks, ntok, &err)) { ctx->set_err(err); return -1; }
    auto b = std::make_unique<jg_batch>();
    b->ctx = ctx;
    b->dev = ctx->devs[device_slot].get();
    b->lane = &b->dev->lane0;
    b->own = std::make_unique<Bufs>();
    b->b = b->own.get();
    std::lock_guard<std::mutex> g(b->dev->mu);
    HIPCHK(hipSetDevice(b->dev->id));
    PlanScratch X;
    if (arena_len >= (uint64_t(1) << 32) - ARENA_SLACK) {
      ctx->set_err("a resident batch's arena must be smaller than 4 GiB");
      return -1;
    }
    std::vector<JobDev> jobs;
    std::vector<int32_t> perm;
    plan_layout(ctx, toks, ntok, b->plan, X, true);
    jobs.resize(b->plan.npad);
    perm.resize(b->plan.npad);
    plan_fill_host(ctx, toks, ntok, b->plan, X, jobs.data(), perm.data());
    upload(b->b, b->lane->stream, b->plan, arena, arena_len, jobs.data(), perm.data());
    // the host vectors die here: the copies above must complete first
    HIPCHK(hipStreamSynchronize(b->lane->stream));
    b->arena_len = arena_len;
    b->epoch = ctx->epoch;
    *out = b.release();
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

namespace {
void run_resident(jg_ctx* ctx, jg_batch* b, bool timed) {
  HIPCHK(hipSetDevice(b->dev->id));
  if (b->epoch != ctx->epoch) throw std::runtime_error("key table reloaded since this batch was staged");
  b->timing = timed;
  b->marks_used = 0;
  run_plan(b->dev, b->lane, b->b, b->plan, b);
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
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return nullptr;
  return p;
}

void jg_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

const char* jg_version(void) { return "capjwt 0.2 (gfx950, HIP)"; }

}  // extern "C"
