// cap_jwt.cpp -- see cap_jwt.hpp.
//
// Batch flow of KeySet::verify_batch:
//   1. host threads parse every token (go-jose ParseSigned, R1-R8); compact
//      tokens take a fast path whose protected-header decode is memoised per
//      header segment (tokens signed by one issuer share it byte for byte);
//   2. each token becomes one arena entry  signing-input '.' base64url(sig):
//      canonical tokens are copied as they are, anything else is re-encoded
//      (R6), so the device always sees go-jose's computeAuthData bytes;
//   3. candidate keys per token -- static set: every key of the alg's family,
//      in order (R33); JWKS: keys whose kid matches, all keys when the token
//      has none (R34) -- become jg_tok jobs, verified in ONE jg_verify_batch;
//   4. host threads turn verdicts into (claims, error) exactly as the
//      reference's per-token loop would (first verifying key wins; the claims
//      do not depend on which key verified).
#include "cap_jwt.hpp"

#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "../../../include/jg.h"
#include "hostmem.hpp"

namespace capjwt {

const char* const kSupportedAlgorithms[10] = {"RS256", "RS384", "RS512", "ES256", "ES384",
                                              "ES512", "PS256", "PS384", "PS512", "EdDSA"};

std::string SupportedSigningAlgorithm(const std::vector<std::string>& algs) {
  for (const auto& a : algs)
    if (!alg_id(a)) return "unsupported signing algorithm \"" + a + "\"";
  return "";
}

// CPUs this process may run on: the affinity mask, capped by a cgroup v2 CPU
// quota (a container's share of a large host), never a fixed number.
int available_cpus() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0) {
      const long q = std::atol(quota);
      if (q > 0) n = std::min<int>(n, (int)((q + period - 1) / period));
    }
    std::fclose(f);
  }
  return std::max(1, n);
}

int host_threads() {
  static const int n = [] {
    if (const char* e = std::getenv("CAPJWT_HOST_THREADS")) {
      const int v = std::atoi(e);
      if (v > 0) return v;
    }
    return available_cpus();
  }();
  return n;
}

namespace {

// The batch passes' worker threads, started once per process (host_threads()
// - 1 of them; the calling thread takes part too).  A ValidateBatch call runs
// ~8 parallel passes; creating 15 threads for each cost the caller a few
// hundred microseconds per pass.  A pass started from inside a pass (a nested
// call) gets threads of its own, as before.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool(host_threads() - 1);   // never destroyed: threads live as long as the process
    return *p;
  }
  static bool inside() { return tl_inside_; }
  // task(i) for i in [0, nt), on the pool's threads and the caller's
  void run(size_t nt, const std::function<void(size_t)>& task) {
    Job j;
    j.fn = &task;
    j.nt = nt;
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(&j);
    }
    cv_.notify_all();
    size_t i;
    while ((i = take(&j)) < nt) run_one(&j, i);
    // every index finishes (a throwing task counts as finished) before j,
    // which pool threads still reference, leaves this frame
    std::unique_lock<std::mutex> lk(j.m);
    j.cv.wait(lk, [&] { return j.done == nt; });
    if (j.err) std::rethrow_exception(j.err);
  }

 private:
  struct Job {
    const std::function<void(size_t)>* fn = nullptr;
    size_t nt = 0, next = 0;        // next: under the pool's m_
    size_t done = 0;                // under m
    std::exception_ptr err;         // the first task exception, under m; rethrown by run()
    std::mutex m;
    std::condition_variable cv;
  };
  explicit HostPool(int n) {
    for (int t = 0; t < n; ++t) th_.emplace_back([this] { worker(); });
    for (auto& t : th_) t.detach();
  }
  // the next index of j (nt when none is left; the job leaves the queue with its last index)
  size_t take(Job* j) {
    std::lock_guard<std::mutex> g(m_);
    if (j->next >= j->nt) return j->nt;
    const size_t i = j->next++;
    if (j->next == j->nt) q_.erase(std::find(q_.begin(), q_.end(), j));
    return i;
  }
  static void finish(Job* j) {
    std::lock_guard<std::mutex> g(j->m);     // the owner destroys j only after taking this lock
    if (++j->done == j->nt) j->cv.notify_all();
  }
  static void run_one(Job* j, size_t i) {
    try {
      (*j->fn)(i);
    } catch (...) {
      std::lock_guard<std::mutex> g(j->m);
      if (!j->err) j->err = std::current_exception();
    }
    finish(j);
  }
  void worker() {
    pthread_setname_np(pthread_self(), "capjwt-host");
    tl_inside_ = true;
    std::unique_lock<std::mutex> lk(m_);
    while (true) {
      cv_.wait(lk, [&] { return !q_.empty(); });
      Job* j = q_.front();
      const size_t i = j->next++;
      if (j->next == j->nt) q_.pop_front();
      lk.unlock();
      run_one(j, i);
      lk.lock();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<Job*> q_;
  std::vector<std::thread> th_;
  static thread_local bool tl_inside_;
};
thread_local bool HostPool::tl_inside_ = false;

// fn(i) for i in [0, nt) on nt threads (the pool's, or new ones for a nested call)
template <class F>
void run_parallel(size_t nt, F&& fn) {
  if (!HostPool::inside() && nt <= (size_t)host_threads()) {
    const std::function<void(size_t)> task = [&fn](size_t i) { fn(i); };
    HostPool::get().run(nt, task);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (size_t t = 0; t < nt; ++t) th.emplace_back([&fn, t] { fn(t); });
  for (auto& t : th) t.join();
}

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  // fn(begin, end): contiguous chunks; small batches stay on the caller's thread
  const size_t min_chunk = 512;
  const size_t nt = std::min<size_t>((size_t)std::max(1, threads), (n + min_chunk - 1) / min_chunk);
  if (nt <= 1) {
    if (n) fn((size_t)0, n);
    return;
  }
  run_parallel(nt, [&](size_t t) { fn(n * t / nt, n * (t + 1) / nt); });
}

// A fixed cut of [0, n) into per-thread ranges, so that several passes over a
// batch (count, prefix, fill) see the same ranges and keep running offsets per
// range instead of one serial prefix sum over every token.
struct Chunks {
  std::vector<size_t> b;        // range c = [b[c], b[c+1])
  size_t count() const { return b.size() - 1; }
};
Chunks make_chunks(size_t n, int threads) {
  const size_t min_chunk = 512;
  const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), (n + min_chunk - 1) / min_chunk));
  Chunks c;
  c.b.resize(nt + 1);
  for (size_t t = 0; t <= nt; ++t) c.b[t] = n * t / nt;
  return c;
}
template <class F>
void run_chunks(const Chunks& c, F&& fn) {
  // fn(chunk, begin, end)
  if (c.count() == 1) {
    fn((size_t)0, c.b[0], c.b[1]);
    return;
  }
  run_parallel(c.count(), [&](size_t t) { fn(t, c.b[t], c.b[t + 1]); });
}

}  // namespace

void* batch_block_alloc(size_t bytes, size_t* cap) {
  if (bytes >= (size_t(1) << 20)) return hostmem::big_get(bytes, cap);
  *cap = bytes;
  return ::operator new(bytes);
}

void batch_block_free(void* p, size_t cap) {
  if (!p) return;
  if (cap >= (size_t(1) << 20)) hostmem::big_put(p, cap);
  else ::operator delete(p);
}

void SetHostMemoryRetention(size_t bytes) { hostmem::set_retention_cap(bytes); }
void TrimHostMemory() { hostmem::trim(); }
size_t HostMemoryRetained() { return hostmem::retained(); }

void batch_parallel(size_t n, int threads, const std::function<void(size_t, size_t)>& fn) {
  parallel_for(n, threads, fn);
}

namespace {

int64_t wall_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// ---------------------------------------------------------------- per-token parse
struct HdrInfo {                 // one decoded protected-header segment (compact form)
  bool b64_ok = false;
  std::string b64_err;
  bool ok = false;               // JSON + sanitize
  std::string err;
  Signature sig;                 // protected_raw / protected_hdr / alg / kid
  bool seg_canonical = false;
  bool verifiable = false;       // crit understood, non-empty protected bytes
  bool needs_b64 = true;
  int alg = 0;
};

std::shared_ptr<const HdrInfo> make_hdr(std::string_view seg) {
  auto h = std::make_shared<HdrInfo>();
  h->b64_ok = b64url_decode(seg, &h->sig.protected_raw, &h->b64_err);
  if (!h->b64_ok) return h;
  // parse the header exactly as parse_signed does, on a minimal token
  JWS j;
  std::string tok = b64url_encode(h->sig.protected_raw) + "..";
  if (!parse_signed(tok, &j, &h->err)) return h;
  h->ok = true;
  h->sig = j.sigs[0];
  h->seg_canonical = b64url_canonical(seg);
  std::string si;
  h->verifiable = signing_input(j, &si);       // payload "" -> crit / protected checks only
  if (const json::Value* b = h->sig.protected_hdr.get("b64"); b && b->kind == json::Value::Bool) h->needs_b64 = b->b;
  h->alg = alg_id(h->sig.alg);
  return h;
}

struct HdrCache {
  // a few recent segments checked by plain compare first (a key set's tokens
  // cycle through a handful of headers), then the map
  static constexpr int NRECENT = 8;
  std::string recent_key[NRECENT];
  std::shared_ptr<const HdrInfo> recent_val[NRECENT];
  int nrecent = 0, next = 0;
  // the cache lives as long as its pool thread and its segments come from
  // callers: it is bounded by bytes, and a segment above kMaxSeg (far above
  // any issuer's header) is decoded for this token only
  static constexpr size_t kMaxSeg = 1024, kMaxBytes = 1 << 20;
  std::unordered_map<std::string, std::shared_ptr<const HdrInfo>> m;
  size_t bytes = 0;
  std::shared_ptr<const HdrInfo> uncached;
  const std::shared_ptr<const HdrInfo>& get(std::string_view seg) {
    for (int i = 0; i < nrecent; ++i)
      if (recent_key[i] == seg) return recent_val[i];
    if (seg.size() > kMaxSeg) {
      uncached = make_hdr(seg);
      return uncached;
    }
    auto it = m.find(std::string(seg));
    if (it == m.end()) {
      if (bytes + seg.size() > kMaxBytes) {
        m.clear();
        bytes = 0;
      }
      it = m.emplace(std::string(seg), make_hdr(seg)).first;
      bytes += seg.size() + 64;
    }
    const int slot = next;
    next = (next + 1) % NRECENT;
    if (nrecent < NRECENT) ++nrecent;
    recent_key[slot].assign(seg);
    recent_val[slot] = it->second;
    return recent_val[slot];
  }
};

// decoded length of a base64url segment with no '=' (Go RawURLEncoding)
inline size_t b64_decoded_len(size_t n) { return n / 4 * 3 + (n % 4 == 2 ? 1 : n % 4 == 3 ? 2 : 0); }

struct PhaseTimer {            // CAPJWT_TRACE=1: per-phase wall times (and page faults) on stderr
  bool on;
  std::chrono::steady_clock::time_point t0;
  long flt0 = 0;
  const char* what;
  static long minflt() {
    rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_minflt;
  }
  explicit PhaseTimer(const char* w) : on(std::getenv("CAPJWT_TRACE") != nullptr), t0(std::chrono::steady_clock::now()), what(w) {
    if (on) flt0 = minflt();
  }
  void lap(const char* phase) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    const long f = minflt();
    std::fprintf(stderr, "[capjwt] %s %-12s %7ld flt %8.2f ms\n", what, phase, f - flt0,
                 std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
    flt0 = f;
  }
};

// Array whose elements are constructed and destroyed by all host threads
// (a 1M-token batch's per-token records are ~200 MB of strings: serial
// construction/destruction cost more than the parse itself).
template <class T>
struct ParArray {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  int threads = 1;
  ParArray() = default;
  ParArray(const ParArray&) = delete;
  ParArray& operator=(const ParArray&) = delete;
  void init(size_t count, int th);
  void release();
  ~ParArray() { release(); }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  size_t size() const { return n; }
};

// Decoded payloads of one parse range, in pooled hostmem blocks (one return
// per block instead of one free per token; no page faults in steady state)
struct ByteArena {
  std::vector<void*> blocks;                      // hostmem::kBlock each
  std::vector<std::unique_ptr<char[]>> big;       // payloads larger than a block
  char* cur = nullptr;
  size_t left = 0;
  ByteArena() = default;
  ByteArena(ByteArena&& o) noexcept
      : blocks(std::move(o.blocks)), big(std::move(o.big)), cur(o.cur), left(o.left), last_big(o.last_big) {
    o.cur = nullptr;
    o.left = 0;
  }
  ByteArena(const ByteArena&) = delete;
  ByteArena& operator=(const ByteArena&) = delete;
  ~ByteArena() {
    for (void* b : blocks) hostmem::block_put(b);
  }
  bool last_big = false;
  char* alloc(size_t n) {
    last_big = n > hostmem::kBlock / 2;
    if (last_big) {
      big.emplace_back(new char[n]);
      return big.back().get();
    }
    if (n > left) {
      blocks.push_back(hostmem::block_get());
      cur = static_cast<char*>(blocks.back());
      left = hostmem::kBlock;
    }
    char* r = cur;
    cur += n;
    left -= n;
    return r;
  }
  void give_back(size_t n) {     // the unused tail of the last alloc (a block's, not a big one's)
    if (last_big) return;
    cur -= n;
    left += n;
  }
};

struct GeneralParse {            // storage of a token that took jose.ParseSigned's general path
  std::string alg, kid, payload;
};

struct Tok {
  // ParseSigned outcome (validateSigningAlgorithm's inputs)
  bool parsed = false;
  bool verifiable = false;     // DetachedVerify gets as far as verifyPayload
  int alg = 0;
  uint32_t nsigs = 0;
  size_t sig0_len = 0;
  std::string parse_err;
  std::string_view alg_name, kid, payload;     // into hdr / gen / the batch's ByteArena
  std::shared_ptr<const HdrInfo> hdr;           // compact path: the shared header decode
  std::unique_ptr<GeneralParse> gen;
  // arena entry: literal token span, or owned bytes
  const char* lit = nullptr;
  size_t lit_len = 0;
  std::string owned;
  uint32_t si_len = 0, sig_b64_len = 0;
  uint32_t ncand = 0;          // candidate keys (jobs) in the current GPU batch
  uint64_t job0 = 0;           // first job of this token in that batch
  size_t entry_len() const { return lit ? lit_len : owned.size(); }
  TokenView view() const { return TokenView{parsed, parse_err, nsigs, sig0_len, alg_name}; }
};

template <class T>
void ParArray<T>::init(size_t count, int th) {
  release();
  threads = th;
  p = static_cast<T*>(batch_block_alloc(sizeof(T) * (count ? count : 1), &cap));
  n = count;
  parallel_for(n, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) new (p + i) T();
  });
}

template <class T>
void ParArray<T>::release() {
  if (!p) return;
  parallel_for(n, threads, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) p[i].~T();
  });
  batch_block_free(p, cap);
  p = nullptr;
  n = 0;
}

void parse_one(std::string_view token, HdrCache& cache, ByteArena& pay, Tok* t) {
  // compact fast path: no whitespace / non-ASCII, exactly three segments
  if (!token.empty() && token[0] != '{' && !has_go_space_or_nonascii(token)) {
    const size_t d1 = token.find('.');
    const size_t d2 = d1 == std::string_view::npos ? d1 : token.find('.', d1 + 1);
    if (d1 == std::string_view::npos || d2 == std::string_view::npos ||
        token.find('.', d2 + 1) != std::string_view::npos) {
      t->parse_err = "square/go-jose: compact JWS format must have three parts";
      return;
    }
    const std::string_view hs = token.substr(0, d1), ps = token.substr(d1 + 1, d2 - d1 - 1),
                           ss = token.substr(d2 + 1);
    const std::shared_ptr<const HdrInfo>& h = cache.get(hs);
    // parseSignedCompact order: protected, payload, signature decodes, then sanitize
    if (!h->b64_ok) { t->parse_err = h->b64_err; return; }
    bool pay_canon = false;
    {
      const size_t cap = ps.size() / 4 * 3 + 2;
      char* dst = pay.alloc(cap);
      const long len = b64url_decode_fast(ps, dst, &pay_canon);
      if (len >= 0) {
        pay.give_back(cap - (size_t)len);
        t->payload = std::string_view(dst, (size_t)len);
      } else {                 // '=', CR/LF or an illegal byte: Go's skipping and error text
        pay.give_back(cap);
        t->gen = std::make_unique<GeneralParse>();
        if (!b64url_decode(ps, &t->gen->payload, &t->parse_err)) return;
        t->payload = t->gen->payload;
        pay_canon = false;
      }
    }
    // the signature bytes themselves are only needed when the segment is not
    // canonical (the device decodes canonical base64url itself)
    const bool sig_canon = b64url_canonical(ss);
    std::string sig;
    size_t siglen;
    if (sig_canon) {
      siglen = b64_decoded_len(ss.size());
    } else {
      if (!b64url_decode(ss, &sig, &t->parse_err)) return;
      siglen = sig.size();
    }
    if (!h->ok) { t->parse_err = h->err; return; }
    t->parsed = true;
    t->nsigs = 1;
    t->sig0_len = siglen;
    t->hdr = h;
    t->alg_name = h->sig.alg;
    t->kid = h->sig.kid;
    t->alg = h->alg;
    t->verifiable = h->verifiable && t->alg != 0;
    if (!t->verifiable) return;
    if (h->seg_canonical && h->needs_b64 && pay_canon && sig_canon) {
      t->lit = token.data();
      t->lit_len = token.size();
      t->si_len = (uint32_t)d2;
      t->sig_b64_len = (uint32_t)ss.size();
      return;
    }
    JWS j;
    j.payload = std::string(t->payload);
    j.sigs.push_back(h->sig);
    std::string si;
    signing_input(j, &si);
    t->si_len = (uint32_t)si.size();
    t->owned = std::move(si);
    t->owned.push_back('.');
    const std::string sb = sig_canon ? std::string(ss) : b64url_encode(sig);
    t->sig_b64_len = (uint32_t)sb.size();
    t->owned += sb;
    return;
  }
  // general path: jose.ParseSigned
  JWS j;
  if (!parse_signed(token, &j, &t->parse_err)) return;
  t->parsed = true;
  t->nsigs = (uint32_t)j.sigs.size();
  t->sig0_len = j.sigs.empty() ? 0 : j.sigs[0].signature.size();
  t->gen = std::make_unique<GeneralParse>();
  t->gen->alg = j.sigs.empty() ? "" : j.sigs[0].alg;
  t->gen->kid = j.sigs.empty() ? "" : j.sigs[0].kid;      // go-oidc: the first signature's kid
  t->gen->payload = j.payload;
  t->alg_name = t->gen->alg;
  t->kid = t->gen->kid;
  t->payload = t->gen->payload;
  std::string si;
  if (!signing_input(j, &si)) return;
  t->alg = alg_id(j.sigs[0].alg);
  t->verifiable = t->alg != 0;
  if (!t->verifiable) return;
  t->si_len = (uint32_t)si.size();
  t->owned = std::move(si);
  t->owned.push_back('.');
  const std::string sb = b64url_encode(j.sigs[0].signature);
  t->sig_b64_len = (uint32_t)sb.size();
  t->owned += sb;
}

// json.Unmarshal(payload, &map[string]interface{})  [R33, R35, R40]
bool claims_map(std::string_view payload, json::Value* out, std::string* err) {
  if (!json::parse(payload, out, err)) return false;
  if (out->is_null()) return true;
  if (out->kind != json::Value::Object) {
    static const char* names[] = {"null", "bool", "number", "string", "array", "object"};
    *err = std::string("json: cannot unmarshal ") + names[out->kind] + " into Go value of type map[string]interface {}";
    return false;
  }
  if (json::has_range_error(*out)) {
    *err = "json: cannot unmarshal number into Go value of type float64";
    return false;
  }
  return true;
}

jg_key to_jg(const PublicKey& k) {
  jg_key o{};
  switch (k.kind) {
    case PublicKey::RSA:
      o.kind = JG_KEY_RSA;
      o.n = (const uint8_t*)k.n.data();
      o.n_len = (int32_t)k.n.size();
      o.e = k.e;
      break;
    case PublicKey::EC:
      o.kind = JG_KEY_EC;
      o.curve = k.curve;
      o.x = (const uint8_t*)k.x.data();
      o.y = (const uint8_t*)k.y.data();
      o.coord_len = (int32_t)k.x.size();
      break;
    case PublicKey::Ed25519:
      o.kind = JG_KEY_ED25519;
      o.x = (const uint8_t*)k.x.data();
      o.coord_len = (int32_t)k.x.size();
      break;
    default:
      o.kind = 0;         // HMAC secret / private key / nothing: verifies no token on this path
  }
  return o;
}

int key_family(const PublicKey& k) {
  switch (k.kind) {
    case PublicKey::RSA: return JG_KEY_RSA;
    case PublicKey::EC: return JG_KEY_EC;
    case PublicKey::Ed25519: return k.x.size() == 32 ? JG_KEY_ED25519 : 0;
    default: return 0;
  }
}

// The GPU half shared by both key sets: parse, pack, verify.  `cand(t, push)`
// pushes the key indices to try for token t.  `keys_lock` (may be null) is the
// caller's lock on its key list, held from the first cand() call until the
// jobs are queued on the device and released there (jg_submit captures the
// device key table that the candidate indices refer to).
}  // namespace

// A batch after parse and device verification, before claims (KeySet::verify_raw)
struct Verified {
  ParArray<Tok> toks;
  std::vector<ByteArena> payloads;   // one per parse range
  std::vector<uint8_t> any;          // some candidate key verified
  // degraded path (SURVEY §5 failure row): when the device call fails (a HIP
  // error, a lost device) the tokens it carried are marked here and get
  // dev_err as their error -- no CPU verification, no exception out of the
  // batch; dev_seen = the engine's error count then (for Engine::recover)
  std::vector<uint8_t> failed;
  std::string dev_err;
  uint64_t dev_seen = 0;
  bool dev_failed = false;
  std::string miss_err;              // JWKS: the error of a parsed token no key verified
};

namespace {

template <class Cand>
void gpu_verify(Engine& eng, const std::vector<std::string_view>& tokens, Verified* V, Cand&& cand,
                const std::vector<size_t>* subset = nullptr, std::shared_lock<std::shared_mutex>* keys_lock = nullptr,
                const KeySet::Overlap* overlap = nullptr) {
  const size_t n = subset ? subset->size() : tokens.size();
  auto tok_index = [&](size_t i) { return subset ? (*subset)[i] : i; };
  auto release_keys = [&] {
    if (keys_lock && keys_lock->owns_lock()) keys_lock->unlock();
  };
  PhaseTimer pt("verify");
  const Chunks ch = make_chunks(n, eng.threads());
  if (!subset) {
    V->toks.init(tokens.size(), eng.threads());
    V->any.assign(tokens.size(), 0);
    V->failed.assign(tokens.size(), 0);
    V->payloads.resize(ch.count());
    run_chunks(ch, [&](size_t c, size_t lo, size_t hi) {
      // per thread and kept across batches: a coalesced single-token batch
      // finds its issuer's header decoded already (make_hdr is a pure function
      // of the segment; entries are immutable and shared)
      thread_local HdrCache cache;
      for (size_t i = lo; i < hi; ++i) parse_one(tokens[i], cache, V->payloads[c], &V->toks[i]);
    });
    pt.lap("parse");
  }
  // pass 1: candidate keys per token, arena bytes and jobs per range
  std::vector<uint64_t> rbytes(ch.count() + 1, 0), rjobs(ch.count() + 1, 0);
  run_chunks(ch, [&](size_t c, size_t lo, size_t hi) {
    std::vector<uint16_t> ks;
    uint64_t bytes = 0, jobs = 0;
    for (size_t i = lo; i < hi; ++i) {
      Tok& t = V->toks[tok_index(i)];
      ks.clear();
      if (t.verifiable) cand(t, ks);
      t.ncand = (uint32_t)ks.size();
      if (t.ncand) bytes += t.entry_len();
      jobs += t.ncand;
    }
    rbytes[c + 1] = bytes;
    rjobs[c + 1] = jobs;
  });
  for (size_t c = 0; c < ch.count(); ++c) {
    rbytes[c + 1] += rbytes[c];
    rjobs[c + 1] += rjobs[c];
  }
  const size_t total_jobs = rjobs[ch.count()];
  pt.lap("plan");
  if (total_jobs == 0) {
    release_keys();
    return;
  }
  const uint64_t arena_len = rbytes[ch.count()];
  Engine::Pinned arena = eng.pinned(arena_len);
  std::unique_ptr<jg_tok[]> jobs(new jg_tok[total_jobs]);      // filled below, not zeroed first
  std::unique_ptr<uint8_t[]> verdict(new uint8_t[total_jobs]);
  // pass 2: pack the arena and the jobs, each range from its own offsets
  run_chunks(ch, [&](size_t c, size_t lo, size_t hi) {
    std::vector<uint16_t> ks;
    uint64_t off = rbytes[c], jn = rjobs[c];
    for (size_t i = lo; i < hi; ++i) {
      Tok& t = V->toks[tok_index(i)];
      if (!t.ncand) continue;
      const size_t len = t.entry_len();
      std::memcpy(arena.get() + off, t.lit ? t.lit : t.owned.data(), len);
      ks.clear();
      cand(t, ks);
      t.job0 = jn;
      for (size_t k = 0; k < ks.size(); ++k) {
        jg_tok& j = jobs[jn + k];
        j.off = off;
        j.sig_in_len = t.si_len;
        j.sig_rel_off = t.si_len + 1;
        j.sig_b64_len = t.sig_b64_len;
        j.key_idx = ks[k];
        j.alg = (uint8_t)t.alg;
        j.flags = 0;
      }
      off += len;
      jn += ks.size();
    }
  });
  pt.lap("pack");
  try {
    eng.verify(arena.get(), arena_len, jobs.get(), total_jobs, verdict.get(), [&] {
      release_keys();
      if (overlap) {
        (*overlap)(*V);
        pt.lap("overlap");
      }
    });
  } catch (const DeviceError& e) {
    release_keys();
    V->dev_err = std::string("capjwt: signature verification unavailable: ") + e.what();
    V->dev_seen = eng.errors();
    V->dev_failed = true;
    run_chunks(ch, [&](size_t, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i)
        if (V->toks[tok_index(i)].ncand) V->failed[tok_index(i)] = 1;
    });
    return;
  }
  pt.lap("gpu");
  run_chunks(ch, [&](size_t, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const size_t ti = tok_index(i);
      const Tok& t = V->toks[ti];
      for (uint32_t k = 0; k < t.ncand; ++k)
        if (verdict[t.job0 + k] == JG_ACCEPT) V->any[ti] = 1;
    }
  });
  pt.lap("verdicts");
}

// After a batch whose device call failed: recreate the context so that the
// next call verifies again (Engine::recover; no key refetch)
void recover_after(Engine& eng, const Verified& V) {
  if (V.dev_failed) (void)eng.recover(V.dev_seen);
}

// ---------------------------------------------------------------- static key set
class StaticKeySet final : public KeySet {
 public:
  StaticKeySet(const std::vector<PublicKey>& keys, const std::vector<int>& devices) : keys_(keys), eng_(devices) {
    eng_.load(keys_);
    for (const auto& k : keys_) fam_.push_back(key_family(k));
  }
  void WaitTables() override { eng_.wait_tables(); }
  std::string DeviceStatus() override { return eng_.status(); }
  int DeviceRecoveries() override { return eng_.recoveries(); }
  int DebugFailVerify(int n) override { return eng_.debug_fail_verify(n); }
  // The key list never changes: no lock; concurrent calls pipeline on the device.
  std::shared_ptr<Verified> verify_raw(const std::vector<std::string_view>& tokens,
                                       const Overlap* overlap = nullptr) override {
    auto V = std::make_shared<Verified>();
    gpu_verify(eng_, tokens, V.get(), [&](const Tok& t, std::vector<uint16_t>& out) {
      // staticKeySet: every key in order (jwt/keyset.go:162-168); a key of
      // another family fails newVerifier/verifyPayload without arithmetic (R10)
      const int fam = alg_key_kind(t.alg);
      for (size_t k = 0; k < keys_.size(); ++k)
        if (fam_[k] == fam) out.push_back((uint16_t)k);
    }, nullptr, nullptr, overlap);
    recover_after(eng_, *V);
    return V;
  }
  void finish(const Verified& V, size_t i, Result& r) override {
    const Tok& t = V.toks[i];
    if (!t.parsed) {
      r.err = t.parse_err;                                           // jwt.ParseSigned error
    } else if (V.failed[i]) {
      r.err = V.dev_err;
    } else {
      std::string jerr;
      // parsedJWT.Claims(key, &allClaims): verify, then unmarshal; a JSON
      // error moves on to the next key, so it ends as "no known key"
      if (V.any[i] && claims_map(t.payload, &r.claims, &jerr)) {
        r.ok = true;
      } else {
        r.claims = json::Value();
        r.err = "no known key successfully validated the token signature";
      }
    }
  }
  void finish_pre(const Verified& V, size_t i, Result& r, bool json_ok) override {
    if (V.failed[i]) {
      r.claims = json::Value();
      r.err = V.dev_err;
    } else if (V.any[i] && json_ok) {
      r.err.clear();
      r.ok = true;
    } else {
      r.claims = json::Value();
      r.err = "no known key successfully validated the token signature";
    }
  }
  const char* trace_name() const override { return "static"; }

 private:
  std::vector<PublicKey> keys_;
  std::vector<int> fam_;
  Engine eng_;
};

// ---------------------------------------------------------------- JWKS key set (go-oidc v2.2.1 remoteKeySet)
bool ca_pem_ok(const std::string& pem) {
  // x509.CertPool.AppendCertsFromPEM: true iff at least one CERTIFICATE block parses
  std::string_view rest = pem;
  bool any = false;
  while (true) {
    const size_t b = rest.find("-----BEGIN CERTIFICATE-----");
    if (b == std::string_view::npos) break;
    const size_t e = rest.find("-----END CERTIFICATE-----", b);
    if (e == std::string_view::npos) break;
    const std::string_view block = rest.substr(b, e + 25 - b);
    std::string body;
    const size_t hs = block.find('\n');
    for (char c : block.substr(hs == std::string_view::npos ? 0 : hs, block.size() - 25 - (hs == std::string_view::npos ? 0 : hs)))
      if (c != ' ' && c != '\t' && c != '\r' && c != '\n') body.push_back(c);
    std::string der, err;
    PublicKey pk;
    if (b64std_decode(body, &der) && parse_certificate_public_key(der, &pk, &err)) any = true;
    rest = rest.substr(e + 25);
  }
  return any;
}

class JSONWebKeySet final : public KeySet {
 public:
  JSONWebKeySet(std::string url, std::string ca, Fetcher f, const std::vector<int>& devices)
      : url_(std::move(url)), ca_(std::move(ca)), fetch_(std::move(f)), eng_(devices) {}

  void WaitTables() override { eng_.wait_tables(); }
  std::string DeviceStatus() override { return eng_.status(); }
  int DeviceRecoveries() override { return eng_.recoveries(); }
  int DebugFailVerify(int n) override { return eng_.debug_fail_verify(n); }
  std::shared_ptr<Verified> verify_raw(const std::vector<std::string_view>& tokens,
                                       const Overlap* overlap = nullptr) override {
    auto V = std::make_shared<Verified>();
    remote_verify(tokens, V.get(), &V->miss_err, overlap);
    return V;
  }
  void finish(const Verified& V, size_t i, Result& r) override {
    const Tok& t = V.toks[i];
    if (!t.parsed) {
      r.err = "oidc: malformed jwt: " + t.parse_err;
    } else if (V.failed[i]) {
      r.err = V.dev_err;
    } else if (!V.any[i]) {
      r.err = V.miss_err;
    } else {
      std::string jerr;       // jsonWebKeySet.VerifySignature: json.Unmarshal(payload)
      if (claims_map(t.payload, &r.claims, &jerr)) r.ok = true;
      else { r.claims = json::Value(); r.err = jerr; }
    }
  }
  void finish_pre(const Verified& V, size_t i, Result& r, bool json_ok) override {
    if (V.failed[i]) {
      r.claims = json::Value();
      r.err = V.dev_err;
    } else if (!V.any[i]) {
      r.claims = json::Value();
      r.err = V.miss_err;
    } else if (json_ok) {
      r.err.clear();
      r.ok = true;
    } else {
      r.claims = json::Value();                  // r.err: the JSON error
    }
  }
  const char* trace_name() const override { return "jwks"; }

  // go-oidc remoteKeySet.VerifySignature itself: token i's verified payload bytes
  static PayloadResult payload_result(const Verified& V, size_t i) {
    PayloadResult r;
    const Tok& t = V.toks[i];
    if (!t.parsed) r.err = "oidc: malformed jwt: " + t.parse_err;
    else if (V.failed[i]) r.err = V.dev_err;
    else if (!V.any[i]) r.err = V.miss_err;
    else { r.ok = true; r.payload = std::string(t.payload); }
    return r;
  }
  std::vector<PayloadResult> verify_payload_batch(const std::vector<std::string_view>& tokens) {
    auto V = verify_raw(tokens);
    std::vector<PayloadResult> res(tokens.size());
    parallel_for(tokens.size(), eng_.threads(), [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) res[i] = payload_result(*V, i);
    });
    return res;
  }

 private:
  // remoteKeySet.verify over a batch: kid-filtered keys from the cache, then
  // (for the tokens that missed) one refresh if the cache has expired and a
  // retry.  *miss_err = the error every unverified, parsed token gets.
  //
  // Concurrency: the key list (keys_, fam_) is read under a shared lock from
  // candidate selection until the jobs are queued (gpu_verify), and replaced
  // under the exclusive lock by refresh() -- a refresh never waits for a device
  // call, and no call's jobs can name a key of a list the device does not hold.
  // Refreshes are serialised.  As in go-oidc, the expiry a call tests is the
  // one it read with the cached keys; a call that needs remote keys while
  // another call's refresh completed since its read takes that refresh's
  // outcome (go-oidc's keysFromRemote shares an in-flight request the same way).
  void remote_verify(const std::vector<std::string_view>& tokens, Verified* V, std::string* miss_err,
                     const Overlap* overlap) {
    auto cand = [&](const Tok& t, std::vector<uint16_t>& out) {
      // remoteKeySet.verify: keyID == "" || key.KeyID == keyID   [R31, R34]
      const int fam = alg_key_kind(t.alg);
      for (size_t k = 0; k < keys_.size(); ++k)
        if ((t.kid.empty() || keys_[k].kid == t.kid) && fam_[k] == fam) out.push_back((uint16_t)k);
    };
    uint64_t seen_refreshes;
    int64_t seen_expiry;
    bool seen_have;
    {
      std::shared_lock<std::shared_mutex> lk(keys_mu_);
      seen_refreshes = refreshes_;
      seen_expiry = expiry_ns_;
      seen_have = have_keys_;
      if (have_keys_) gpu_verify(eng_, tokens, V, cand, nullptr, &lk, overlap);
      else gpu_verify(eng_, tokens, V, [](const Tok&, std::vector<uint16_t>&) {}, nullptr, &lk, overlap);
    }
    recover_after(eng_, *V);
    // tokens that parsed but did not verify: refresh once if the cache has
    // expired (now + keysExpiryDelta(30s) after expiry), then retry them.  A
    // token whose device call failed is no miss: it keeps the device error and
    // triggers no refetch
    std::vector<size_t> miss;
    for (size_t i = 0; i < tokens.size(); ++i)
      if (V->toks[i].parsed && !V->any[i] && !V->failed[i]) miss.push_back(i);
    std::string fetch_err;
    bool refreshed = false;
    if (!miss.empty() && (!seen_have || wall_now_ns() + 30 * kSecond > seen_expiry)) {
      refreshed = true;
      std::lock_guard<std::mutex> rg(refresh_mu_);
      bool ok;
      if (refreshes_ != seen_refreshes) {            // joined a refresh that completed meanwhile
        ok = last_refresh_ok_;
        fetch_err = last_fetch_err_;
      } else {
        ok = refresh(&fetch_err);
        std::unique_lock<std::shared_mutex> lk(keys_mu_);
        ++refreshes_;
        last_refresh_ok_ = ok;
        last_fetch_err_ = fetch_err;
      }
      if (ok) {
        std::shared_lock<std::shared_mutex> lk(keys_mu_);
        gpu_verify(eng_, tokens, V, cand, &miss, &lk);
      }
    }
    recover_after(eng_, *V);
    *miss_err = refreshed && !fetch_err.empty() ? "fetching keys " + fetch_err : "failed to verify id token signature";
  }

  // go-oidc updateKeys; the caller holds refresh_mu_
  bool refresh(std::string* err) {
    FetchResponse resp;
    try {
      resp = fetch_(url_, ca_);
    } catch (const std::exception& e) {
      *err = std::string("oidc: get keys failed ") + e.what();
      return false;
    }
    if (resp.status != 200) {
      *err = "oidc: get keys failed: " + resp.status_text + " " + resp.body;
      return false;
    }
    const int64_t expiry = wall_now_ns() + (resp.max_age_s > 0 ? resp.max_age_s * kSecond : 0);
    // an unchanged document (the usual refresh-on-miss answer for a tampered
    // token): the cached keys stand as they are -- no decode, no device work
    {
      std::unique_lock<std::shared_mutex> lk(keys_mu_);
      if (have_keys_ && resp.body == body_) {
        expiry_ns_ = expiry;
        return true;
      }
    }
    std::vector<JSONWebKey> keys;
    std::string derr;
    if (!jwks_decode(resp.body, &keys, &derr)) {
      *err = "oidc: failed to decode keys: " + derr + " " + resp.body;
      return false;
    }
    if (keys.size() > 65535) { *err = "oidc: too many keys"; return false; }
    // the new key list is committed only once the device table holds it: a
    // failed staging keeps the previous cache, as go-oidc keeps its cached
    // keys when updateKeys fails
    std::vector<PublicKey> pk;
    std::vector<int> fam;
    for (const auto& k : keys) {
      pk.push_back(k.key);
      fam.push_back(key_family(k.key));
    }
    std::unique_lock<std::shared_mutex> lk(keys_mu_);
    try {
      eng_.load(pk);
    } catch (const std::exception& e) {
      *err = std::string("oidc: failed to stage keys: ") + e.what();
      return false;
    }
    fam_ = std::move(fam);
    keys_ = std::move(keys);
    body_ = std::move(resp.body);
    have_keys_ = true;
    expiry_ns_ = expiry;
    return true;
  }

  std::string url_, ca_;
  Fetcher fetch_;
  Engine eng_;
  std::shared_mutex keys_mu_;     // keys_, fam_, body_, have_keys_, expiry_ns_, refreshes_, last_*
  std::mutex refresh_mu_;         // one refresh at a time
  std::vector<JSONWebKey> keys_;
  std::vector<int> fam_;
  std::string body_;              // the JWKS document keys_ came from
  bool have_keys_ = false;
  int64_t expiry_ns_ = 0;
  uint64_t refreshes_ = 0;        // refresh attempts completed
  bool last_refresh_ok_ = false;  // ... and the last one's outcome
  std::string last_fetch_err_;
};

// ---------------------------------------------------------------- Go time arithmetic
constexpr int64_t kUnixToInternal = 62135596800LL;   // time.unixToInternal
struct GoTime {
  int64_t sec;     // seconds since year 1 (Time.ext without monotonic)
  int64_t nsec;    // [0, 1e9)
};
GoTime go_now(int64_t unix_ns) {
  int64_t s = unix_ns / kSecond, ns = unix_ns % kSecond;
  if (ns < 0) { ns += kSecond; --s; }
  return {s + kUnixToInternal, ns};
}
GoTime go_add(GoTime t, int64_t d) {                  // Time.Add
  int64_t dsec = d / kSecond;
  int64_t nsec = t.nsec + d % kSecond;
  if (nsec >= kSecond) { ++dsec; nsec -= kSecond; }
  else if (nsec < 0) { --dsec; nsec += kSecond; }
  const int64_t sum = (int64_t)((uint64_t)t.sec + (uint64_t)dsec);
  if ((sum > t.sec) == (dsec > 0)) t.sec = sum;
  else if (dsec > 0) t.sec = INT64_MAX;
  else t.sec = -INT64_MAX;
  t.nsec = nsec;
  return t;
}
GoTime go_unix(int64_t sec) { return {(int64_t)((uint64_t)sec + (uint64_t)kUnixToInternal), 0}; }   // time.Unix(sec, 0)
bool go_before(GoTime a, GoTime b) { return a.sec < b.sec || (a.sec == b.sec && a.nsec < b.nsec); }
bool go_after(GoTime a, GoTime b) { return a.sec > b.sec || (a.sec == b.sec && a.nsec > b.nsec); }

double dur_seconds(int64_t d) {                       // time.Duration.Seconds
  const int64_t s = d / kSecond, ns = d % kSecond;
  return (double)s + (double)ns / 1e9;
}
int64_t go_f64_to_i64(double f) {                     // int64(f) on amd64 (CVTTSD2SQ)
  if (std::isnan(f) || f >= 9223372036854775808.0 || f < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)f;
}

// encoding/json field matching: fold(key) == fold(field name) (Go 1.21 foldName)
bool fold_eq(const std::string& key, const char* upper_field) {
  const unsigned char* p = (const unsigned char*)key.data();
  size_t i = 0, j = 0;
  const size_t n = key.size(), m = std::strlen(upper_field);
  while (i < n) {
    if (j >= m) return false;
    uint32_t r;
    size_t w;
    r = json::decode_rune(p + i, n - i, &w);
    if (r >= 'a' && r <= 'z') r -= 32;
    else if (r == 0x17F) r = 'S';          // LATIN SMALL LETTER LONG S folds to S
    else if (r == 0x212A) r = 'K';         // KELVIN SIGN folds to K
    if (r != (unsigned char)upper_field[j]) return false;
    i += w;
    ++j;
  }
  return j == m;
}

}  // namespace

// ====================================================================== Engine
Engine::Engine(const std::vector<int>& devices) : devices_(devices) {
  ctx_ = jg_create(devices.empty() ? nullptr : devices.data(), (int)devices.size());
  if (!ctx_) throw std::runtime_error(std::string("capjwt: no GPU verifier: ") + jg_last_error(nullptr));
  threads_ = host_threads();
}

Engine::~Engine() {
  for (auto& b : pin_free_) jg_host_free(b.first);
  if (ctx_) jg_destroy(ctx_);
}

void Engine::wait_tables() {
  std::shared_lock<std::shared_mutex> life(life_);
  if (ctx_) (void)jg_keys_wait_tables(ctx_);
}

void Engine::load(const std::vector<PublicKey>& keys) {
  std::vector<jg_key> jk;
  jk.reserve(keys.size());
  for (const auto& k : keys) jk.push_back(to_jg(k));
  std::shared_lock<std::shared_mutex> life(life_);
  std::lock_guard<std::mutex> g(load_mu_);
  if (!ctx_) throw DeviceError("capjwt: device lost: " + lost_);
  const int rc = jg_keys_load(ctx_, jk.data(), (int)jk.size());
  if (rc != 0) throw std::runtime_error(std::string("capjwt: jg_keys_load: ") + jg_last_error(ctx_));
  keys_ = keys;
  has_keys_ = true;
}

Engine::Pinned Engine::pinned(size_t bytes) {
  bytes = std::max<size_t>(bytes, 1);
  {
    std::lock_guard<std::mutex> g(pin_mu_);
    // the smallest free block that holds it
    size_t best = pin_free_.size();
    for (size_t i = 0; i < pin_free_.size(); ++i)
      if (pin_free_[i].second >= bytes && (best == pin_free_.size() || pin_free_[i].second < pin_free_[best].second))
        best = i;
    if (best < pin_free_.size()) {
      auto b = pin_free_[best];
      pin_free_.erase(pin_free_.begin() + (std::ptrdiff_t)best);
      return Pinned(this, b.first, b.second);
    }
  }
  // 64 KiB granules, 1/8 headroom: a stream of similar batches reuses one block
  const size_t cap = ((bytes + bytes / 8) + 65535) & ~size_t(65535);
  uint8_t* p = (uint8_t*)jg_host_alloc(cap);
  if (!p) throw std::runtime_error("capjwt: pinned host allocation failed");
  return Pinned(this, p, cap);
}

Engine::Pinned::~Pinned() {
  if (!p_) return;
  std::lock_guard<std::mutex> g(e_->pin_mu_);
  // keep a few blocks (one per concurrent call, typically); drop the smallest beyond that
  e_->pin_free_.emplace_back(p_, cap_);
  if (e_->pin_free_.size() > 4) {
    auto it = std::min_element(e_->pin_free_.begin(), e_->pin_free_.end(),
                               [](const auto& x, const auto& y) { return x.second < y.second; });
    jg_host_free(it->first);
    e_->pin_free_.erase(it);
  }
}

void Engine::fail_device(const std::string& what) {
  errors_.fetch_add(1);
  throw DeviceError(what);
}

void Engine::verify(const uint8_t* arena, size_t arena_len, const void* jobs, size_t njobs, uint8_t* verdicts,
                    const std::function<void()>& submitted) {
  // a lost context: try to recreate it (at most once a second) before failing
  bool lost;
  uint64_t seen;
  {
    std::shared_lock<std::shared_mutex> life(life_);
    lost = ctx_ == nullptr;
    seen = errors_.load();
  }
  if (lost) {
    bool retry;
    {
      std::unique_lock<std::shared_mutex> life(life_);
      retry = std::chrono::steady_clock::now() - last_try_ > std::chrono::seconds(1);
    }
    if (retry) (void)recover(seen + 1);
  }
  std::shared_lock<std::shared_mutex> life(life_);
  if (!ctx_) {
    if (submitted) submitted();
    fail_device("capjwt: device lost: " + lost_);
  }
  jg_ticket* t = nullptr;
  const int rc = jg_submit(ctx_, arena, arena_len, (const jg_tok*)jobs, njobs, verdicts, &t);
  if (submitted) {
    // the device worker reads `jobs` and the arena and writes `verdicts` until
    // jg_wait returns: an exception from the overlapped host work must not
    // unwind the caller's buffers (or return a pooled arena) before that
    try {
      submitted();
    } catch (...) {
      if (rc == 0) (void)jg_wait(ctx_, t);
      throw;
    }
  }
  if (rc == -1) throw std::logic_error(std::string("capjwt: jg_submit rejected the host's jobs: ") + jg_last_error(ctx_));
  if (rc != 0) fail_device(std::string("capjwt: jg_verify_batch: ") + jg_last_error(ctx_));
  const int wc = jg_wait(ctx_, t);
  if (wc == -1) throw std::logic_error(std::string("capjwt: jg_wait rejected the host's jobs: ") + jg_last_error(ctx_));
  if (wc != 0) fail_device(std::string("capjwt: jg_verify_batch: ") + jg_last_error(ctx_));
}

bool Engine::recover(uint64_t seen) {
  std::unique_lock<std::shared_mutex> life(life_);
  if (recovered_at_ >= seen && ctx_) return true;          // already recovered since that error
  last_try_ = std::chrono::steady_clock::now();
  if (ctx_) jg_destroy(ctx_);                              // its streams, workers, staged tables
  ctx_ = jg_create(devices_.empty() ? nullptr : devices_.data(), (int)devices_.size());
  recovered_at_ = errors_.load();
  if (!ctx_) {
    lost_ = std::string("jg_create: ") + jg_last_error(nullptr);
    return false;
  }
  if (has_keys_) {
    std::vector<jg_key> jk;
    jk.reserve(keys_.size());
    for (const auto& k : keys_) jk.push_back(to_jg(k));
    if (jg_keys_load(ctx_, jk.data(), (int)jk.size()) != 0) {
      lost_ = std::string("jg_keys_load: ") + jg_last_error(ctx_);
      jg_destroy(ctx_);
      ctx_ = nullptr;
      return false;
    }
  }
  lost_.clear();
  recoveries_.fetch_add(1);
  return true;
}

std::string Engine::status() {
  std::shared_lock<std::shared_mutex> life(life_);
  return ctx_ ? std::string() : lost_.empty() ? std::string("device lost") : lost_;
}

int Engine::debug_fail_verify(int n) {
  std::shared_lock<std::shared_mutex> life(life_);
  return ctx_ ? jg_debug_fail_verify(ctx_, n) : -1;
}

// ====================================================================== request coalescing
// Concurrent single-token calls (VerifySignature / Validate) become device
// batches.  A caller pushes its request onto a lock-free stack.  If fewer than
// max_inflight batches are being carried, the caller itself takes everything
// pushed so far (one exchange) and carries it as one batch (parse + device
// verification) -- an idle key set verifies a lone token with no thread
// hand-off; otherwise it sleeps on its own state word.  Dispatcher threads
// (max_inflight of them) serve what the callers leave: whoever finishes a
// batch and finds the stack non-empty wakes one, so pending requests never
// wait for a caller.  Batches pipeline on the device up to max_inflight deep
// and grow with the load.
//
// No lock is taken per call.  A first version (a queue under one mutex, the
// callers leading batches in turn) lost 20x at 1024 callers on a box with 256
// CPUs and a 16-CPU cgroup quota: 243 us of system time per call, the quota
// throttled for most of every period (profiles/r05_s2/session_c.log); the same
// code pinned to 16 CPUs ran 1.2 M calls/s.
namespace {
// process-private futex on a 32-bit word
void futex_wait(void* w, uint32_t expect) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, expect, nullptr, nullptr, 0);
}
void futex_wake(void* w, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}
}  // namespace

Coalescer::~Coalescer() {
  std::lock_guard<std::mutex> g(threads_mu_);
  stop_locked();
}

void Coalescer::start_locked() {
  stop_.store(false);
  for (int i = 0; i < cfg_.max_inflight; ++i) threads_.emplace_back([this] { dispatch_loop(); });
  started_.store(true, std::memory_order_release);
}

void Coalescer::stop_locked() {
  if (threads_.empty()) return;
  stop_.store(true);
  seq_.fetch_add(1);
  futex_wake(&seq_, INT_MAX);
  for (auto& t : threads_) t.join();
  threads_.clear();
  started_.store(false);
}

void Coalescer::configure(const CoalesceConfig& c) {
  std::lock_guard<std::mutex> g(threads_mu_);
  cfg_ = c;
  cfg_.max_inflight = std::max(1, cfg_.max_inflight);
  cfg_.max_batch = std::max<size_t>(1, cfg_.max_batch);
  cfg_.window_us = std::max<int64_t>(0, cfg_.window_us);
  max_batch_.store(cfg_.max_batch);
  window_us_.store(cfg_.window_us);
  max_inflight_.store(cfg_.max_inflight);
  if (!threads_.empty()) {        // restart with the new count (requests pushed meanwhile wait on the stack)
    stop_locked();
    start_locked();
    kick();
    futex_wake(&seq_, INT_MAX);
  }
}

void Coalescer::kick() {
  seq_.fetch_add(1, std::memory_order_seq_cst);
  futex_wake(&seq_, 1);
}

CoalesceConfig Coalescer::config() {
  std::lock_guard<std::mutex> g(threads_mu_);
  return cfg_;
}

Coalescer::Stats Coalescer::stats() {
  Stats s;
  s.calls = calls_.load();
  s.batches = batches_.load();
  s.max_batch_seen = max_seen_.load();
  return s;
}

// Wake position i of a finished batch's wake-up list
void Coalescer::release(const std::vector<Req*>& wake, size_t i) {
  if (i >= wake.size()) return;
  Req* x = wake[i];
  x->state.store(Req::DONE, std::memory_order_release);
  futex_wake(&x->state, 1);                      // x may be touched no more after this (its owner returns)
}

void Coalescer::run(Req* r) {
  if (!started_.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> g(threads_mu_);
    if (threads_.empty()) start_locked();
  }
  calls_.fetch_add(1, std::memory_order_relaxed);
  Req* h = head_.load(std::memory_order_relaxed);
  do {
    r->next = h;
  } while (!head_.compare_exchange_weak(h, r, std::memory_order_seq_cst, std::memory_order_relaxed));
  if (active_.fetch_add(1, std::memory_order_seq_cst) < max_inflight_.load(std::memory_order_relaxed)) {
    // a free slot: carry everything pushed so far (normally this request too)
    thread_local std::vector<Req*> all, batch;
    serve_stack(all, batch);
    active_.fetch_sub(1, std::memory_order_seq_cst);
    if (head_.load(std::memory_order_seq_cst)) kick();   // what arrived meanwhile: a dispatcher takes it
  } else {
    // every slot busy: whoever finishes a batch finds this request on the stack
    // (the push precedes this caller's view of the slots, which precedes the
    // holder's release, which precedes the holder's look at the stack -- all
    // sequentially consistent).  But the dispatcher that holder kicks may
    // itself be refused by this caller's brief increment and go back to
    // sleep; so if this decrement leaves a slot free while requests wait, kick
    // again.  With every slot truly busy (the heavy-load case) no kick: one
    // futex call per request from 1024 callers cost 25 s of system time per
    // 131 k calls on the box.
    const int prev = active_.fetch_sub(1, std::memory_order_seq_cst);
    if (prev - 1 < max_inflight_.load(std::memory_order_relaxed) && head_.load(std::memory_order_seq_cst)) kick();
  }
  int st;
  while ((st = r->state.load(std::memory_order_acquire)) != Req::DONE) futex_wait(&r->state, (uint32_t)st);
  // carried by a batch: wake this caller's two children in its wake-up tree
  auto peers = std::move(r->peers);
  release(*peers, 2 * r->wpos + 1);
  release(*peers, 2 * r->wpos + 2);
  if (r->ex) std::rethrow_exception(r->ex);
}

void Coalescer::serve_stack(std::vector<Req*>& all, std::vector<Req*>& batch) {
  const int64_t win = window_us_.load(std::memory_order_relaxed);
  if (win > 0) std::this_thread::sleep_for(std::chrono::microseconds(win));
  Req* list = head_.exchange(nullptr, std::memory_order_acquire);
  all.clear();
  for (Req* p = list; p; p = p->next) all.push_back(p);
  std::reverse(all.begin(), all.end());          // oldest first
  const size_t mb = max_batch_.load(std::memory_order_relaxed);
  for (size_t lo = 0; lo < all.size(); lo += mb) {
    batch.assign(all.begin() + (std::ptrdiff_t)lo, all.begin() + (std::ptrdiff_t)std::min(all.size(), lo + mb));
    carry(batch);
  }
}

void Coalescer::dispatch_loop() {
  pthread_setname_np(pthread_self(), "capjwt-batch");
  std::vector<Req*> all, batch;
  while (!stop_.load()) {
    // seq_ is read before the stack and the slots: a kick after this read
    // makes the futex_wait below return at once
    const uint32_t s = seq_.load(std::memory_order_seq_cst);
    if (!head_.load(std::memory_order_seq_cst)) {
      futex_wait(&seq_, s);
      continue;
    }
    if (active_.fetch_add(1, std::memory_order_seq_cst) >= max_inflight_.load(std::memory_order_relaxed)) {
      // every slot busy: the holder kicks when done.  A slot seen busy only
      // through another thread's brief increment is free by now: look again
      // instead of sleeping through the kick that thread may already have sent
      const int prev = active_.fetch_sub(1, std::memory_order_seq_cst);
      if (prev - 1 < max_inflight_.load(std::memory_order_relaxed)) {
        std::this_thread::yield();
        continue;
      }
      futex_wait(&seq_, s);
      continue;
    }
    serve_stack(all, batch);
    active_.fetch_sub(1, std::memory_order_seq_cst);
  }
}

// Run one batch and wake its callers
void Coalescer::carry(std::vector<Req*>& batch) {
  batches_.fetch_add(1, std::memory_order_relaxed);
  uint64_t m = max_seen_.load(std::memory_order_relaxed);
  while (batch.size() > m && !max_seen_.compare_exchange_weak(m, batch.size())) {
  }
  std::exception_ptr ex;
  std::shared_ptr<const Verified> V;
  try {
    std::vector<std::string_view> toks;
    toks.reserve(batch.size());
    for (Req* x : batch) toks.push_back(x->tok);
    V = exec_(toks);
  } catch (...) {
    ex = std::current_exception();
  }
  // the callers wake as a binary tree: the dispatcher wakes the first, each
  // woken caller its own two -- log2(batch) rounds of wake-ups
  auto wake = std::make_shared<std::vector<Req*>>(batch);
  for (size_t i = 0; i < batch.size(); ++i) {
    Req* x = batch[i];
    x->batch = V;
    x->idx = i;
    x->ex = ex;                                  // a host-side bug in the batch reaches every caller in it
    x->wpos = i;
    x->peers = wake;
  }
  release(*wake, 0);
}

// ====================================================================== KeySet
KeySet::KeySet()
    : co_([this](const std::vector<std::string_view>& toks) -> std::shared_ptr<const Verified> {
        return verify_raw(toks);
      }) {}

Results KeySet::verify_batch(const std::vector<std::string_view>& tokens, const PostFn* post) {
  const int th = host_threads();
  Results res(tokens.size(), th);
  // Claims maps are read -- and, with a post step (Validator's claim checks),
  // checked -- while the device verifies (Overlap): a parsed token's payload
  // is JSON-decoded before its verdict is known, and the result of a token no
  // key verifies is replaced afterwards.  pre[i]: 0 not read (finish reads
  // it), 1 read, 2 JSON error (the message in res[i].err), 3 read and post-
  // processed as if verified (kept iff it was).
  std::vector<uint8_t> pre(tokens.size(), 0);
  const Overlap overlap = [&](const Verified& V) {
    parallel_for(tokens.size(), th, [&](size_t lo, size_t hi) {
      auto arena = std::make_unique<json::Arena>();   // this range's claims trees (owned by res)
      json::ArenaScope scope(arena.get());
      res.adopt(std::move(arena));
      std::string jerr;
      for (size_t i = lo; i < hi; ++i) {
        const Tok& t = V.toks[i];
        if (!t.parsed) continue;
        if (claims_map(t.payload, &res[i].claims, &jerr)) {
          pre[i] = 1;
          if (post) {
            res[i].ok = true;
            (*post)(i, res[i], t.view());
            pre[i] = 3;
          }
        } else {
          res[i].claims = json::Value();
          res[i].err = jerr;
          pre[i] = 2;
        }
      }
    });
  };
  std::shared_ptr<Verified> V = verify_raw(tokens, &overlap);
  PhaseTimer pt(trace_name());
  parallel_for(tokens.size(), th, [&](size_t lo, size_t hi) {
    auto arena = std::make_unique<json::Arena>();   // this range's claims trees (owned by res)
    json::ArenaScope scope(arena.get());
    res.adopt(std::move(arena));
    for (size_t i = lo; i < hi; ++i) {
      if (pre[i] == 3) {
        if (!V->failed[i] && V->any[i]) continue;            // verified: the checked result stands
        res[i] = Result();
        finish_pre(*V, i, res[i], true);
      } else if (pre[i]) {
        finish_pre(*V, i, res[i], pre[i] == 1);
      } else {
        finish(*V, i, res[i]);
      }
      if (post) (*post)(i, res[i], V->toks[i].view());
    }
  });
  pt.lap("payload-json");
  V->toks.release();
  pt.lap("free-toks");
  return res;
}

// One token of a coalesced batch: the leader ran parse + device verify for
// everyone; the claims map is built here, on the caller's own thread, straight
// into heap storage (it leaves the batch with the caller)
Result KeySet::VerifySignature(std::string_view token) {
  Coalescer::Req q;
  q.tok = token;
  co_.run(&q);
  Result r;
  finish(*q.batch, q.idx, r);
  return r;
}

Result KeySet::verify_one(std::string_view token, TokenInfo* info) {
  Coalescer::Req q;
  q.tok = token;
  co_.run(&q);
  Result r;
  finish(*q.batch, q.idx, r);
  const TokenView t = q.batch->toks[q.idx].view();
  info->parsed = t.parsed;
  info->parse_err = std::string(t.parse_err);
  info->nsigs = t.nsigs;
  info->sig0_len = t.sig0_len;
  info->alg = std::string(t.alg);
  return r;
}

Results KeySet::VerifySignatureBatch(const std::vector<std::string_view>& tokens) {
  return verify_batch(tokens, nullptr);
}

std::unique_ptr<KeySet> NewStaticKeySet(const std::vector<PublicKey>& keys, std::string* err,
                                        const std::vector<int>& devices) {
  if (keys.empty()) { *err = "publicKeys must not be empty"; return nullptr; }
  if (keys.size() > 65535) { *err = "at most 65535 keys"; return nullptr; }
  return std::make_unique<StaticKeySet>(keys, devices);
}

std::unique_ptr<KeySet> NewJSONWebKeySet(const std::string& jwks_url, const std::string& jwks_ca_pem, Fetcher fetch,
                                         std::string* err, const std::vector<int>& devices) {
  if (jwks_url.empty()) { *err = "jwksURL must not be empty"; return nullptr; }
  if (!jwks_ca_pem.empty() && !ca_pem_ok(jwks_ca_pem)) { *err = "could not parse CA PEM value successfully"; return nullptr; }
  return std::make_unique<JSONWebKeySet>(jwks_url, jwks_ca_pem, std::move(fetch), devices);
}

// go-oidc's oidc.KeySet over the same GPU JWKS machinery
class RemoteKeySet::Impl {
 public:
  Impl(const std::string& url, Fetcher f, const std::vector<int>& devices)
      : ks(url, "", std::move(f), devices),
        co([this](const std::vector<std::string_view>& toks) -> std::shared_ptr<const Verified> {
          return ks.verify_raw(toks);
        }) {}
  JSONWebKeySet ks;
  Coalescer co;
};
RemoteKeySet::RemoteKeySet(const std::string& jwks_url, Fetcher fetch, const std::vector<int>& devices)
    : impl_(std::make_unique<Impl>(jwks_url, std::move(fetch), devices)) {}
RemoteKeySet::~RemoteKeySet() = default;
PayloadResult RemoteKeySet::VerifySignature(std::string_view jwt) {
  Coalescer::Req q;
  q.tok = jwt;
  impl_->co.run(&q);
  return JSONWebKeySet::payload_result(*q.batch, q.idx);
}
std::vector<PayloadResult> RemoteKeySet::VerifySignatureBatch(const std::vector<std::string_view>& jwts) {
  return impl_->ks.verify_payload_batch(jwts);
}
void RemoteKeySet::SetCoalescing(const CoalesceConfig& c) { impl_->co.configure(c); }
std::unique_ptr<RemoteKeySet> NewRemoteKeySet(const std::string& jwks_url, Fetcher fetch,
                                              const std::vector<int>& devices) {
  return std::make_unique<RemoteKeySet>(jwks_url, std::move(fetch), devices);
}

std::unique_ptr<KeySet> NewOIDCDiscoveryKeySet(const std::string& issuer, const std::string& issuer_ca_pem,
                                               Fetcher fetch, std::string* err, const std::vector<int>& devices) {
  // jwt/keyset.go:49-104
  if (issuer.empty()) { *err = "issuer must not be empty"; return nullptr; }
  if (!issuer_ca_pem.empty() && !ca_pem_ok(issuer_ca_pem)) { *err = "could not parse CA PEM value successfully"; return nullptr; }
  std::string base = issuer;
  if (!base.empty() && base.back() == '/') base.pop_back();          // strings.TrimSuffix(issuer, "/")
  FetchResponse resp;
  try {
    resp = fetch(base + "/.well-known/openid-configuration", issuer_ca_pem);
  } catch (const std::exception& e) {
    *err = e.what();
    return nullptr;
  }
  if (resp.status != 200) { *err = resp.status_text + ": " + resp.body; return nullptr; }
  json::Value doc;
  std::string jerr;
  std::string iss, jwks;
  bool ok = json::parse(resp.body, &doc, &jerr);
  if (ok && !doc.is_null() && doc.kind != json::Value::Object) { ok = false; jerr = "json: cannot unmarshal into struct"; }
  if (ok && doc.kind == json::Value::Object) {
    // encoding/json into struct { Issuer `json:"issuer"`; JWKSURL `json:"jwks_uri"` }
    for (const auto& m : doc.obj) {
      std::string* dst = fold_eq(m.first, "ISSUER") ? &iss : fold_eq(m.first, "JWKS_URI") ? &jwks : nullptr;
      if (!dst || m.second.is_null()) continue;
      if (m.second.kind != json::Value::String) { ok = false; jerr = "json: cannot unmarshal into string"; break; }
      *dst = m.second.str;
    }
  }
  if (!ok) {
    // unmarshalResp (jwt/keyset.go:229-241)
    std::string media = resp.content_type.substr(0, resp.content_type.find(';'));
    while (!media.empty() && media.back() == ' ') media.pop_back();
    for (auto& c : media) c = (char)std::tolower((unsigned char)c);
    if (media == "application/json")
      *err = "failed to decode OIDC discovery document: got Content-Type = application/json, but could not unmarshal as JSON: " + jerr;
    else
      *err = "failed to decode OIDC discovery document: expected Content-Type = application/json, got \"" +
             resp.content_type + "\": " + jerr;
    return nullptr;
  }
  if (iss != issuer) {
    *err = "issuer did not match the returned issuer, expected \"" + issuer + "\" got \"" + iss + "\"";
    return nullptr;
  }
  return std::make_unique<JSONWebKeySet>(jwks, issuer_ca_pem, std::move(fetch), devices);
}

bool ParsePublicKeyPEM(std::string_view data, PublicKey* out, std::string* err) {
  return parse_public_key_pem(data, out, err);
}

// ====================================================================== Validator
std::unique_ptr<Validator> NewValidator(KeySet* ks, std::string* err) {
  if (!ks) { *err = "keySet must not be nil"; return nullptr; }
  return std::make_unique<Validator>(ks);
}

namespace {
// The jwt.Claims field a claims-map member lands in under encoding/json's
// case-insensitive matching (fold_eq).  Every field name is 3 letters: a
// 3-byte ASCII key is matched by upper-casing it; a key with non-ASCII runes
// (the 'ſ' and Kelvin-sign foldings) takes fold_eq.
enum ClaimField { F_NONE, F_ISS, F_SUB, F_JTI, F_AUD, F_EXP, F_NBF, F_IAT };
ClaimField claim_field(const std::string& key) {
  static const char* const names[] = {"", "ISS", "SUB", "JTI", "AUD", "EXP", "NBF", "IAT"};
  const size_t n = key.size();
  if (n < 3 || n > 9) return F_NONE;         // 3 runes of 1..3 bytes
  if (n == 3) {
    char u[3];
    for (int i = 0; i < 3; ++i) {
      const unsigned char c = (unsigned char)key[i];
      if (c >= 0x80) return F_NONE;          // a multi-byte rune cannot fit 3 bytes with 2 more
      u[i] = (char)(c >= 'a' && c <= 'z' ? c - 32 : c);
    }
    for (int f = F_ISS; f <= F_IAT; ++f)
      if (u[0] == names[f][0] && u[1] == names[f][1] && u[2] == names[f][2]) return (ClaimField)f;
    return F_NONE;
  }
  for (int f = F_ISS; f <= F_IAT; ++f)
    if (fold_eq(key, names[f])) return (ClaimField)f;
  return F_NONE;
}
}  // namespace

Result validate_claims(const json::Value& all_claims, const TokenInfo& info, const Expected& expected,
                       int64_t now_unix_ns) {
  return validate_claims(all_claims, TokenView{info.parsed, info.parse_err, info.nsigs, info.sig0_len, info.alg},
                         expected, now_unix_ns);
}

Result validate_claims(const json::Value& all_claims, const TokenView& info, const Expected& expected,
                       int64_t now_unix_ns) {
  Result r;
  // validateSigningAlgorithm (jwt/jwt.go:207-239)  [R36]
  {
    std::string e = SupportedSigningAlgorithm(expected.SigningAlgorithms);
    if (e.empty() && !info.parsed) e = std::string(info.parse_err);
    if (e.empty() && (info.nsigs == 0 || (info.nsigs == 1 && info.sig0_len == 0))) e = "token must be signed";
    if (e.empty() && info.nsigs > 1) e = "token with multiple signatures not supported";
    if (e.empty()) {
      bool found = false;
      if (expected.SigningAlgorithms.empty()) found = info.alg == "RS256";
      for (const auto& a : expected.SigningAlgorithms) found = found || a == info.alg;
      if (!found) e = "token signed with unexpected algorithm";
    }
    if (!e.empty()) {
      r.err = "invalid algorithm (alg) header parameter: " + e;
      return r;
    }
  }
  // json.Marshal(allClaims) -> json.Unmarshal(&jwt.Claims{})  [R37]: members in
  // sorted key order, each assigned to the case-insensitively matching field.
  // The fields are views into all_claims (which outlives this call).
  std::string_view iss, sub, jti;
  const json::Value* aud = nullptr;            // a String, or an Array of Strings
  bool has_iat = false, has_exp = false, has_nbf = false;
  int64_t iat = 0, exp = 0, nbf = 0;
  if (all_claims.kind == json::Value::Object) {
    const json::Member* small[32];
    std::vector<const json::Member*> big;
    const json::Member** ms = small;
    const size_t nm = all_claims.obj.size();
    if (nm > 32) {
      big.resize(nm);
      ms = big.data();
    }
    for (size_t k = 0; k < nm; ++k) ms[k] = &all_claims.obj[k];
    std::sort(ms, ms + nm, [](const json::Member* a, const json::Member* b) { return a->first < b->first; });
    for (size_t mk = 0; mk < nm; ++mk) {
      const json::Member* m = ms[mk];
      const json::Value& v = m->second;
      const ClaimField f = claim_field(m->first);
      if (f == F_NONE) continue;
      if (f == F_ISS || f == F_SUB || f == F_JTI) {
        if (v.is_null()) continue;
        if (v.kind != json::Value::String) {
          r.err = "json: cannot unmarshal into Go struct field Claims." + m->first + " of type string";
          return r;
        }
        (f == F_ISS ? iss : f == F_SUB ? sub : jti) = v.str;
        continue;
      }
      if (f == F_AUD) {
        // jwt.Audience.UnmarshalJSON: string or array of strings; null included
        bool ok = v.kind == json::Value::String || v.kind == json::Value::Array;
        if (v.kind == json::Value::Array)
          for (const auto& e : v.arr)
            if (e.kind != json::Value::String) { ok = false; break; }
        if (!ok) {
          r.err = "square/go-jose/jwt: expected string or array value to unmarshal to Audience";
          return r;
        }
        aud = &v;
        continue;
      }
      bool* has = f == F_EXP ? &has_exp : f == F_NBF ? &has_nbf : &has_iat;
      int64_t* dst = f == F_EXP ? &exp : f == F_NBF ? &nbf : &iat;
      if (v.is_null()) { *has = false; *dst = 0; continue; }       // *NumericDate = nil
      if (v.kind != json::Value::Number) {
        r.err = "square/go-jose/jwt: expected number value to unmarshal NumericDate";
        return r;
      }
      *has = true;
      *dst = go_f64_to_i64(v.num);                                 // NumericDate(f)
    }
  }
  // time defaulting (jwt/jwt.go:117-170)  [R38]
  if (!has_iat) iat = 0;
  if (!has_exp) exp = 0;
  if (!has_nbf) nbf = 0;
  if (iat == 0 && exp == 0 && nbf == 0) {
    r.err = "no issued at (iat), not before (nbf), or expiration time (exp) claims in token";
    return r;
  }
  if (exp == 0) {
    const int64_t latest = nbf > iat ? nbf : iat;
    double lw = dur_seconds(expected.ExpirationLeeway);
    if (lw < 0) lw = 0;
    else if (lw == 0) lw = DefaultLeewaySeconds;
    exp = (int64_t)((uint64_t)latest + (uint64_t)go_f64_to_i64(lw));
  }
  if (nbf == 0) {
    if (iat != 0) {
      nbf = iat;
    } else {
      double lw = dur_seconds(expected.NotBeforeLeeway);
      if (lw < 0) lw = 0;
      else if (lw == 0) lw = DefaultLeewaySeconds;
      nbf = (int64_t)((uint64_t)exp - (uint64_t)go_f64_to_i64(lw));
    }
  }
  int64_t cks = expected.ClockSkewLeeway;
  if (dur_seconds(cks) < 0) cks = 0;
  else if (dur_seconds(cks) == 0) cks = 60 * kSecond;           // jwt.DefaultLeeway = 1 minute
  // registered claims (jwt/jwt.go:172-184)  [R39]
  if (!expected.Issuer.empty() && expected.Issuer != iss) { r.err = "invalid issuer (iss) claim"; return r; }
  if (!expected.Subject.empty() && expected.Subject != sub) { r.err = "invalid subject (sub) claim"; return r; }
  if (!expected.ID.empty() && expected.ID != jti) { r.err = "invalid ID (jti) claim"; return r; }
  if (!expected.Audiences.empty()) {
    bool found = false;
    for (const auto& e : expected.Audiences) {
      if (!aud) break;
      if (aud->kind == json::Value::String) found = found || aud->str == e;
      else
        for (const auto& a : aud->arr) found = found || a.str == e;
    }
    if (!found) {
      r.err = "invalid audience (aud) claim: audience claim does not match any expected audience";
      return r;
    }
  }
  // time window (jwt/jwt.go:186-199)
  const GoTime now = go_now(now_unix_ns);
  if (go_before(go_add(now, cks), go_unix(nbf))) { r.err = "invalid not before (nbf) claim: token not yet valid"; return r; }
  if (go_after(go_add(now, -cks), go_unix(exp))) { r.err = "invalid expiration time (exp) claim: token is expired"; return r; }
  if (go_before(go_add(now, cks), go_unix(iat))) { r.err = "invalid issued at (iat) claim: token issued in the future"; return r; }
  r.ok = true;                 // the caller attaches all_claims (returned unchanged)
  return r;
}

void release_results(Results& rs) { rs.release(); }

// jwt/jwt.go:95-202 for one token: the signature through the key set's
// coalescer (concurrent Validate calls share device batches), the claim
// checks on the caller's thread with the caller's Expected
Result Validator::Validate(std::string_view token, const Expected& expected) {
  TokenInfo info;
  Result r = ks_->verify_one(token, &info);
  if (!r.ok) {
    r.err = "error verifying token signature: " + r.err;
    return r;
  }
  const int64_t now = expected.has_now ? expected.now_unix_ns : wall_now_ns();
  Result v = validate_claims(r.claims, info, expected, now);
  if (v.ok) v.claims = std::move(r.claims);
  return v;
}

Results Validator::ValidateBatch(const std::vector<std::string_view>& tokens, const Expected& expected) {
  const int64_t now = expected.has_now ? expected.now_unix_ns : wall_now_ns();
  // the claim checks run inside the key set's per-token pass, on the host
  // threads, while each token's claims map is still in cache; a claims map
  // that fails validation is destroyed there
  const PostFn post = [&](size_t, Result& r, const TokenView& t) {
    if (!r.ok) {
      r.err = "error verifying token signature: " + r.err;
      return;
    }
    Result v = validate_claims(r.claims, t, expected, now);
    if (v.ok) v.claims = std::move(r.claims);
    r = std::move(v);
  };
  return ks_->verify_batch(tokens, &post);
}

// ====================================================================== oidc hash claims
void Engine::hash(const uint8_t* arena, size_t arena_len, const void* jobs, size_t njobs, uint8_t* digests) {
  std::shared_lock<std::shared_mutex> life(life_);
  if (!ctx_) fail_device("capjwt: device lost: " + lost_);
  const int rc = jg_hash_batch(ctx_, arena, arena_len, (const jg_hjob*)jobs, njobs, digests);
  if (rc == -1) throw std::logic_error(std::string("capjwt: jg_hash_batch rejected the host's jobs: ") + jg_last_error(ctx_));
  if (rc != 0) fail_device(std::string("capjwt: jg_hash_batch: ") + jg_last_error(ctx_));
}

namespace {

// unicode.IsPrint for the runes an alg header can carry: ASCII graphic + space,
// and every other rune except the C0/C1 controls and the common non-printing
// format / separator runes (Go's tables list more unassigned code points; an
// alg name with those is not a supported alg either way, only its %q differs).
bool go_is_print(uint32_t r) {
  if (r < 0x80) return r >= 0x20 && r < 0x7f;
  if (r < 0xa0 || r == 0xad) return false;
  if (r == 0xa0 || r == 0x1680 || (r >= 0x2000 && r <= 0x200f) || (r >= 0x2028 && r <= 0x202f) ||
      (r >= 0x205f && r <= 0x2064) || r == 0x3000 || r == 0xfeff || (r >= 0xfff9 && r <= 0xfffb) ||
      r == 0xfffe || r == 0xffff || (r >= 0xd800 && r <= 0xdfff) || r > 0x10ffff)
    return false;
  return true;
}

// fmt %q of a string (strconv.Quote)
std::string go_quote(std::string_view s) {
  static const char* hex = "0123456789abcdef";
  std::string o = "\"";
  size_t i = 0;
  while (i < s.size()) {
    size_t w = 1;
    const uint32_t r = json::decode_rune((const unsigned char*)s.data() + i, s.size() - i, &w);
    if (r == 0xfffd && w == 1) {                       // invalid byte
      const unsigned char b = (unsigned char)s[i];
      o += "\\x";
      o.push_back(hex[b >> 4]);
      o.push_back(hex[b & 15]);
    } else if (r == '"' || r == '\\') {
      o.push_back('\\');
      o.push_back((char)r);
    } else if (go_is_print(r)) {
      o.append(s.substr(i, w));
    } else if (r == '\a') { o += "\\a"; } else if (r == '\b') { o += "\\b"; } else if (r == '\f') { o += "\\f"; }
    else if (r == '\n') { o += "\\n"; } else if (r == '\r') { o += "\\r"; } else if (r == '\t') { o += "\\t"; }
    else if (r == '\v') { o += "\\v"; }
    else if (r < ' ' || r == 0x7f) {
      o += "\\x";
      o.push_back(hex[r >> 4]);
      o.push_back(hex[r & 15]);
    } else {
      const int nd = r < 0x10000 ? 4 : 8;
      o += nd == 4 ? "\\u" : "\\U";
      for (int k = nd - 1; k >= 0; --k) o.push_back(hex[(r >> (4 * k)) & 15]);
    }
    i += w;
  }
  o.push_back('"');
  return o;
}

// oidc.UnmarshalClaims(rawToken, &map[string]interface{})   (oidc/token.go:170-184)
bool unmarshal_claims(std::string_view raw, json::Value* claims, std::string* err) {
  size_t parts = 1;
  for (char c : raw) parts += c == '.';
  if (parts != 3) {
    *err = "UnmarshalClaims: malformed jwt, expected 3 parts got " + std::to_string(parts) + ": invalid parameter";
    return false;
  }
  const size_t d1 = raw.find('.'), d2 = raw.find('.', d1 + 1);
  std::string payload, e;
  if (!b64rawurl_decode(raw.substr(d1 + 1, d2 - d1 - 1), &payload, &e)) {
    *err = "UnmarshalClaims: malformed jwt claims: " + e;
    return false;
  }
  if (!claims_map(payload, claims, &e)) {
    *err = "UnmarshalClaims: unable to marshal jwt JSON: " + e;
    return false;
  }
  return true;
}

struct HashPlan {
  int fam = 0;                   // jg_hash_fam, 0 = no hash (decided already)
  std::string want;              // the claim's value
};

// verifyHashClaim up to the hash: fills r (decided) or p (hash needed)
void hash_claim_plan(const std::string& claim, std::string_view t, HashClaimResult* r, HashPlan* p) {
  const std::string op = "verifyHashClaim";
  json::Value claims;
  std::string e;
  if (t.empty()) {
    r->err = op + ": IDToken.Claims: id_token is empty: invalid parameter";
    return;
  }
  if (!unmarshal_claims(t, &claims, &e)) {
    r->err = op + ": " + e;
    return;
  }
  const json::Value* v = claims.kind == json::Value::Object ? claims.get(claim) : nullptr;
  if (!v || v->kind != json::Value::String) return;        // (false, nil)
  JWS jws;
  if (!parse_signed(t, &jws, &e)) {
    r->err = op + ": malformed jwt (" + e + "): token malformed";
    return;
  }
  if (jws.sigs.empty()) {
    r->err = op + ": id_token not signed: token is not signed";
    return;
  }
  if (jws.sigs.size() > 1) {
    r->err = op + ": multiple signatures on id_token not supported";
    return;
  }
  const int alg = alg_id(jws.sigs[0].alg);
  if (!alg) {
    r->err = op + ": id_token signed with algorithm " + go_quote(jws.sigs[0].alg) + ": unsupported signing algorithm";
    return;
  }
  switch (alg) {
    case JG_RS256: case JG_ES256: case JG_PS256: p->fam = JG_SHA256; break;
    case JG_RS384: case JG_ES384: case JG_PS384: p->fam = JG_SHA384; break;
    case JG_RS512: case JG_ES512: case JG_PS512: p->fam = JG_SHA512; break;
    default: return;                                        // EdDSA: (false, nil)
  }
  p->want = v->str;
}

std::vector<HashClaimResult> verify_hash_claim_batch(Engine& eng, const std::string& claim,
                                                     const std::vector<std::string_view>& id_tokens,
                                                     const std::vector<std::string_view>& values) {
  if (id_tokens.size() != values.size()) throw std::invalid_argument("id_tokens and values differ in length");
  const size_t n = id_tokens.size();
  std::vector<HashClaimResult> out(n);
  std::vector<HashPlan> plan(n);
  parallel_for(n, host_threads(), [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) hash_claim_plan(claim, id_tokens[i], &out[i], &plan[i]);
  });
  // one GPU batch over the values that need hashing
  std::vector<size_t> idx;
  size_t bytes = 0;
  for (size_t i = 0; i < n; ++i)
    if (plan[i].fam) {
      idx.push_back(i);
      bytes += values[i].size();
    }
  if (!idx.empty()) {
    std::string arena;
    arena.reserve(bytes);
    std::vector<jg_hjob> jobs(idx.size());
    for (size_t k = 0; k < idx.size(); ++k) {
      jobs[k] = jg_hjob{};
      jobs[k].off = arena.size();
      jobs[k].len = (uint32_t)values[idx[k]].size();
      jobs[k].fam = (uint8_t)plan[idx[k]].fam;
      arena.append(values[idx[k]]);
    }
    std::vector<uint8_t> dig(64 * idx.size());
    try {
      eng.hash((const uint8_t*)arena.data(), arena.size(), jobs.data(), jobs.size(), dig.data());
    } catch (const DeviceError& e) {
      // degraded path, as the key sets': the pairs that needed the device get
      // its error, the batch returns, and the context is recreated for the next
      for (size_t i : idx) out[i].err = std::string("capjwt: hash unavailable: ") + e.what();
      idx.clear();
      (void)eng.recover(eng.errors());
    }
    parallel_for(idx.size(), host_threads(), [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k) {
        const size_t i = idx[k];
        const size_t half = (plan[i].fam == JG_SHA256 ? 32 : plan[i].fam == JG_SHA384 ? 48 : 64) / 2;
        const std::string actual = b64url_encode(std::string_view((const char*)dig.data() + 64 * k, half));
        if (actual != plan[i].want) {
          out[i].err = claim == "at_hash" ? "verifyHashClaim: access_token hash does not match value in id_token"
                                          : "verifyHashClaim: authorization code hash does not match value in id_token";
        } else {
          out[i].verified = true;
        }
      }
    });
  }
  for (auto& r : out)
    if (!r.err.empty()) r.err = "VerifyAccessToken: " + r.err;     // both public methods use this op
  return out;
}

}  // namespace

std::vector<HashClaimResult> VerifyAccessTokenBatch(Engine& eng, const std::vector<std::string_view>& id_tokens,
                                                    const std::vector<std::string_view>& access_tokens) {
  return verify_hash_claim_batch(eng, "at_hash", id_tokens, access_tokens);
}

std::vector<HashClaimResult> VerifyAuthorizationCodeBatch(Engine& eng, const std::vector<std::string_view>& id_tokens,
                                                          const std::vector<std::string_view>& codes) {
  return verify_hash_claim_batch(eng, "c_hash", id_tokens, codes);
}

}  // namespace capjwt
