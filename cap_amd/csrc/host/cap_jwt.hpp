// cap_jwt.hpp -- C++ mirror of cap's jwt package API (jwt/keyset.go, jwt/jwt.go,
// jwt/algs.go) on top of the GPU verifier's C ABI (include/jg.h).
//
// Go is absent from this image, so this layer stands where the Go host code of
// BASELINE.json's north star would: it keeps base64url/JSON header parsing,
// kid -> key lookup and claims validation on the host and hands every
// signature check to libcapjwt.so in one batch.  Names, argument meaning and
// error strings follow the reference:
//
//   Go (reference)                                   here
//   KeySet.VerifySignature    jwt/keyset.go:27-32     KeySet::VerifySignature / VerifySignatureBatch
//   NewStaticKeySet           jwt/keyset.go:142-150   NewStaticKeySet
//   NewJSONWebKeySet          jwt/keyset.go:109-123   NewJSONWebKeySet (HTTP GET via a Fetcher)
//   NewOIDCDiscoveryKeySet    jwt/keyset.go:49-104    NewOIDCDiscoveryKeySet
//   ParsePublicKeyPEM         jwt/keyset.go:178-200   ParsePublicKeyPEM
//   NewValidator / Validate   jwt/jwt.go:25-202       NewValidator / Validator::Validate
//   (north star) ValidateBatch                        Validator::ValidateBatch
//   SupportedSigningAlgorithm jwt/algs.go:38-46       SupportedSigningAlgorithm
//
// There is no CPU verification path: a KeySet whose GPU context cannot be
// created fails at construction.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "jose.hpp"
#include "json.hpp"

struct jg_ctx;

namespace capjwt {

// ---------------------------------------------------------------- algs (jwt/algs.go)
extern const char* const kSupportedAlgorithms[10];
// "" if every alg is supported, else `unsupported signing algorithm "X"`
std::string SupportedSigningAlgorithm(const std::vector<std::string>& algs);

// ---------------------------------------------------------------- results
// (claims, error): ok == true <=> Go's err == nil.  claims is the
// map[string]interface{} (Object) or nil (Null, for a `null` payload).
struct Result {
  bool ok = false;
  json::Value claims;
  std::string err;
};

// ---------------------------------------------------------------- batch arrays
// Runs fn(begin, end) over [0, n) on `threads` host threads (contiguous ranges;
// small n stays on the caller's thread).
void batch_parallel(size_t n, int threads, const std::function<void(size_t, size_t)>& fn);
int host_threads();

// Storage of the batch arrays (BatchArray, the key sets' per-token records):
// blocks of 1 MiB and more come from the hostmem pool (hostmem.hpp) and go
// back to it when freed, instead of going back to the OS.  A 1M-token batch
// frees ~200 MB of records twice per ValidateBatch call; returned to the OS
// each time, the unmap cost ~30 ms per array and the next call paid the page
// faults again (bench e2e phases "free-toks", "blob release").  A pooled
// block is reused for a request of at least half its size; *cap receives the
// block's true capacity, which batch_block_free takes back.
void* batch_block_alloc(size_t bytes, size_t* cap);
void batch_block_free(void* p, size_t cap);

// Host memory the batches keep for reuse (hostmem pools): at most `bytes`
// (default 4 GiB, or CAPJWT_HOST_CACHE_GB); TrimHostMemory hands all of it
// back to the OS now.  HostMemoryRetained: bytes held right now.
void SetHostMemoryRetention(size_t bytes);
void TrimHostMemory();
size_t HostMemoryRetained();

// The per-token records of a batch, constructed and destroyed by all host
// threads: a 1M-token batch's results are ~150 MB of records plus their claims
// maps, and a serial std::vector construction or free of that costs more than
// the batch's parse.  Move-only; indexable and iterable like a vector.  The
// array also owns the arenas its records' claims trees live in (adopt): they
// are released after the records.
template <class T>
class BatchArray {
 public:
  BatchArray() = default;
  explicit BatchArray(size_t n, int threads = host_threads()) : threads_(threads) {
    p_ = static_cast<T*>(batch_block_alloc(sizeof(T) * (n ? n : 1), &cap_));
    batch_parallel(n, threads_, [this](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) new (p_ + i) T();
    });
    n_ = n;
  }
  BatchArray(BatchArray&& o) noexcept
      : p_(o.p_), n_(o.n_), cap_(o.cap_), threads_(o.threads_), arenas_(std::move(o.arenas_)) {
    o.p_ = nullptr; o.n_ = 0;
  }
  BatchArray& operator=(BatchArray&& o) noexcept {
    if (this != &o) {
      release();
      p_ = o.p_; n_ = o.n_; cap_ = o.cap_; threads_ = o.threads_; arenas_ = std::move(o.arenas_);
      o.p_ = nullptr; o.n_ = 0;
    }
    return *this;
  }
  BatchArray(const BatchArray&) = delete;
  BatchArray& operator=(const BatchArray&) = delete;
  ~BatchArray() { release(); }
  void release() {
    if (p_) {
      batch_parallel(n_, threads_, [this](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) p_[i].~T();
      });
      batch_block_free(p_, cap_);
    }
    p_ = nullptr;
    n_ = 0;
    arenas_.clear();
  }
  // keep `a` alive as long as the records (thread-safe)
  void adopt(std::unique_ptr<json::Arena> a) {
    std::lock_guard<std::mutex> g(amu_);
    arenas_.push_back(std::move(a));
  }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  size_t size() const { return n_; }
  T* begin() { return p_; }
  T* end() { return p_ + n_; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
  int threads_ = 1;
  std::vector<std::unique_ptr<json::Arena>> arenas_;
  std::mutex amu_;
};
using Results = BatchArray<Result>;

// ---------------------------------------------------------------- HTTP
// The JWKS / discovery GET.  The reference uses net/http with a TLS client
// built from the CA PEM (createCAContext, jwt/keyset.go:204-227); here the
// caller supplies the transport.  Throw std::runtime_error for a transport
// error (Go: client.Do error).
struct FetchResponse {
  int status = 200;
  std::string status_text = "200 OK";   // resp.Status
  std::string body;
  std::string content_type = "application/json";
  int64_t max_age_s = -1;               // Cache-Control max-age; -1 = none (go-oidc: expire at once)
};
using Fetcher = std::function<FetchResponse(const std::string& url, const std::string& ca_pem)>;

// ---------------------------------------------------------------- GPU engine
// A failed device call: jg_* returned -2 (a HIP error, a lost device).  The key
// sets turn it into per-token errors and recover the context (Engine::recover).
// A -1 (a job outside the key table or the arena: the host layer packed it
// wrong) is a std::logic_error and propagates -- it is a bug, not a device fault.
struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// One jg_ctx (HIP devices + staged key table).  Thread-safe: concurrent verify
// calls are separate submissions that pipeline on the devices (jg_submit).
class Engine {
 public:
  explicit Engine(const std::vector<int>& devices);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  void load(const std::vector<PublicKey>& keys);      // jg_keys_load (returns once the keys verify)
  void wait_tables();                                 // jg_keys_wait_tables: wide comb tables in place
  // verify (arena entry, key, alg) jobs; verdicts[i] = 1 accept, 0 reject.
  // `submitted` runs once the jobs are queued (before the wait): a key set
  // releases its key-list lock there, so refreshes never wait for the device.
  void verify(const uint8_t* arena, size_t arena_len, const void* jobs, size_t njobs, uint8_t* verdicts,
              const std::function<void()>& submitted = {});
  // SHA-2 of (arena span, family) jobs: digests njobs x 64 bytes (jg_hash_batch)
  void hash(const uint8_t* arena, size_t arena_len, const void* jobs, size_t njobs, uint8_t* digests);
  // Pinned host memory for one call's arena (jg_host_alloc), from a small pool
  // of blocks the engine keeps; back to the pool when the Pinned dies.
  class Pinned {
   public:
    Pinned(Engine* e, uint8_t* p, size_t cap) : e_(e), p_(p), cap_(cap) {}
    Pinned(Pinned&& o) noexcept : e_(o.e_), p_(o.p_), cap_(o.cap_) { o.p_ = nullptr; }
    Pinned(const Pinned&) = delete;
    Pinned& operator=(const Pinned&) = delete;
    ~Pinned();
    uint8_t* get() const { return p_; }
   private:
    Engine* e_;
    uint8_t* p_;
    size_t cap_;
  };
  Pinned pinned(size_t bytes);
  // Recreate the device context after a DeviceError: its streams and
  // per-device state are torn down and rebuilt and the current key list is
  // re-staged (no process restart, no key refetch).  `seen` = errors() when
  // the caller's call failed: a recovery since then is not repeated.  True
  // when the engine verifies again; false leaves it marked lost (status()).
  bool recover(uint64_t seen);
  uint64_t errors() const { return errors_.load(); }  // DeviceErrors so far
  int recoveries() const { return recoveries_.load(); }
  std::string status();                               // "" healthy, else why the device is lost
  int debug_fail_verify(int n);                       // jg_debug_fail_verify (test hook)
  int threads() const { return threads_; }
 private:
  void fail_device(const std::string& what);          // count the error; throws DeviceError
  std::vector<int> devices_;
  jg_ctx* ctx_ = nullptr;
  std::shared_mutex life_;        // shared: calls on ctx_; unique: recover (ctx_ replaced)
  std::mutex load_mu_;            // serialises loads; guards keys_
  std::vector<PublicKey> keys_;   // the list the context holds (re-staged by recover)
  bool has_keys_ = false;
  std::atomic<uint64_t> errors_{0};
  uint64_t recovered_at_ = 0;     // errors_ when the last recovery ran (under life_)
  std::atomic<int> recoveries_{0};
  std::string lost_;              // why ctx_ is null (under life_)
  std::chrono::steady_clock::time_point last_try_{};
  std::mutex pin_mu_;
  std::vector<std::pair<uint8_t*, size_t>> pin_free_;
  int threads_ = 1;
};

// ---------------------------------------------------------------- KeySet
struct TokenInfo {          // what validateSigningAlgorithm needs from ParseSigned
  bool parsed = false;
  std::string parse_err;
  size_t nsigs = 0;
  size_t sig0_len = 0;
  std::string alg;
};
// The same, as views into a batch's parse records (valid during a PostFn call)
struct TokenView {
  bool parsed = false;
  std::string_view parse_err;
  size_t nsigs = 0;
  size_t sig0_len = 0;
  std::string_view alg;
};
// Per-token continuation of a batch verify: called on the host threads, once
// per token (i = its index in the batch), right after that token's (claims,
// error) is final -- the Validator's claim checks run there while the claims
// map is still in cache.
using PostFn = std::function<void(size_t i, Result& r, const TokenView& t)>;

// Request coalescing of single-token calls (KeySet::VerifySignature,
// Validator::Validate, RemoteKeySet::VerifySignature): a Go service calls
// these once per request from many goroutines.  Each call queues its token;
// while fewer than `max_inflight` batches are on the device, a caller takes
// everything queued (up to `max_batch` tokens, after waiting at most
// `window_us` for more to arrive) and runs it as ONE batch, then wakes the
// callers it carried.  Under load the batches grow by themselves (everything
// that arrived while the device was busy goes in the next); an idle device
// takes a lone token at once.  No lock is held across a device call.
struct CoalesceConfig {
  int max_inflight = 4;
  size_t max_batch = 65536;
  int64_t window_us = 0;
};
struct Verified;                  // a batch after parse and device verification (cap_jwt.cpp)
class Coalescer {
 public:
  struct Req {
    std::string_view tok;
    std::shared_ptr<const Verified> batch;   // the verified batch that carried this token ...
    size_t idx = 0;                          // ... and its index there
    std::exception_ptr ex;        // the batch threw (a host-side bug): re-thrown to every caller in it
    std::shared_ptr<std::vector<Req*>> peers;   // the batch's callers to wake (a binary tree) ...
    size_t wpos = 0;                            // ... and this one's position there
    Req* next = nullptr;          // the submission stack's link
    enum { WAITING = 0, DONE = 1 };
    std::atomic<int> state{WAITING};   // futex word: DONE once a dispatcher has carried it
  };
  // parse + verify a batch of tokens (KeySet::verify_raw)
  using Exec = std::function<std::shared_ptr<const Verified>(const std::vector<std::string_view>&)>;
  explicit Coalescer(Exec exec) : exec_(std::move(exec)) {}
  ~Coalescer();
  void run(Req* r);               // blocks until r->batch is set (exceptions of the batch re-thrown)
  void configure(const CoalesceConfig& c);
  CoalesceConfig config();
  struct Stats { uint64_t calls = 0, batches = 0, max_batch_seen = 0; };
  Stats stats();
 private:
  static void release(const std::vector<Req*>& wake, size_t i);
  void dispatch_loop();
  void serve_stack(std::vector<Req*>& all, std::vector<Req*>& batch);   // one exchange of the stack, carried
  void carry(std::vector<Req*>& batch);
  void kick();                    // wake one idle dispatcher
  void start_locked();            // spawn the dispatchers (threads_mu_ held)
  void stop_locked();             // stop and join them (threads_mu_ held)
  Exec exec_;
  std::atomic<Req*> head_{nullptr};        // submissions not yet taken (LIFO, lock-free)
  std::atomic<uint32_t> seq_{0};           // futex word of idle dispatchers (kick)
  std::atomic<int> active_{0};             // batches being carried (callers leading + dispatchers)
  std::atomic<int> max_inflight_{4};
  std::atomic<bool> stop_{false};
  std::atomic<bool> started_{false};
  std::mutex threads_mu_;
  std::vector<std::thread> threads_;
  CoalesceConfig cfg_;                      // threads_mu_
  std::atomic<size_t> max_batch_{65536};
  std::atomic<int64_t> window_us_{0};
  std::atomic<uint64_t> calls_{0}, batches_{0}, max_seen_{0};
};

class KeySet {
 public:
  KeySet();
  virtual ~KeySet() = default;
  // jwt/keyset.go:27-32 (one token; concurrent calls are coalesced into
  // batches, and each caller builds its own claims map on its own thread)
  Result VerifySignature(std::string_view token);
  Results VerifySignatureBatch(const std::vector<std::string_view>& tokens);
  // batch verify; `post` (may be null) continues each token's result with what
  // the parse learned (Validator::ValidateBatch)
  Results verify_batch(const std::vector<std::string_view>& tokens, const PostFn* post);
  // one token through the coalescer, with its parse info (Validator::Validate)
  Result verify_one(std::string_view token, TokenInfo* info);
  // the two halves of a batch: parse + device verification, then token i's
  // (claims, error) -- the key set's own error strings and JSON rules
  // overlap (may be null): run while the batch's device call is in flight
  // (after parse, before the verdicts) -- verify_batch parses the claims then
  using Overlap = std::function<void(const Verified&)>;
  virtual std::shared_ptr<Verified> verify_raw(const std::vector<std::string_view>& tokens,
                                               const Overlap* overlap = nullptr) = 0;
  virtual void finish(const Verified& V, size_t i, Result& r) = 0;
  // finish() for a parsed token whose claims map was already read into r
  // (json_ok; else r.err holds the JSON error) while the device verified
  virtual void finish_pre(const Verified& V, size_t i, Result& r, bool json_ok) = 0;
  virtual const char* trace_name() const = 0;
  // block until background comb-table widening of the last key load is done
  // (keys verify before that, on narrower tables; a measurement hook)
  virtual void WaitTables() {}
  void SetCoalescing(const CoalesceConfig& c) { co_.configure(c); }
  Coalescer::Stats CoalescingStats() { return co_.stats(); }
  // the device context behind the key set: "" healthy, else why it is lost;
  // how many times it was recovered after a device error
  virtual std::string DeviceStatus() = 0;
  virtual int DeviceRecoveries() = 0;
  virtual int DebugFailVerify(int n) = 0;            // jg_debug_fail_verify on its context (tests)
 private:
  Coalescer co_;
};

std::unique_ptr<KeySet> NewStaticKeySet(const std::vector<PublicKey>& keys, std::string* err,
                                        const std::vector<int>& devices = {});
std::unique_ptr<KeySet> NewJSONWebKeySet(const std::string& jwks_url, const std::string& jwks_ca_pem, Fetcher fetch,
                                         std::string* err, const std::vector<int>& devices = {});
std::unique_ptr<KeySet> NewOIDCDiscoveryKeySet(const std::string& issuer, const std::string& issuer_ca_pem,
                                               Fetcher fetch, std::string* err, const std::vector<int>& devices = {});

// ---------------------------------------------------------------- go-oidc KeySet adapter
// go-oidc v2.2.1's `oidc.KeySet` (VerifySignature(ctx, jwt) ([]byte, error)) as
// returned by oidc.NewRemoteKeySet: the interface cap's jsonWebKeySet wraps
// (jwt/keyset.go:101,120,127) and go-oidc's IDTokenVerifier calls -- the path
// behind cap's oidc.Provider.VerifyIDToken (oidc/provider.go:418-441).  Same
// kid filtering, refresh-on-miss and error strings as the JWKS key set above
// ("oidc: malformed jwt: ...", "failed to verify id token signature",
// "fetching keys ..."), returning the verified payload bytes.
struct PayloadResult {
  bool ok = false;
  std::string payload;
  std::string err;
};
class RemoteKeySet {
 public:
  RemoteKeySet(const std::string& jwks_url, Fetcher fetch, const std::vector<int>& devices);
  ~RemoteKeySet();
  PayloadResult VerifySignature(std::string_view jwt);            // coalesced, as KeySet's
  std::vector<PayloadResult> VerifySignatureBatch(const std::vector<std::string_view>& jwts);
  void SetCoalescing(const CoalesceConfig& c);
 private:
  class Impl;
  std::unique_ptr<Impl> impl_;
};
std::unique_ptr<RemoteKeySet> NewRemoteKeySet(const std::string& jwks_url, Fetcher fetch,
                                              const std::vector<int>& devices = {});

// ---------------------------------------------------------------- Validator
constexpr int64_t kSecond = 1000000000LL;
constexpr int64_t DefaultLeewaySeconds = 150;          // jwt/jwt.go:16

struct Expected {                                      // jwt/jwt.go:38-83
  std::string Issuer, Subject, ID;
  std::vector<std::string> Audiences;
  std::vector<std::string> SigningAlgorithms;
  int64_t NotBeforeLeeway = 0;                         // time.Duration (ns)
  int64_t ExpirationLeeway = 0;
  int64_t ClockSkewLeeway = 0;
  bool has_now = false;                                // Now == nil -> time.Now()
  int64_t now_unix_ns = 0;
};

class Validator {
 public:
  explicit Validator(KeySet* ks) : ks_(ks) {}
  Result Validate(std::string_view token, const Expected& expected);
  Results ValidateBatch(const std::vector<std::string_view>& tokens, const Expected& expected);
 private:
  KeySet* ks_;
};
// nil keySet -> error "keySet must not be nil"
std::unique_ptr<Validator> NewValidator(KeySet* ks, std::string* err);

// The claim checks of Validate after the signature (jwt/jwt.go:103-201), on a
// verified claims map and the token's parse info.  Exposed for tests.
Result validate_claims(const json::Value& all_claims, const TokenInfo& info, const Expected& expected,
                       int64_t now_unix_ns);
Result validate_claims(const json::Value& all_claims, const TokenView& info, const Expected& expected,
                       int64_t now_unix_ns);

bool ParsePublicKeyPEM(std::string_view data, PublicKey* out, std::string* err);

// Frees a batch's results now (all host threads; the destructor does the same).
void release_results(Results& rs);

// Host threads used by batch parsing / claims (CAPJWT_HOST_THREADS, default
// available_cpus()): declared above.
// CPUs available to this process (affinity mask, cgroup v2 quota)
int available_cpus();

// ---------------------------------------------------------------- oidc hash claims
// IDToken.VerifyAccessToken / VerifyAuthorizationCode (oidc/id_token.go:59-145,
// verifyHashClaim) for many (id_token, value) pairs: claims via UnmarshalClaims
// (oidc/token.go:170-184), the claim as a string, jose.ParseSigned, exactly one
// signature with a supported alg, then base64url(left half of SHA-2(value)) ==
// claim.  The SHA-2 runs on the GPU in one jg_hash_batch.  verified/err are Go's
// (bool, error); err == "" <=> nil.  Error strings follow the reference,
// including its "VerifyAccessToken" op prefix on the c_hash path.
struct HashClaimResult {
  bool verified = false;
  std::string err;
};
std::vector<HashClaimResult> VerifyAccessTokenBatch(Engine& eng, const std::vector<std::string_view>& id_tokens,
                                                    const std::vector<std::string_view>& access_tokens);
std::vector<HashClaimResult> VerifyAuthorizationCodeBatch(Engine& eng, const std::vector<std::string_view>& id_tokens,
                                                          const std::vector<std::string_view>& codes);

}  // namespace capjwt
