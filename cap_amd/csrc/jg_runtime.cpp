// jg_runtime.cpp -- host runtime behind include/jg.h.
//
// Owns the per-device state (stream, generator / base-point comb tables, the
// staged key table) and turns a flat job list into a dispatch plan:
//   1. classify every (alg, key) pair into a kernel class (RSA-2K/3K/4K, P-256,
//      P-384, P-521, Ed25519, or reject -- go-jose newVerifier/verifyPayload
//      type dispatch);
//   2. counting-sort the jobs by (class, key) and pad every key's run to a
//      whole 64-lane wave, so each wave's key is uniform (scalar key loads,
//      broadcast modulus limbs);
//   3. launch prep (base64url + SHA-2) and the class's arithmetic kernels over
//      the padded ranges on the device's stream; scatter verdicts back.
// Multiple devices: jobs are split into contiguous chunks weighted by the
// per-alg cost model and run concurrently, one host thread per device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
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

static_assert(sizeof(jg_tok) == sizeof(jg_tok_dev), "jg_tok layout");
static_assert(offsetof(jg_tok, key_idx) == offsetof(jg_tok_dev, key_idx), "jg_tok layout");
static_assert(offsetof(jg_tok, alg) == offsetof(jg_tok_dev, alg), "jg_tok layout");

using namespace jgk;

namespace {

constexpr size_t ARENA_SLACK = 256;   // aligned SHA word reads may run past the last string

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

int cls_rows_sig(int c) {
  switch (c) {
    case CLS_RSA2K: case CLS_RSA3K: case CLS_RSA4K: return rsa_sig_rows(c);
    case CLS_P256: case CLS_P384: case CLS_P521: return EC_S_ROW + 17;
    case CLS_ED25519: return 16;
    default: return 0;
  }
}
int cls_rows_scratch(int c) {
  switch (c) {
    case CLS_RSA2K: case CLS_RSA3K: case CLS_RSA4K: return 2 * rsa_limbs(c) + SIGW_ROWS;
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

struct Grow {                     // grow-only device allocation
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t n) {
    if (n == 0) n = 16;
    if (n > cap) {
      if (p) (void)hipFree(p);
      p = nullptr;
      HIPCHK(hipMalloc(&p, n));
      cap = n;
    }
    return p;
  }
  ~Grow() { if (p) (void)hipFree(p); }
};

struct HostKey {
  int kind = 0, cls = CLS_REJECT, valid = 0;
};

// Fixed-base tables of the curve generators / Ed25519 base point depend only
// on (device, curve), so every jg_ctx of the process shares one copy per device
// (the P-256 one is 7.4 GB and takes 0.3 s to build).  Freed with the last
// context that holds it.
struct SharedTable {
  uint32_t* p = nullptr;
  ~SharedTable() { if (p) (void)hipFree(p); }
};
std::mutex g_tab_mu;
std::map<std::pair<int, int>, std::weak_ptr<SharedTable>> g_tabs;   // (device id, class) -> table

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  uint32_t* gtab[NCLS] = {};
  uint32_t* btab = nullptr;
  std::shared_ptr<SharedTable> tab_ref[NCLS];   // keeps gtab / btab alive
  // untimed runs with several classes: one stream per class so the classes'
  // kernel chains overlap (a mixed batch's per-class ranges are each too small
  // to fill 256 CUs alone); joined back into `stream` before the scatter
  hipStream_t cstream[NCLS] = {};
  hipEvent_t ev_start = nullptr, ev_done[NCLS] = {};
  // comb tables of the current key blob by key content (class, coordinates):
  // a reload (JWKS refresh) copies the tables of keys it already had instead
  // of rebuilding them (D2D copy ~0.2 ms vs ~80 ms per P-256 key)
  std::unordered_map<std::string, std::pair<uint64_t, uint64_t>> tab_cache;   // id -> (word offset, words)
  DevKey* dkeys = nullptr;
  uint32_t* dblob = nullptr;
  int32_t* didx = nullptr;
  std::mutex mu;
  std::unique_ptr<struct Bufs> sync_bufs;
};

struct Bufs {
  Grow arena, toks, perm, wave_key, sigw, dig, status, siglen, vpad, verdict, rows, pss, exc, exc_cnt;
};

}  // namespace

struct jg_batch {
  jg_ctx* ctx = nullptr;
  Device* dev = nullptr;
  std::unique_ptr<Bufs> own;
  Bufs* b = nullptr;
  int64_t ntok = 0, npad = 0;
  size_t arena_len = 0;
  int sig_rows = 0, scratch_rows = 0;
  int64_t pss_tokens = 0;          // PSS scratch tokens: the RSA classes' ranges back to back
  int64_t pss_off[NCLS] = {};
  ClassRange ranges[NCLS] = {};
  int hash_mask[NCLS] = {};       // per class: bit 0 SHA-256 present, bit 1 SHA-384/512
  int pss_any[NCLS] = {};         // per class: some token uses RSASSA-PSS (PS256/384/512)
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

struct jg_ctx {
  std::vector<std::unique_ptr<Device>> devs;
  std::vector<HostKey> keys;
  uint64_t epoch = 0;
  std::mutex key_mu;
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

int classify(const jg_ctx* ctx, const jg_tok& t) {
  if (t.key_idx >= ctx->keys.size()) return -1;
  const HostKey& k = ctx->keys[t.key_idx];
  if (!k.valid || alg_family(t.alg) != k.kind) return CLS_REJECT;
  return k.cls;
}

void mark(jg_batch* b, const char* name) {
  if (!b->timing) return;
  if (b->marks_used == b->mark_events.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    b->mark_events.push_back(e);
    b->mark_names.emplace_back();
  }
  HIPCHK(hipEventRecord(b->mark_events[b->marks_used], b->dev->stream));
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
  g_mark_ctx = MarkCtx{b, cls};
  Marker mk;
  mk.ctx = &g_mark_ctx;
  mk.fn = mark_cb;
  return mk;
}

// Build the plan and upload everything for toks[0..ntok) (indices are the caller's).
void stage(jg_ctx* ctx, jg_batch* b, const uint8_t* arena, size_t arena_len, const jg_tok* toks, size_t ntok) {
  Device* d = b->dev;
  HIPCHK(hipSetDevice(d->id));
  const int nkeys = (int)ctx->keys.size();
  const size_t nbuck = (size_t)NCLS * (nkeys > 0 ? nkeys : 1);
  std::vector<int64_t> cnt(nbuck, 0);
  std::vector<int> tcls(ntok);
  for (int c = 0; c < NCLS; ++c) b->hash_mask[c] = b->pss_any[c] = 0;
  for (size_t i = 0; i < ntok; ++i) {
    const int c = classify(ctx, toks[i]);
    if (c < 0) throw std::invalid_argument("jg_tok.key_idx out of range of the loaded key table");
    tcls[i] = c;
    const int alg = toks[i].alg;
    b->hash_mask[c] |= (alg == JG_RS256 || alg == JG_PS256 || alg == JG_ES256) ? 1 : 2;
    if (alg >= JG_PS256 && alg <= JG_PS512) b->pss_any[c] = 1;
    cnt[(size_t)c * nkeys + (c == CLS_REJECT ? 0 : toks[i].key_idx)]++;
  }
  // bucket order: classes 1..NCLS-1 by key, then the reject bucket
  std::vector<int64_t> off(nbuck, 0);
  int64_t pos = 0;
  for (int c = 1; c <= NCLS; ++c) {
    const int cc = c % NCLS;
    b->ranges[cc].begin = pos;
    const int kmax = cc == CLS_REJECT ? 1 : nkeys;
    for (int k = 0; k < kmax; ++k) {
      const size_t i = (size_t)cc * nkeys + k;
      off[i] = pos;
      pos += (cnt[i] + WAVE - 1) / WAVE * WAVE;
    }
    b->ranges[cc].end = pos;
  }
  const int64_t npad = pos > 0 ? pos : WAVE;
  b->npad = npad;
  b->ntok = (int64_t)ntok;
  std::vector<int32_t> perm((size_t)npad, -1);
  std::vector<int32_t> wkey((size_t)(npad / WAVE), 0);
  std::vector<int64_t> fill = off;
  for (size_t i = 0; i < ntok; ++i) {
    const int c = tcls[i];
    const size_t bi = (size_t)c * nkeys + (c == CLS_REJECT ? 0 : toks[i].key_idx);
    const int64_t p = fill[bi]++;
    perm[(size_t)p] = (int32_t)i;
    wkey[(size_t)(p / WAVE)] = c == CLS_REJECT ? 0 : toks[i].key_idx;
  }
  b->sig_rows = 1;
  b->scratch_rows = 1;
  b->pss_tokens = 0;
  for (int c = 1; c < NCLS; ++c) {
    if (b->ranges[c].end <= b->ranges[c].begin) continue;
    b->sig_rows = std::max(b->sig_rows, cls_rows_sig(c));
    b->scratch_rows = std::max(b->scratch_rows, cls_rows_scratch(c));
    if (c <= CLS_RSA4K) {
      b->pss_off[c] = b->pss_tokens;
      b->pss_tokens += b->ranges[c].end - b->ranges[c].begin;
    }
  }
  Bufs* B = b->b;
  hipStream_t s = d->stream;
  b->arena_len = arena_len;
  uint8_t* da = (uint8_t*)B->arena.get(arena_len + ARENA_SLACK);
  HIPCHK(hipMemcpyAsync(da, arena, arena_len, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(da + arena_len, 0, ARENA_SLACK, s));
  HIPCHK(hipMemcpyAsync(B->toks.get(sizeof(jg_tok) * std::max<size_t>(ntok, 1)), toks, sizeof(jg_tok) * ntok,
                        hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(B->perm.get(sizeof(int32_t) * npad), perm.data(), sizeof(int32_t) * npad,
                        hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(B->wave_key.get(sizeof(int32_t) * wkey.size()), wkey.data(), sizeof(int32_t) * wkey.size(),
                        hipMemcpyHostToDevice, s));
  B->sigw.get(sizeof(uint32_t) * b->sig_rows * npad);
  B->dig.get(sizeof(uint32_t) * DIG_ROWS * npad);
  B->status.get(npad);
  B->siglen.get(sizeof(uint16_t) * npad);
  B->vpad.get(npad);
  B->verdict.get(std::max<size_t>(ntok, 1));
  B->rows.get(sizeof(uint32_t) * (size_t)b->scratch_rows * npad);
  B->pss.get((size_t)std::max<int64_t>(b->pss_tokens, 1) * 2048);
  B->exc.get(sizeof(int32_t) * npad);
  B->exc_cnt.get(sizeof(uint32_t) * NCLS);
  // the host vectors die here: the copies above must complete first
  HIPCHK(hipStreamSynchronize(s));
  b->epoch = ctx->epoch;
}

// timed: per-kernel HIP events (classes in sequence on the device stream);
// untimed: classes on their own streams, overlapping.
void run(jg_ctx* ctx, jg_batch* b, bool timed) {
  Device* d = b->dev;
  HIPCHK(hipSetDevice(d->id));
  if (b->epoch != ctx->epoch) throw std::runtime_error("key table reloaded since this batch was staged");
  Bufs* B = b->b;
  hipStream_t s = d->stream;
  b->timing = timed;
  b->marks_used = 0;
  int nact = 0;
  for (int c = 1; c < NCLS; ++c) nact += b->ranges[c].end > b->ranges[c].begin;
  const bool conc = !timed && nact > 1;
  const int64_t np = b->npad;
  mark(b, "begin");
  HIPCHK(hipMemsetAsync(B->vpad.p, 0, np, s));
  PrepArgs pa{};
  pa.arena = (const uint8_t*)B->arena.p;
  pa.toks = (const jg_tok_dev*)B->toks.p;
  pa.perm = (const int32_t*)B->perm.p;
  pa.wave_key = (const int32_t*)B->wave_key.p;
  pa.keys = d->dkeys;
  pa.keyblob = d->dblob;
  pa.sigw = (uint32_t*)B->sigw.p;
  pa.dig = (uint32_t*)B->dig.p;
  pa.status = (uint8_t*)B->status.p;
  pa.siglen = (uint16_t*)B->siglen.p;
  pa.npad = np;
  uint32_t* rows = (uint32_t*)B->rows.p;
  if (conc) HIPCHK(hipEventRecord(d->ev_start, s));
  const hipStream_t s0 = s;
  for (int c = 1; c < NCLS; ++c) {
    const ClassRange r = b->ranges[c];
    if (r.end <= r.begin) continue;
    // every class reads and writes only columns [r.begin, r.end) of the shared
    // scratch rows, its own exception counter and its own PSS scratch
    hipStream_t s = s0;
    if (conc) {
      s = d->cstream[c];
      HIPCHK(hipStreamWaitEvent(s, d->ev_start, 0));
    }
    pa.begin = r.begin;
    pa.end = r.end;
    pa.zrows = cls_rows_sig(c);
    launch_prep(c, b->hash_mask[c], pa, s);
    mark(b, (std::string(cls_name(c)) + "_prep").c_str());
    if (c <= CLS_RSA4K) {
      RsaArgs ra{};
      ra.toks = pa.toks; ra.perm = pa.perm; ra.wave_key = pa.wave_key; ra.keys = pa.keys; ra.keyblob = pa.keyblob;
      ra.sigw = pa.sigw; ra.dig = pa.dig;
      const int L = rsa_limbs(c);
      ra.xmw = rows;
      ra.xlr = rows + (size_t)L * np;
      ra.yw = rows + (size_t)2 * L * np;
      ra.status = pa.status; ra.siglen = pa.siglen; ra.verdict_pad = (uint8_t*)B->vpad.p;
      ra.pss_scratch = (uint8_t*)B->pss.p + b->pss_off[c] * 2048;
      ra.has_pss = b->pss_any[c];
      ra.npad = np; ra.begin = r.begin; ra.end = r.end;
      launch_rsa(c, ra, s, marker(b, c));
    } else if (c <= CLS_P521) {
      if (!d->gtab[c]) throw std::runtime_error("curve table missing");
      EcArgs ea{};
      ea.toks = pa.toks; ea.perm = pa.perm; ea.wave_key = pa.wave_key; ea.keys = pa.keys; ea.keyblob = pa.keyblob;
      ea.sigw = pa.sigw; ea.dig = pa.dig; ea.status = pa.status; ea.verdict_pad = (uint8_t*)B->vpad.p;
      ea.digs = rows;
      ea.u1w = rows + (size_t)ec_digit_rows(c) * np;
      ea.u2w = rows + (size_t)(ec_digit_rows(c) + ec_limbs(c)) * np;
      ea.gtab = d->gtab[c];
      ea.exc_list = (int32_t*)B->exc.p + r.begin;
      ea.exc_count = (uint32_t*)B->exc_cnt.p + c;
      ea.npad = np; ea.begin = r.begin; ea.end = r.end;
      launch_ec(c, ea, s, marker(b, c));
    } else {
      EdArgs ea{};
      ea.perm = pa.perm; ea.wave_key = pa.wave_key; ea.keys = pa.keys; ea.keyblob = pa.keyblob;
      ea.sigw = pa.sigw; ea.dig = pa.dig; ea.status = pa.status; ea.siglen = pa.siglen;
      ea.verdict_pad = (uint8_t*)B->vpad.p;
      ea.xyz = rows;
      ea.btab = d->btab;
      ea.npad = np; ea.begin = r.begin; ea.end = r.end;
      launch_ed(ea, s, marker(b, c));
    }
    if (conc) {
      HIPCHK(hipEventRecord(d->ev_done[c], s));
      HIPCHK(hipStreamWaitEvent(s0, d->ev_done[c], 0));
    }
  }
  launch_scatter((const int32_t*)B->perm.p, (const uint8_t*)B->vpad.p, (uint8_t*)B->verdict.p, np, s);
  mark(b, "scatter");
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

// ---------------------------------------------------------------- keys
struct StagedKeys {
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

void build_keys(jg_ctx* ctx, const jg_key* keys, int nkeys, StagedKeys& S) {
  ctx->keys.assign((size_t)nkeys, HostKey{});
  S.dk.assign((size_t)nkeys, DevKey{});
  S.tab_id.assign((size_t)nkeys, std::string());
  for (int i = 0; i < nkeys; ++i) {
    const jg_key& k = keys[i];
    HostKey& hk = ctx->keys[i];
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
      int cls = bits <= rsa_limbs(CLS_RSA2K) * 28 - 2 ? CLS_RSA2K : bits <= 112 * 28 - 2 ? CLS_RSA3K : bits <= 148 * 28 - 2 ? CLS_RSA4K : -1;
      if (cls < 0) {
        ok = false;
        ctx->set_err("RSA key " + std::to_string(i) + " has " + std::to_string(bits) +
                     " bits; the GPU path supports up to 4142-bit moduli (key marked unusable)");
        cls = CLS_RSA4K;
      }
      const int L = rsa_limbs(cls);
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
    } else if (k.kind == JG_KEY_EC) {
      const int cls = k.curve == JG_P256 ? CLS_P256 : k.curve == JG_P384 ? CLS_P384 : k.curve == JG_P521 ? CLS_P521 : -1;
      if (cls < 0) { hk.valid = 0; continue; }
      const int L = ec_limbs(cls);
      const int cb = cls == CLS_P256 ? 32 : cls == CLS_P384 ? 48 : 66;
      K.cls = cls;
      K.kbytes = cb;
      K.aux_off = blob_alloc(S.blob, 2 * L);
      K.tab_off = tab_alloc(S, i, (uint64_t)ec_table_words(cls, false));
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
      K.tab_off = tab_alloc(S, i, (uint64_t)ed_table_words(false));
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
                               std::to_string(ec_table_words(c, false) * 4 >> 20) + " MiB each)");
  if ((int)S.ed_idx.size() > ED_MAX_KEYS)
    throw std::runtime_error("Ed25519: at most " + std::to_string(ED_MAX_KEYS) + " keys per table (comb tables are " +
                             std::to_string(ed_table_words(false) * 4 >> 20) + " MiB each)");
  blob_alloc(S.blob, 0);                                      // align the host part
  for (int k : S.tab_keys) S.dk[k].tab_off += S.blob.size();
}

// the process-wide table of (device, class), built on this device's stream
// and complete before any other context can see it
template <class Build>
std::shared_ptr<SharedTable> shared_table(Device* d, int cls, size_t bytes, Build&& build) {
  std::lock_guard<std::mutex> g(g_tab_mu);
  const auto key = std::make_pair(d->id, cls);
  if (auto t = g_tabs[key].lock()) return t;
  auto t = std::make_shared<SharedTable>();
  HIPCHK(hipMalloc(&t->p, bytes));
  build(t->p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(d->stream));
  g_tabs[key] = t;
  return t;
}

void ensure_tables(Device* d, const StagedKeys& S) {
  HIPCHK(hipSetDevice(d->id));
  for (int c = CLS_P256; c <= CLS_P521; ++c) {
    if (S.ec_idx[c].empty() || d->gtab[c]) continue;
    d->tab_ref[c] = shared_table(d, c, sizeof(uint32_t) * ec_table_words(c, true),
                                 [&](uint32_t* t) { launch_ec_gtable(c, t, d->stream); });
    d->gtab[c] = d->tab_ref[c]->p;
  }
  if (!S.ed_idx.empty() && !d->btab) {
    d->tab_ref[CLS_ED25519] = shared_table(d, CLS_ED25519, sizeof(uint32_t) * ed_table_words(true),
                                           [&](uint32_t* t) { launch_ed_btable(t, d->stream); });
    d->btab = d->tab_ref[CLS_ED25519]->p;
  }
}

void load_keys_device(Device* d, const StagedKeys& S) {
  HIPCHK(hipSetDevice(d->id));
  hipStream_t s = d->stream;
  HIPCHK(hipStreamSynchronize(s));
  if (d->dkeys) (void)hipFree(d->dkeys);
  if (d->didx) (void)hipFree(d->didx);
  d->dkeys = nullptr; d->didx = nullptr;
  uint32_t* old_blob = d->dblob;                   // kept until its reusable tables are copied
  auto old_cache = std::move(d->tab_cache);
  d->tab_cache.clear();
  d->dblob = nullptr;
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
  for (int c = CLS_P256; c <= CLS_P521; ++c) split(S.ec_idx[c], (uint64_t)ec_table_words(c, false), build_ec[c]);
  split(S.ed_idx, (uint64_t)ed_table_words(false), build_ed);
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
    launch_ec_keyprep(c, d->dkeys, d->dblob, d->didx + at[1 + c - CLS_P256], (int)S.ec_idx[c].size(),
                      d->didx + at[5 + c - CLS_P256], (int)build_ec[c].size(), s);
  launch_ed_keyprep(d->dkeys, d->dblob, d->didx + at[4], (int)S.ed_idx.size(), d->didx + at[8],
                    (int)build_ed.size(), s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  if (old_blob) (void)hipFree(old_blob);
}

thread_local std::string g_tls_err;

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
      HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
      for (int c = 1; c < NCLS; ++c) {
        HIPCHK(hipStreamCreateWithFlags(&d->cstream[c], hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&d->ev_done[c], hipEventDisableTiming));
      }
      HIPCHK(hipEventCreateWithFlags(&d->ev_start, hipEventDisableTiming));
      d->sync_bufs = std::make_unique<Bufs>();
      ctx->devs.push_back(std::move(d));
    }
    return ctx.release();
  } catch (const std::exception& e) {
    g_tls_err = e.what();
    return nullptr;
  }
}

void jg_destroy(jg_ctx* ctx) {
  if (!ctx) return;
  for (auto& d : ctx->devs) {
    (void)hipSetDevice(d->id);
    (void)hipStreamSynchronize(d->stream);
    d->sync_bufs.reset();
    for (auto& t : d->tab_ref) t.reset();         // shared fixed-base tables: last holder frees
    if (d->dkeys) (void)hipFree(d->dkeys);
    if (d->dblob) (void)hipFree(d->dblob);
    if (d->didx) (void)hipFree(d->didx);
    for (int c = 1; c < NCLS; ++c) {
      if (d->cstream[c]) (void)hipStreamSynchronize(d->cstream[c]);
      if (d->cstream[c]) (void)hipStreamDestroy(d->cstream[c]);
      if (d->ev_done[c]) (void)hipEventDestroy(d->ev_done[c]);
    }
    if (d->ev_start) (void)hipEventDestroy(d->ev_start);
    (void)hipStreamDestroy(d->stream);
  }
  delete ctx;
}

int jg_keys_load(jg_ctx* ctx, const jg_key* keys, int nkeys) {
  if (!ctx || nkeys < 0 || (nkeys > 0 && !keys)) return -1;
  if (nkeys > 65535) { ctx->set_err("at most 65535 keys"); return -1; }
  try {
    std::lock_guard<std::mutex> g(ctx->key_mu);
    for (auto& d : ctx->devs) d->mu.lock();
    StagedKeys S;
    build_keys(ctx, keys, nkeys, S);
    try {
      for (auto& d : ctx->devs) load_keys_device(d.get(), S);
    } catch (...) {
      for (auto& d : ctx->devs) d->mu.unlock();
      throw;
    }
    // device-side validity (on-curve, Ed25519 decoding) back into the host view
    Device* d0 = ctx->devs[0].get();
    std::vector<DevKey> back(S.dk.size());
    if (!back.empty()) {
      HIPCHK(hipSetDevice(d0->id));
      HIPCHK(hipMemcpy(back.data(), d0->dkeys, sizeof(DevKey) * back.size(), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < back.size(); ++i) ctx->keys[i].valid = ctx->keys[i].valid && back[i].valid;
    }
    ++ctx->epoch;
    for (auto& d : ctx->devs) d->mu.unlock();
    return 0;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_batch_stage(jg_ctx* ctx, int device_slot, const uint8_t* arena, size_t arena_len,
                   const jg_tok* toks, size_t ntok, jg_batch** out) {
  if (!ctx || !out || (ntok > 0 && (!toks || !arena))) return -1;
  if (device_slot < 0 || device_slot >= (int)ctx->devs.size()) return -1;
  if (ntok > (size_t)INT32_MAX / 2) { ctx->set_err("batch too large"); return -1; }
  try {
    auto b = std::make_unique<jg_batch>();
    b->ctx = ctx;
    b->dev = ctx->devs[device_slot].get();
    b->own = std::make_unique<Bufs>();
    b->b = b->own.get();
    std::lock_guard<std::mutex> g(b->dev->mu);
    stage(ctx, b.get(), arena, arena_len, toks, ntok);
    *out = b.release();
    return 0;
  } catch (const std::invalid_argument& e) {
    ctx->set_err(e.what());
    return -1;
  } catch (const std::exception& e) {
    ctx->set_err(e.what());
    return -2;
  }
}

int jg_batch_run(jg_ctx* ctx, jg_batch* b, uint8_t* verdict_out) {
  if (!ctx || !b) return -1;
  try {
    std::lock_guard<std::mutex> g(b->dev->mu);
    run(ctx, b, true);
    if (verdict_out) {
      if (b->ntok > 0)
        HIPCHK(hipMemcpyAsync(verdict_out, b->b->verdict.p, (size_t)b->ntok, hipMemcpyDeviceToHost, b->dev->stream));
      HIPCHK(hipStreamSynchronize(b->dev->stream));
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
    run(ctx, b, false);
    if (verdict_out && b->ntok > 0)
      HIPCHK(hipMemcpyAsync(verdict_out, b->b->verdict.p, (size_t)b->ntok, hipMemcpyDeviceToHost, b->dev->stream));
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
    HIPCHK(hipStreamSynchronize(b->dev->stream));
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
  (void)hipStreamSynchronize(b->dev->stream);
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

int jg_verify_batch(jg_ctx* ctx, const uint8_t* arena, size_t arena_len,
                    const jg_tok* toks, size_t ntok, uint8_t* verdict_out) {
  if (!ctx || (ntok > 0 && (!toks || !arena || !verdict_out))) return -1;
  if (ntok == 0) return 0;
  // split over devices by the cost model
  const size_t nd = ctx->devs.size();
  std::vector<size_t> cut(nd + 1, 0);
  cut[nd] = ntok;
  if (nd > 1) {
    std::vector<double> pre(ntok + 1, 0.0);
    for (size_t i = 0; i < ntok; ++i) {
      int c = classify(ctx, toks[i]);
      pre[i + 1] = pre[i] + cls_cost(c < 0 ? 0 : c);
    }
    size_t j = 0;
    for (size_t k = 1; k < nd; ++k) {
      const double target = pre[ntok] * (double)k / (double)nd;
      while (j < ntok && pre[j] < target) ++j;
      cut[k] = j;
    }
  }
  std::vector<int> rc(nd, 0);
  std::vector<std::string> errs(nd);
  auto work = [&](size_t k) {
    Device* d = ctx->devs[k].get();
    const size_t lo = cut[k], hi = cut[k + 1];
    if (hi <= lo) return;
    try {
      std::lock_guard<std::mutex> g(d->mu);
      jg_batch b;
      b.ctx = ctx;
      b.dev = d;
      b.b = d->sync_bufs.get();
      b.timing = false;
      stage(ctx, &b, arena, arena_len, toks + lo, hi - lo);
      run(ctx, &b, false);
      HIPCHK(hipMemcpyAsync(verdict_out + lo, b.b->verdict.p, hi - lo, hipMemcpyDeviceToHost, d->stream));
      HIPCHK(hipStreamSynchronize(d->stream));
    } catch (const std::invalid_argument& e) {
      rc[k] = -1;
      errs[k] = e.what();
    } catch (const std::exception& e) {
      rc[k] = -2;
      errs[k] = e.what();
    }
  };
  if (nd == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (size_t k = 0; k < nd; ++k) th.emplace_back(work, k);
    for (auto& t : th) t.join();
  }
  for (size_t k = 0; k < nd; ++k)
    if (rc[k]) {
      ctx->set_err(errs[k]);
      return rc[k];
    }
  return 0;
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
    Grow da, dj, dout;
    uint8_t* a = (uint8_t*)da.get(arena_len + ARENA_SLACK);
    HIPCHK(hipMemsetAsync(a + arena_len, 0, ARENA_SLACK, d->stream));
    if (arena_len) HIPCHK(hipMemcpyAsync(a, arena, arena_len, hipMemcpyHostToDevice, d->stream));
    jg_hjob* j = (jg_hjob*)dj.get(sizeof(jg_hjob) * njobs);
    HIPCHK(hipMemcpyAsync(j, jobs, sizeof(jg_hjob) * njobs, hipMemcpyHostToDevice, d->stream));
    uint32_t* o = (uint32_t*)dout.get(64 * njobs);
    launch_hash(a, j, (int64_t)njobs, o, d->stream);
    HIPCHK(hipGetLastError());
    std::vector<uint32_t> w(16 * njobs);
    HIPCHK(hipMemcpyAsync(w.data(), o, 64 * njobs, hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
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
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void jg_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

const char* jg_version(void) { return "capjwt 0.1 (gfx950, HIP)"; }

}  // extern "C"
