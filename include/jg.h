/*
 * jg.h -- C ABI of the MI355X batched JWS signature verifier (libcapjwt.so).
 *
 * This is the drop-in boundary for cap's signature-verification hot path.  A Go
 * maintainer binds it with cgo underneath a GPU-backed
 * implementation of cap's KeySet interface:
 *
 *   type KeySet interface {                                 jwt/keyset.go:27-32
 *     VerifySignature(ctx, token string) (map[string]interface{}, error)
 *   }
 *
 * Each entry point replaces one piece of the reference's per-token call stack
 *  with a batched, device-side equivalent:
 *
 *   jg_keys_load     <- key ingestion: NewStaticKeySet (jwt/keyset.go:142-150),
 *                       JWKS decode in go-oidc RemoteKeySet (jwt/keyset.go:101,120)
 *   jg_verify_batch  <- the signature arithmetic of parsedJWT.Claims(key, ...)
 *                       (jwt/keyset.go:163) / remoteJWKS.VerifySignature
 *                       (jwt/keyset.go:127): go-jose verifyPayload -> crypto/rsa
 *                       VerifyPKCS1v15 | VerifyPSS, crypto/ecdsa.Verify,
 *                       crypto/ed25519.Verify, for MANY (token, key) pairs at once
 *
 * Plain C types only: pointers + sizes, no Go or torch types.  All byte strings
 * are big-endian as in JWK / Go's big.Int.Bytes(), except the Ed25519 public key
 * (32 raw bytes, RFC 8032 encoding).
 */
#ifndef CAPJWT_JG_H
#define CAPJWT_JG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* JWS algorithms -- jwt/algs.go:12-21 */
enum jg_alg {
  JG_ALG_NONE = 0, /* anything not in jwt/algs.go:24-35 (HS256, none, ...) -> reject */
  JG_RS256 = 1, JG_RS384 = 2, JG_RS512 = 3,
  JG_PS256 = 4, JG_PS384 = 5, JG_PS512 = 6,
  JG_ES256 = 7, JG_ES384 = 8, JG_ES512 = 9,
  JG_EDDSA = 10
};

enum jg_key_kind { JG_KEY_RSA = 1, JG_KEY_EC = 2, JG_KEY_ED25519 = 3 };
enum jg_curve { JG_P256 = 1, JG_P384 = 2, JG_P521 = 3 };

/* One public key: *rsa.PublicKey | *ecdsa.PublicKey | ed25519.PublicKey. */
typedef struct jg_key {
  int32_t kind;            /* jg_key_kind */
  int32_t curve;           /* jg_curve, EC only */
  const uint8_t* n;        /* RSA modulus, big-endian (leading zeros allowed) */
  int32_t n_len;
  uint64_t e;              /* RSA public exponent as decoded (Go rejects e<2, e>2^31-1) */
  const uint8_t* x;        /* EC X / Ed25519 public key (32 bytes) */
  const uint8_t* y;        /* EC Y */
  int32_t coord_len;       /* EC coordinate length in bytes (32/48/66) */
} jg_key;

/* One verification job.  `off`/`sig_in_len` locate the JWS signing input
 * (go-jose computeAuthData: BASE64URL(protected) '.' BASE64URL(payload), or the
 * raw payload when b64=false) inside the arena; the signature is the base64url
 * string at arena[off + sig_rel_off, +sig_b64_len) with any trailing '='
 * already trimmed by the caller (go-jose base64URLDecode).
 * The verdict is the crypto outcome for (alg, key) on those bytes. */
typedef struct jg_tok {
  uint64_t off;
  uint32_t sig_in_len;
  uint32_t sig_rel_off;
  uint32_t sig_b64_len;
  uint16_t key_idx;        /* index into the last jg_keys_load table */
  uint8_t alg;             /* jg_alg */
  uint8_t flags;           /* reserved, 0 */
} jg_tok;

/* verdict_out[i] values */
enum { JG_REJECT = 0, JG_ACCEPT = 1 };

typedef struct jg_ctx jg_ctx;
typedef struct jg_batch jg_batch;

/* Create a context on the given HIP devices (NULL/0 = device 0). */
jg_ctx* jg_create(const int* devices, int ndev);
void jg_destroy(jg_ctx* ctx);

/* Replace the key table (copied; may be reloaded on JWKS refresh -- go-oidc
 * RemoteKeySet updateKeys behind jwt/keyset.go:127).  Invalid keys (off-curve
 * EC point, Ed25519 point that does not decode, even or unusable RSA modulus,
 * e out of range) load fine and verify nothing -- the same outcome Go produces
 * per token.
 *  - A key list identical to the loaded one (same bytes, same table budget)
 *    returns 0 at once: no device work, nothing drained, staged batches stay
 *    valid.
 *  - Otherwise the new table is staged beside running verifications (no
 *    drain): work submitted before the call finishes against the old table,
 *    work submitted after it returns runs against the new one.  A key that was
 *    already loaded keeps its comb table (shared by content, no copy); a new
 *    EC / Ed25519 key gets a narrow table first (P-256 W = 20: 436 MB, about
 *    0.1 s) so it verifies as soon as this returns, and its budgeted wide table
 *    is built in the background and swapped in when complete
 *    (jg_keys_wait_tables).  CAPJWT_TABLES_SYNC=1 builds full width here.
 * Returns 0, -1 on bad arguments, or -2 when the table cannot be staged (more
 * than 256 EC keys of one curve, not enough free HBM for the new tables, a
 * device allocation or kernel failure): the previous table then stays in force
 * on every device, as go-oidc keeps its cached keys when updateKeys fails. */
int jg_keys_load(jg_ctx* ctx, const jg_key* keys, int nkeys);

/* Block until the background comb-table widening of the last jg_keys_load has
 * finished (every key verifying with its budgeted table width).  Returns 0, 1
 * when some table stayed narrower because it did not fit free HBM (see
 * jg_last_error), -1 on bad arguments. */
int jg_keys_wait_tables(jg_ctx* ctx);

/* Comb width of each loaded key's table on the context's first device (0 for
 * RSA and invalid keys): widths[0..min(n, cap)).  Returns n, the key count. */
int jg_keys_table_widths(jg_ctx* ctx, int* widths, int cap);

/* Test / A-B hook: small submissions (at most 64 jobs, every job ECDSA or
 * rejected) run as one launch per (curve, key-table width) that does the whole
 * verification per token -- enable 1: on (the default), 0: off (they take the
 * batch chain: arena DMA, plan fill, prep, scalar, point, exact, scatter),
 * -1: unchanged.  Verdicts are identical either way.  Applies to later
 * submissions.  *launches (may be NULL) receives the number of such one-launch
 * verifications this context has enqueued.  Returns 0 or -1. */
int jg_debug_small_path(jg_ctx* ctx, int enable, uint64_t* launches);

/* Test hook: the n-th device allocation of later key loads (counting from 1)
 * fails as if hipMalloc ran out of memory; 0 disables.  Returns 0 or -1. */
int jg_debug_fail_alloc(jg_ctx* ctx, int n);

/* Test hook of the degraded path (SURVEY §5 failure row): the n-th later
 * jg_submit / jg_verify_batch of this context (counting from 1) fails as a
 * device fault would -- its jg_wait returns -2 -- and the context is then
 * unusable, as after a sticky HIP error: every later submission returns -2
 * until the context is destroyed and recreated (the host layer's Engine does
 * that, re-staging its key list).  0 disables.  Returns 0 or -1. */
int jg_debug_fail_verify(jg_ctx* ctx, int n);

/* Test hook: the background upgrader widens at most n more comb tables of
 * this context (-1 = no limit, the default; CAPJWT_DEBUG_MAX_UPGRADES sets
 * the initial value), so a class can be held at mixed widths; raising it
 * resumes widening.  Returns 0 or -1. */
int jg_debug_max_upgrades(jg_ctx* ctx, int n);

/* Debug check of the key-memory lifetime rule (process-wide; also
 * CAPJWT_CHECK_LIFETIME=1): every stream that launches against a key
 * generation records an event, and releasing the generation queries them --
 * one still pending is a violation (logged to stderr).  enable: 1 on, 0 off,
 * -1 unchanged; *violations / *checked (either may be NULL) receive the
 * counts so far.  Returns 0. */
int jg_debug_lifetime_check(int enable, uint64_t* violations, uint64_t* checked);

/* Test hook: a 64-bit digest of key `key`'s current comb table on the first
 * device (0 when it has none) -- tables built at different times or on
 * different paths must agree.  Returns 0, -1 or -2. */
int jg_debug_table_digest(jg_ctx* ctx, int key, uint64_t* digest);

/* Test hook: the number of key comb tables this context has built so far, on
 * every device (key loads and background width upgrades; a table reused from
 * the per-device cache -- same key content and width -- is not a build).
 * Returns 0 or -1. */
int jg_debug_tables_built(jg_ctx* ctx, uint64_t* built);

/* Verify ntok jobs, blocking (= jg_submit + jg_wait).  Host buffers; copied to
 * the device(s) in chunks whose H2D copies overlap the kernels of the previous
 * chunk (direct DMA when `arena` is pinned -- jg_host_alloc -- else through
 * pinned staging).  A batch whose jobs span two or more kernel classes (e.g.
 * RSA and ECDSA keys) and whose arena (16-byte aligned) lies in one
 * jg_host_alloc block is not DMAed: it runs as one class-major plan, each
 * class's token bytes gathered from the pinned arena over PCIe by a kernel,
 * costliest class first, while earlier classes compute -- when zero-copy
 * plans are on (jg_set_zero_copy; off by default, CAPJWT_ZC=1).  Returns 0 on success, -1 on bad arguments (a key_idx
 * outside the loaded table, a signing-input or signature span past
 * arena_len), -2 on an infrastructure error (see jg_last_error); per-token
 * outcomes are only in verdict_out[i] (JG_ACCEPT / JG_REJECT).  ntok == 0
 * returns 0 without touching the buffers.
 * Replaces the per-token loops of jwt/keyset.go:162-167 (staticKeySet) and
 * jwt/keyset.go:127 (go-oidc remoteKeySet) for a whole batch. */
int jg_verify_batch(jg_ctx* ctx, const uint8_t* arena, size_t arena_len,
                    const jg_tok* toks, size_t ntok, uint8_t* verdict_out);

/* Asynchronous form: jg_submit checks its arguments, queues the jobs on the
 * context's devices and returns at once with a ticket (-1 on bad arguments, -2
 * on an infrastructure error); arena, toks and verdict_out must stay valid and
 * unmodified until jg_wait(ticket) returns.  Consecutive submissions pipeline
 * back to back on each device.  The jobs themselves are validated by the
 * device workers chunk by chunk, in the same pass that plans each chunk, so a
 * bad job (a key_idx outside the table, a span past arena_len) is reported by
 * jg_wait: it returns -1 and verdict_out is then only partly written (chunks
 * before the bad one are verified; the rest are not).  jg_wait blocks until
 * the batch is complete, frees the ticket and returns 0, -1 or -2.  A batch
 * runs entirely against the key table current at submit time, even when a
 * jg_keys_load replaces it while the batch is queued. */
typedef struct jg_ticket jg_ticket;
int jg_submit(jg_ctx* ctx, const uint8_t* arena, size_t arena_len, const jg_tok* toks, size_t ntok,
              uint8_t* verdict_out, jg_ticket** ticket);
int jg_wait(jg_ctx* ctx, jg_ticket* ticket);

/* Jobs per pipeline chunk of jg_submit / jg_verify_batch (default 65536, or
 * CAPJWT_CHUNK; >= 64).  Applies to later submissions.  Returns 0 or -1. */
int jg_set_chunk(jg_ctx* ctx, size_t jobs);

/* Class-major zero-copy plans of jg_verify_batch / jg_submit (see above): on
 * (enable != 0) or off (the default unless CAPJWT_ZC=1), and the jobs per plan
 * (max_jobs >= 64; 0 keeps the current value; default 2M or CAPJWT_ZC_MAX) --
 * a longer submission runs as equal plans of at most that many jobs.  Applies
 * to later submissions.  Returns 0 or -1. */
int jg_set_zero_copy(jg_ctx* ctx, int enable, size_t max_jobs);

/* HBM (bytes per device, one total over all curves) the context may spend on
 * the comb tables of its EC and Ed25519 keys (default 32 GiB, or
 * CAPJWT_TABLE_BUDGET_GB).  The next jg_keys_load first gives every key its
 * curve's narrowest table (always allowed: P-256 W = 20, 436 MB; P-384 16,
 * 105 MB; P-521 16, 173 MB; Ed25519 16, 67 MB), then widens P-256, P-384,
 * Ed25519 and P-521 in that order, each curve to the widest width whose tables
 * for all of its keys still fit what is left: P-256 W = 26 (21.5 GB per key,
 * 20 point additions per token), 24 (5.9 GB, 21) or 22 (1.6 GB); P-384 W = 24
 * (18.3 GB), 20 (1.34 GB) or 18 (369 MB); Ed25519 24 (11.8 GB), 22 (3.2 GB),
 * 20 (872 MB) or 18 (252 MB); P-521 20 (2.26 GB) or 18 (629 MB: 30 windows)
 * -- HBM traded for fewer additions, as the shared generator tables do.  At
 * the default 32 GiB a lone P-256 key gets W = 26, 2-5 keys 24, 6-21 keys 22;
 * bench.py key_widths mirrors the rule (tests/test_bench_contract.py).
 * New tables are also sized against free HBM: a load narrows them rather than
 * fail.  Besides the budget, each device holds the generator / base-point
 * tables (about 54 GB with all four curves) for the life of the process
 * (CAPJWT_RELEASE_GTABLES=1 frees them with the last context).  Returns 0 or -1. */
int jg_set_table_budget(jg_ctx* ctx, uint64_t bytes);

const char* jg_last_error(jg_ctx* ctx);

/* Pinned host memory for arenas / job arrays (hipHostMalloc).  The block
 * carries 256 readable bytes past `bytes`, so kernels may read an arena in it
 * in place (jg_verify_batch's zero-copy plans). */
void* jg_host_alloc(size_t bytes);
void jg_host_free(void* p);

/* ---- device-resident batches (throughput measurement, pipelining) ----
 * jg_batch_stage copies a batch to the device of `device_slot` and precomputes
 * its dispatch plan (bucketing by algorithm family and key); jg_batch_run runs
 * the verify kernels on the resident inputs (no H2D) and, if verdict_out is
 * non-NULL, copies verdicts back.  jg_batch_run is asynchronous when
 * verdict_out is NULL; jg_batch_sync waits.  Consecutively staged batches of a
 * device alternate between two compute lanes on different hardware queues:
 * runs of one batch are in order, runs of two batches enqueued back to back
 * overlap on the device. */
int jg_batch_stage(jg_ctx* ctx, int device_slot, const uint8_t* arena, size_t arena_len,
                   const jg_tok* toks, size_t ntok, jg_batch** out);
int jg_batch_run(jg_ctx* ctx, jg_batch* b, uint8_t* verdict_out);
/* Enqueue one run (kernels + verdict copy into verdict_out, which must be
 * pinned -- jg_host_alloc -- and stay valid until jg_batch_sync) and return
 * without waiting: consecutive runs stream back to back on the device. */
int jg_batch_enqueue(jg_ctx* ctx, jg_batch* b, uint8_t* verdict_out);
int jg_batch_sync(jg_ctx* ctx, jg_batch* b);
void jg_batch_free(jg_ctx* ctx, jg_batch* b);

/* Per-kernel device time (ms) of the last jg_batch_run, measured with HIP
 * events on the batch's stream.  names/ms arrays of length cap; returns count. */
int jg_batch_kernel_times(jg_batch* b, const char** names, float* ms, int cap);

/* Diagnostics of the last run of a resident batch: counts[c] = tokens of kernel
 * class c (0 reject, 1-3 RSA-2K/3K/4K, 4-6 P-256/384/521, 7 Ed25519) whose
 * ECDSA comb sum hit an exceptional case of the group law and were recomputed
 * by the complete-formula path.  Returns the number of classes (8) or <0. */
int jg_batch_exceptions(jg_batch* b, uint32_t* counts, int cap);

/* ---- batched SHA-2 of byte strings ----
 * The hash of cap's OIDC hash-claim checks: oidc/id_token.go:121-135
 * (verifyHashClaim, behind IDToken.VerifyAccessToken :59 and
 * VerifyAuthorizationCode :83) hashes the access token / authorization code
 * with SHA-256, SHA-384 or SHA-512 by the id_token's alg.  Job i hashes
 * arena[off, off + len) with `fam`; digest_out receives njobs x 64 bytes, the
 * digest (32 / 48 / 64 bytes) left-aligned and zero-filled.  Blocking; runs on
 * the context's first device.  Returns 0, or <0 on bad arguments (a span past
 * arena_len, unknown fam) or an infrastructure error. */
enum jg_hash_fam { JG_SHA256 = 1, JG_SHA384 = 2, JG_SHA512 = 3 };
typedef struct jg_hjob {
  uint64_t off;
  uint32_t len;
  uint8_t fam;             /* jg_hash_fam */
  uint8_t pad_[3];
} jg_hjob;
int jg_hash_batch(jg_ctx* ctx, const uint8_t* arena, size_t arena_len,
                  const jg_hjob* jobs, size_t njobs, uint8_t* digest_out);

/* Library build information (gfx target, version). */
const char* jg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CAPJWT_JG_H */
