/*
 * cpuverify -- all-core CPU JWS verifier on OpenSSL libcrypto: the labelled
 * "OpenSSL" leg of bench.py's CPU baseline (the reference Go
 * verifier cannot run here -- Go is absent on the GPU box -- so the baseline
 * is stood in for by (a) the repo's C oracle and (b) this, a much closer proxy
 * for Go's assembly-backed crypto/rsa, crypto/ecdsa and crypto/ed25519).
 * Measurement only: never on the GPU path, never the parity checker.
 *
 *   cpuverify <ALG> <threads> <min_seconds> <tokens.txt> <key.pem> [key.pem ...]
 *
 * Token i (one per line, as tools/tokgen writes them) is verified with key
 * i % nkeys, the way a JWT verifier does it: split the compact form, base64url
 * decode the signature, hash the signing input and verify (RSA PKCS#1 v1.5,
 * RSA-PSS with auto-detected salt length as Go's VerifyPSS(nil), ECDSA from the
 * r||s form, Ed25519).  The whole token list is verified repeatedly across
 * `threads` threads until min_seconds have passed; prints one JSON line.
 */
#include <openssl/bn.h>
#include <openssl/ecdsa.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  const char* alg;
  EVP_PKEY** keys;
  int nkeys;
  char** toks;
  long ntok, lo, hi;
  long verified, accepted;
  double min_seconds;
  double t0;
} job;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int b64val(int c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '-') return 62;
  if (c == '_') return 63;
  return -1;
}

static long b64url_decode(const char* s, size_t n, unsigned char* out, size_t cap) {
  unsigned acc = 0;
  int bits = 0;
  size_t o = 0;
  for (size_t i = 0; i < n; ++i) {
    const int v = b64val((unsigned char)s[i]);
    if (v < 0) return -1;
    acc = (acc << 6) | (unsigned)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      if (o >= cap) return -1;
      out[o++] = (unsigned char)(acc >> bits);
    }
  }
  return (long)o;
}

static const EVP_MD* alg_md(const char* alg) {
  if (!strcmp(alg, "EdDSA")) return NULL;
  const char* h = alg + 2;
  if (!strcmp(h, "256")) return EVP_sha256();
  if (!strcmp(h, "384")) return EVP_sha384();
  return EVP_sha512();
}

// per-thread, per-key verify contexts initialised once (OpenSSL 3 re-fetches
// the digest / key methods on every EVP_DigestVerifyInit); each token copies one
static EVP_MD_CTX* make_template(const char* alg, EVP_PKEY* key) {
  EVP_MD_CTX* t = EVP_MD_CTX_new();
  EVP_PKEY_CTX* pc = NULL;
  if (EVP_DigestVerifyInit(t, &pc, alg_md(alg), NULL, key) != 1) return NULL;
  if (alg[0] == 'P') {
    EVP_PKEY_CTX_set_rsa_padding(pc, RSA_PKCS1_PSS_PADDING);
    EVP_PKEY_CTX_set_rsa_pss_saltlen(pc, RSA_PSS_SALTLEN_AUTO);
  }
  return t;
}

static int verify_one(const job* j, EVP_MD_CTX* mc, EVP_MD_CTX* tmpl, const char* tok, EVP_PKEY* key) {
  const char* d2 = strrchr(tok, '.');
  if (!d2) return 0;
  unsigned char sig[1100], der[200];
  long sl = b64url_decode(d2 + 1, strlen(d2 + 1), sig, sizeof sig);
  if (sl <= 0) return 0;
  const unsigned char* s = sig;
  size_t slen = (size_t)sl;
  if (j->alg[0] == 'E' && j->alg[1] == 'S') {            /* r || s -> DER */
    const size_t half = (size_t)sl / 2;
    ECDSA_SIG* es = ECDSA_SIG_new();
    ECDSA_SIG_set0(es, BN_bin2bn(sig, (int)half, NULL), BN_bin2bn(sig + half, (int)half, NULL));
    unsigned char* p = der;
    const int dl = i2d_ECDSA_SIG(es, &p);
    ECDSA_SIG_free(es);
    if (dl <= 0) return 0;
    s = der;
    slen = (size_t)dl;
  }
  (void)key;
  if (tmpl) {
    if (EVP_MD_CTX_copy_ex(mc, tmpl) != 1) return 0;
  } else {                                                /* EdDSA: one-shot init per message */
    if (EVP_DigestVerifyInit(mc, NULL, NULL, NULL, key) != 1) return 0;
  }
  return EVP_DigestVerify(mc, s, slen, (const unsigned char*)tok, (size_t)(d2 - tok)) == 1;
}

static void* worker(void* arg) {
  job* j = (job*)arg;
  EVP_MD_CTX* mc = EVP_MD_CTX_new();
  EVP_MD_CTX** tm = calloc((size_t)j->nkeys, sizeof(EVP_MD_CTX*));
  const int ed = !strcmp(j->alg, "EdDSA");
  for (int k = 0; k < j->nkeys && !ed; ++k) tm[k] = make_template(j->alg, j->keys[k]);
  do {
    for (long i = j->lo; i < j->hi; ++i) {
      const int k = (int)(i % j->nkeys);
      j->accepted += verify_one(j, mc, tm[k], j->toks[i], j->keys[k]);
      ++j->verified;
      EVP_MD_CTX_reset(mc);
    }
  } while (now_s() - j->t0 < j->min_seconds);
  for (int k = 0; k < j->nkeys; ++k) EVP_MD_CTX_free(tm[k]);
  free(tm);
  EVP_MD_CTX_free(mc);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: cpuverify ALG threads min_seconds tokens.txt key.pem...\n");
    return 2;
  }
  const char* alg = argv[1];
  int threads = atoi(argv[2]);
  if (threads < 1) threads = 1;
  const double min_s = atof(argv[3]);
  FILE* f = fopen(argv[4], "r");
  if (!f) { perror(argv[4]); return 2; }
  long cap = 1024, n = 0;
  char** toks = malloc(sizeof(char*) * (size_t)cap);
  char* line = NULL;
  size_t lcap = 0;
  ssize_t len;
  while ((len = getline(&line, &lcap, f)) > 0) {
    while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
    if (!len) continue;
    if (n == cap) toks = realloc(toks, sizeof(char*) * (size_t)(cap *= 2));
    toks[n++] = strdup(line);
  }
  fclose(f);
  free(line);
  const int nkeys = argc - 5;
  EVP_PKEY** keys = calloc((size_t)nkeys, sizeof(EVP_PKEY*));
  for (int i = 0; i < nkeys; ++i) {
    FILE* kf = fopen(argv[5 + i], "r");
    if (!kf) { perror(argv[5 + i]); return 2; }
    keys[i] = PEM_read_PrivateKey(kf, NULL, NULL, NULL);
    fclose(kf);
    if (!keys[i]) { fprintf(stderr, "bad key %s\n", argv[5 + i]); return 2; }
  }
  pthread_t* th = calloc((size_t)threads, sizeof(pthread_t));
  job* js = calloc((size_t)threads, sizeof(job));
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    js[t] = (job){alg, keys, nkeys, toks, n, n * t / threads, n * (t + 1) / threads, 0, 0, min_s, t0};
    pthread_create(&th[t], NULL, worker, &js[t]);
  }
  long ver = 0, acc = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    ver += js[t].verified;
    acc += js[t].accepted;
  }
  const double el = now_s() - t0;
  printf("{\"alg\":\"%s\",\"tokens\":%ld,\"verified\":%ld,\"accepted\":%ld,\"threads\":%d,\"seconds\":%.4f,"
         "\"per_second\":%.1f,\"openssl\":\"%s\"}\n",
         alg, n, ver, acc, threads, el, (double)ver / el, OpenSSL_version(OPENSSL_VERSION));
  return 0;
}
