/*
 * tokgen -- synthetic signed-JWT generator for bench.py and the large-batch
 * GPU tests (input generation only; never on the measured path, never the
 * checker).  Signs with OpenSSL libcrypto, multi-threaded.
 *
 *   tokgen <ALG> <count> <threads> <out.txt> <key.pem> [key.pem ...]
 *
 * Token i uses key i % nkeys; header {"alg":ALG,"kid":"kid-KK","typ":"JWT"},
 * payload shaped like cap's testJWTClaims (jwt/keyset_test.go:666-677) with
 * jti = i.  One token per line.  PS* use salt length = hash length (go-jose).
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

static const char B64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

static size_t b64url(const unsigned char* in, size_t n, char* out) {
  size_t o = 0, i = 0;
  for (; i + 3 <= n; i += 3) {
    unsigned v = (unsigned)in[i] << 16 | (unsigned)in[i + 1] << 8 | in[i + 2];
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63]; out[o++] = B64[(v >> 6) & 63]; out[o++] = B64[v & 63];
  }
  if (n - i == 1) {
    unsigned v = (unsigned)in[i] << 16;
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63];
  } else if (n - i == 2) {
    unsigned v = (unsigned)in[i] << 16 | (unsigned)in[i + 1] << 8;
    out[o++] = B64[v >> 18]; out[o++] = B64[(v >> 12) & 63]; out[o++] = B64[(v >> 6) & 63];
  }
  out[o] = 0;
  return o;
}

typedef struct {
  const char* alg;
  EVP_PKEY** keys;
  int nkeys;
  long lo, hi;
  char** out;
  int kid_base;           /* TOKGEN_KID_BASE: first kid number ("kid-NN") */
} job;

static const EVP_MD* alg_md(const char* alg) {
  if (!strcmp(alg, "EdDSA")) return NULL;
  const char* h = alg + 2;
  if (!strcmp(h, "256")) return EVP_sha256();
  if (!strcmp(h, "384")) return EVP_sha384();
  return EVP_sha512();
}

static int es_size(const char* alg) {
  return !strcmp(alg, "ES256") ? 32 : !strcmp(alg, "ES384") ? 48 : 66;
}

static void* worker(void* arg) {
  job* j = (job*)arg;
  /* TOKGEN_PAD=n: a "pad" claim of n 'x' bytes (long signing inputs) */
  const char* pe = getenv("TOKGEN_PAD");
  const size_t padn = pe ? (size_t)atol(pe) : 0;
  char hdr[256], hb[512], sb[1500];
  char* pay = malloc(512 + padn);
  char* pb = malloc(2 * (512 + padn) + 8);
  char* padv = malloc(padn + 1);
  memset(padv, 'x', padn);
  padv[padn] = 0;
  unsigned char sig[1024], raw[200];
  for (long i = j->lo; i < j->hi; ++i) {
    const int k = (int)(i % j->nkeys);
    snprintf(hdr, sizeof hdr, "{\"alg\":\"%s\",\"kid\":\"kid-%02d\",\"typ\":\"JWT\"}", j->alg, j->kid_base + k);
    if (padn)
      snprintf(pay, 512 + padn,
               "{\"aud\":[\"www.example.com\"],\"exp\":1611699944,\"iat\":1611699344,"
               "\"iss\":\"https://example.com/\",\"jti\":\"%ld\",\"nbf\":1611699344,\"pad\":\"%s\","
               "\"sub\":\"alice@example.com\"}", i, padv);
    else
      snprintf(pay, 512,
               "{\"aud\":[\"www.example.com\"],\"exp\":1611699944,\"iat\":1611699344,"
               "\"iss\":\"https://example.com/\",\"jti\":\"%ld\",\"nbf\":1611699344,\"sub\":\"alice@example.com\"}", i);
    size_t hl = b64url((const unsigned char*)hdr, strlen(hdr), hb);
    size_t pl = b64url((const unsigned char*)pay, strlen(pay), pb);
    char* si = malloc(hl + pl + 2);
    memcpy(si, hb, hl); si[hl] = '.'; memcpy(si + hl + 1, pb, pl); si[hl + pl + 1] = 0;
    const size_t slen_in = hl + pl + 1;
    EVP_MD_CTX* mc = EVP_MD_CTX_new();
    EVP_PKEY_CTX* pc = NULL;
    size_t sl = sizeof sig;
    if (EVP_DigestSignInit(mc, &pc, alg_md(j->alg), NULL, j->keys[k]) != 1) { fprintf(stderr, "init\n"); exit(2); }
    if (j->alg[0] == 'P') {
      EVP_PKEY_CTX_set_rsa_padding(pc, RSA_PKCS1_PSS_PADDING);
      EVP_PKEY_CTX_set_rsa_pss_saltlen(pc, RSA_PSS_SALTLEN_DIGEST);
    }
    if (EVP_DigestSign(mc, sig, &sl, (const unsigned char*)si, slen_in) != 1) { fprintf(stderr, "sign\n"); exit(2); }
    EVP_MD_CTX_free(mc);
    const unsigned char* s = sig;
    size_t n = sl;
    if (j->alg[0] == 'E' && j->alg[1] == 'S') {             /* DER -> r || s */
      const unsigned char* p = sig;
      ECDSA_SIG* es = d2i_ECDSA_SIG(NULL, &p, (long)sl);
      const BIGNUM *r, *ss;
      ECDSA_SIG_get0(es, &r, &ss);
      const int sz = es_size(j->alg);
      memset(raw, 0, sizeof raw);
      BN_bn2binpad(r, raw, sz);
      BN_bn2binpad(ss, raw + sz, sz);
      ECDSA_SIG_free(es);
      s = raw;
      n = 2 * (size_t)sz;
    }
    size_t bl = b64url(s, n, sb);
    char* tok = malloc(slen_in + bl + 2);
    memcpy(tok, si, slen_in); tok[slen_in] = '.'; memcpy(tok + slen_in + 1, sb, bl + 1);
    free(si);
    j->out[i] = tok;
  }
  free(pay);
  free(pb);
  free(padv);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: tokgen ALG count threads out.txt key.pem...\n");
    return 2;
  }
  const char* alg = argv[1];
  long count = atol(argv[2]);
  int threads = atoi(argv[3]);
  if (threads < 1) threads = 1;
  int nkeys = argc - 5;
  EVP_PKEY** keys = calloc((size_t)nkeys, sizeof(EVP_PKEY*));
  for (int i = 0; i < nkeys; ++i) {
    FILE* f = fopen(argv[5 + i], "r");
    if (!f) { perror(argv[5 + i]); return 2; }
    keys[i] = PEM_read_PrivateKey(f, NULL, NULL, NULL);
    fclose(f);
    if (!keys[i]) { fprintf(stderr, "bad key %s\n", argv[5 + i]); return 2; }
  }
  char** out = calloc((size_t)count, sizeof(char*));
  pthread_t* th = calloc((size_t)threads, sizeof(pthread_t));
  job* js = calloc((size_t)threads, sizeof(job));
  for (int t = 0; t < threads; ++t) {
    const char* kb = getenv("TOKGEN_KID_BASE");
    js[t] = (job){alg, keys, nkeys, count * t / threads, count * (t + 1) / threads, out, kb ? atoi(kb) : 0};
    pthread_create(&th[t], NULL, worker, &js[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  FILE* f = fopen(argv[4], "w");
  for (long i = 0; i < count; ++i) { fputs(out[i], f); fputc('\n', f); free(out[i]); }
  fclose(f);
  return 0;
}
