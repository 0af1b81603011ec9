/*
 * jws_oracle.h -- CPU restatement of the JWS signature arithmetic on cap's
 * verify path.  TEST INFRASTRUCTURE ONLY: imported by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg.
 * The product (cap_amd/, libcapjwt.so) never links or calls this.
 *
 * The reference (hashicorp/cap, Go) delegates this arithmetic to third-party
 * code that is NOT under /root/reference:
 *   gopkg.in/square/go-jose.v2 v2.5.1            (go.mod:19, go.sum:48)
 *   Go stdlib crypto/rsa, crypto/ecdsa, crypto/ed25519, crypto/sha256|512
 *   golang.org/x/crypto v0.0.0-20200622213623    (go.sum:24, ed25519 alias)
 * reached from jwt/keyset.go:155,163 and jwt/jwt.go:212.  Each function below
 * restates the published algorithm of those pinned versions (SURVEY.md
 * Appendix A rule numbers in brackets).  Parity pinning: see DESIGN.md
 * "Oracle" -- OpenSSL-generated golden vectors (tests/golden), FIPS 180-4 and
 * RFC 8032 known answers.
 */
#ifndef JWS_ORACLE_H
#define JWS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* algorithm ids (match include/jg.h JG_ALG_*) -- jwt/algs.go:12-21 */
enum { OR_RS256 = 1, OR_RS384, OR_RS512, OR_PS256, OR_PS384, OR_PS512,
       OR_ES256, OR_ES384, OR_ES512, OR_EDDSA };
enum { OR_P256 = 1, OR_P384 = 2, OR_P521 = 3 };

void or_sha256(const uint8_t* m, size_t n, uint8_t out[32]);
void or_sha384(const uint8_t* m, size_t n, uint8_t out[48]);
void or_sha512(const uint8_t* m, size_t n, uint8_t out[64]);

/* go-jose base64URLDecode [R3]: TrimRight '=', RawURLEncoding, '\r' '\n'
 * skipped, non-zero trailing bits accepted.  Returns decoded length or -1. */
long or_b64url_decode(const char* s, size_t n, uint8_t* out, size_t cap);

/* crypto/rsa VerifyPKCS1v15 / VerifyPSS(opts=nil) behind go-jose's
 * rsaEncrypterVerifier [R9, R12-R17].  n big-endian (leading zeros ok).
 * Returns 1 accept, 0 reject. */
int or_rsa_verify(int alg, const uint8_t* n, size_t nlen, uint64_t e,
                  const uint8_t* msg, size_t mlen, const uint8_t* sig, size_t slen);

/* go-jose ecEncrypterVerifier + crypto/ecdsa.Verify [R18-R22]; curve from the
 * key, sig size and hash from the alg.  x,y big-endian coord_len bytes. */
int or_ecdsa_verify(int alg, int curve, const uint8_t* x, const uint8_t* y, size_t coord_len,
                    const uint8_t* msg, size_t mlen, const uint8_t* sig, size_t slen);

/* 1 if (x,y) is a valid point of the curve with coordinates in [0,p). */
int or_ec_point_valid(int curve, const uint8_t* x, const uint8_t* y, size_t coord_len);

/* crypto/ed25519.Verify [R23-R26]. */
int or_ed25519_verify(const uint8_t pub[32], const uint8_t* msg, size_t mlen,
                      const uint8_t* sig, size_t slen);

/* Raw RSA public operation for tests: out = sig^e mod n (k bytes, big-endian).
 * Returns 0, or -1 if sig >= n. */
int or_rsa_public(const uint8_t* n, size_t nlen, uint64_t e, const uint8_t* sig, size_t slen,
                  uint8_t* out);

/* Verify `count` (alg,key,msg,sig) jobs on `threads` pthreads (bench CPU leg).
 * key_kind: 0 RSA (n,nlen,e), 1 EC (curve,x,y,coord_len), 2 Ed25519 (x).   */
typedef struct {
  int alg, key_kind, curve;
  const uint8_t *n, *x, *y; size_t nlen, coord_len; uint64_t e;
  const uint8_t* msg; size_t mlen; const uint8_t* sig; size_t slen;
} or_job;
void or_verify_many(const or_job* jobs, size_t count, int threads, uint8_t* verdicts);

#ifdef __cplusplus
}
#endif
#endif
