// jose.hpp -- host-side restatement of the go-jose v2.5.1 pieces that sit in
// front of the signature arithmetic on cap's verify path (SURVEY.md §8 rows
// a5, a6, a15; Appendix A R1-R8, R27-R32).  Everything here is byte/JSON
// handling; the signature checks themselves run on the GPU (include/jg.h).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "json.hpp"

namespace capjwt {

// ---------------------------------------------------------------- algorithms
// jwt/algs.go:12-21 -- index = enum jg_alg (0 = not one of the 10)
int alg_id(std::string_view alg);
const char* alg_name(int id);
int alg_key_kind(int id);           // JG_KEY_RSA / JG_KEY_EC / JG_KEY_ED25519, 0 for none

// ---------------------------------------------------------------- base64url
// go-jose base64URLDecode (encoding.go): TrimRight(s, "="), then
// base64.RawURLEncoding.DecodeString -- '\r' and '\n' are skipped, non-zero
// trailing bits are accepted, a final group of one character is an error.
// Returns false on error (err = Go's "illegal base64 data at input byte N").
bool b64url_decode(std::string_view s, std::string* out, std::string* err = nullptr);
// base64.RawURLEncoding.DecodeString itself ('=' is an illegal byte), as cap's
// oidc.UnmarshalClaims calls it (oidc/token.go:176).
bool b64rawurl_decode(std::string_view s, std::string* out, std::string* err = nullptr);
std::string b64url_encode(std::string_view raw);
// Go base64.StdEncoding.DecodeString (x5c entries): padded, strict length.
bool b64std_decode(std::string_view s, std::string* out);
// True iff decoding s and re-encoding it gives s back: no '=', no CR/LF, no
// unused non-zero bits.  Only then is the literal token text the
// signing input.
bool b64url_canonical(std::string_view s);
// Fast path of b64url_decode for a segment of alphabet characters only (no
// '=', CR, LF or other byte): decodes into out[0 .. s.size()*3/4] and returns
// the length, with *canonical = b64url_canonical(s).  Returns -1 if s holds any
// other byte or ends in a 1-character group; the caller then takes
// b64url_decode (which reproduces Go's skipping and error text).
long b64url_decode_fast(std::string_view s, char* out, bool* canonical);

// go-jose stripWhitespace: removes every rune for which unicode.IsSpace holds;
// invalid UTF-8 bytes become U+FFFD (ranging over a Go string).
bool has_go_space_or_nonascii(std::string_view s);
std::string strip_whitespace(std::string_view s);

// ---------------------------------------------------------------- keys
// crypto.PublicKey as go-jose/cap see it.
struct PublicKey {
  enum Kind { None = 0, RSA = 1, EC = 2, Ed25519 = 3, Symmetric = 4 };
  Kind kind = None;
  std::string n;          // RSA modulus, big-endian, leading zeros stripped
  uint64_t e = 0;         // RSA exponent: low 64 bits of big.Int (go-jose toInt)
  int curve = 0;          // 1 = P-256, 2 = P-384, 3 = P-521
  std::string x, y;       // EC coordinates, fixed width; Ed25519: x = 32 raw bytes
  std::string k;          // oct (HMAC) secret -- never verifies on this path
  bool operator==(const PublicKey& o) const {
    return kind == o.kind && n == o.n && e == o.e && curve == o.curve && x == o.x && y == o.y && k == o.k;
  }
};

struct JSONWebKey {
  PublicKey key;
  std::string kid, alg, use;
};

// go-jose JSONWebKey.UnmarshalJSON (jwk.go) for public keys; private members
// (d, p, q, ...) are parsed for validity and then dropped.  False + err on the
// errors go-jose returns (unknown kty/crv, wrong coordinate length, point not
// on the curve, missing n/e/x/y, x5c that does not parse or does not match).
bool jwk_from_json(const json::Value& v, JSONWebKey* out, std::string* err);
// go-oidc v2.2.1 updateKeys: jose.JSONWebKeySet decode of a JWKS document; any
// bad key fails the whole document (R28, R30).
bool jwks_decode(std::string_view doc, std::vector<JSONWebKey>* out, std::string* err);

// curve.IsOnCurve(x, y) for P-256/384/521 (big-endian, any length)
bool ec_on_curve(int curve, std::string_view x, std::string_view y);

// cap ParsePublicKeyPEM (jwt/keyset.go:178-200): first PEM block, PKIX public
// key, else X.509 certificate; RSA or ECDSA only.
bool parse_public_key_pem(std::string_view data, PublicKey* out, std::string* err);
// x509.ParsePKIXPublicKey subset: RSA, ECDSA (named P-256/384/521), Ed25519.
bool parse_pkix_public_key(std::string_view der, PublicKey* out, std::string* err);
// x509.ParseCertificate, reduced to what this path needs: the structure is
// walked and the SubjectPublicKeyInfo decoded.
bool parse_certificate_public_key(std::string_view der, PublicKey* out, std::string* err);

// ---------------------------------------------------------------- JWS parse
struct Signature {
  std::string protected_raw;     // decoded protected header bytes ("" if absent)
  bool has_protected = false;
  json::Value protected_hdr;     // parsed protected header (Object) if has_protected
  json::Value unprotected_hdr;   // JSON serialization "header" member (Object) or Null
  std::string signature;         // decoded signature bytes
  // merged header (protected wins over unprotected), sanitised
  std::string alg, kid;
  bool has_jwk = false;
};

struct JWS {
  std::string payload;               // decoded payload
  std::vector<Signature> sigs;
  bool compact = true;
  // compact form: spans of the literal token text (valid when compact)
  size_t seg1_end = 0, seg2_end = 0;
};

// jose.ParseSigned (jws.go): whitespace strip, compact or JSON serialization,
// header sanitisation.  False + err = a parse error (the token is rejected).
bool parse_signed(std::string_view token, JWS* out, std::string* err);

// What DetachedVerify checks before the arithmetic, for signature 0:
// len(sigs) == 1, crit members understood, then computeAuthData.  False if
// the token can never verify (go-jose returns ErrCryptoFailure).
bool signing_input(const JWS& jws, std::string* out);

}  // namespace capjwt
