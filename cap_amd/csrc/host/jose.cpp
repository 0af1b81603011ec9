// jose.cpp -- see jose.hpp.  Restates go-jose v2.5.1 (jws.go, encoding.go,
// jwk.go, shared.go), Go's encoding/pem, crypto/x509 public-key parsing and
// crypto/elliptic IsOnCurve for the verify path.  SURVEY.md Appendix A rules
// are cited inline.
#include "jose.hpp"

#include <algorithm>
#include <cstring>

#include "../../../include/jg.h"

namespace capjwt {

// ====================================================================== algs
namespace {
const char* const kAlgNames[11] = {"", "RS256", "RS384", "RS512", "PS256", "PS384",
                                   "PS512", "ES256", "ES384", "ES512", "EdDSA"};
}

int alg_id(std::string_view alg) {
  for (int i = 1; i <= 10; ++i)
    if (alg == kAlgNames[i]) return i;
  return 0;
}
const char* alg_name(int id) { return id >= 1 && id <= 10 ? kAlgNames[id] : ""; }
int alg_key_kind(int id) {
  if (id >= JG_RS256 && id <= JG_PS512) return JG_KEY_RSA;
  if (id >= JG_ES256 && id <= JG_ES512) return JG_KEY_EC;
  if (id == JG_EDDSA) return JG_KEY_ED25519;
  return 0;
}

// ====================================================================== base64
namespace {
struct B64Tables {
  int8_t url[256], std_[256];
  B64Tables() {
    std::memset(url, -1, sizeof(url));
    std::memset(std_, -1, sizeof(std_));
    const char* u = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    const char* s = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) {
      url[(unsigned char)u[i]] = (int8_t)i;
      std_[(unsigned char)s[i]] = (int8_t)i;
    }
  }
};
const B64Tables& tabs() {
  static const B64Tables t;
  return t;
}
const char kUrlAlpha[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

// encoding/base64 Decode without padding (RawURLEncoding, non-strict):
// CR/LF anywhere are skipped; a final quantum of 1 symbol is an error.
bool raw_decode(const int8_t* tab, std::string_view s, std::string* out, std::string* err) {
  out->clear();
  out->reserve(s.size() * 3 / 4 + 3);
  uint32_t acc = 0;
  int nq = 0;
  size_t last = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = (unsigned char)s[i];
    if (c == '\r' || c == '\n') continue;
    const int v = tab[c];
    if (v < 0) {
      if (err) *err = "illegal base64 data at input byte " + std::to_string(i);
      return false;
    }
    last = i;
    acc = acc << 6 | (uint32_t)v;
    if (++nq == 4) {
      out->push_back((char)(acc >> 16));
      out->push_back((char)(acc >> 8));
      out->push_back((char)acc);
      acc = 0;
      nq = 0;
    }
  }
  if (nq == 1) {
    if (err) *err = "illegal base64 data at input byte " + std::to_string(last);
    return false;
  }
  if (nq == 2) {
    out->push_back((char)(acc >> 4));
  } else if (nq == 3) {
    out->push_back((char)(acc >> 10));
    out->push_back((char)(acc >> 2));
  }
  return true;
}
}  // namespace

bool b64url_decode(std::string_view s, std::string* out, std::string* err) {
  // go-jose base64URLDecode: strings.TrimRight(value, "=")   [R3]
  size_t n = s.size();
  while (n > 0 && s[n - 1] == '=') --n;
  out->resize(n / 4 * 3 + 2);
  bool canon;
  const long len = b64url_decode_fast(s.substr(0, n), out->data(), &canon);
  if (len >= 0) {
    out->resize((size_t)len);
    return true;
  }
  return raw_decode(tabs().url, s.substr(0, n), out, err);
}

bool b64rawurl_decode(std::string_view s, std::string* out, std::string* err) {
  return raw_decode(tabs().url, s, out, err);
}

std::string b64url_encode(std::string_view raw) {
  std::string o;
  o.reserve((raw.size() * 4 + 2) / 3);
  const unsigned char* p = (const unsigned char*)raw.data();
  size_t i = 0;
  for (; i + 3 <= raw.size(); i += 3) {
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    o.push_back(kUrlAlpha[v >> 18]);
    o.push_back(kUrlAlpha[(v >> 12) & 63]);
    o.push_back(kUrlAlpha[(v >> 6) & 63]);
    o.push_back(kUrlAlpha[v & 63]);
  }
  const size_t r = raw.size() - i;
  if (r == 1) {
    const uint32_t v = (uint32_t)p[i] << 16;
    o.push_back(kUrlAlpha[v >> 18]);
    o.push_back(kUrlAlpha[(v >> 12) & 63]);
  } else if (r == 2) {
    const uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8;
    o.push_back(kUrlAlpha[v >> 18]);
    o.push_back(kUrlAlpha[(v >> 12) & 63]);
    o.push_back(kUrlAlpha[(v >> 6) & 63]);
  }
  return o;
}

bool b64std_decode(std::string_view s, std::string* out) {
  // base64.StdEncoding.DecodeString: padded quanta, CR/LF skipped
  std::string clean;
  clean.reserve(s.size());
  for (char c : s)
    if (c != '\r' && c != '\n') clean.push_back(c);
  if (clean.size() % 4) return false;
  size_t pad = 0;
  while (pad < 2 && pad < clean.size() && clean[clean.size() - 1 - pad] == '=') ++pad;
  const std::string_view body(clean.data(), clean.size() - pad);
  if (body.find('=') != std::string_view::npos) return false;
  std::string err;
  return raw_decode(tabs().std_, body, out, &err);
}

bool b64url_canonical(std::string_view s) {
  const int8_t* t = tabs().url;
  for (char c : s)
    if (t[(unsigned char)c] < 0) return false;          // also rejects '=', CR, LF
  const size_t r = s.size() % 4;
  if (r == 1) return false;
  if (r == 0 || s.empty()) return true;
  const int v = t[(unsigned char)s.back()];
  return r == 2 ? (v & 15) == 0 : (v & 3) == 0;          // unused low bits must be zero
}

long b64url_decode_fast(std::string_view s, char* out, bool* canonical) {
  // 4 characters -> 3 bytes per step; an invalid symbol has the table's sign
  // bit, so one OR over the group detects it
  const int8_t* t = tabs().url;
  const unsigned char* p = (const unsigned char*)s.data();
  const size_t n = s.size(), full = n / 4 * 4;
  unsigned char* o = (unsigned char*)out;
  for (size_t i = 0; i < full; i += 4) {
    const int32_t a = t[p[i]], b = t[p[i + 1]], c = t[p[i + 2]], d = t[p[i + 3]];
    if ((a | b | c | d) < 0) return -1;
    const uint32_t v = (uint32_t)a << 18 | (uint32_t)b << 12 | (uint32_t)c << 6 | (uint32_t)d;
    o[0] = (unsigned char)(v >> 16);
    o[1] = (unsigned char)(v >> 8);
    o[2] = (unsigned char)v;
    o += 3;
  }
  const size_t r = n - full;
  bool canon = true;
  if (r == 1) return -1;
  if (r == 2) {
    const int32_t a = t[p[full]], b = t[p[full + 1]];
    if ((a | b) < 0) return -1;
    *o++ = (unsigned char)((a << 2) | (b >> 4));
    canon = (b & 15) == 0;
  } else if (r == 3) {
    const int32_t a = t[p[full]], b = t[p[full + 1]], c = t[p[full + 2]];
    if ((a | b | c) < 0) return -1;
    const uint32_t v = (uint32_t)a << 12 | (uint32_t)b << 6 | (uint32_t)c;
    *o++ = (unsigned char)(v >> 10);
    *o++ = (unsigned char)(v >> 2);
    canon = (c & 3) == 0;
  }
  *canonical = canon;
  return (long)(o - (unsigned char*)out);
}

// ====================================================================== whitespace
namespace {
bool go_is_space(uint32_t r) {
  switch (r) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
    case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000:
      return true;
    default:
      return r >= 0x2000 && r <= 0x200A;
  }
}
}  // namespace

bool has_go_space_or_nonascii(std::string_view s) {
  // 8 bytes at a time: a byte >= 0x80, or a byte < 0x21 (SWAR "has less than")
  constexpr uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
  size_t i = 0;
  for (; i + 8 <= s.size(); i += 8) {
    uint64_t w;
    std::memcpy(&w, s.data() + i, 8);
    if ((w & highs) | ((w - ones * 0x21) & ~w & highs)) return true;
  }
  for (char ch : s.substr(i)) {
    const unsigned char c = (unsigned char)ch;
    if (c >= 0x80 || c <= ' ') return true;
  }
  return false;
}

std::string strip_whitespace(std::string_view s) {
  // go-jose stripWhitespace: `for _, r := range data { if !unicode.IsSpace(r) { buf.WriteRune(r) } }`  [R1]
  std::string o;
  o.reserve(s.size());
  const unsigned char* p = (const unsigned char*)s.data();
  for (size_t i = 0; i < s.size();) {
    size_t w;
    const uint32_t r = json::decode_rune(p + i, s.size() - i, &w);
    if (!go_is_space(r)) {
      if (r == 0xFFFD && w == 1) json::put_utf8(o, 0xFFFD);
      else o.append((const char*)p + i, w);
    }
    i += w;
  }
  return o;
}

// ====================================================================== bignum (key ingestion only)
namespace {
struct Big {
  std::vector<uint32_t> w;   // little-endian 32-bit words, trimmed
  void trim() { while (!w.empty() && w.back() == 0) w.pop_back(); }
  static Big from_be(std::string_view b) {
    Big r;
    r.w.assign((b.size() + 3) / 4, 0);
    for (size_t i = 0; i < b.size(); ++i) {
      const size_t bit = (b.size() - 1 - i) * 8;
      r.w[bit / 32] |= (uint32_t)(unsigned char)b[i] << (bit % 32);
    }
    r.trim();
    return r;
  }
  static Big from_hex(const char* h) {
    std::string b;
    const size_t n = std::strlen(h);
    for (size_t i = 0; i + 1 < n; i += 2) {
      auto hv = [](char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; };
      b.push_back((char)(hv(h[i]) << 4 | hv(h[i + 1])));
    }
    return from_be(b);
  }
  size_t bits() const {
    if (w.empty()) return 0;
    size_t n = (w.size() - 1) * 32;
    uint32_t t = w.back();
    while (t) { ++n; t >>= 1; }
    return n;
  }
  bool bit(size_t i) const { return i / 32 < w.size() && ((w[i / 32] >> (i % 32)) & 1); }
};
int cmp(const Big& a, const Big& b) {
  if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
  for (size_t i = a.w.size(); i-- > 0;)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
Big add(const Big& a, const Big& b) {
  Big r;
  const size_t n = std::max(a.w.size(), b.w.size());
  r.w.assign(n + 1, 0);
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c += (uint64_t)(i < a.w.size() ? a.w[i] : 0) + (i < b.w.size() ? b.w[i] : 0);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  r.w[n] = (uint32_t)c;
  r.trim();
  return r;
}
Big sub(const Big& a, const Big& b) {   // a >= b
  Big r;
  r.w.assign(a.w.size(), 0);
  int64_t br = 0;
  for (size_t i = 0; i < a.w.size(); ++i) {
    int64_t d = (int64_t)a.w[i] - (i < b.w.size() ? b.w[i] : 0) - br;
    br = d < 0;
    r.w[i] = (uint32_t)(d + (br << 32));
  }
  r.trim();
  return r;
}
Big mul(const Big& a, const Big& b) {
  Big r;
  r.w.assign(a.w.size() + b.w.size() + 1, 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.w.size(); ++j) {
      c += (uint64_t)a.w[i] * b.w[j] + r.w[i + j];
      r.w[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r.w[i + b.w.size()] += (uint32_t)c;
  }
  r.trim();
  return r;
}
Big mod(const Big& a, const Big& m) {   // binary long division
  Big r;
  for (size_t i = a.bits(); i-- > 0;) {
    r = add(r, r);
    if (a.bit(i)) r = add(r, Big{{1}});
    if (cmp(r, m) >= 0) r = sub(r, m);
  }
  return r;
}

const char* const kCurveP[4] = {
    nullptr, "ffffffff00000001000000000000000000000000ffffffffffffffffffffffff",
    "fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffeffffffff0000000000000000ffffffff",
    "01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff"
    "ffffffffffffffffffffffffffffff"};
const char* const kCurveB[4] = {
    nullptr, "5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b",
    "b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef",
    "0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf07357"
    "3df883d2c34f1ef451fd46b503f00"};
}  // namespace

bool ec_on_curve(int curve, std::string_view xb, std::string_view yb) {
  if (curve < 1 || curve > 3) return false;
  const Big p = Big::from_hex(kCurveP[curve]), b = Big::from_hex(kCurveB[curve]);
  const Big x = Big::from_be(xb), y = Big::from_be(yb);
  if (cmp(x, p) >= 0 || cmp(y, p) >= 0) return false;        // IsOnCurve: 0 <= x, y < p
  // y^2 == x^3 - 3x + b  (mod p)
  const Big y2 = mod(mul(y, y), p);
  const Big x3 = mod(mul(mod(mul(x, x), p), x), p);
  const Big three_x = mod(mul(x, Big{{3}}), p);
  Big rhs = add(x3, b);
  rhs = mod(add(rhs, sub(p, three_x)), p);
  return cmp(y2, rhs) == 0;
}

// ====================================================================== DER / PKIX
namespace {
struct Der {
  const unsigned char* p;
  const unsigned char* end;
  // read one TLV; out = contents
  bool read(unsigned tag, std::string_view* out) {
    if (end - p < 2 || *p != tag) return false;
    ++p;
    size_t len = *p++;
    if (len & 0x80) {
      const size_t nb = len & 0x7F;
      if (nb == 0 || nb > 4 || (size_t)(end - p) < nb) return false;
      len = 0;
      for (size_t i = 0; i < nb; ++i) len = len << 8 | *p++;
      if (len < 128 || (nb > 1 && (len >> ((nb - 1) * 8)) == 0)) return false;   // non-minimal length
    }
    if ((size_t)(end - p) < len) return false;
    *out = std::string_view((const char*)p, len);
    p += len;
    return true;
  }
  bool peek(unsigned tag) const { return p < end && *p == tag; }
  bool skip_any() {
    if (end - p < 2) return false;
    const unsigned tag = *p;
    std::string_view t;
    return read(tag, &t);
  }
  bool empty() const { return p == end; }
  static Der of(std::string_view s) { return Der{(const unsigned char*)s.data(), (const unsigned char*)s.data() + s.size()}; }
};

// DER INTEGER contents -> big-endian magnitude; false if negative / non-minimal
bool der_uint(std::string_view c, std::string* mag, bool* positive) {
  if (c.empty()) return false;
  if (c.size() > 1 && ((c[0] == 0 && !((unsigned char)c[1] & 0x80)) || ((unsigned char)c[0] == 0xFF && ((unsigned char)c[1] & 0x80))))
    return false;                                   // cryptobyte: non-minimal encoding
  if ((unsigned char)c[0] & 0x80) { *positive = false; mag->clear(); return true; }
  size_t i = 0;
  while (i < c.size() && c[i] == 0) ++i;
  mag->assign(c.substr(i));
  *positive = !mag->empty();
  return true;
}

const std::string_view kOidRSA("\x2a\x86\x48\x86\xf7\x0d\x01\x01\x01", 9);
const std::string_view kOidEC("\x2a\x86\x48\xce\x3d\x02\x01", 7);
const std::string_view kOidEd25519("\x2b\x65\x70", 3);
const std::string_view kOidP256("\x2a\x86\x48\xce\x3d\x03\x01\x07", 8);
const std::string_view kOidP384("\x2b\x81\x04\x00\x22", 5);
const std::string_view kOidP521("\x2b\x81\x04\x00\x23", 5);
}  // namespace

bool parse_pkix_public_key(std::string_view der, PublicKey* out, std::string* err) {
  auto bad = [&](const char* m) { if (err) *err = m; return false; };
  Der d = Der::of(der);
  std::string_view spki, alg, bits;
  if (!d.read(0x30, &spki) || !d.empty()) return bad("x509: malformed public key");
  Der s = Der::of(spki);
  // encoding/asn1 (ParsePKIXPublicKey) and cryptobyte (ParseCertificate) both
  // ignore elements after the ones they read, in the SubjectPublicKeyInfo and
  // in its AlgorithmIdentifier ("We allow extra bytes at the end of the
  // SEQUENCE because adding elements to the end has been used in X.509")
  if (!s.read(0x30, &alg) || !s.read(0x03, &bits)) return bad("x509: malformed public key");
  Der a = Der::of(alg);
  std::string_view oid, params;
  if (!a.read(0x06, &oid)) return bad("x509: malformed public key algorithm identifier");
  const bool has_params = !a.empty();
  const unsigned ptag = has_params ? *a.p : 0;
  const unsigned char* pstart = a.p;
  if (has_params && !a.skip_any()) return bad("x509: malformed public key algorithm identifier");
  if (has_params) params = std::string_view((const char*)pstart, (size_t)(a.p - pstart));   // the first element only
  if (bits.empty() || bits[0] != 0) return bad("x509: malformed public key");   // unused bits must be 0
  const std::string_view key = bits.substr(1);
  if (oid == kOidRSA) {
    // x509 parsePublicKey RSA: NULL parameters, RSAPublicKey ::= SEQUENCE { n, e }
    if (!has_params || ptag != 0x05 || params.size() != 2 || params[1] != 0)
      return bad("x509: RSA key missing NULL parameters");
    Der k = Der::of(key);
    std::string_view seq, ni, ei;
    if (!k.read(0x30, &seq)) return bad("x509: invalid RSA public key");
    Der q = Der::of(seq);                         // trailing bytes are not checked (cryptobyte reads)
    if (!q.read(0x02, &ni)) return bad("x509: invalid RSA modulus");
    if (!q.read(0x02, &ei)) return bad("x509: invalid RSA public exponent");
    std::string n, e;
    bool npos, epos;
    if (!der_uint(ni, &n, &npos)) return bad("x509: invalid RSA modulus");
    if (!der_uint(ei, &e, &epos) || e.size() > 8 || (e.size() == 8 && ((unsigned char)e[0] & 0x80)))
      return bad("x509: invalid RSA public exponent");
    if (!npos) return bad("x509: RSA modulus is not a positive number");
    if (!epos) return bad("x509: RSA public exponent is not a positive number");
    uint64_t ev = 0;
    for (unsigned char c : e) ev = ev << 8 | c;
    out->kind = PublicKey::RSA;
    out->n = n;
    out->e = ev;
    return true;
  }
  if (oid == kOidEC) {
    std::string_view cur;
    Der pp = Der::of(params);
    if (!has_params || !pp.read(0x06, &cur)) return bad("x509: invalid ECDSA parameters");
    const int curve = cur == kOidP256 ? 1 : cur == kOidP384 ? 2 : cur == kOidP521 ? 3 : 0;
    if (!curve) return bad("x509: unsupported elliptic curve");
    const size_t cb = curve == 1 ? 32 : curve == 2 ? 48 : 66;
    // elliptic.Unmarshal: uncompressed point only, coordinates < p, on the curve
    if (key.size() != 1 + 2 * cb || key[0] != 4) return bad("x509: failed to unmarshal elliptic curve point");
    const std::string_view x = key.substr(1, cb), y = key.substr(1 + cb, cb);
    if (!ec_on_curve(curve, x, y)) return bad("x509: failed to unmarshal elliptic curve point");
    out->kind = PublicKey::EC;
    out->curve = curve;
    out->x.assign(x);
    out->y.assign(y);
    return true;
  }
  if (oid == kOidEd25519) {
    if (has_params) return bad("x509: Ed25519 key encoded with illegal parameters");
    if (key.size() != 32) return bad("x509: wrong Ed25519 public key size");
    out->kind = PublicKey::Ed25519;
    out->x.assign(key);
    return true;
  }
  return bad("x509: unknown public key algorithm");
}

bool parse_certificate_public_key(std::string_view der, PublicKey* out, std::string* err) {
  auto bad = [&](const char* m) { if (err) *err = m; return false; };
  Der d = Der::of(der);
  std::string_view cert, tbs, sigalg, sigval;
  if (!d.read(0x30, &cert) || !d.empty()) return bad("x509: malformed certificate");
  Der c = Der::of(cert);
  if (!c.read(0x30, &tbs) || !c.read(0x30, &sigalg) || !c.read(0x03, &sigval) || !c.empty())
    return bad("x509: malformed certificate");
  Der t = Der::of(tbs);
  std::string_view f;
  if (t.peek(0xA0) && !t.read(0xA0, &f)) return bad("x509: malformed version");
  if (!t.read(0x02, &f)) return bad("x509: malformed serial number");
  if (!t.read(0x30, &f)) return bad("x509: malformed signature algorithm identifier");
  if (!t.read(0x30, &f)) return bad("x509: malformed issuer");
  if (!t.read(0x30, &f)) return bad("x509: malformed validity");
  if (!t.read(0x30, &f)) return bad("x509: malformed subject");
  const unsigned char* spki_begin = t.p;
  if (!t.read(0x30, &f)) return bad("x509: malformed spki");
  const std::string_view spki((const char*)spki_begin, (size_t)(t.p - spki_begin));
  std::string e2;
  if (!parse_pkix_public_key(spki, out, &e2)) {
    // Go: an unknown algorithm leaves cert.PublicKey nil (no error)
    if (e2 == "x509: unknown public key algorithm") { out->kind = PublicKey::None; return true; }
    return bad(e2.c_str());
  }
  return true;
}

bool parse_public_key_pem(std::string_view data, PublicKey* out, std::string* err) {
  // encoding/pem.Decode: the first well-formed block (any type)
  const std::string_view kBegin("-----BEGIN ");
  const std::string_view kEnd("-----END ");
  std::string_view rest = data;
  while (true) {
    size_t at;
    if (rest.substr(0, kBegin.size()) == kBegin) {
      at = 0;
    } else {
      const size_t q = rest.find(std::string("\n") + std::string(kBegin));
      if (q == std::string_view::npos) break;
      at = q + 1;
    }
    rest = rest.substr(at + kBegin.size());
    const size_t nl = rest.find('\n');
    std::string_view type_line = rest.substr(0, nl);
    while (!type_line.empty() && (type_line.back() == '\r' || type_line.back() == ' ' || type_line.back() == '\t'))
      type_line.remove_suffix(1);
    rest = nl == std::string_view::npos ? std::string_view() : rest.substr(nl + 1);
    if (type_line.size() < 5 || type_line.substr(type_line.size() - 5) != "-----") continue;
    const std::string_view type = type_line.substr(0, type_line.size() - 5);
    // headers ("Key: value" lines) are skipped
    while (!rest.empty()) {
      const size_t e = rest.find('\n');
      const std::string_view line = rest.substr(0, e);
      if (line.find(':') == std::string_view::npos) break;
      rest = e == std::string_view::npos ? std::string_view() : rest.substr(e + 1);
    }
    size_t end_idx;
    if (rest.substr(0, kEnd.size()) == kEnd) {
      end_idx = 0;
    } else {
      end_idx = rest.find(std::string("\n") + std::string(kEnd));
      if (end_idx == std::string_view::npos) continue;
      end_idx += 1;
    }
    const std::string_view trailer = rest.substr(end_idx + kEnd.size());
    if (trailer.substr(0, type.size()) != type || trailer.substr(type.size(), 5) != "-----") continue;
    std::string b64;
    for (char ch : rest.substr(0, end_idx))
      if (ch != ' ' && ch != '\t') b64.push_back(ch);
    std::string der;
    if (!b64std_decode(b64, &der)) continue;
    // cap ParsePublicKeyPEM: PKIX, else certificate; RSA or ECDSA only  [R32]
    PublicKey k;
    std::string e1, e2;
    if (!parse_pkix_public_key(der, &k, &e1)) {
      if (!parse_certificate_public_key(der, &k, &e2)) {
        if (err) *err = e2;                       // Go returns the certificate error
        return false;
      }
    }
    if (k.kind == PublicKey::RSA || k.kind == PublicKey::EC) {
      *out = k;
      return true;
    }
    break;
  }
  if (err) *err = "data does not contain any valid RSA or ECDSA public keys";
  return false;
}

// ====================================================================== JWK
namespace {
// go-jose byteBuffer member: absent/null -> not present; "" -> present, empty
struct BB {
  bool present = false;
  std::string data;
};

bool get_bb(const json::Value& o, const char* name, BB* out, std::string* err) {
  const json::Value* v = o.get(name);
  if (!v || v->is_null()) return true;
  if (v->kind != json::Value::String) { *err = std::string("json: cannot unmarshal into byteBuffer field ") + name; return false; }
  out->present = true;
  if (v->str.empty()) return true;
  return b64url_decode(v->str, &out->data, err);
}
bool get_str(const json::Value& o, const char* name, std::string* out, std::string* err) {
  const json::Value* v = o.get(name);
  if (!v || v->is_null()) return true;
  if (v->kind != json::Value::String) { *err = std::string("json: cannot unmarshal into string field ") + name; return false; }
  *out = v->str;
  return true;
}
std::string strip_zeros(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && s[i] == 0) ++i;
  return s.substr(i);
}
// big.Int.Int64() of a big-endian magnitude: the low 64 bits
uint64_t low64(const std::string& s) {
  uint64_t v = 0;
  const size_t from = s.size() > 8 ? s.size() - 8 : 0;
  for (size_t i = from; i < s.size(); ++i) v = v << 8 | (unsigned char)s[i];
  return v;
}
}  // namespace

bool jwk_from_json(const json::Value& v, JSONWebKey* out, std::string* err) {
  if (v.kind != json::Value::Object) {
    *err = "json: cannot unmarshal into rawJSONWebKey";
    return false;
  }
  std::string kty, crv;
  JSONWebKey k;
  std::string dummy;
  BB n, e, x, y, d, kk, p, q;
  if (!get_str(v, "kty", &kty, err) || !get_str(v, "crv", &crv, err) || !get_str(v, "kid", &k.kid, err) ||
      !get_str(v, "alg", &k.alg, err) || !get_str(v, "use", &k.use, err) || !get_str(v, "x5u", &dummy, err) ||
      !get_str(v, "x5t", &dummy, err) || !get_str(v, "x5t#S256", &dummy, err))
    return false;
  if (!get_bb(v, "n", &n, err) || !get_bb(v, "e", &e, err) || !get_bb(v, "x", &x, err) || !get_bb(v, "y", &y, err) ||
      !get_bb(v, "d", &d, err) || !get_bb(v, "k", &kk, err) || !get_bb(v, "p", &p, err) || !get_bb(v, "q", &q, err))
    return false;
  for (const char* nm : {"dp", "dq", "qi"}) {
    BB t;
    if (!get_bb(v, nm, &t, err)) return false;
  }
  // x5c: []string of std-base64 DER certificates
  PublicKey cert_pub;
  bool have_cert = false;
  if (const json::Value* c = v.get("x5c"); c && !c->is_null()) {
    if (c->kind != json::Value::Array) { *err = "json: cannot unmarshal x5c"; return false; }
    for (size_t i = 0; i < c->arr.size(); ++i) {
      const json::Value& s = c->arr[i];
      if (s.kind != json::Value::String) { *err = "json: cannot unmarshal x5c"; return false; }
      std::string der;
      if (!b64std_decode(s.str, &der)) {
        *err = "square/go-jose: failed to unmarshal x5c field: illegal base64 data";
        return false;
      }
      PublicKey pk;
      std::string e2;
      if (!parse_certificate_public_key(der, &pk, &e2)) {
        *err = "square/go-jose: failed to unmarshal x5c field: " + e2;
        return false;
      }
      if (i == 0) { cert_pub = pk; have_cert = true; }
    }
  }
  bool is_public = !d.present;
  if (kty == "EC") {
    const int curve = crv == "P-256" ? 1 : crv == "P-384" ? 2 : crv == "P-521" ? 3 : 0;
    if (!curve) { *err = "square/go-jose: unsupported elliptic curve '" + crv + "'"; return false; }
    if (!x.present || !y.present) {
      *err = d.present ? "square/go-jose: invalid EC private key, missing x/y/d values"
                       : "square/go-jose: invalid EC key, missing x/y values";
      return false;
    }
    const size_t cb = curve == 1 ? 32 : curve == 2 ? 48 : 66;
    if (d.present && d.data.size() != cb) {      // dSize(curve): byte length of the group order
      *err = "square/go-jose: invalid EC private key, wrong length for d";
      return false;
    }
    if (x.data.size() != cb) { *err = "square/go-jose: invalid EC public key, wrong length for x"; return false; }
    if (y.data.size() != cb) { *err = "square/go-jose: invalid EC public key, wrong length for y"; return false; }
    if (!ec_on_curve(curve, x.data, y.data)) {
      *err = "square/go-jose: invalid EC key, X/Y are not on declared curve";
      return false;
    }
    k.key.kind = PublicKey::EC;
    k.key.curve = curve;
    k.key.x = x.data;
    k.key.y = y.data;
  } else if (kty == "RSA") {
    if (!n.present || !e.present) { *err = "square/go-jose: invalid RSA key, missing n/e values"; return false; }
    if (d.present && (!p.present || !q.present)) {
      *err = "square/go-jose: invalid RSA private key, missing values";
      return false;
    }
    k.key.kind = PublicKey::RSA;
    k.key.n = strip_zeros(n.data);
    k.key.e = low64(e.data);          // go-jose toInt: int(bigInt.Int64())  [R27]
  } else if (kty == "oct") {
    if (have_cert) { *err = "square/go-jose: invalid JWK, found 'oct' (symmetric) key with cert chain"; return false; }
    if (!kk.present) { *err = "square/go-jose: invalid OCT (symmetric) key, missing k value"; return false; }
    k.key.kind = PublicKey::Symmetric;
    k.key.k = kk.data;
    is_public = false;
  } else if (kty == "OKP") {
    if (crv != "Ed25519" || !x.present) { *err = "square/go-jose: unknown curve " + crv + "'"; return false; }
    k.key.kind = PublicKey::Ed25519;
    k.key.x.assign(32, '\0');                       // copy(publicKey, X) into 32 bytes  [R23]
    std::memcpy(&k.key.x[0], x.data.data(), std::min<size_t>(32, x.data.size()));
  } else {
    *err = "square/go-jose: unknown json web key type '" + kty + "'";
    return false;
  }
  if (have_cert && cert_pub.kind != PublicKey::None && k.key.kind != PublicKey::Symmetric) {
    PublicKey mine = k.key;
    if (!(cert_pub == mine)) {
      *err = "square/go-jose: invalid JWK, public keys in key and x5c fields do not match";
      return false;
    }
  }
  if (!is_public && k.key.kind != PublicKey::Symmetric) {
    // a private key decodes, but newVerifier has no case for it: it never verifies
    k.key.kind = PublicKey::None;
  }
  *out = std::move(k);
  return true;
}

bool jwks_decode(std::string_view doc, std::vector<JSONWebKey>* out, std::string* err) {
  json::Value v;
  if (!json::parse(doc, &v, err)) return false;
  out->clear();
  if (v.is_null()) return true;
  if (v.kind != json::Value::Object) { *err = "json: cannot unmarshal into jose.JSONWebKeySet"; return false; }
  // encoding/json struct field "keys": case-insensitive match, last match wins
  const json::Value* keys = nullptr;
  for (const auto& m : v.obj) {
    std::string low = m.first;
    for (auto& c : low) c = (char)std::tolower((unsigned char)c);
    if (low == "keys") keys = &m.second;
  }
  if (!keys || keys->is_null()) return true;
  if (keys->kind != json::Value::Array) { *err = "json: cannot unmarshal into []jose.JSONWebKey"; return false; }
  for (const auto& kv : keys->arr) {
    JSONWebKey k;
    if (kv.is_null()) { out->push_back(k); continue; }
    if (!jwk_from_json(kv, &k, err)) return false;
    out->push_back(std::move(k));
  }
  return true;
}

// ====================================================================== JWS
namespace {

// rawHeader: JSON object of raw values; `null` members are absent  (shared.go)
bool header_from_bytes(std::string_view raw, json::Value* out, std::string* err) {
  if (!json::parse(raw, out, err)) return false;
  if (out->is_null()) { *out = json::Value(); out->kind = json::Value::Object; return true; }
  if (out->kind != json::Value::Object) { *err = "json: cannot unmarshal into rawHeader"; return false; }
  return true;
}

// rawHeader.isSet: present, non-null, and not the empty string
bool is_set(const json::Value& h, const std::string& k) {
  const json::Value* v = h.get(k);
  if (!v || v->is_null()) return false;
  if (v->kind == json::Value::String) return !v->str.empty();
  return true;
}

json::Value merge_headers(const json::Value* prot, const json::Value* unprot) {
  json::Value out;
  out.kind = json::Value::Object;
  for (const json::Value* src : {prot, unprot}) {
    if (!src || src->kind != json::Value::Object) continue;
    for (const auto& m : src->obj) {
      if (m.second.is_null()) continue;
      if (is_set(out, m.first)) continue;
      bool replaced = false;
      for (auto& o : out.obj)
        if (o.first == m.first) { o.second = m.second; replaced = true; }
      if (!replaced) out.obj.push_back(m);
    }
  }
  return out;
}

// rawHeader.sanitized(): typed members must have their type  [R4]
bool sanitize(const json::Value& h, std::string* alg, std::string* kid, bool* has_jwk, std::string* err) {
  for (const auto& m : h.obj) {
    const json::Value& v = m.second;
    if (v.is_null()) continue;
    const std::string& k = m.first;
    if (k == "alg" || k == "kid" || k == "nonce") {
      if (v.kind != json::Value::String) { *err = "failed to unmarshal " + k; return false; }
      if (k == "alg" && alg) *alg = v.str;
      if (k == "kid" && kid) *kid = v.str;
    } else if (k == "jwk") {
      JSONWebKey jk;
      if (!jwk_from_json(v, &jk, err)) { *err = "failed to unmarshal JWK: " + *err; return false; }
      // RFC 7515 4.1.3 (jws.go sanitized): only valid public keys may be embedded
      const PublicKey& pk = jk.key;
      const bool valid = pk.kind == PublicKey::EC || pk.kind == PublicKey::Ed25519 ||
                         (pk.kind == PublicKey::RSA && !pk.n.empty() && pk.e != 0);
      if (!valid) { *err = "square/go-jose: invalid embedded jwk, must be public key"; return false; }
      if (has_jwk) *has_jwk = true;
    } else if (k == "x5c") {
      if (v.kind != json::Value::Array) { *err = "failed to unmarshal x5c"; return false; }
      for (const auto& s : v.arr) {
        std::string der, e2;
        PublicKey pk;
        if (s.kind != json::Value::String || !b64std_decode(s.str, &der) ||
            !parse_certificate_public_key(der, &pk, &e2)) {
          *err = "failed to unmarshal x5c";
          return false;
        }
      }
    } else if (json::has_range_error(v)) {
      *err = "failed to unmarshal value: number out of range";
      return false;
    }
  }
  return true;
}

bool finish_signature(Signature* s, const json::Value* unprot, std::string* err) {
  // nonce in the unprotected header is refused (ErrUnprotectedNonce)
  if (unprot && unprot->kind == json::Value::Object) {
    const json::Value* nv = unprot->get("nonce");
    if (nv && nv->kind == json::Value::String && !nv->str.empty()) {
      *err = "square/go-jose: Nonce parameter included in unprotected header";
      return false;
    }
    s->unprotected_hdr = *unprot;
  }
  const json::Value merged = merge_headers(s->has_protected ? &s->protected_hdr : nullptr, unprot);
  if (!sanitize(merged, &s->alg, &s->kid, &s->has_jwk, err)) return false;
  if (unprot && unprot->kind == json::Value::Object && !sanitize(*unprot, nullptr, nullptr, nullptr, err)) return false;
  if (s->has_protected && !sanitize(s->protected_hdr, nullptr, nullptr, nullptr, err)) return false;
  return true;
}

// byteBuffer member of rawJSONWebSignature: (present, decoded)
bool full_bb(const json::Value& o, const char* name, bool* present, std::string* out, std::string* err) {
  *present = false;
  out->clear();
  const json::Value* v = o.get(name);
  if (!v || v->is_null()) return true;
  if (v->kind != json::Value::String) { *err = std::string("json: cannot unmarshal ") + name; return false; }
  *present = true;
  if (v->str.empty()) return true;
  return b64url_decode(v->str, out, err);
}

bool parse_full(std::string_view input, JWS* out, std::string* err) {
  json::Value v;
  if (!json::parse(input, &v, err)) return false;
  if (v.is_null()) { *err = "square/go-jose: missing payload in JWS message"; return false; }
  if (v.kind != json::Value::Object) { *err = "json: cannot unmarshal into rawJSONWebSignature"; return false; }
  out->compact = false;
  bool has_payload;
  if (!full_bb(v, "payload", &has_payload, &out->payload, err)) return false;
  const json::Value* hdr = v.get("header");
  if (hdr && !hdr->is_null() && hdr->kind != json::Value::Object) { *err = "json: cannot unmarshal header"; return false; }
  if (hdr && hdr->is_null()) hdr = nullptr;
  const json::Value* sigs = v.get("signatures");
  if (sigs && !sigs->is_null() && sigs->kind != json::Value::Array) { *err = "json: cannot unmarshal signatures"; return false; }
  // validate every member's type before the payload check (json.Unmarshal runs first)
  bool has_prot, has_sig;
  std::string prot, sig;
  if (!full_bb(v, "protected", &has_prot, &prot, err) || !full_bb(v, "signature", &has_sig, &sig, err)) return false;
  std::vector<std::tuple<bool, std::string, const json::Value*, std::string>> raw_sigs;
  if (sigs && sigs->kind == json::Value::Array) {
    for (const auto& e : sigs->arr) {
      if (e.is_null()) { raw_sigs.emplace_back(false, std::string(), nullptr, std::string()); continue; }
      if (e.kind != json::Value::Object) { *err = "json: cannot unmarshal signature"; return false; }
      bool hp, hs;
      std::string p2, s2;
      if (!full_bb(e, "protected", &hp, &p2, err) || !full_bb(e, "signature", &hs, &s2, err)) return false;
      const json::Value* h2 = e.get("header");
      if (h2 && !h2->is_null() && h2->kind != json::Value::Object) { *err = "json: cannot unmarshal header"; return false; }
      if (h2 && h2->is_null()) h2 = nullptr;
      raw_sigs.emplace_back(hp, p2, h2, s2);
    }
  }
  if (!has_payload) { *err = "square/go-jose: missing payload in JWS message"; return false; }
  auto one = [&](bool hp, const std::string& p2, const json::Value* h2, const std::string& s2) {
    Signature s;
    s.has_protected = hp;
    s.protected_raw = p2;
    if (hp && !p2.empty()) {
      if (!header_from_bytes(p2, &s.protected_hdr, err)) return false;
    } else {
      s.protected_hdr.kind = json::Value::Object;
    }
    s.signature = s2;
    if (!finish_signature(&s, h2, err)) return false;
    out->sigs.push_back(std::move(s));
    return true;
  };
  if (raw_sigs.empty()) return one(has_prot, prot, hdr, sig);
  for (auto& r : raw_sigs)
    if (!one(std::get<0>(r), std::get<1>(r), std::get<2>(r), std::get<3>(r))) return false;
  return true;
}

}  // namespace

bool parse_signed(std::string_view token, JWS* out, std::string* err) {
  *out = JWS();
  std::string stripped;
  std::string_view t = token;
  if (has_go_space_or_nonascii(token)) {
    stripped = strip_whitespace(token);
    t = stripped;
  }
  if (!t.empty() && t[0] == '{') return parse_full(t, out, err);
  // parseSignedCompact  [R2]
  const size_t d1 = t.find('.');
  const size_t d2 = d1 == std::string_view::npos ? d1 : t.find('.', d1 + 1);
  if (d1 == std::string_view::npos || d2 == std::string_view::npos || t.find('.', d2 + 1) != std::string_view::npos) {
    *err = "square/go-jose: compact JWS format must have three parts";
    return false;
  }
  Signature s;
  if (!b64url_decode(t.substr(0, d1), &s.protected_raw, err)) return false;
  if (!b64url_decode(t.substr(d1 + 1, d2 - d1 - 1), &out->payload, err)) return false;
  if (!b64url_decode(t.substr(d2 + 1), &s.signature, err)) return false;
  s.has_protected = true;                      // newBuffer(rawProtected) is never nil here
  if (!s.protected_raw.empty()) {
    if (!header_from_bytes(s.protected_raw, &s.protected_hdr, err)) return false;
  } else {
    s.protected_hdr.kind = json::Value::Object;
  }
  if (!finish_signature(&s, nullptr, err)) return false;
  out->sigs.push_back(std::move(s));
  out->compact = true;
  out->seg1_end = d1;
  out->seg2_end = d2;
  return true;
}

bool signing_input(const JWS& jws, std::string* out) {
  // DetachedVerify (jws.go): one signature, understood crit, computeAuthData  [R5-R8]
  if (jws.sigs.size() != 1) return false;
  const Signature& s = jws.sigs[0];
  const json::Value merged = merge_headers(s.has_protected ? &s.protected_hdr : nullptr,
                                           s.unprotected_hdr.kind == json::Value::Object ? &s.unprotected_hdr : nullptr);
  if (const json::Value* crit = merged.get("crit"); crit && !crit->is_null()) {
    if (crit->kind != json::Value::Array) return false;
    for (const auto& c : crit->arr) {
      if (c.kind != json::Value::String) return false;
      if (c.str != "b64") return false;           // supportedCritical = {b64}
    }
  }
  bool needs_b64 = true;
  out->clear();
  if (s.has_protected) {
    // the original protected bytes must unmarshal again (empty -> error)
    if (s.protected_raw.empty()) return false;
    out->append(b64url_encode(s.protected_raw));
    // getB64 on the protected header only; a non-bool value counts as true
    if (const json::Value* b = s.protected_hdr.get("b64"); b && b->kind == json::Value::Bool) needs_b64 = b->b;
  }
  out->push_back('.');
  if (needs_b64) out->append(b64url_encode(jws.payload));
  else out->append(jws.payload);
  return true;
}

}  // namespace capjwt
