"""CPU restatement of cap's token-level verify semantics (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg import this module.  The product never does.

Restates, in order of the call stack:
  * Go encoding/json into interface{} (duplicate keys: last wins; invalid
    UTF-8 -> U+FFFD; float64 overflow is an error)           -> go_json()
  * go-jose v2.5.1 `jose.ParseSigned` / `parseSignedCompact` /
    `parseSignedFull` / `rawJSONWebSignature.sanitized` / `mergedHeaders`
    and `DetachedVerify`'s pre-checks + `computeAuthData`  [Appendix A R1-R8]
                                                               -> parse_jws()
  * go-jose `JSONWebKey.UnmarshalJSON` / go-oidc JWKS decode [R27-R31]
                                                               -> jwk_decode(), jwks_decode()
  * go-jose `newVerifier` + `verifyPayload` dispatch [R9-R11] -> verify_sig()
    whose arithmetic is the C oracle (jws_oracle.c, loaded via ctypes)
  * cap `staticKeySet.VerifySignature`   jwt/keyset.go:154-173  [R33]
  * cap `jsonWebKeySet.VerifySignature`  jwt/keyset.go:126-139 with go-oidc
    v2.2.1 remoteKeySet.verify (kid filter)  [R34, R35]
  * cap `Validator.Validate` / `validateSigningAlgorithm` / `validateAudience`
    jwt/jwt.go:95-265 with go-jose jwt.Claims unmarshalling  [R36-R40]
                                                               -> validate()
"""
import base64
import ctypes
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None

ALGS = {"RS256": 1, "RS384": 2, "RS512": 3, "PS256": 4, "PS384": 5, "PS512": 6,
        "ES256": 7, "ES384": 8, "ES512": 9, "EdDSA": 10}
CURVES = {"P-256": 1, "P-384": 2, "P-521": 3}
CURVE_BYTES = {"P-256": 32, "P-384": 48, "P-521": 66}
CURVE_PB = {   # (p, b) of y^2 = x^3 - 3x + b
    "P-256": (0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff,
              0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b),
    "P-384": (int("fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffeffffffff0000000000000000ffffffff", 16),
              int("b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef", 16)),
    "P-521": ((1 << 521) - 1,
              int("0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1"
                  "bf073573df883d2c34f1ef451fd46b503f00", 16)),
}


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        c_p = ctypes.c_char_p
        L.or_rsa_verify.argtypes = [ctypes.c_int, c_p, ctypes.c_size_t, ctypes.c_uint64, c_p, ctypes.c_size_t,
                                    c_p, ctypes.c_size_t]
        L.or_ecdsa_verify.argtypes = [ctypes.c_int, ctypes.c_int, c_p, c_p, ctypes.c_size_t, c_p, ctypes.c_size_t,
                                      c_p, ctypes.c_size_t]
        L.or_ed25519_verify.argtypes = [c_p, c_p, ctypes.c_size_t, c_p, ctypes.c_size_t]
        L.or_ec_point_valid.argtypes = [ctypes.c_int, c_p, c_p, ctypes.c_size_t]
        L.or_b64url_decode.argtypes = [c_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.or_b64url_decode.restype = ctypes.c_long
        for h in ("or_sha256", "or_sha384", "or_sha512"):
            getattr(L, h).argtypes = [c_p, ctypes.c_size_t, ctypes.c_char_p]
        L.or_rsa_public.argtypes = [c_p, ctypes.c_size_t, ctypes.c_uint64, c_p, ctypes.c_size_t, ctypes.c_char_p]
        _lib = L
    return _lib


# ---------------------------------------------------------------- keys
class Key:
    """A public key as go-jose sees it: *rsa.PublicKey / *ecdsa.PublicKey / ed25519.PublicKey
    ("oct" = an HMAC secret; "none" = a private JWK, which newVerifier refuses)."""

    def __init__(self, kty, kid=None, n=None, e=None, crv=None, x=None, y=None, k=None):
        self.kty, self.kid, self.n, self.e, self.crv, self.x, self.y, self.k = kty, kid, n, e, crv, x, y, k

    @staticmethod
    def from_fixture(d):
        if d["kty"] == "RSA":
            n = int(d["n"], 16)
            return Key("RSA", d["kid"], n=n.to_bytes((n.bit_length() + 7) // 8, "big"), e=int(d["e"]))
        if d["kty"] == "EC":
            sz = CURVE_BYTES[d["crv"]]
            return Key("EC", d["kid"], crv=d["crv"], x=int(d["x"], 16).to_bytes(sz, "big"),
                       y=int(d["y"], 16).to_bytes(sz, "big"))
        return Key("OKP", d["kid"], crv="Ed25519", x=bytes.fromhex(d["x"]))

    def __eq__(self, o):
        return isinstance(o, Key) and (self.kty, self.n, self.e, self.crv, self.x, self.y, self.k) == \
            (o.kty, o.n, o.e, o.crv, o.x, o.y, o.k)


def b64url_decode(s: str):
    """go-jose base64URLDecode via the C restatement; None on error [R3]."""
    raw = s.encode("utf-8", "surrogatepass")
    out = ctypes.create_string_buffer(len(raw) + 4)
    n = lib().or_b64url_decode(raw, len(raw), out, len(out))
    return None if n < 0 else out.raw[:n]


def b64url_encode(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def b64std_decode(s: str):
    """base64.StdEncoding.DecodeString (padded; CR/LF ignored; non-strict tail bits)."""
    s = s.replace("\r", "").replace("\n", "")
    if len(s) % 4:
        return None
    body = s.rstrip("=")
    if len(s) - len(body) > 2 or "=" in body:
        return None
    return b64url_decode(body.replace("+", "-").replace("/", "_")) if all(
        c.isalnum() and c.isascii() or c in "+/" for c in body) else None


def hash_bytes(hbits, m: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    getattr(lib(), f"or_sha{hbits}")(m, len(m), out)
    return out.raw[:hbits // 8]


# ---------------------------------------------------------------- Go encoding/json
def go_utf8(b: bytes) -> str:
    """Decode the way Go coerces to valid UTF-8: every byte that does not start
    a valid sequence becomes one U+FFFD (utf8.DecodeRune returns width 1)."""
    out = []
    i, n = 0, len(b)
    while i < n:
        c = b[i]
        if c < 0x80:
            out.append(chr(c)); i += 1; continue
        w = 0
        if 0xC2 <= c <= 0xDF:
            w = 2 if i + 1 < n and 0x80 <= b[i + 1] <= 0xBF else 0
        elif 0xE0 <= c <= 0xEF:
            lo = 0xA0 if c == 0xE0 else 0x80
            hi = 0x9F if c == 0xED else 0xBF
            w = 3 if i + 2 < n and lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF else 0
        elif 0xF0 <= c <= 0xF4:
            lo = 0x90 if c == 0xF0 else 0x80
            hi = 0x8F if c == 0xF4 else 0xBF
            w = 4 if i + 3 < n and lo <= b[i + 1] <= hi and 0x80 <= b[i + 2] <= 0xBF and 0x80 <= b[i + 3] <= 0xBF else 0
        if w:
            out.append(b[i:i + w].decode("utf-8")); i += w
        else:
            out.append("�"); i += 1
    return "".join(out)


class GoJSONError(ValueError):
    pass


def _no_surrogates(v):
    if isinstance(v, str):
        return "".join("�" if 0xD800 <= ord(ch) < 0xE000 else ch for ch in v)
    if isinstance(v, list):
        return [_no_surrogates(x) for x in v]
    if isinstance(v, dict):
        return {_no_surrogates(k): _no_surrogates(x) for k, x in v.items()}
    return v


def _go_float(s):
    f = float(s)
    if math.isinf(f):
        raise GoJSONError("json: cannot unmarshal number " + s + " into Go value of type float64")
    return f


def _no_const(s):
    raise GoJSONError("invalid character")


def go_json(raw):
    """json.Unmarshal(raw, &interface{}) -> value; raises GoJSONError.  Numbers are float64."""
    text = go_utf8(raw) if isinstance(raw, (bytes, bytearray)) else raw
    try:
        v = json.loads(text, object_pairs_hook=dict, parse_float=_go_float, parse_int=_go_float,
                       parse_constant=_no_const)
    except GoJSONError:
        raise
    except (ValueError, RecursionError) as e:
        raise GoJSONError(str(e))
    return _no_surrogates(v)


# ---------------------------------------------------------------- DER (x5c / certificates)
def _der(b, i, tag):
    if i + 2 > len(b) or b[i] != tag:
        return None
    ln, j = b[i + 1], i + 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or j + nb > len(b):
            return None
        ln = int.from_bytes(b[j:j + nb], "big")
        if ln < 128 or b[j] == 0:                    # DER: non-minimal length (asn1 / cryptobyte reject)
            return None
        j += nb
    if j + ln > len(b):
        return None
    return b[j:j + ln], j + ln


class UnknownAlgorithm(Exception):
    """x509: unknown public key algorithm (x509.ParseCertificate leaves
    PublicKey nil for it instead of failing)"""


def spki_key(spki: bytes):
    """x509.ParsePKIXPublicKey subset -> Key or None."""
    try:
        return spki_key_ex(spki)
    except UnknownAlgorithm:
        return None


def spki_key_ex(spki: bytes):
    """Key, None for a malformed SubjectPublicKeyInfo or an invalid key of a
    known algorithm (Go's parsePublicKey errors), UnknownAlgorithm raised for an
    algorithm OID Go does not know."""
    r = _der(spki, 0, 0x30)
    if not r:
        return None
    body = r[0]
    a = _der(body, 0, 0x30)
    if not a:
        return None
    alg, i = a
    bits = _der(body, i, 0x03)
    if not bits or not bits[0] or bits[0][0] != 0:
        return None
    key = bits[0][1:]
    o = _der(alg, 0, 0x06)
    if not o:
        return None
    oid, j = o
    # AlgorithmIdentifier.Parameters: the first element after the OID (Go
    # ignores any further ones, as it ignores elements after the BIT STRING)
    params = b""
    if j < len(alg):
        pr = _der(alg, j, alg[j])
        if not pr:
            return None
        params = alg[j:pr[1]]
    if oid == bytes.fromhex("2a864886f70d010101"):
        if params != b"\x05\x00":
            return None
        s = _der(key, 0, 0x30)
        if not s:
            return None
        n = _der(s[0], 0, 0x02)
        e = n and _der(s[0], n[1], 0x02)
        if not n or not e:
            return None
        nv, ev = int.from_bytes(n[0], "big", signed=True), int.from_bytes(e[0], "big", signed=True)
        if nv <= 0 or ev <= 0:
            return None
        return Key("RSA", n=nv.to_bytes((nv.bit_length() + 7) // 8, "big"), e=ev)
    if oid == bytes.fromhex("2a8648ce3d0201"):
        c = _der(params, 0, 0x06)
        names = {bytes.fromhex("2a8648ce3d030107"): "P-256", bytes.fromhex("2b81040022"): "P-384",
                 bytes.fromhex("2b81040023"): "P-521"}
        crv = c and names.get(c[0])
        if not crv:
            return None
        sz = CURVE_BYTES[crv]
        if len(key) != 1 + 2 * sz or key[0] != 4 or not ec_on_curve(crv, key[1:1 + sz], key[1 + sz:]):
            return None
        return Key("EC", crv=crv, x=key[1:1 + sz], y=key[1 + sz:])
    if oid == bytes.fromhex("2b6570"):
        if params or len(key) != 32:
            return None
        return Key("OKP", crv="Ed25519", x=key)
    raise UnknownAlgorithm()


def cert_key(der: bytes):
    """Certificate -> its SubjectPublicKeyInfo's Key (or "unknown")."""
    c = _der(der, 0, 0x30)
    if not c or c[1] != len(der):                    # x509: trailing data
        return None
    # Certificate ::= SEQUENCE { tbsCertificate, signatureAlgorithm, signatureValue BIT STRING }
    t = _der(c[0], 0, 0x30)
    sa = t and _der(c[0], t[1], 0x30)
    sv = sa and _der(c[0], sa[1], 0x03)
    if not sv or sv[1] != len(c[0]):
        return None
    tbs, i = t[0], 0
    if tbs[:1] == b"\xa0":
        v = _der(tbs, 0, 0xA0)
        if not v:                                    # x509: malformed version
            return None
        i = v[1]
    for tag in (0x02, 0x30, 0x30, 0x30, 0x30):
        r = _der(tbs, i, tag)
        if not r:
            return None
        i = r[1]
    s = _der(tbs, i, 0x30)
    if not s:
        return None
    # x509.ParseCertificate: an invalid key of a known algorithm (an EC point
    # off the curve, RSA without NULL parameters, ...) fails the parse; an
    # unknown algorithm parses with PublicKey nil
    try:
        return spki_key_ex(tbs[i:s[1]])
    except UnknownAlgorithm:
        return "unknown"


def ec_on_curve(crv, x: bytes, y: bytes) -> bool:
    p, b = CURVE_PB[crv]
    X, Y = int.from_bytes(x, "big"), int.from_bytes(y, "big")
    return X < p and Y < p and (Y * Y - (X ** 3 - 3 * X + b)) % p == 0


# ---------------------------------------------------------------- JWK (go-jose jwk.go)
class JWKError(ValueError):
    pass


def jwk_decode(obj) -> Key:
    """JSONWebKey.UnmarshalJSON (go-jose json: case-sensitive members)."""
    if not isinstance(obj, dict):
        raise JWKError("not an object")

    def s(name):
        v = obj.get(name)
        if v is not None and not isinstance(v, str):
            raise JWKError("type " + name)
        return v or ""

    def bb(name):                       # byteBuffer: absent/null -> None, "" -> b""
        v = obj.get(name)
        if v is None:
            return None
        if not isinstance(v, str):
            raise JWKError("type " + name)
        if v == "":
            return b""
        d = b64url_decode(v)
        if d is None:
            raise JWKError("base64 " + name)
        return d
    kty, crv, kid = s("kty"), s("crv"), s("kid")
    for nm in ("alg", "use", "x5u", "x5t", "x5t#S256"):
        s(nm)
    vals = {nm: bb(nm) for nm in ("n", "e", "x", "y", "d", "k", "p", "q", "dp", "dq", "qi")}
    cert = None
    x5c = obj.get("x5c")
    if x5c is not None:
        if not isinstance(x5c, list) or not all(isinstance(c, str) for c in x5c):
            raise JWKError("x5c type")
        for i, c in enumerate(x5c):
            der = b64std_decode(c)
            k = der is not None and cert_key(der)
            if not k:
                raise JWKError("x5c parse")
            if i == 0:
                cert = k
    d = vals["d"]
    if kty == "EC":
        if crv not in CURVE_BYTES:
            raise JWKError("unsupported elliptic curve")
        x, y = vals["x"], vals["y"]
        if x is None or y is None:
            raise JWKError("missing x/y")
        sz = CURVE_BYTES[crv]
        if d is not None and len(d) != sz:
            raise JWKError("wrong length for d")
        if len(x) != sz or len(y) != sz:
            raise JWKError("wrong length")
        if not ec_on_curve(crv, x, y):
            raise JWKError("not on curve")
        key = Key("EC", kid, crv=crv, x=x, y=y)
    elif kty == "RSA":
        if vals["n"] is None or vals["e"] is None:
            raise JWKError("missing n/e")
        if d is not None and (vals["p"] is None or vals["q"] is None):
            raise JWKError("private key missing values")
        nv = int.from_bytes(vals["n"], "big")
        e64 = int.from_bytes(vals["e"], "big") & ((1 << 64) - 1)      # int(bigInt.Int64())
        key = Key("RSA", kid, n=nv.to_bytes((nv.bit_length() + 7) // 8, "big"), e=e64)
    elif kty == "oct":
        if cert is not None:
            raise JWKError("oct with cert chain")
        if vals["k"] is None:
            raise JWKError("missing k")
        return Key("oct", kid, k=vals["k"])
    elif kty == "OKP":
        if crv != "Ed25519" or vals["x"] is None:
            raise JWKError("unknown curve")
        key = Key("OKP", kid, crv="Ed25519", x=(vals["x"][:32] + bytes(32))[:32])
    else:
        raise JWKError("unknown kty")
    if cert is not None and cert != "unknown":
        mine = Key(key.kty, None, key.n, key.e, key.crv, key.x, key.y)
        if cert != mine:
            raise JWKError("x5c mismatch")
    if d is not None:
        return Key("none", kid)
    return key


def jwks_decode(doc: bytes):
    """go-oidc updateKeys: json.Unmarshal(body, &jose.JSONWebKeySet) -> [Key]; raises."""
    v = go_json(doc)
    if v is None:
        return []
    if not isinstance(v, dict):
        raise JWKError("not an object")
    keys = None
    for k, val in v.items():                    # encoding/json: case-insensitive field "keys"
        if k.lower() == "keys":
            keys = val
    if keys is None:
        return []
    if not isinstance(keys, list):
        raise JWKError("keys not an array")
    return [Key("none") if k is None else jwk_decode(k) for k in keys]


# ---------------------------------------------------------------- parse (go-jose jws.go)
_GO_SPACE = set("\t\n\v\f\r \x85\xa0     　") | {chr(c) for c in range(0x2000, 0x200b)}


def strip_whitespace(s: str) -> str:
    """go-jose stripWhitespace: drop every rune with unicode.IsSpace [R1]."""
    return "".join(ch for ch in s if ch not in _GO_SPACE)


class ParsedJWS:
    def __init__(self, payload, sigs):
        self.payload = payload
        self.sigs = sigs                    # [dict(protected, protected_raw, header, signature, merged)]
        self.nsigs = len(sigs)
        s0 = sigs[0]
        self.protected_raw = s0["protected_raw"] or b""
        self.header = s0["merged"]
        self.signature = s0["signature"]
        self.alg = s0["merged"].get("alg") or ""
        self.kid = s0["merged"].get("kid") or ""
        self.signing_input = _auth_data(self)
        self.crit_ok = self.signing_input is not None


def _is_set(h, k):
    v = h.get(k)
    if v is None:
        return False
    return v != "" if isinstance(v, str) else True


def _merge(prot, unprot):
    out = {}
    for src in (prot, unprot):
        for k, v in (src or {}).items():
            if not _is_set(out, k):
                out[k] = v
    return out


def _sanitize(h) -> bool:
    for k, v in h.items():
        if v is None:
            continue
        if k in ("alg", "kid", "nonce"):
            if not isinstance(v, str):
                return False
        elif k == "jwk":
            try:
                key = jwk_decode(v)
            except JWKError:
                return False
            if key.kty in ("oct", "none") or (key.kty == "RSA" and (not key.n or not key.e)):
                return False                    # embedded jwk must be a valid public key
        elif k == "x5c":
            if not isinstance(v, list):
                return False
            for c in v:
                der = b64std_decode(c) if isinstance(c, str) else None
                if der is None or not cert_key(der):
                    return False
    return True


def _header_obj(raw: bytes):
    v = go_json(raw)                            # raises GoJSONError
    if v is None:
        return {}
    if not isinstance(v, dict):
        raise GoJSONError("header not an object")
    return v


def _sanitized(payload, raw_sigs):
    """rawJSONWebSignature.sanitized for each (protected bytes|None, header dict|None, signature)."""
    sigs = []
    for prot_raw, unprot, sig in raw_sigs:
        prot = _header_obj(prot_raw) if prot_raw else None
        if unprot is not None:
            n = unprot.get("nonce")
            if isinstance(n, str) and n != "":
                return None                     # ErrUnprotectedNonce
        merged = _merge(prot, unprot)
        if not _sanitize(merged) or (unprot and not _sanitize(unprot)) or (prot and not _sanitize(prot)):
            return None
        sigs.append(dict(protected=prot, protected_raw=prot_raw, header=unprot, signature=sig or b"",
                         merged=merged))
    return ParsedJWS(payload, sigs)


def _auth_data(p):
    """DetachedVerify pre-checks + computeAuthData; None => ErrCryptoFailure."""
    if p.nsigs != 1:
        return None
    s = p.sigs[0]
    crit = s["merged"].get("crit")
    if crit is not None:
        if not isinstance(crit, list) or not all(isinstance(c, str) for c in crit):
            return None
        if any(c != "b64" for c in crit):
            return None
    needs_b64 = True
    out = b""
    if s["protected_raw"] is not None:
        if s["protected_raw"] == b"":
            return None                         # json.Unmarshal of empty input fails
        out = b64url_encode(s["protected_raw"]).encode()
        b = (s["protected"] or {}).get("b64")
        if isinstance(b, bool):
            needs_b64 = b
    return out + b"." + (b64url_encode(p.payload).encode() if needs_b64 else p.payload)


def parse_jws(token: str):
    """jose.ParseSigned: returns ParsedJWS or None (parse error => reject)."""
    if isinstance(token, bytes):
        token = go_utf8(token)
    token = strip_whitespace(token)
    try:
        if token.startswith("{"):
            return _parse_full(token)
        parts = token.split(".")
        if len(parts) != 3:
            return None
        prot = b64url_decode(parts[0])
        payload = b64url_decode(parts[1])
        sig = b64url_decode(parts[2])
        if prot is None or payload is None or sig is None:
            return None
        return _sanitized(payload, [(prot, None, sig)])
    except GoJSONError:
        return None


def _parse_full(token):
    obj = go_json(token)
    if obj is None or not isinstance(obj, dict):
        return None

    def bb(o, k):                       # byteBuffer: absent/null -> None; "" -> b""
        v = o.get(k)
        if v is None:
            return None
        if not isinstance(v, str):
            raise GoJSONError(k)
        if v == "":
            return b""
        d = b64url_decode(v)
        if d is None:
            raise GoJSONError(k)
        return d

    def hdr(o):
        h = o.get("header")
        if h is not None and not isinstance(h, dict):
            raise GoJSONError("header")
        return h
    payload = bb(obj, "payload")
    top = (bb(obj, "protected"), hdr(obj), bb(obj, "signature"))
    sigs = obj.get("signatures")
    if sigs is not None and not isinstance(sigs, list):
        return None
    raw = []
    for e in sigs or []:
        if e is None:
            raw.append((None, None, None))
            continue
        if not isinstance(e, dict):
            return None
        raw.append((bb(e, "protected"), hdr(e), bb(e, "signature")))
    if payload is None:
        return None                     # missing payload in JWS message
    return _sanitized(payload, raw if raw else [top])


# ---------------------------------------------------------------- verify
def verify_sig(p: ParsedJWS, key: Key) -> bool:
    """JSONWebSignature.Verify(key) -> newVerifier + verifyPayload [R9-R11]."""
    if p is None or not p.crit_ok:
        return False
    a = ALGS.get(p.alg)
    if a is None:
        return False
    L = lib()
    m, s = p.signing_input, p.signature
    if key.kty == "RSA":
        return bool(L.or_rsa_verify(a, key.n, len(key.n), key.e, m, len(m), s, len(s)))
    if key.kty == "EC":
        return bool(L.or_ecdsa_verify(a, CURVES[key.crv], key.x, key.y, len(key.x), m, len(m), s, len(s)))
    if key.kty == "OKP":
        if a != ALGS["EdDSA"] or len(key.x) != 32:
            return False
        return bool(L.or_ed25519_verify(key.x, m, len(m), s, len(s)))
    return False


def verify_alg_sig(alg: str, key: Key, signing_input: bytes, sig: bytes) -> bool:
    """Signature arithmetic alone for an (alg, key, signing input, signature) job."""
    if alg not in ALGS:
        return False
    L = lib()
    a, m, s = ALGS[alg], signing_input, sig
    if key.kty == "RSA":
        return bool(L.or_rsa_verify(a, key.n, len(key.n), key.e, m, len(m), s, len(s)))
    if key.kty == "EC":
        return bool(L.or_ecdsa_verify(a, CURVES[key.crv], key.x, key.y, len(key.x), m, len(m), s, len(s)))
    if key.kty == "OKP" and a == ALGS["EdDSA"] and len(key.x) == 32:
        return bool(L.or_ed25519_verify(key.x, m, len(m), s, len(s)))
    return False


class ErrNoKey(Exception):
    pass


def _claims_map(payload: bytes):
    """json.Unmarshal(payload, &map[string]interface{}) [R33, R35]; raises on error."""
    obj = go_json(payload)
    if obj is None:
        return None
    if not isinstance(obj, dict):
        raise GoJSONError("json: cannot unmarshal into map")
    return obj


def static_keyset_verify(token: str, keys):
    """staticKeySet.VerifySignature (jwt/keyset.go:154-173): keys in order, first success wins."""
    p = parse_jws(token)
    if p is None:
        raise ErrNoKey("parse")
    for k in keys:
        if verify_sig(p, k):
            try:
                return _claims_map(p.payload)
            except GoJSONError:
                continue
    raise ErrNoKey("no known key successfully validated the token signature")


def jwks_keyset_verify(token: str, keys):
    """jsonWebKeySet.VerifySignature (jwt/keyset.go:126-139) over go-oidc remoteKeySet.verify:
    keys whose kid matches the header kid (or all, when the header has none) [R34]."""
    p = parse_jws(token)
    if p is None:
        raise ErrNoKey("oidc: malformed jwt")
    for k in keys:
        if p.kid == "" or k.kid == p.kid:
            if verify_sig(p, k):
                try:
                    return _claims_map(p.payload)   # json error => reject (keyset.go:134)
                except GoJSONError as e:
                    raise ErrNoKey(str(e))
    raise ErrNoKey("failed to verify id token signature")


# ---------------------------------------------------------------- Validator (jwt/jwt.go:95-239)
SECOND = 1_000_000_000
I64 = 1 << 64


def _wrap64(v):
    v %= I64
    return v - I64 if v >= 1 << 63 else v


def _f64_to_i64(f):
    """int64(float64) as amd64 CVTTSD2SQ does it."""
    if f != f or f >= 2.0 ** 63 or f < -(2.0 ** 63):
        return -(1 << 63)
    return int(f)


def _trunc_div(a, b):
    """Go integer division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _dur_seconds(d):
    """time.Duration.Seconds: sec + nsec/1e9 with Go's truncating d / Second, d % Second."""
    s = _trunc_div(d, SECOND)
    return float(s) + float(d - s * SECOND) / 1e9


def _fold(k):
    out = []
    for ch in k:
        if "a" <= ch <= "z":
            out.append(ch.upper())
        elif ch == "ſ":
            out.append("S")
        elif ch == "K":
            out.append("K")
        else:
            out.append(ch)
    return "".join(out)


def _claims_struct(all_claims):
    """json.Marshal(allClaims) then json.Unmarshal(&jwt.Claims{}) [R37] -> (fields, err)."""
    f = {"iss": "", "sub": "", "jti": "", "aud": [], "exp": None, "nbf": None, "iat": None}
    if all_claims is None:
        return f, None
    for k in sorted(all_claims, key=lambda s: s.encode("utf-8")):
        v = all_claims[k]
        name = _fold(k)
        if name in ("ISS", "SUB", "JTI"):
            if v is None:
                continue
            if not isinstance(v, str):
                return None, "json: cannot unmarshal into Go struct field Claims." + k + " of type string"
            f[name.lower()] = v
        elif name == "AUD":
            if isinstance(v, str):
                f["aud"] = [v]
            elif isinstance(v, list) and all(isinstance(x, str) for x in v):
                f["aud"] = list(v)
            else:
                return None, "square/go-jose/jwt: expected string or array value to unmarshal to Audience"
        elif name in ("EXP", "NBF", "IAT"):
            if v is None:
                f[name.lower()] = None
            elif isinstance(v, float) and not isinstance(v, bool):
                f[name.lower()] = _f64_to_i64(v)
            else:
                return None, "square/go-jose/jwt: expected number value to unmarshal NumericDate"
    return f, None


def validate_claims(all_claims, alg, nsigs, sig_len, expected, now_ns):
    """Validate after KeySet.VerifySignature succeeded. `expected` is a dict with the
    jwt.Expected field names (durations in ns).  Returns (claims, err)."""
    # validateSigningAlgorithm [R36]
    algs = expected.get("SigningAlgorithms") or []
    err = None
    for a in algs:
        if a not in ALGS:
            err = f'unsupported signing algorithm "{a}"'
            break
    if err is None:
        if nsigs == 0 or (nsigs == 1 and sig_len == 0):
            err = "token must be signed"
        elif nsigs > 1:
            err = "token with multiple signatures not supported"
        elif alg not in (algs or ["RS256"]):
            err = "token signed with unexpected algorithm"
    if err:
        return None, "invalid algorithm (alg) header parameter: " + err
    f, err = _claims_struct(all_claims)
    if err:
        return None, err
    iat, exp, nbf = f["iat"] or 0, f["exp"] or 0, f["nbf"] or 0
    if iat == 0 and exp == 0 and nbf == 0:
        return None, "no issued at (iat), not before (nbf), or expiration time (exp) claims in token"

    def leeway(d):
        s = _dur_seconds(d)
        return 0.0 if s < 0 else float(150) if s == 0 else s
    if exp == 0:
        exp = _wrap64(max(iat, nbf) + _f64_to_i64(leeway(expected.get("ExpirationLeeway", 0))))
    if nbf == 0:
        nbf = iat if iat != 0 else _wrap64(exp - _f64_to_i64(leeway(expected.get("NotBeforeLeeway", 0))))
    cks = expected.get("ClockSkewLeeway", 0)
    cks = 0 if _dur_seconds(cks) < 0 else 60 * SECOND if _dur_seconds(cks) == 0 else cks
    if expected.get("Issuer") and expected["Issuer"] != f["iss"]:
        return None, "invalid issuer (iss) claim"
    if expected.get("Subject") and expected["Subject"] != f["sub"]:
        return None, "invalid subject (sub) claim"
    if expected.get("ID") and expected["ID"] != f["jti"]:
        return None, "invalid ID (jti) claim"
    auds = expected.get("Audiences") or []
    if auds and not any(a in f["aud"] for a in auds):
        return None, "invalid audience (aud) claim: audience claim does not match any expected audience"
    # time.Time comparisons on (seconds since year 1, ns); time.Unix wraps int64
    U = 62135596800

    def t_unix(sec):
        return (_wrap64(sec + U), 0)
    s, ns = divmod(now_ns, SECOND)

    def add(d):                                 # Time.Add
        ds = _trunc_div(d, SECOND)
        n2 = ns + (d - ds * SECOND)
        if n2 >= SECOND:
            ds, n2 = ds + 1, n2 - SECOND
        elif n2 < 0:
            ds, n2 = ds - 1, n2 + SECOND
        return (s + U + ds, n2)
    if add(cks) < t_unix(nbf):
        return None, "invalid not before (nbf) claim: token not yet valid"
    if add(-cks) > t_unix(exp):
        return None, "invalid expiration time (exp) claim: token is expired"
    if add(cks) < t_unix(iat):
        return None, "invalid issued at (iat) claim: token issued in the future"
    return all_claims, None


def validate(token, keyset_verify, expected, now_ns):
    """Validator.Validate with a restated KeySet (keyset_verify(token) -> claims, raises ErrNoKey)."""
    try:
        claims = keyset_verify(token)
    except ErrNoKey as e:
        return None, "error verifying token signature: " + str(e)
    p = parse_jws(token)
    return validate_claims(claims, p.alg, p.nsigs, len(p.signature), expected, now_ns)
