"""CPU restatement of cap's token-level verify semantics (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg import this module.  The product never does.

Restates, in order of the call stack:
  * go-jose v2.5.1 `jose.ParseSigned` / `parseSignedCompact` / `sanitized`
    and `computeAuthData` [Appendix A R1-R8]   -> parse_jws()
  * go-jose `newVerifier` + `verifyPayload` dispatch [R9-R11]  -> verify_sig()
    whose arithmetic is the C oracle (jws_oracle.c, loaded via ctypes)
  * cap `staticKeySet.VerifySignature`   jwt/keyset.go:154-173  [R33]
  * cap `jsonWebKeySet.VerifySignature`  jwt/keyset.go:126-139 with go-oidc
    v2.2.1 remoteKeySet.verify (kid filter)  [R34, R35]
  * cap `Validator.Validate` / `validateSigningAlgorithm` / `validateAudience`
    jwt/jwt.go:95-265  [R36-R40]
"""
import base64
import ctypes
import json
import os
import unicodedata

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None

ALGS = {"RS256": 1, "RS384": 2, "RS512": 3, "PS256": 4, "PS384": 5, "PS512": 6,
        "ES256": 7, "ES384": 8, "ES512": 9, "EdDSA": 10}
CURVES = {"P-256": 1, "P-384": 2, "P-521": 3}
CURVE_BYTES = {"P-256": 32, "P-384": 48, "P-521": 66}


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
    """A public key as go-jose sees it: *rsa.PublicKey / *ecdsa.PublicKey / ed25519.PublicKey."""

    def __init__(self, kty, kid=None, n=None, e=None, crv=None, x=None, y=None):
        self.kty, self.kid, self.n, self.e, self.crv, self.x, self.y = kty, kid, n, e, crv, x, y

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


def b64url_decode(s: str):
    """go-jose base64URLDecode via the C restatement; None on error [R3]."""
    raw = s.encode("utf-8", "surrogatepass")
    out = ctypes.create_string_buffer(len(raw) + 4)
    n = lib().or_b64url_decode(raw, len(raw), out, len(out))
    return None if n < 0 else out.raw[:n]


def b64url_encode(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def hash_bytes(hbits, m: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    getattr(lib(), f"or_sha{hbits}")(m, len(m), out)
    return out.raw[:hbits // 8]


# ---------------------------------------------------------------- parse
_GO_SPACE = set(" \t\n\v\f\r\x85\xa0     　") | {chr(c) for c in range(0x2000, 0x200b)}


def strip_whitespace(s: str) -> str:
    """go-jose stripWhitespace: drop every rune with unicode.IsSpace [R1]."""
    return "".join(ch for ch in s if ch not in _GO_SPACE)


class ParsedJWS:
    def __init__(self, protected_raw, header, payload, signature, signing_input, alg, kid, crit_ok):
        self.protected_raw = protected_raw
        self.header = header
        self.payload = payload
        self.signature = signature
        self.signing_input = signing_input
        self.alg = alg
        self.kid = kid
        self.crit_ok = crit_ok


def _pairs_last_wins(pairs):
    return dict(pairs)          # encoding/json: duplicate keys, the last one wins


def _sanitize_header(raw: bytes):
    """rawHeader unmarshal + sanitized(): alg and kid must be strings [R4, R8]."""
    try:
        hdr = json.loads(raw.decode("utf-8"), object_pairs_hook=_pairs_last_wins)
    except Exception:
        return None
    if not isinstance(hdr, dict):
        return None
    alg = hdr.get("alg")
    if alg is not None and not isinstance(alg, str):
        return None
    kid = hdr.get("kid")
    if kid is not None and not isinstance(kid, str):
        return None
    return hdr


def parse_jws(token: str):
    """jose.ParseSigned: returns ParsedJWS or None (parse error => reject)."""
    token = strip_whitespace(token)
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
    return _finish(prot, payload, sig)


def _parse_full(token):
    try:
        obj = json.loads(token, object_pairs_hook=_pairs_last_wins)
    except Exception:
        return None
    if not isinstance(obj, dict):
        return None
    if "signatures" in obj and obj["signatures"] is not None:
        return None                               # multiple-signature form: not compact-equivalent
    def dec(k):
        v = obj.get(k)
        if v is None:
            return b""
        if not isinstance(v, str):
            raise ValueError
        return b64url_decode(v)
    try:
        prot, payload, sig = dec("protected"), dec("payload"), dec("signature")
    except ValueError:
        return None
    if prot is None or payload is None or sig is None:
        return None
    if obj.get("payload") is None:
        return None
    return _finish(prot, payload, sig)


def _finish(prot, payload, sig):
    hdr = {}
    if len(prot) > 0:
        hdr = _sanitize_header(prot)
        if hdr is None:
            return None
    alg = hdr.get("alg") or ""
    kid = hdr.get("kid") or ""
    crit = hdr.get("crit")
    crit_ok = True
    if crit is not None:
        if not isinstance(crit, list) or not all(isinstance(c, str) for c in crit):
            crit_ok = False
        elif any(c != "b64" for c in crit):
            crit_ok = False
    needs_b64 = True
    if "b64" in hdr:
        if not isinstance(hdr["b64"], bool):
            crit_ok = False
        else:
            needs_b64 = hdr["b64"]
    # computeAuthData: canonical re-encoding of the decoded protected header / payload [R6, R7]
    si = b64url_encode(prot).encode() + b"." + (b64url_encode(payload).encode() if needs_b64 else payload)
    return ParsedJWS(prot, hdr, payload, sig, si, alg, kid, crit_ok)


# ---------------------------------------------------------------- verify
def verify_sig(p: ParsedJWS, key: Key) -> bool:
    """JSONWebSignature.Verify(key) -> newVerifier + verifyPayload [R9-R11]."""
    if not p.crit_ok:
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
    p = ParsedJWS(b"", {}, b"", sig, signing_input, alg, "", True)
    return verify_sig(p, key)


class ErrNoKey(Exception):
    pass


def _claims_map(payload: bytes):
    """json.Unmarshal(payload, &map[string]interface{}) [R33, R35]; raises on error."""
    obj = json.loads(payload.decode("utf-8"), object_pairs_hook=_pairs_last_wins)
    if obj is None:
        return None
    if not isinstance(obj, dict):
        raise ValueError("json: cannot unmarshal into map")
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
            except Exception:
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
                return _claims_map(p.payload)   # json error => reject (keyset.go:134)
    raise ErrNoKey("failed to verify id token signature")
