"""CPU restatement of cap's OIDC hash-claim checks (TEST INFRASTRUCTURE ONLY).

Only tests/ import this module; the product never does.

Restates oidc/id_token.go:59-145 -- IDToken.VerifyAccessToken (at_hash),
IDToken.VerifyAuthorizationCode (c_hash) and their shared verifyHashClaim --
with the claims read by oidc.UnmarshalClaims (oidc/token.go:170-184):

  1. IDToken.Claims: empty token -> error; else strings.Split on "." must give
     3 parts, base64.RawURLEncoding of part 2 ('=' is illegal), json.Unmarshal
     into map[string]interface{}                         (error -> "claims")
  2. claims[name].(string): absent / not a string       -> (False, None)
  3. jose.ParseSigned(token)                            (error -> "malformed")
  4. exactly one signature ("multi"); its alg one of the 10 supported
     ("unsupported"); EdDSA                             -> (False, None)
  5. base64url(left half of SHA-256/384/512(value)) == claim
                                                        (else "mismatch")

Returns (verified, kind) with kind None for Go's nil error, else one of the
strings above; tests map kinds to the reference's error text.  Parse errors
come from oracle.jws (go-jose restatement); the hash is the C oracle's SHA-2.
"""
from . import jws

HASH_BITS = {"RS256": 256, "ES256": 256, "PS256": 256,
             "RS384": 384, "ES384": 384, "PS384": 384,
             "RS512": 512, "ES512": 512, "PS512": 512}


def raw_url_decode(s: str):
    """base64.RawURLEncoding.DecodeString: None on error ('=' is not in the alphabet)."""
    if "=" in s:
        return None
    return jws.b64url_decode(s)


def unmarshal_claims(token: str):
    """oidc.UnmarshalClaims into map[string]interface{}: (claims, ok)."""
    parts = token.split(".")
    if len(parts) != 3:
        return None, False
    raw = raw_url_decode(parts[1])
    if raw is None:
        return None, False
    try:
        return jws._claims_map(raw), True
    except jws.GoJSONError:
        return None, False


def verify_hash_claim(claim: str, token: str, value: bytes):
    """verifyHashClaim(claim, value) on IDToken(token) -> (verified, kind)."""
    if token == "":
        return False, "claims"
    claims, ok = unmarshal_claims(token)
    if not ok:
        return False, "claims"
    want = claims.get(claim) if isinstance(claims, dict) else None
    if not isinstance(want, str):
        return False, None
    p = jws.parse_jws(token)
    if p is None:
        return False, "malformed"
    if p.nsigs != 1:
        return False, "multi"
    if p.alg not in jws.ALGS:
        return False, "unsupported"
    if p.alg == "EdDSA":
        return False, None
    bits = HASH_BITS[p.alg]
    h = jws.hash_bytes(bits, value)
    if jws.b64url_encode(h[:len(h) // 2]) != want:
        return False, "mismatch"
    return True, None


def verify_access_token(token: str, access_token: bytes):
    return verify_hash_claim("at_hash", token, access_token)


def verify_authorization_code(token: str, code: bytes):
    return verify_hash_claim("c_hash", token, code)
