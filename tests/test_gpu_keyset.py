"""GPU parity of cap's KeySet / Validator API (C++ host mirror over libcapjwt.so).

Mirrors the reference's own tests -- jwt/keyset_test.go (static + JWKS key
sets, all 10 algs, wrong key, HS256 swap, malformed tokens, JWKS fetch
failure) and jwt/jwt_test.go (Validate valid/invalid cases, allow-list) --
and checks every outcome (claims map and error string) against the oracle's
restatement (oracle/jws.py), single-token and batched."""
import base64
import json
import os

import pytest

from oracle import jws

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SECOND = 1_000_000_000


@pytest.fixture(scope="module")
def J():
    from cap_amd import jwt
    return jwt


@pytest.fixture(scope="module")
def cases():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "host_cases.json")))


@pytest.fixture(scope="module")
def keys(golden, J):
    """kid -> (native PublicKey, oracle Key, JWK dict)"""
    out = {}
    for d in golden["keys_raw"]:
        k = jws.Key.from_fixture(d)
        if k.kty == "RSA":
            nat = J.PublicKey.rsa(k.n, k.e)
            jwk = {"kty": "RSA", "kid": d["kid"], "n": b64u(k.n), "e": b64u(k.e.to_bytes(4, "big").lstrip(b"\0"))}
        elif k.kty == "EC":
            nat = J.PublicKey.ec(k.crv, k.x, k.y)
            jwk = {"kty": "EC", "kid": d["kid"], "crv": k.crv, "x": b64u(k.x), "y": b64u(k.y)}
        else:
            nat = J.PublicKey.ed25519(k.x)
            jwk = {"kty": "OKP", "kid": d["kid"], "crv": "Ed25519", "x": b64u(k.x)}
        out[d["kid"]] = (nat, k, jwk)
    return out


def b64u(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def oracle_static(token, okeys):
    try:
        return jws.static_keyset_verify(token, okeys), None
    except jws.ErrNoKey as e:
        return None, str(e)


def oracle_jwks(token, okeys):
    try:
        return jws.jwks_keyset_verify(token, okeys), None
    except jws.ErrNoKey as e:
        return None, str(e)


# ---------------------------------------------------------------- staticKeySet (jwt/keyset.go:154-173)
def test_static_keyset_golden_tokens(golden, keys, J):
    """Every golden token through a one-key static set: accept <=> the oracle
    accepts (signature verdict AND payload is a JSON map), claims identical."""
    by_key = {}
    for t in golden["tokens"]:
        by_key.setdefault(t["key"], []).append(t)
    for kid, toks in by_key.items():
        ks, err = J.NewStaticKeySet([keys[kid][0]])
        assert err is None
        got = ks.VerifySignatureBatch([t["token"] for t in toks])
        for t, (claims, gerr) in zip(toks, got):
            want, werr = oracle_static(t["token"], [keys[kid][1]])
            assert (gerr is None) == (werr is None), (t["name"], gerr, werr)
            if gerr is None:
                assert claims == want, t["name"]
                assert t["verdict"] == 1, t["name"]
            else:
                assert gerr == "no known key successfully validated the token signature" or werr == "parse", t["name"]


def test_static_keyset_all_algs_and_wrong_keys(cases, keys, J):
    toks = [t for t in cases["tokens"] if t["name"].startswith(("alg-", "nokid-"))]
    assert len(toks) == 20
    all_keys = [keys[k][0] for k in ("ed-b", "p256-a", "rsa2048-b", "p384-a", "rsa2048-a", "rsa3072-a",
                                     "rsa4096-a", "p256-b", "p521-a", "ed-a")]
    ks, _ = J.NewStaticKeySet(all_keys)
    res = ks.VerifySignatureBatch([t["token"] for t in toks])
    for t, (claims, err) in zip(toks, res):
        assert err is None, (t["name"], err)
        assert claims == jws.go_json(jws.parse_jws(t["token"]).payload)
        assert claims["exp"] == float(cases["t0"] + 600)     # numbers are float64, as in Go
    # wrong key: every token against a set lacking its key
    for t in toks:
        others = [keys[k][0] for k in keys if k != t["key"] and not k.startswith("ed-A")]
        ks2, _ = J.NewStaticKeySet(others)
        claims, err = ks2.VerifySignature(t["token"])
        assert claims is None and err == "no known key successfully validated the token signature", t["name"]


def test_static_keyset_single_equals_batch(golden, keys, J):
    ks, _ = J.NewStaticKeySet([keys["p256-a"][0], keys["rsa2048-a"][0], keys["ed-a"][0]])
    toks = [t["token"] for t in golden["tokens"]]
    batch = ks.VerifySignatureBatch(toks)
    for tok, b in zip(toks[::5], batch[::5]):
        assert ks.VerifySignature(tok) == b


def test_new_static_keyset_errors(J):
    ks, err = J.NewStaticKeySet([])
    assert ks is None and err == "publicKeys must not be empty"


def test_hs256_and_malformed(cases, keys, J):
    t = next(x for x in cases["tokens"] if x["name"] == "alg-RS256-rsa2048-a")["token"]
    h, p, s = t.split(".")
    swapped = b64u(b'{"alg":"HS256","typ":"JWT"}') + "." + p + "." + s
    ks, _ = J.NewStaticKeySet([keys["rsa2048-a"][0]])
    assert ks.VerifySignature(swapped) == (None, "no known key successfully validated the token signature")
    claims, err = ks.VerifySignature("not.a.jwt.token")
    assert claims is None and "three parts" in err
    claims, err = ks.VerifySignature("")
    assert claims is None and err


# ---------------------------------------------------------------- jsonWebKeySet (go-oidc remoteKeySet)
class FakeJWKS:
    """Stands in for oidc.StartTestProvider's JWKS endpoint (jwt/keyset_test.go)."""

    def __init__(self, jwks):
        self.docs = [jwks] if not isinstance(jwks, list) else jwks
        self.calls = 0

    def __call__(self, url, ca_pem):
        doc = self.docs[min(self.calls, len(self.docs) - 1)]
        self.calls += 1
        if isinstance(doc, Exception):
            raise doc
        if isinstance(doc, tuple):
            return {"status": doc[0], "status_text": doc[1], "body": doc[2]}
        return {"status": 200, "body": json.dumps(doc).encode()}


def test_jwks_keyset_all_algs(cases, keys, J):
    kids = ["rsa2048-a", "rsa3072-a", "rsa4096-a", "p256-a", "p256-b", "p384-a", "p521-a", "ed-a"]
    fetch = FakeJWKS({"keys": [keys[k][2] for k in kids]})
    ks, err = J.NewJSONWebKeySet(None, "https://idp.example/.well-known/jwks.json", "", fetch)
    assert err is None
    toks = [t for t in cases["tokens"] if t["name"].startswith(("alg-", "nokid-", "kid-", "key_id-"))]
    res = ks.VerifySignatureBatch([t["token"] for t in toks])
    okeys = [keys[k][1] for k in kids]
    for k, kid in zip(okeys, kids):
        k.kid = kid
    for t, (claims, err) in zip(toks, res):
        want, werr = oracle_jwks(t["token"], okeys)
        assert (err is None) == (werr is None), (t["name"], err, werr)
        if err is None:
            assert claims == want
        else:
            assert err == "failed to verify id token signature", t["name"]
    assert fetch.calls >= 1
    # kid routing facts from the reference semantics (R34)
    by = {t["name"]: r for t, r in zip(toks, res)}
    assert by["kid-mismatch-p256-a"][1] is not None        # header kid names p256-b, signed by p256-a
    assert by["key_id-field-p256-a"][1] is None             # no "kid": every key is tried
    assert by["nokid-ES256-p256-b"][1] is None


def test_jwks_refresh_on_miss_and_rotation(cases, keys, J):
    tok = next(t for t in cases["tokens"] if t["name"] == "alg-ES256-p256-b")["token"]
    fetch = FakeJWKS([{"keys": [keys["p256-a"][2]]}, {"keys": [keys["p256-a"][2], keys["p256-b"][2]]}])
    ks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", fetch)
    # go-oidc remoteKeySet.verify refreshes at most once per call
    claims, err = ks.VerifySignature(tok)                   # cache empty -> fetch #1 (no p256-b): miss
    assert err == "failed to verify id token signature" and fetch.calls == 1
    claims, err = ks.VerifySignature(tok)                   # miss, cache expired -> fetch #2 has p256-b
    assert err is None and fetch.calls == 2
    claims, err = ks.VerifySignature(tok)                   # cached hit: no fetch
    assert err is None and fetch.calls == 2


def test_jwks_fetch_failures(cases, keys, J):
    tok = next(t for t in cases["tokens"] if t["name"] == "alg-ES256-p256-b")["token"]
    ks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", FakeJWKS(RuntimeError("connection refused")))
    claims, err = ks.VerifySignature(tok)
    assert claims is None and err.startswith("fetching keys oidc: get keys failed")
    ks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", FakeJWKS((500, "500 Internal Server Error", b"x")))
    claims, err = ks.VerifySignature(tok)
    assert err == "fetching keys oidc: get keys failed: 500 Internal Server Error x"
    bad = dict(keys["p256-b"][2], crv="P-384")
    ks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", FakeJWKS({"keys": [keys["p256-a"][2], bad]}))
    claims, err = ks.VerifySignature(tok)                   # one bad key fails the whole JWKS (R28)
    assert err.startswith("fetching keys oidc: failed to decode keys")
    claims, err = ks.VerifySignature("a.b")
    assert err.startswith("oidc: malformed jwt")


def test_jwks_payload_json_errors(cases, keys, J):
    fetch = FakeJWKS({"keys": [keys["p256-a"][2]]})
    ks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", fetch)
    toks = [t for t in cases["tokens"] if t["name"].startswith("claims-")]
    res = ks.VerifySignatureBatch([t["token"] for t in toks])
    ok = keys["p256-a"][1]
    ok.kid = "p256-a"
    for t, (claims, err) in zip(toks, res):
        want, werr = oracle_jwks(t["token"], [ok])
        assert (err is None) == (werr is None), (t["name"], err, werr)
        if err is None:
            assert claims == want, t["name"]
    names = {t["name"]: r for t, r in zip(toks, res)}
    assert names["claims-null"] == (None, None)             # nil map, no error (R33/R35)
    assert names["claims-array"][1] is not None
    assert names["claims-number-overflow"][1] is not None
    assert names["claims-invalid-utf8"][0]["iss"] == "a��b"


def test_remote_keyset_adapter_payloads(cases, keys, J):
    """go-oidc oidc.KeySet (NewRemoteKeySet): the verified payload bytes, and
    the same outcome as cap's jsonWebKeySet minus its json.Unmarshal step
    (jwt/keyset.go:126-139 wraps exactly this call)."""
    from cap_amd import oidc
    kids = ["rsa2048-a", "rsa3072-a", "rsa4096-a", "p256-a", "p256-b", "p384-a", "p521-a", "ed-a"]
    doc = {"keys": [keys[k][2] for k in kids]}
    rks = oidc.NewRemoteKeySet(None, "https://idp.example/jwks", FakeJWKS(doc))
    jks, _ = J.NewJSONWebKeySet(None, "https://idp.example/jwks", "", FakeJWKS(doc))
    toks = [t for t in cases["tokens"] if t["name"].startswith(("alg-", "nokid-", "kid-", "key_id-", "claims-"))]
    res = rks.VerifySignatureBatch(None, [t["token"] for t in toks])
    jres = jks.VerifySignatureBatch([t["token"] for t in toks])
    nverified = 0
    for t, (payload, err), (claims, jerr) in zip(toks, res, jres):
        if err is None:
            nverified += 1
            assert payload == jws.parse_jws(t["token"]).payload, t["name"]
            if jerr is not None:                       # only the JSON step may still fail
                with pytest.raises(jws.GoJSONError):
                    jws._claims_map(payload)
        else:
            assert payload is None and err == jerr, (t["name"], err, jerr)
    assert nverified >= 20
    single = rks.VerifySignature(None, toks[0]["token"])
    assert single == tuple(res[0])
    assert rks.VerifySignature(None, "a.b")[1].startswith("oidc: malformed jwt")


def test_new_json_web_keyset_errors(J):
    assert J.NewJSONWebKeySet(None, "", "", FakeJWKS({})) == (None, "jwksURL must not be empty")
    assert J.NewJSONWebKeySet(None, "https://x", "not a pem", FakeJWKS({})) == \
        (None, "could not parse CA PEM value successfully")


def test_oidc_discovery_keyset(cases, keys, J):
    iss = "https://idp.example"
    jwks = {"keys": [keys["p256-b"][2]]}

    def fetch(url, ca):
        if url == iss + "/.well-known/openid-configuration":
            return {"status": 200, "body": json.dumps({"issuer": iss, "jwks_uri": iss + "/jwks"})}
        assert url == iss + "/jwks"
        return {"status": 200, "body": json.dumps(jwks)}
    ks, err = J.NewOIDCDiscoveryKeySet(None, iss, "", fetch)
    assert err is None
    tok = next(t for t in cases["tokens"] if t["name"] == "alg-ES256-p256-b")["token"]
    assert ks.VerifySignature(tok)[1] is None
    ks, err = J.NewOIDCDiscoveryKeySet(None, iss + "/", "", fetch)
    assert ks is None and err == f'issuer did not match the returned issuer, expected "{iss}/" got "{iss}"'
    assert J.NewOIDCDiscoveryKeySet(None, "", "", fetch) == (None, "issuer must not be empty")

    def bad(url, ca):
        return {"status": 404, "status_text": "404 Not Found", "body": "nope"}
    assert J.NewOIDCDiscoveryKeySet(None, iss, "", bad) == (None, "404 Not Found: nope")

    def html(url, ca):
        return {"status": 200, "body": "<html>", "content_type": "text/html"}
    ks, err = J.NewOIDCDiscoveryKeySet(None, iss, "", html)
    assert ks is None and err.startswith('failed to decode OIDC discovery document: expected Content-Type = '
                                         'application/json, got "text/html"')


# ---------------------------------------------------------------- Validator (jwt/jwt.go)
def _now(cases, d=1):
    return lambda: cases["t0"] + d


def test_validator_reference_cases(cases, keys, J):
    """jwt/jwt_test.go TestValidator_Validate_Valid_JWT / _Invalid_JWT."""
    ks, _ = J.NewStaticKeySet([keys["p256-a"][0]])
    v, err = J.NewValidator(ks)
    assert err is None
    tok = {t["name"]: t["token"] for t in cases["tokens"]}
    E = J.Expected
    now = _now(cases)
    ok = [
        (tok["claims-std"], E(Issuer="https://example.com/", SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-std"], E(Subject="alice@example.com", SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-std"], E(ID="std", SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-std"], E(Audiences=["www.example.com"], SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-std"], E(Issuer="https://example.com/", Subject="alice@example.com", ID="std",
                              Audiences=["x", "www.example.com"], SigningAlgorithms=["RS256", "ES256"], Now=now)),
        (tok["claims-exp-past-in-skew"], E(SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-only-nbf"], E(SigningAlgorithms=["ES256"], Now=now)),
        (tok["claims-only-nbf"], E(SigningAlgorithms=["ES256"], NotBeforeLeeway=5, Now=now)),
    ]
    for t, e in ok:
        claims, err = v.Validate(t, e)
        assert err is None, err
        assert "iss" not in claims or claims["iss"] == "https://example.com/"
    bad = [
        (tok["claims-std"], E(Issuer="x", SigningAlgorithms=["ES256"], Now=now), "invalid issuer (iss) claim"),
        (tok["claims-std"], E(SigningAlgorithms=["RS256"], Now=now),
         "invalid algorithm (alg) header parameter: token signed with unexpected algorithm"),
        (tok["claims-std"], E(Now=now), "invalid algorithm (alg) header parameter: token signed with unexpected "
                                        "algorithm"),
        (tok["claims-std"], E(SigningAlgorithms=["HS256"], Now=now),
         'invalid algorithm (alg) header parameter: unsupported signing algorithm "HS256"'),
        (tok["claims-no-time-claims"], E(SigningAlgorithms=["ES256"], Now=now),
         "no issued at (iat), not before (nbf), or expiration time (exp) claims in token"),
        (tok["claims-nbf-future"], E(SigningAlgorithms=["ES256"], Now=now),
         "invalid not before (nbf) claim: token not yet valid"),
        (tok["claims-exp-past"], E(SigningAlgorithms=["ES256"], Now=now),
         "invalid expiration time (exp) claim: token is expired"),
        (tok["claims-iat-future"], E(SigningAlgorithms=["ES256"], Now=now),
         "invalid issued at (iat) claim: token issued in the future"),
        (tok["alg-ES256-p256-b"], E(SigningAlgorithms=["ES256"], Now=now),
         "error verifying token signature: no known key successfully validated the token signature"),
        ("malformed", E(Now=now), "error verifying token signature: square/go-jose: compact JWS format must have "
                                  "three parts"),
    ]
    for t, e, msg in bad:
        assert v.Validate(t, e) == (None, msg)
    assert J.NewValidator(None) == (None, "keySet must not be nil")


def test_validate_batch_matches_validate_and_oracle(golden, cases, keys, J):
    kids = ["p256-a", "rsa2048-a", "ed-a", "p384-a"]
    ks, _ = J.NewStaticKeySet([keys[k][0] for k in kids])
    v, _ = J.NewValidator(ks)
    okeys = [keys[k][1] for k in kids]
    toks = [t["token"] for t in cases["tokens"]] + [t["token"] for t in golden["tokens"]]
    for ex in [dict(SigningAlgorithms=["ES256", "RS256", "EdDSA", "PS256", "ES384"]),
               dict(SigningAlgorithms=["ES256"], Issuer="https://example.com/", Audiences=["www.example.com"]),
               dict(), dict(SigningAlgorithms=["ES256"], ClockSkewLeeway=-1, ExpirationLeeway=-1)]:
        for d in (1, 650, -300):
            e = J.Expected(Now=_now(cases, d), **ex)
            batch = v.ValidateBatch(toks, e)
            assert len(batch) == len(toks)
            now_ns = (cases["t0"] + d) * SECOND
            exd = {k: (x * SECOND if k.endswith("Leeway") else x) for k, x in ex.items()}
            n_ok = 0
            for tok, got in zip(toks, batch):
                want = jws.validate(tok, lambda t: jws.static_keyset_verify(t, okeys), exd, now_ns)
                if want[1] == "error verifying token signature: parse":
                    # the oracle does not restate go-jose's parse error texts
                    assert got[0] is None and got[1].startswith("error verifying token signature: "), tok[:60]
                    continue
                assert got == want, (tok[:60], got[1], want[1])
                n_ok += got[1] is None
            if d == 1 and ex.get("SigningAlgorithms") and len(ex) == 1:
                assert n_ok > 50
    e = J.Expected(SigningAlgorithms=["ES256"], Now=_now(cases))
    for tok in toks[:40]:
        assert v.Validate(tok, e) == v.ValidateBatch([tok], e)[0]


def test_validate_blob_throughput_entry(cases, keys, J):
    ks, _ = J.NewStaticKeySet([keys["p256-a"][0]])
    v, _ = J.NewValidator(ks)
    toks = [t["token"] for t in cases["tokens"]]
    e = J.Expected(SigningAlgorithms=["ES256"], Now=_now(cases))
    blob = "\n".join(toks * 50).encode()
    ok = v.ValidateBlob(blob, e)
    want = [r[1] is None for r in v.ValidateBatch(toks, e)] * 50
    assert list(ok) == [int(x) for x in want]
