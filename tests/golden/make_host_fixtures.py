#!/usr/bin/env python3
"""Generate tests/golden/host_cases.json: signed tokens for the KeySet /
Validator parity tests (claims validation, kid routing, JWKS, PEM/certificates).

Test infrastructure only (run here, never on the GPU box).  Signing reuses the
OpenSSL-backed helpers of make_fixtures.py and its committed private keys.

Claim shapes follow the reference's tests: testJWTClaims (jwt/keyset_test.go:
666-677) and the claim variations of jwt/jwt_test.go:17-498 (missing
iat/nbf/exp, now before nbf / after exp / before iat, audience as string or
list), plus encoding/json corner cases the claims round trip must reproduce
(case-insensitive member names, null members, non-string
iss, fractional or huge NumericDates).

Usage: python tests/golden/make_host_fixtures.py
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_fixtures as MF  # noqa: E402

T0 = 1611699344            # the fixtures' iat; tests validate at now = T0 + 1


def cert_pem(key):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "c.pem")
        MF.must(["openssl", "req", "-x509", "-new", "-key", key["_path"], "-subj", "/CN=" + key["kid"],
                 "-days", "3650", "-set_serial", "1", "-out", out])
        return open(out).read()


def payload_variants():
    std = MF.claims("std")
    v = {
        "std": std,
        "aud-string": dict(std, aud="www.example.com"),
        "aud-two": dict(std, aud=["a.example.com", "www.example.com"]),
        "aud-number-elem": dict(std, aud=["www.example.com", 5]),
        "aud-null": dict(std, aud=None),
        "aud-object": dict(std, aud={"x": 1}),
        "no-time-claims": {"iss": "https://example.com/", "sub": "alice@example.com"},
        "only-exp": {"exp": T0 + 600},
        "only-iat": {"iat": T0},
        "only-nbf": {"nbf": T0 - 10},
        "nbf-future": dict(std, nbf=T0 + 1000),
        "nbf-future-in-skew": dict(std, nbf=T0 + 30),
        "exp-past": dict(std, exp=T0 - 1000, nbf=T0 - 2000, iat=T0 - 2000),
        "exp-past-in-skew": dict(std, exp=T0 - 30, nbf=T0 - 2000, iat=T0 - 2000),
        "iat-future": dict(std, iat=T0 + 1000),
        "iat-null": dict(std, iat=None),
        "exp-null-EXP-set": dict(std, EXP=T0 + 5, exp=None),
        "exp-string": dict(std, exp=str(T0 + 600)),
        "exp-bool": dict(std, exp=True),
        "exp-fraction": dict(std, exp=T0 + 0.9, nbf=T0 - 100, iat=T0 - 100),
        "exp-huge": dict(std, exp=1e300),
        "exp-negative": dict(std, exp=-5.0),
        "iss-number": dict(std, iss=7),
        "iss-null": dict(std, iss=None),
        "iss-upper": {k: v for k, v in std.items() if k != "iss"} | {"ISS": "https://upper.example/"},
        "iss-both-cases": dict(std, ISS="https://upper.example/"),
        "sub-long-s": {k: v for k, v in std.items() if k != "sub"} | {"ſub": "bob@example.com"},
        "jti-mixed-case": {k: v for k, v in std.items() if k != "jti"} | {"JtI": "mixed"},
        "nested": dict(std, groups=["a", "b"], extra={"k": [1, 2.5, None, True], "s": "é中"}),
        "big-int-claim": dict(std, big=12345678901234567890),
    }
    out = {k: MF.enc_json(x) for k, x in v.items()}
    # raw payloads (not expressible through json.dumps)
    out["dup-keys"] = b'{"aud":["www.example.com"],"exp":%d,"iat":%d,"iss":"first","iss":"second","nbf":%d}' % (
        T0 + 600, T0, T0)
    out["null"] = b"null"
    out["array"] = b"[1,2,3]"
    out["not-json"] = b"{not json"
    out["empty"] = b""
    out["number-overflow"] = b'{"exp":%d,"x":1e400}' % (T0 + 600)
    out["invalid-utf8"] = b'{"exp":%d,"iss":"a\xff\xfeb","iat":%d}' % (T0 + 600, T0)
    out["lone-surrogate"] = b'{"exp":%d,"iss":"a\\ud800b","iat":%d}' % (T0 + 600, T0)
    out["whitespace"] = b' \n{"exp" : %d , "iat":%d}\t' % (T0 + 600, T0)
    return out


def main():
    K = MF.Keys()
    K.rsa("rsa2048-a", 2048); K.rsa("rsa2048-b", 2048)
    K.rsa("rsa3072-a", 3072); K.rsa("rsa4096-a", 4096)
    K.ec("p256-a", "P-256"); K.ec("p256-b", "P-256")
    K.ec("p384-a", "P-384"); K.ec("p521-a", "P-521")
    K.ed("ed-a"); K.ed("ed-b")
    keys = K.keys
    toks = []

    def sign(name, alg, kid, payload: bytes, hdr_kid="same", key_field="kid", extra=None):
        key = keys[kid]
        hdr = {"alg": alg, "typ": "JWT"}
        if hdr_kid == "same":
            hdr[key_field] = kid
        elif hdr_kid is not None:
            hdr[key_field] = hdr_kid
        if extra:
            hdr.update(extra)
        sinp = (MF.b64u(MF.enc_json(hdr)) + "." + MF.b64u(payload)).encode()
        sig = MF.ossl_sign(key, alg, sinp)
        toks.append(dict(name=name, alg=alg, key=kid, token=sinp.decode() + "." + MF.b64u(sig)))

    for pname, p in payload_variants().items():
        sign("claims-" + pname, "ES256", "p256-a", p)
    std = MF.enc_json(MF.claims("std"))
    for alg, kid in [("RS256", "rsa2048-a"), ("RS384", "rsa3072-a"), ("RS512", "rsa4096-a"),
                     ("PS256", "rsa2048-a"), ("PS384", "rsa3072-a"), ("PS512", "rsa4096-a"),
                     ("ES256", "p256-b"), ("ES384", "p384-a"), ("ES512", "p521-a"), ("EdDSA", "ed-a")]:
        sign(f"alg-{alg}-{kid}", alg, kid, std)
        sign(f"nokid-{alg}-{kid}", alg, kid, std, hdr_kid=None)
    sign("kid-mismatch-p256-a", "ES256", "p256-a", std, hdr_kid="p256-b")
    sign("kid-unknown-p256-a", "ES256", "p256-a", std, hdr_kid="rotated-kid")
    sign("key_id-field-p256-a", "ES256", "p256-a", std, key_field="key_id")
    sign("kid-rsa2048-b", "RS256", "rsa2048-b", std)
    certs = {kid: cert_pem(keys[kid]) for kid in ("rsa2048-a", "p256-a", "p384-a", "ed-a")}
    out = dict(t0=T0, certs=certs, tokens=toks)
    with open(os.path.join(HERE, "host_cases.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(toks)} tokens, {len(certs)} certificates")


if __name__ == "__main__":
    main()
