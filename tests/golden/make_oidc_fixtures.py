"""Generate tests/golden/oidc_cases.json: id_token / value pairs for cap's
IDToken.VerifyAccessToken / VerifyAuthorizationCode (oidc/id_token.go:59-145),
each labelled by hand from the reference's rules (not by running any oracle):

  * the reference's own test matrix (oidc/id_token_test.go:98-350): every one
    of the 10 algs verifies its own at_hash / c_hash; EdDSA -> (false, nil);
    missing claim -> (false, nil); a hash of another value -> ErrInvalidAtHash /
    ErrInvalidCodeHash;
  * the OpenID Connect Core 1.0 example access token (published at_hash);
  * the error branches of verifyHashClaim / UnmarshalClaims: empty token,
    wrong part count, '=' or a bad byte in the claims segment, non-object and
    null claims, non-string claim, go-jose parse failure, unsupported alg.

verifyHashClaim never checks the signature, so signatures here are random
bytes.  Run:  python tests/golden/make_oidc_fixtures.py
"""
import base64
import hashlib
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
OP = "VerifyAccessToken: verifyHashClaim: "
HASH = {"RS256": hashlib.sha256, "ES256": hashlib.sha256, "PS256": hashlib.sha256,
        "RS384": hashlib.sha384, "ES384": hashlib.sha384, "PS384": hashlib.sha384,
        "RS512": hashlib.sha512, "ES512": hashlib.sha512, "PS512": hashlib.sha512}
ALGS = list(HASH) + ["EdDSA"]
rng = random.Random(0x0DC)


def b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def half_hash(alg, value: bytes) -> str:
    h = HASH[alg](value).digest()
    return b64(h[:len(h) // 2])


def token(header: dict, claims, sig_len=64, raw_claims=None) -> str:
    hs = b64(json.dumps(header, separators=(",", ":")).encode())
    cs = raw_claims if raw_claims is not None else b64(json.dumps(claims, separators=(",", ":")).encode())
    return f"{hs}.{cs}.{b64(bytes(rng.randrange(256) for _ in range(sig_len)))}"


def base_claims():
    return {"iss": "https://example.com/", "iat": 1600000000, "exp": 1600000600,
            "aud": ["www.example.com"], "sub": "alice@example.com"}


def main():
    cases = []

    def add(name, claim, tok, value, verified, err):
        cases.append(dict(name=name, claim=claim, token=tok, value=value, verified=verified, err=err))

    mism = {"at_hash": OP + "access_token hash does not match value in id_token",
            "c_hash": OP + "authorization code hash does not match value in id_token"}
    for claim, value in (("at_hash", "test-access-token"), ("c_hash", "test-code")):
        for alg in ALGS:
            c = base_claims()
            c[claim] = half_hash(alg if alg != "EdDSA" else "RS256", value.encode())
            tok = token({"alg": alg, "kid": "k1", "typ": "JWT"}, c)
            add(f"{claim}-{alg}", claim, tok, value, alg != "EdDSA", None)
        c = base_claims()
        add(f"{claim}-missing", claim, token({"alg": "RS256"}, c), value, False, None)
        c[claim] = half_hash("RS256", b"this-isn't-going-to-match")
        add(f"{claim}-not-equal", claim, token({"alg": "RS256"}, c), value, False, mism[claim])
        c[claim] = 12345
        add(f"{claim}-not-string", claim, token({"alg": "RS256"}, c), value, False, None)

    # OpenID Connect Core 1.0 example (id_token + access_token, RS256)
    at = "jHkWEdUXMU1BwAsC4vtUsZwnNvTIxEl0z9K3vx5KF0Y"
    c = base_claims()
    c["at_hash"] = "77QmUPtjPfzWtF2AnpK9RQ"
    add("oidc-core-example", "at_hash", token({"alg": "RS256", "kid": "1e9gdk7"}, c, 256), at, True, None)

    # lengths around the SHA block boundaries
    for alg in ("RS256", "ES384", "PS512"):
        for n in (0, 1, 55, 56, 63, 64, 65, 111, 112, 119, 120, 127, 128, 129, 300):
            v = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789-_.~") for _ in range(n))
            c = base_claims()
            c["at_hash"] = half_hash(alg, v.encode())
            add(f"len-{alg}-{n}", "at_hash", token({"alg": alg}, c), v, True, None)

    # error branches
    c = base_claims()
    c["at_hash"] = half_hash("RS256", b"x")
    good = token({"alg": "RS256"}, c)
    add("empty-token", "at_hash", "", "x", False, OP + "IDToken.Claims: id_token is empty: invalid parameter")
    two = good.rsplit(".", 1)[0]
    add("two-parts", "at_hash", two, "x", False,
        OP + "UnmarshalClaims: malformed jwt, expected 3 parts got 2: invalid parameter")
    add("four-parts", "at_hash", good + ".x", "x", False,
        OP + "UnmarshalClaims: malformed jwt, expected 3 parts got 4: invalid parameter")
    h, p, s = good.split(".")
    add("claims-padded", "at_hash", f"{h}.{p}==.{s}", "x", False,
        OP + f"UnmarshalClaims: malformed jwt claims: illegal base64 data at input byte {len(p)}")
    add("claims-bad-byte", "at_hash", f"{h}.{p[:5]}*{p[5:]}.{s}", "x", False,
        OP + "UnmarshalClaims: malformed jwt claims: illegal base64 data at input byte 5")
    add("claims-array", "at_hash", f"{h}.{b64(b'[1,2]')}.{s}", "x", False,
        OP + "UnmarshalClaims: unable to marshal jwt JSON: json: cannot unmarshal array into Go value of type "
        "map[string]interface {}")
    add("claims-null", "at_hash", f"{h}.{b64(b'null')}.{s}", "x", False, None)
    add("claims-newline", "at_hash", f"{h}.{p[:8]}\n{p[8:]}.{s}", "x", True, None)
    add("header-bad-b64", "at_hash", f"!{h}.{p}.{s}", "x", False,
        OP + "malformed jwt (illegal base64 data at input byte 0): token malformed")
    add("unsupported-alg", "at_hash", token({"alg": "HS256"}, c), "x", False,
        OP + 'id_token signed with algorithm "HS256": unsupported signing algorithm')
    add("unsupported-alg-quoted", "at_hash", token({"alg": "R\"S\t256é"}, c), "x", False,
        OP + 'id_token signed with algorithm "R\\"S\\t256é": unsupported signing algorithm')
    add("alg-none-empty", "at_hash", token({"typ": "JWT"}, c), "x", False,
        OP + 'id_token signed with algorithm "": unsupported signing algorithm')
    # c_hash mismatch keeps the reference's "VerifyAccessToken" op name
    c2 = base_claims()
    c2["c_hash"] = half_hash("ES512", b"other")
    add("c_hash-mismatch-es512", "c_hash", token({"alg": "ES512"}, c2), "code", False, mism["c_hash"])

    with open(os.path.join(HERE, "oidc_cases.json"), "w") as f:
        json.dump(cases, f, indent=1, ensure_ascii=False)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
