"""cap's oidc at_hash / c_hash checks (oidc/id_token.go:59-145).

CPU: the oracle (oracle/oidc.py) against the hand-labelled fixtures of
tests/golden/make_oidc_fixtures.py (the reference's test matrix of
oidc/id_token_test.go:98-350, the OpenID Connect Core example at_hash, and
every error branch).  GPU: the product (cap_amd.oidc -> C++ host mirror ->
jg_hash_batch) against the same labels with the reference's exact error
strings, and against the oracle on a seeded random batch.
"""
import base64
import hashlib
import json
import os
import random

import pytest

from oracle import oidc as ooidc

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "oidc_cases.json")))


def _kind_ok(kind, err):
    if err is None:
        return kind is None
    marks = {"claims": ("UnmarshalClaims:", "IDToken.Claims:"), "malformed": ("malformed jwt (",),
             "unsupported": ("id_token signed with algorithm",), "mismatch": ("hash does not match",)}
    return kind is not None and any(m in err for m in marks[kind])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_labels(case):
    v, kind = ooidc.verify_hash_claim(case["claim"], case["token"], case["value"].encode())
    assert v == case["verified"]
    assert _kind_ok(kind, case["err"]), (kind, case["err"])


def test_oracle_oidc_core_example():
    # OpenID Connect Core 1.0: at_hash of this access token under RS256
    h = hashlib.sha256(b"jHkWEdUXMU1BwAsC4vtUsZwnNvTIxEl0z9K3vx5KF0Y").digest()
    assert base64.urlsafe_b64encode(h[:16]).rstrip(b"=") == b"77QmUPtjPfzWtF2AnpK9RQ"


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_labels_exact():
    from cap_amd import oidc
    for claim in ("at_hash", "c_hash"):
        cs = [c for c in CASES if c["claim"] == claim]
        fn = oidc.VerifyAccessTokenBatch if claim == "at_hash" else oidc.VerifyAuthorizationCodeBatch
        got = fn([c["token"] for c in cs], [c["value"] for c in cs])
        for c, (v, err) in zip(cs, got):
            assert (v, err) == (c["verified"], c["err"]), c["name"]


@pytest.mark.gpu
def test_gpu_single_token_methods():
    from cap_amd import oidc
    c = next(x for x in CASES if x["name"] == "oidc-core-example")
    assert oidc.IDToken(c["token"]).VerifyAccessToken(c["value"]) == (True, None)
    c = next(x for x in CASES if x["name"] == "c_hash-ES384")
    assert oidc.IDToken(c["token"]).VerifyAuthorizationCode(c["value"]) == (True, None)
    assert oidc.IDToken(c["token"]).VerifyAuthorizationCode("other")[0] is False


@pytest.mark.gpu
def test_gpu_random_batch_vs_oracle():
    from cap_amd import oidc
    rng = random.Random(7)
    algs = list(ooidc.HASH_BITS) + ["EdDSA", "HS256"]
    toks, vals = [], []
    for i in range(3000):
        alg = rng.choice(algs)
        n = rng.choice([0, 1, 55, 56, 64, 111, 112, 128, rng.randrange(600)])
        v = bytes(rng.randrange(32, 127) for _ in range(n))
        claims = {"sub": f"user-{i}"}
        if rng.random() < 0.9:
            hb = ooidc.HASH_BITS.get(alg, 256)
            h = {256: hashlib.sha256, 384: hashlib.sha384, 512: hashlib.sha512}[hb](v).digest()
            claims["at_hash"] = base64.urlsafe_b64encode(h[:len(h) // 2]).rstrip(b"=").decode()
            if rng.random() < 0.1:
                v = v + b"!"                                   # mismatch
        hdr = base64.urlsafe_b64encode(json.dumps({"alg": alg}).encode()).rstrip(b"=").decode()
        pl = base64.urlsafe_b64encode(json.dumps(claims).encode()).rstrip(b"=").decode()
        toks.append(f"{hdr}.{pl}.c2ln")
        vals.append(v)
    got = oidc.VerifyAccessTokenBatch(toks, vals)
    for t, v, (gv, gerr) in zip(toks, vals, got):
        ov, kind = ooidc.verify_access_token(t, v)
        assert gv == ov and _kind_ok(kind, gerr), (t, v, gv, gerr, ov, kind)
