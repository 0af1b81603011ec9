"""GPU parity on the verify branches random tokens do not reach, and on the
mixed-alg JWKS workload of BASELINE configs[4]:

* tests/golden/ec_edge.json (make_ec_edge_fixtures.py): comb sums that meet
  P == +-Q (the exact recompute, k_ec_exact -- counted through
  jg_batch_exceptions), accepting tokens whose R has x(R) >= n, an ES256 token
  on a P-521 key, and the reference's own example token (jwt/docs_test.go:35);
* 32 kids over all 10 algs with ~5 % tampered tokens (signature bit flip,
  payload flip, kid swap, alg swap) through the JWKS KeySet and
  Validator.ValidateBatch, every claims map and error string against the
  oracle (oracle/jws.py jwks_keyset_verify / validate)."""
import base64
import json
import os

import numpy as np
import pytest

from oracle import jws
from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu

ROOT = H.ROOT


def edge():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "ec_edge.json")))


def test_ec_edge_fixtures_through_the_abi():
    """Every crafted token against its key: GPU verdict == fixture (Go rule) ==
    oracle, via jg_verify_batch (streaming path) and a resident batch."""
    from cap_amd import _lib
    d = edge()
    kid_index = {k["kid"]: i for i, k in enumerate(d["keys"])}
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in d["keys"]}
    toks = d["tokens"]
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in d["keys"]])
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    out = ctx.verify(arena)
    for t, s in zip(toks, slots):
        p = jws.parse_jws(t["token"])
        want = int(jws.verify_sig(p, okeys[t["key"]])) if p is not None else 0
        assert want == t["verdict"], t["name"]
        assert (0 if s is None else out[s]) == t["verdict"], t["name"]
    assert sum(t["verdict"] for t in toks) >= 7
    ctx.close()


def test_exact_path_is_exercised_per_curve():
    """The exceptional tokens really go down k_ec_exact: the resident batch's
    per-class exception counters are non-zero for P-256, P-384 and P-521, the
    counts equal the number of exceptional fixtures per curve, and those
    verdicts (accepting ones included) equal the fixture's."""
    from cap_amd import _lib
    d = edge()
    kid_index = {k["kid"]: i for i, k in enumerate(d["keys"])}
    crv_of = {k["kid"]: k["crv"] for k in d["keys"]}
    exc = [t for t in d["tokens"] if t.get("exceptional")]
    assert {crv_of[t["key"]] for t in exc} == {"P-256", "P-384", "P-521"}
    assert any(t["verdict"] == 1 for t in exc)
    ctx = _lib.Context()
    # the fixtures' accepting exceptional tokens were searched for the 26/20
    # comb (make_ec_edge_fixtures.py COMB_W): P-256 key tables at W = 20
    ctx.set_table_budget(0)
    ctx.load_keys([H.abi_key(k) for k in d["keys"]])
    arena, slots = H.jobs_from_tokens(exc, kid_index)
    b = ctx.stage(arena)
    out = b.run(want_verdicts=True)
    assert [out[s] for s in slots] == [t["verdict"] for t in exc]
    counts = b.exceptions()
    want = {4: 0, 5: 0, 6: 0}
    for t in exc:
        want[{"P-256": 4, "P-384": 5, "P-521": 6}[crv_of[t["key"]]]] += 1
    assert {c: counts[c] for c in (4, 5, 6)} == want, counts
    # streamed (untimed, classes on their own streams) agrees too
    pinned = _lib.PinnedBuffer(len(exc))
    b.enqueue(pinned)
    b.sync()
    assert list(pinned.bytes()) == list(out)
    pinned.free()
    b.free()
    ctx.close()


def test_reference_docs_example_token_rejects(golden, J_keys):
    """jwt/docs_test.go:35 -- RS256, signed by a key nobody here holds: the
    static and JWKS key sets reject it with the reference's error strings."""
    from cap_amd import jwt
    tok = next(t for t in edge()["tokens"] if t["name"] == "reference-docs-example-RS256")["token"]
    nat = [v[0] for v in J_keys.values()]
    ks, _ = jwt.NewStaticKeySet(nat)
    assert ks.VerifySignature(tok) == (None, "no known key successfully validated the token signature")
    doc = {"keys": [v[2] for v in J_keys.values()]}
    jks, _ = jwt.NewJSONWebKeySet(None, "https://idp.example/jwks", "",
                                  lambda url, ca: {"status": 200, "body": json.dumps(doc).encode()})
    assert jks.VerifySignature(tok) == (None, "failed to verify id token signature")
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="your_expected_issuer", SigningAlgorithms=["RS256"], Now=lambda: 1526239022 - 10)
    assert v.Validate(tok, e) == (None, "error verifying token signature: no known key successfully validated "
                                        "the token signature")
    okeys = [v[1] for v in J_keys.values()]
    with pytest.raises(jws.ErrNoKey):
        jws.static_keyset_verify(tok, okeys)


@pytest.fixture(scope="module")
def J_keys(golden):
    from cap_amd import jwt
    out = {}
    for d in golden["keys_raw"]:
        k = jws.Key.from_fixture(d)
        if k.kty == "RSA":
            nat = jwt.PublicKey.rsa(k.n, k.e)
            jwk = {"kty": "RSA", "kid": d["kid"], "n": b64u(k.n), "e": b64u(k.e.to_bytes(4, "big").lstrip(b"\0"))}
        elif k.kty == "EC":
            nat = jwt.PublicKey.ec(k.crv, k.x, k.y)
            jwk = {"kty": "EC", "kid": d["kid"], "crv": k.crv, "x": b64u(k.x), "y": b64u(k.y)}
        else:
            nat = jwt.PublicKey.ed25519(k.x)
            jwk = {"kty": "OKP", "kid": d["kid"], "crv": "Ed25519", "x": b64u(k.x)}
        k.kid = d["kid"]
        out[d["kid"]] = (nat, k, jwk)
    return out


def b64u(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


# ---------------------------------------------------------------- configs[4]: 32 kids, 10 algs, 5 % tampered
def _c5_pool(per_kid=48, frac=0.05, seed=1):
    """Tokens of every bench kid (tools/benchkeys, signed by tools/tokgen) in a
    seeded random order, ~5 % tampered as header/payload/signature strings:
    signature bit flip, payload character flip, kid swap (header names the
    next kid), alg swap within the family."""
    import bench
    meta = bench.bench_keys()
    pool = []
    for ki, (kid, alg, pem, _, _) in enumerate(meta):
        pool += [t.decode() for t in bench.gen_tokens(alg, per_kid, [pem], 4, "c5test", kid_base=ki)]
    rng = np.random.default_rng(seed)
    pool = [pool[i] for i in rng.permutation(len(pool))]
    sel = rng.choice(len(pool), int(len(pool) * frac), replace=False)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    fam = {"RS": ["RS256", "RS384", "RS512", "PS256", "PS384", "PS512"], "PS": None, "ES": ["ES256", "ES384", "ES512"]}
    fam["PS"] = fam["RS"]
    for j, i in enumerate(sel):
        h, p, s = pool[i].split(".")
        mode = j % 4
        if mode == 0:
            s = alpha[alpha.index(s[0]) ^ 1] + s[1:]
        elif mode == 1:
            p = p[:5] + alpha[alpha.index(p[5]) ^ 2] + p[6:]
        else:
            hdr = json.loads(base64.urlsafe_b64decode(h + "=" * (-len(h) % 4)))
            if mode == 2 or hdr["alg"] == "EdDSA":
                n = int(hdr["kid"].split("-")[1])
                hdr["kid"] = f"kid-{(n + 1) % len(meta):02d}"
            else:
                alts = [a for a in fam[hdr["alg"][:2]] if a != hdr["alg"]]
                hdr["alg"] = alts[j % len(alts)]
            h = b64u(json.dumps(hdr, separators=(",", ":")).encode())
        pool[i] = ".".join((h, p, s))
    okeys = []
    for kid, alg, pem, _, jwk in meta:
        k = jws.jwk_decode(jwk)
        k.kid = kid
        okeys.append(k)
    return meta, pool, set(int(i) for i in sel), okeys


class CountingJWKS:
    def __init__(self, doc, max_age=0):
        self.body = json.dumps(doc).encode()
        self.max_age = max_age
        self.calls = 0

    def __call__(self, url, ca):
        self.calls += 1
        return {"status": 200, "body": self.body, "max_age": self.max_age}


def test_config5_jwks_32_kids_tampered_batch_vs_oracle():
    from cap_amd import jwt
    meta, pool, tampered, okeys = _c5_pool()
    doc = {"keys": [m[4] for m in meta]}
    fetch = CountingJWKS(doc)
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "", fetch)
    assert err is None
    res = ks.VerifySignatureBatch(pool)
    assert fetch.calls == 1          # the first fetch, for the empty cache's misses (R34)
    n_ok = 0
    for i, (tok, (claims, gerr)) in enumerate(zip(pool, res)):
        try:
            want, werr = jws.jwks_keyset_verify(tok, okeys), None
        except jws.ErrNoKey as e:
            want, werr = None, str(e)
        assert (gerr, claims) == (werr, want), (i, gerr, werr)
        n_ok += gerr is None
        assert (gerr is None) == (i not in tampered), i
    assert n_ok == len(pool) - len(tampered)
    # Validator.ValidateBatch over the same key set: claims + error strings
    v, _ = jwt.NewValidator(ks)
    algs = sorted({m[1] for m in meta})
    for exp in (dict(SigningAlgorithms=algs, Issuer="https://example.com/", Audiences=["www.example.com"]),
                dict(SigningAlgorithms=["ES256", "RS256"])):
        e = jwt.Expected(Now=lambda: 1611699344 + 60, **exp)
        got = v.ValidateBatch(pool, e)
        now_ns = (1611699344 + 60) * jws.SECOND
        for i, (tok, g) in enumerate(zip(pool, got)):
            want = jws.validate(tok, lambda t: jws.jwks_keyset_verify(t, okeys), exp, now_ns)
            assert tuple(g) == tuple(want), (i, g[1], want[1])
    assert fetch.calls == 3          # max_age 0: each later batch with misses refreshes once


def test_config5_raw_abi_every_token_every_kid():
    """The same pool through the C ABI with jobs for EVERY kid of the token's
    family (the static-set candidate list, R33), streamed in small chunks over
    two device slots: each verdict equals the oracle's verify_sig."""
    from cap_amd import _lib
    meta, pool, _, okeys = _c5_pool(per_kid=16, seed=2)
    ctx = _lib.Context([0, 0])
    ctx.load_keys([m[3] for m in meta])
    ctx.set_chunk(256)
    arena = _lib.Arena()
    want = []
    for tok in pool:
        p = jws.parse_jws(tok)
        sig_b64 = jws.b64url_encode(p.signature).encode()
        for ki, k in enumerate(okeys):
            fam = "RSA" if p.alg[:2] in ("RS", "PS") else "EC" if p.alg[:2] == "ES" else "OKP"
            if k.kty != fam:
                continue
            arena.add(p.signing_input, sig_b64, p.alg, ki)
            want.append(int(jws.verify_sig(p, k)))
    out = ctx.verify(arena)
    assert list(out) == want
    assert sum(want) > len(pool) * 0.8
    ctx.close()
