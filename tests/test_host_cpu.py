"""CPU parity of the C++ host mirror (cap_amd/csrc/host) against the oracle's
restatement of go-jose / encoding/json / cap semantics -- no GPU needed.

Covers SURVEY.md §8 rows a5 (ParseSigned), a6 (computeAuthData), a12
(validateSigningAlgorithm), a13 (claims), a15 (JWK / JWKS / PEM ingestion).
The C++ side and the oracle are independent restatements; the golden tokens
pin the oracle (tests/test_oracle.py)."""
import base64
import json
import os
import random

import pytest

from oracle import jws

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = pytest.importorskip("cap_amd._capjwt_host")

SECOND = 1_000_000_000
# mutation-fuzz rounds scale with CAPJWT_FUZZ_SCALE (tools/sanitize/run.sh runs 10x under ASan + UBSan)
FUZZ = max(1, int(os.environ.get("CAPJWT_FUZZ_SCALE", "1")))


@pytest.fixture(scope="module")
def cases():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "host_cases.json")))


def b64u(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


# ---------------------------------------------------------------- encoding/json
JSON_DOCS = [
    b'{}', b'[]', b'null', b'true', b'0', b'-0', b'1e5', b'-1.5E-3', b'"x"', b'{"a":1,"a":2}',
    b'{"a":{"b":[1,{"c":null}]}}', b' {"a" : 1 } ', b'{"a":"\\u00e9\\ud83d\\ude00"}', b'{"a":"\\ud800"}',
    b'{"a":"\\ud800\\u0041"}', b'{"a":"\\udc00"}', b'"\xff\xfe"', b'"\xed\xa0\x80"', b'"\xe2\x82"', b'"\xf0\x9f\x98\x80"',
    b'1e400', b'[1e400]', b'1e-400', b'{"a":1}x', b'{"a":1,}', b'[1,]', b'01', b'1.', b'.5', b'+1', b'NaN',
    b'Infinity', b'"a\x01"', b'"\\x"', b'{"a"}', b'', b' ', b'tru', b'nul', b'{"a":1', b'[1 2]', b'"\\u12"',
    b'{"a":"\\/\\b\\f\\n\\r\\t"}', b'123456789012345678901234567890', b'1.7976931348623157e308', b'-1.8e308',
    # integer literals around the parser's exact fast path (<= 15 digits)
    b'999999999999999', b'-999999999999999', b'1000000000000000', b'9007199254740993', b'[0,-0,7,1611699344]',
]


def _big_object(n, dups):
    # n distinct members k00..k{n-1}, then re-assignments of the members in `dups`
    mem = [f'"k{i:02d}":{i}' for i in range(n)] + [f'"k{i:02d}":"again{i}"' for i in dups]
    return ("{" + ",".join(mem) + "}").encode()


# objects across the linear-scan / index switch (16 members): a duplicate of
# each position must replace the earlier member (the last duplicate wins)
JSON_DOCS += [_big_object(n, d) for n, d in [(15, [14]), (16, [15]), (16, [0, 15]), (17, [15, 16]), (20, [15, 3, 19]),
                                              (40, [15, 16, 39, 0])]]


@pytest.mark.parametrize("doc", JSON_DOCS)
def test_json_matches_go_semantics(doc):
    v, err = H.json_loads(doc)
    try:
        want = jws.go_json(doc)
        ok = True
    except jws.GoJSONError:
        ok = False
    assert (err is None) == ok, (doc, err)
    if ok:
        assert v == want


@pytest.mark.parametrize("n,dups", [(15, [14]), (16, [15]), (17, [15, 16]), (20, [15, 3, 19]), (40, [15, 16, 39, 0])])
def test_json_duplicate_members_replace_in_place(n, dups):
    """map assignment: a re-assigned member keeps one entry holding the last
    value, on both sides of the parser's 16-member index switch"""
    out = H.json_marshal(_big_object(n, dups))
    for i in range(n):
        assert out.count(f'"k{i:02d}":'.encode()) == 1, (i, out)
    for i in dups:
        assert f'"k{i:02d}":"again{i}"'.encode() in out


# ---------------------------------------------------------------- base64url / whitespace
def test_b64url_decode_fuzz():
    rnd = random.Random(1)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_=+/\r\n. "
    for _ in range(3000 * FUZZ):
        s = "".join(rnd.choice(alpha) for _ in range(rnd.randint(0, 13)))
        assert H.b64url_decode(s) == jws.b64url_decode(s), s


def test_strip_whitespace_matches_go():
    s = "a b　c\u0085d e​f \t\n\v\f\rg h i j"
    assert H.strip_whitespace(s.encode()).decode() == jws.strip_whitespace(s)
    assert H.strip_whitespace(b"a\xffb") == "a�b".encode()


# ---------------------------------------------------------------- ParseSigned / computeAuthData
def _cmp_parse(tok):
    got = H.parse_signed(tok.encode("utf-8", "surrogatepass") if isinstance(tok, str) else tok)
    want = jws.parse_jws(tok)
    assert (got["error"] is None) == (want is not None), (tok, got["error"])
    if want is None:
        return
    assert got["alg"] == want.alg
    assert got["kid"] == want.kid
    assert got["payload"] == want.payload
    assert got["signature"] == want.signature
    assert got["nsigs"] == want.nsigs
    assert got["signing_input"] == want.signing_input, tok


def test_parse_signed_golden(golden, cases):
    for t in golden["tokens"]:
        _cmp_parse(t["token"])
    for t in cases["tokens"]:
        _cmp_parse(t["token"])


def _hdr_tok(hdr: bytes, payload=b'{"a":1}', sig=b"\x01\x02"):
    return b64u(hdr) + "." + b64u(payload) + "." + b64u(sig)


PARSE_CASES = [
    _hdr_tok(b'{"alg":"ES256"}'),
    _hdr_tok(b'null'),
    _hdr_tok(b'[]'),
    _hdr_tok(b''),
    _hdr_tok(b'{"alg":null}'),
    _hdr_tok(b'{"alg":""}'),
    _hdr_tok(b'{"alg":5}'),
    _hdr_tok(b'{"kid":null,"alg":"RS256"}'),
    _hdr_tok(b'{"nonce":5,"alg":"RS256"}'),
    _hdr_tok(b'{"alg":"RS256","b64":false,"crit":["b64"]}'),
    _hdr_tok(b'{"alg":"RS256","b64":"no"}'),
    _hdr_tok(b'{"alg":"RS256","b64":false}'),
    _hdr_tok(b'{"alg":"RS256","crit":"b64"}'),
    _hdr_tok(b'{"alg":"RS256","crit":[1]}'),
    _hdr_tok(b'{"alg":"RS256","crit":null}'),
    _hdr_tok(b'{"alg":"RS256","crit":[]}'),
    _hdr_tok(b'{"alg":"RS256","x":1e400}'),
    _hdr_tok(b'{"alg":"RS256","jwk":{"kty":"oct","k":"AAAA"}}'),
    _hdr_tok(b'{"alg":"RS256","jwk":"x"}'),
    _hdr_tok(b'{"alg":"RS256","jwk":null}'),
    _hdr_tok(b'{"alg":"RS256","x5c":["notbase64!"]}'),
    _hdr_tok(b'{"alg":"RS256","x5c":[]}'),
    _hdr_tok(b'{"alg":"ES256"}', sig=b""),
    _hdr_tok(b'{"alg":"ES256"}', payload=b""),
    _hdr_tok(b'{"alg":"ES256"} '),
    _hdr_tok(b'{"alg":"ES256"}') + "=",
    " " + _hdr_tok(b'{"alg":"ES256"}') + "\n",
    _hdr_tok(b'{"alg":"ES256"}').replace(".", ". ", 1),
    "a.b",
    "a.b.c.d",
    "",
    "..",
    "{",
    json.dumps({"payload": b64u(b'{"a":1}'), "protected": b64u(b'{"alg":"ES256"}'), "signature": "AQI"}),
    json.dumps({"payload": b64u(b'{"a":1}'), "header": {"alg": "ES256", "kid": "k"}, "signature": "AQI"}),
    json.dumps({"payload": b64u(b'{"a":1}'), "protected": b64u(b'{"alg":""}'), "header": {"alg": "ES256"},
                "signature": "AQI"}),
    json.dumps({"payload": b64u(b'{"a":1}'), "protected": b64u(b'{"alg":"RS256"}'), "header": {"alg": "ES256"},
                "signature": "AQI"}),
    json.dumps({"payload": b64u(b'{"a":1}'), "protected": "", "signature": "AQI"}),
    json.dumps({"payload": "", "protected": b64u(b'{"alg":"ES256"}'), "signature": "AQI"}),
    json.dumps({"protected": b64u(b'{"alg":"ES256"}'), "signature": "AQI"}),
    json.dumps({"payload": None, "protected": b64u(b'{"alg":"ES256"}'), "signature": "AQI"}),
    json.dumps({"payload": 5, "signature": "AQI"}),
    json.dumps({"payload": b64u(b"x"), "header": {"alg": "ES256", "nonce": "n"}, "signature": "AQI"}),
    json.dumps({"payload": b64u(b"x"), "header": {"alg": "ES256", "nonce": ""}, "signature": "AQI"}),
    json.dumps({"payload": b64u(b"x"), "header": 5, "signature": "AQI"}),
    json.dumps({"payload": b64u(b"x"), "signatures": [{"protected": b64u(b'{"alg":"ES256","kid":"a"}'),
                                                       "signature": "AQI"}]}),
    json.dumps({"payload": b64u(b"x"), "signatures": [{"protected": b64u(b'{"alg":"ES256"}'), "signature": "AQI"},
                                                      {"header": {"alg": "RS256"}, "signature": "AQI"}]}),
    json.dumps({"payload": b64u(b"x"), "signatures": [], "protected": b64u(b'{"alg":"ES256"}'), "signature": "AQ"}),
    json.dumps({"payload": b64u(b"x"), "signatures": 7}),
    json.dumps({"payload": b64u(b"x"), "signatures": [None]}),
    json.dumps({"payload": b64u(b"x"), "signatures": [{"protected": b64u(b'{"alg":"ES256","crit":["exp"]}'),
                                                       "signature": "AQI"}]}),
    json.dumps({"payload": b64u(b"x"), "protected": b64u(b'{"alg":"ES256","b64":false}'), "signature": "AQI"}),
    "[1]",
    "null",
]


@pytest.mark.parametrize("i", range(len(PARSE_CASES)))
def test_parse_signed_edge_cases(i):
    _cmp_parse(PARSE_CASES[i])


def test_parse_signed_mutation_fuzz(golden):
    rnd = random.Random(7)
    toks = [t["token"] for t in golden["tokens"][:60]]
    alpha = "A.=_-+/ \n{}\" é"
    for _ in range(1500):
        t = list(rnd.choice(toks))
        for _ in range(rnd.randint(1, 3)):
            op = rnd.random()
            i = rnd.randrange(len(t) + 1)
            if op < 0.4 and t:
                t[min(i, len(t) - 1)] = rnd.choice(alpha)
            elif op < 0.7:
                t.insert(i, rnd.choice(alpha))
            elif t:
                del t[min(i, len(t) - 1)]
        _cmp_parse("".join(t))


# ---------------------------------------------------------------- JWK / JWKS / PEM
def _jwk(src, **over):
    d = src
    if d["kty"] == "RSA":
        n = int(d["n"], 16)
        j = {"kty": "RSA", "kid": d["kid"], "n": b64u(n.to_bytes((n.bit_length() + 7) // 8, "big")),
             "e": b64u(int(d["e"]).to_bytes(3, "big").lstrip(b"\0"))}
    elif d["kty"] == "EC":
        sz = jws.CURVE_BYTES[d["crv"]]
        j = {"kty": "EC", "kid": d["kid"], "crv": d["crv"], "x": b64u(int(d["x"], 16).to_bytes(sz, "big")),
             "y": b64u(int(d["y"], 16).to_bytes(sz, "big"))}
    else:
        j = {"kty": "OKP", "kid": d["kid"], "crv": "Ed25519", "x": b64u(bytes.fromhex(d["x"]))}
    j.update(over)
    return {k: v for k, v in j.items() if v is not None}


def _key_eq(native, okey):
    d = native.as_dict()
    if okey.kty in ("none", "oct"):
        return d["kind"] in ("none", "oct")
    if okey.kty == "RSA":
        return d["kind"] == "RSA" and d["n"] == okey.n and d["e"] == okey.e
    if okey.kty == "EC":
        return d["kind"] == "EC" and d["crv"] == okey.crv and d["x"] == okey.x and d["y"] == okey.y
    return d["kind"] == "Ed25519" and d["x"] == okey.x


def _cmp_jwks(doc: bytes):
    try:
        want = jws.jwks_decode(doc)
    except (jws.JWKError, jws.GoJSONError):
        want = None
    try:
        got = H.jwks_decode(doc)
    except ValueError:
        got = None
    assert (got is None) == (want is None), doc
    if want is not None:
        assert len(got) == len(want)
        for (kid, k), w in zip(got, want):
            assert _key_eq(k, w), doc


def test_jwks_decode(golden):
    raw = golden["keys_raw"]
    good = [_jwk(d) for d in raw if not d["kid"].startswith("ed-A")]
    _cmp_jwks(json.dumps({"keys": good}).encode())
    p256 = next(d for d in raw if d["kid"] == "p256-a")
    rsa = next(d for d in raw if d["kid"] == "rsa2048-a")
    bad_y = b64u((int(p256["y"], 16) ^ 1).to_bytes(32, "big"))
    variants = [
        _jwk(p256, y=bad_y), _jwk(p256, x=b64u(b"\0" + bytes(31))[:-1]), _jwk(p256, crv="P-999"), _jwk(p256, y=None),
        _jwk(p256, kty="XYZ"), _jwk(rsa, e=None), _jwk(rsa, n=""), _jwk(rsa, e="AQAB" * 4), _jwk(rsa, d="AQAB"),
        _jwk(rsa, d="AQAB", p="AQ", q="AQ"), _jwk(p256, d=b64u(bytes(32))), _jwk(p256, d=b64u(bytes(31))),
        {"kty": "oct", "k": "c2VjcmV0"}, {"kty": "oct"}, {"kty": "OKP", "crv": "Ed25519", "x": b64u(b"\x01" * 20)},
        {"kty": "OKP", "crv": "X25519", "x": b64u(bytes(32))}, _jwk(rsa, kid=5), _jwk(rsa, n="!!"),
        _jwk(rsa, x5c=["!!"]), _jwk(rsa, x5c="abc"), {"kty": "RSA", "n": "AQAB", "e": "AQAB", "alg": 5},
    ]
    for v in variants:
        _cmp_jwks(json.dumps({"keys": [_jwk(rsa), v]}).encode())
    for doc in [b"null", b"{}", b'{"keys":null}', b'{"KEYS":[]}', b'{"keys":5}', b"[]", b"{", b'{"keys":[null]}']:
        _cmp_jwks(doc)


def test_parse_public_key_pem(golden, cases):
    for d in golden["keys_raw"]:
        if not d.get("pem"):
            continue
        k = jws.Key.from_fixture(d)
        if d["kty"] == "OKP":
            with pytest.raises(ValueError, match="data does not contain any valid RSA or ECDSA public keys"):
                H.parse_public_key_pem(d["pem"].encode())
            continue
        assert _key_eq(H.parse_public_key_pem(d["pem"].encode()), k), d["kid"]
    for kid, pem in cases["certs"].items():
        d = next(x for x in golden["keys_raw"] if x["kid"] == kid)
        if d["kty"] == "OKP":
            with pytest.raises(ValueError):
                H.parse_public_key_pem(pem.encode())
        else:
            assert _key_eq(H.parse_public_key_pem(pem.encode()), jws.Key.from_fixture(d)), kid
    for bad in [b"", b"garbage", b"-----BEGIN PUBLIC KEY-----\nAAAA\n-----END PUBLIC KEY-----\n"]:
        with pytest.raises(ValueError):
            H.parse_public_key_pem(bad)


def _mutate_bytes(rnd, b, alpha):
    b = bytearray(b)
    for _ in range(rnd.randint(1, 4)):
        op = rnd.random()
        i = rnd.randrange(len(b) + 1)
        if op < 0.45 and b:
            b[min(i, len(b) - 1)] = rnd.choice(alpha)
        elif op < 0.75:
            b.insert(i, rnd.choice(alpha))
        elif b:
            del b[min(i, len(b) - 1):min(i, len(b) - 1) + rnd.randint(1, 8)]
    return bytes(b)


def test_json_mutation_fuzz():
    """byte mutations of JSON documents (and of the claims payload shape):
    accept / reject and the decoded value equal Go encoding/json's (oracle)"""
    rnd = random.Random(11)
    seeds = [d for d in JSON_DOCS if len(d) > 1] + [
        b'{"aud":["www.example.com"],"exp":1611699344,"iat":1611699284,"iss":"https://example.com/",'
        b'"jti":"7","nbf":1611699284,"sub":"alice@example.com","n":[1.5e3,-0,null,true,{"x":"\\u00e9"}]}']
    alpha = list(b'{}[]":,.-+0123456789eE\\u tnrfal\x00\x7f\xc3\xa9\xed\xa0\xff')
    for _ in range(2000 * FUZZ):
        doc = _mutate_bytes(rnd, rnd.choice(seeds), alpha)
        v, err = H.json_loads(doc)
        try:
            want = jws.go_json(doc)
            ok = True
        except jws.GoJSONError:
            ok = False
        assert (err is None) == ok, (doc, err)
        if ok:
            assert v == want, doc


def test_jwks_mutation_fuzz(golden, cases):
    """byte mutations of a JWKS document (RSA / EC / OKP members, an x5c
    certificate) and of the certificate's DER under x5c: the decoded key set,
    or the rejection, equals go-jose's (oracle jwks_decode with its own DER walker)"""
    rnd = random.Random(5)
    raw = golden["keys_raw"]
    d = next(x for x in raw if x["kid"] == "p256-a")
    der = base64.b64decode("".join(l for l in cases["certs"]["p256-a"].splitlines() if "-----" not in l))
    good = [_jwk(x) for x in raw if x["kid"] in ("rsa2048-a", "p384-a", "ed-a")]
    doc = json.dumps({"keys": good + [_jwk(d, x5c=[base64.b64encode(der).decode()])]}).encode()
    alpha = list(b'{}[]":,AQBxyz09-_=+/ \x00\xff')
    for _ in range(400 * FUZZ):
        _cmp_jwks(_mutate_bytes(rnd, doc, alpha))
    for _ in range(400 * FUZZ):
        bad = _mutate_bytes(rnd, der, list(range(256)))
        _cmp_jwks(json.dumps({"keys": [_jwk(d, x5c=[base64.b64encode(bad).decode()])]}).encode())


def test_pem_mutation_fuzz(golden, cases):
    """byte mutations of PEM public keys and certificates: ParsePublicKeyPEM
    (jwt/keyset.go:178-200) never crashes and rejects with ValueError; DER-level
    mutations that still parse give the key of the oracle's DER walker"""
    rnd = random.Random(9)
    pems = [x["pem"].encode() for x in golden["keys_raw"] if x.get("pem")] + [p.encode() for p in cases["certs"].values()]
    for _ in range(500 * FUZZ):
        src = rnd.choice(pems)
        if rnd.random() < 0.5:
            bad = _mutate_bytes(rnd, src, list(b"ABCQ019+/=-\n "))
        else:
            lines = src.decode().splitlines()
            body = base64.b64decode("".join(l for l in lines if "-----" not in l))
            body = _mutate_bytes(rnd, body, list(range(256)))
            b64 = base64.b64encode(body).decode()
            bad = ("\n".join([lines[0]] + [b64[i:i + 64] for i in range(0, len(b64), 64)] + [lines[-1]]) + "\n").encode()
        try:
            H.parse_public_key_pem(bad)
        except ValueError:
            pass


def test_x5c_certificate_must_match_key(golden, cases):
    d = next(x for x in golden["keys_raw"] if x["kid"] == "p256-a")
    pem = cases["certs"]["p256-a"]
    der_b64 = "".join(l for l in pem.splitlines() if "-----" not in l)
    _cmp_jwks(json.dumps({"keys": [_jwk(d, x5c=[der_b64])]}).encode())
    assert len(H.jwks_decode(json.dumps({"keys": [_jwk(d, x5c=[der_b64])]}).encode())) == 1
    other = next(x for x in golden["keys_raw"] if x["kid"] == "p256-b")
    with pytest.raises(ValueError, match="do not match"):
        H.jwks_decode(json.dumps({"keys": [_jwk(other, x5c=[der_b64])]}).encode())


def test_ec_on_curve(golden):
    for d in golden["keys_raw"]:
        if d["kty"] != "EC":
            continue
        k = jws.Key.from_fixture(d)
        assert H.ec_on_curve(d["crv"], k.x, k.y)
        assert not H.ec_on_curve(d["crv"], k.x, (int.from_bytes(k.y, "big") + 1).to_bytes(len(k.y), "big"))
        p = jws.CURVE_PB[d["crv"]][0]
        assert not H.ec_on_curve(d["crv"], (int.from_bytes(k.x, "big") + p).to_bytes(len(k.x) + 1, "big"), k.y)


# ---------------------------------------------------------------- Validate claims (jwt/jwt.go:95-202)
def _expected(**kw):
    e = H.Expected()
    d = {}
    for k, v in kw.items():
        setattr(e, k, v)
        d[k] = v
    return e, d


EXPECTEDS = [
    {}, {"Issuer": "https://example.com/"}, {"Issuer": "nope"}, {"Subject": "alice@example.com"},
    {"Subject": "bob@example.com"}, {"ID": "std"}, {"ID": "x"}, {"Audiences": ["www.example.com"]},
    {"Audiences": ["a", "b"]}, {"SigningAlgorithms": ["ES256"]}, {"SigningAlgorithms": ["RS256", "EdDSA"]},
    {"SigningAlgorithms": ["HS256"]}, {"SigningAlgorithms": ["ES256"], "ExpirationLeeway": -1},
    {"SigningAlgorithms": ["ES256"], "NotBeforeLeeway": 5 * SECOND, "ExpirationLeeway": 7 * SECOND + 500_000_000},
    {"SigningAlgorithms": ["ES256"], "ClockSkewLeeway": -1}, {"SigningAlgorithms": ["ES256"], "ClockSkewLeeway": 1},
    {"SigningAlgorithms": ["ES256"], "ClockSkewLeeway": 3600 * SECOND},
    {"SigningAlgorithms": ["ES256"], "Issuer": "https://upper.example/"},
    {"SigningAlgorithms": ["ES256"], "Issuer": "second"}, {"SigningAlgorithms": ["ES256"], "Subject": "bob@example.com"},
    {"SigningAlgorithms": ["ES256"], "ID": "mixed"},
]


def test_validate_claims_matches_oracle(cases):
    t0 = cases["t0"]
    nows = [t0 * SECOND + SECOND, t0 * SECOND - 200 * SECOND, (t0 + 700) * SECOND + 123, (t0 - 31) * SECOND,
            (t0 + 100000) * SECOND]
    n = 0
    for t in cases["tokens"]:
        p = jws.parse_jws(t["token"])
        try:
            claims = jws._claims_map(p.payload)
        except jws.GoJSONError:
            continue
        for ex in EXPECTEDS:
            e, d = _expected(**ex)
            for now in nows:
                got = H.validate_claims(p.payload, p.alg, len(p.signature), e, now)
                want = jws.validate_claims(claims, p.alg, p.nsigs, len(p.signature), d, now)
                assert (got[1] is None) == (want[1] is None), (t["name"], ex, now, got[1], want[1])
                assert got[1] == want[1], (t["name"], ex, now)
                if got[1] is None:
                    assert got[0] == want[0]
                n += 1
    assert n > 1000


def test_reference_claim_cases(cases):
    """jwt/jwt_test.go:17-498 outcomes, stated directly (not via the oracle)."""
    t0 = cases["t0"]
    tok = {t["name"]: t for t in cases["tokens"]}
    now = (t0 + 1) * SECOND

    def run(name, **ex):
        p = jws.parse_jws(tok[name]["token"])
        e, _ = _expected(SigningAlgorithms=ex.pop("SigningAlgorithms", ["ES256"]), **ex)
        return H.validate_claims(p.payload, p.alg, len(p.signature), e, ex.get("now", now))[1]

    assert run("claims-std") is None
    assert run("claims-std", Issuer="https://example.com/", Subject="alice@example.com", ID="std",
               Audiences=["www.example.com"]) is None
    assert run("claims-std", Issuer="x") == "invalid issuer (iss) claim"
    assert run("claims-std", Subject="x") == "invalid subject (sub) claim"
    assert run("claims-std", ID="x") == "invalid ID (jti) claim"
    assert run("claims-std", Audiences=["x"]).startswith("invalid audience (aud) claim")
    assert run("claims-std", SigningAlgorithms=["RS256"]) == \
        "invalid algorithm (alg) header parameter: token signed with unexpected algorithm"
    assert run("claims-no-time-claims") == \
        "no issued at (iat), not before (nbf), or expiration time (exp) claims in token"
    assert run("claims-nbf-future") == "invalid not before (nbf) claim: token not yet valid"
    assert run("claims-nbf-future-in-skew") is None
    assert run("claims-exp-past") == "invalid expiration time (exp) claim: token is expired"
    assert run("claims-exp-past-in-skew") is None
    assert run("claims-iat-future") == "invalid issued at (iat) claim: token issued in the future"
    assert run("claims-only-iat") is None              # exp defaults to iat + 150 s
    assert run("claims-aud-string", Audiences=["www.example.com"]) is None
    assert run("claims-aud-null") is not None
    assert run("claims-iss-number") is not None
