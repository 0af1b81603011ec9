"""Pin the CPU oracle (oracle/) before trusting it as the parity checker.

* golden vectors: tokens signed and verified by OpenSSL 3 (independent of the
  oracle), plus Go-semantics edge cases labelled by SURVEY.md Appendix A rule
  (tests/golden/make_fixtures.py);
* FIPS 180-4 / hashlib cross-checks for SHA-256/384/512;
* RFC 8032 §7.1 Ed25519 known answers.
"""
import hashlib
import os

import pytest

from oracle import jws


def test_golden_tokens_signature_verdicts(golden):
    bad = []
    for t in golden["tokens"]:
        p = jws.parse_jws(t["token"])
        v = 0 if p is None else int(jws.verify_sig(p, golden["keys"][t["key"]]))
        if v != t["verdict"]:
            bad.append((t["name"], v, t["verdict"], t["source"]))
    assert not bad, bad


def test_golden_covers_every_alg_and_rule(golden):
    algs = {t["alg"] for t in golden["tokens"] if t["verdict"] == 1}
    assert algs >= {"RS256", "RS384", "RS512", "PS256", "PS384", "PS512", "ES256", "ES384", "ES512", "EdDSA"}
    rules = {t["source"] for t in golden["tokens"]}
    for r in ("R1", "R2", "R3", "R6", "R7", "R13", "R14", "R15", "R16", "R18", "R19", "R20", "R22", "R24", "R25", "R26"):
        assert r in rules, r


@pytest.mark.parametrize("n", [0, 1, 3, 55, 56, 63, 64, 65, 111, 112, 119, 127, 128, 129, 255, 256, 1000])
def test_sha2_against_hashlib(n):
    m = os.urandom(n)
    assert jws.hash_bytes(256, m) == hashlib.sha256(m).digest()
    assert jws.hash_bytes(384, m) == hashlib.sha384(m).digest()
    assert jws.hash_bytes(512, m) == hashlib.sha512(m).digest()


def test_sha2_fips180_abc():
    assert jws.hash_bytes(256, b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert jws.hash_bytes(384, b"abc").hex() == (
        "cb00753f45a35e8bb5a03d699ac65007272c32ab0eded1631a8b605a43ff5bed8086072ba1e7cc2358baeca134c825a7")
    assert jws.hash_bytes(512, b"abc").hex() == (
        "ddaf35a193617abacc417349ae20413112e6fa4e89a97ea20a9eeee64b55d39a"
        "2192992a274fc1a836ba3c23a3feebbd454d4423643ce80e2a9ac94fa54ca49f")


RFC8032 = [
    ("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
]


@pytest.mark.parametrize("pub,msg,sig", RFC8032)
def test_ed25519_rfc8032(pub, msg, sig):
    L = jws.lib()
    pub, msg, sig = bytes.fromhex(pub), bytes.fromhex(msg), bytes.fromhex(sig)
    assert L.or_ed25519_verify(pub, msg, len(msg), sig, len(sig)) == 1
    bad = bytearray(sig); bad[0] ^= 1
    assert L.or_ed25519_verify(pub, msg, len(msg), bytes(bad), len(bad)) == 0


@pytest.mark.parametrize("s,ok", [("", b""), ("QQ", b"A"), ("QR", b"A"), ("QQ==", b"A"), ("QUI", b"AB"),
                                  ("Q", None), ("QUJD", b"ABC"), ("QU\nJD", b"ABC"), ("Q+", None), ("Q=Q", None)])
def test_b64url_go_semantics(s, ok):
    assert jws.b64url_decode(s) == ok


def test_static_keyset_semantics(golden):
    """staticKeySet: keys tried in order, first verifying key whose payload is a JSON map wins (R33)."""
    k = golden["keys"]
    t = next(t for t in golden["tokens"] if t["name"] == "valid-RS256-rsa2048-a-0")
    claims = jws.static_keyset_verify(t["token"], [k["ed-a"], k["p256-a"], k["rsa2048-a"]])
    assert claims["jti"] == "jti-RS256-rsa2048-a-0"
    with pytest.raises(jws.ErrNoKey):
        jws.static_keyset_verify(t["token"], [k["ed-a"], k["p256-a"], k["rsa2048-b"]])
    for t in golden["tokens"]:
        if "keyset_verdict" in t:
            try:
                jws.static_keyset_verify(t["token"], [k[t["key"]]])
                got = 1
            except jws.ErrNoKey:
                got = 0
            assert got == t["keyset_verdict"], t["name"]


def test_oracle_rsa_keys_above_4096_bits():
    """RSA keys of 4100 to 16384 bits (tests/golden/rsa_big.json): Go's
    crypto/rsa has no 4096-bit ceiling, so valid RS256 / RS512 / PS512 tokens
    accept and signature-flipped ones reject."""
    import json
    import os
    from oracle import jws
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rsa_big.json")))
    keys = {k["kid"]: jws.Key.from_fixture(k) for k in d["keys"]}
    for t in d["tokens"]:
        p = jws.parse_jws(t["token"])
        assert int(jws.verify_sig(p, keys[t["key"]])) == t["want"], t["name"]


def test_oracle_matches_crafted_ec_edge_fixtures():
    """tests/golden/ec_edge.json (make_ec_edge_fixtures.py: verdicts from plain
    affine big-integer arithmetic under the Go rule R22): exceptional comb
    sums, x(R) >= n, an ES256 token on a P-521 key, the reference's example
    token -- the C oracle agrees on every one."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ec_edge.json")))
    keys = {k["kid"]: jws.Key.from_fixture(k) for k in d["keys"]}
    assert len(d["tokens"]) >= 20
    for t in d["tokens"]:
        p = jws.parse_jws(t["token"])
        assert int(jws.verify_sig(p, keys[t["key"]])) == t["verdict"], t["name"]
    assert sum(t["verdict"] for t in d["tokens"]) >= 7
