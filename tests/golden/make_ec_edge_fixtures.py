#!/usr/bin/env python3
"""Crafted ECDSA fixtures for the verify branches random tokens never reach.

Test infrastructure only (run here; writes tests/golden/ec_edge.json).  Every
verdict is the Go rule (crypto/ecdsa.Verify
accepts iff R = u1 G + u2 Q != infinity and x(R) mod n == r), evaluated with
plain affine big-integer arithmetic below -- independent of both the C oracle
and the HIP kernels, which the tests then hold to these verdicts.

1. Exceptional group-law cases of the comb kernel (ecdsa.hip k_ec_point sums
   one table entry per window, mixed additions with no case handling; a sum
   that meets P == +-Q leaves Z == 0 and the token is recomputed by
   k_ec_exact):
   * keys Q = G and Q = -G with r = s = e mod n, so u1 = u2 = 1: window 0 adds
     G onto +-G (a doubling -> 2G, reject; an inverse pair -> infinity, reject);
   * ACCEPTING exceptional tokens: key Q = G (private key 1), a fixed nonce k,
     and messages searched until the lowest signed comb digits of u1 (generator
     window) and u2 (key window) have equal magnitude (ecdsa.hpp ec_comb_w:
     P-256 26/20 bits, P-384 and P-521 20/16 bits).
2. The x(R) >= n acceptance branch (k_ec_point: X == (r + n) Z^2): a point R0
   with x(R0) = r + n for a small r, key Q = r^-1 (R0 - e G), signature
   (r, s = 1) -- then u1 G + u2 Q = e G + r Q = R0 and Go accepts.  Plus the
   same with r + 1 (reject), and an ES256 token on a P-521 key (alg/curve
   mismatch, R19) with r = s = e and Q = R0 - G.
3. The one literal token the reference holds (jwt/docs_test.go:35, RS256, an
   unknown key): it must reject under any key set.

Usage: python tests/golden/make_ec_edge_fixtures.py
"""
import base64
import hashlib
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_fixtures import CURVES, claims, enc_json, b64u  # noqa: E402

GEN = {
    "P-256": (0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296,
              0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5),
    "P-384": (int("aa87ca22be8b05378eb1c71ef320ad746e1d3b628ba79b9859f741e082542a38"
                  "5502f25dbf55296c3a545e3872760ab7", 16),
              int("3617de4a96262c6f5d9e98bf9292dc29f8f41dbd289a147ce9da3113b5f0b8c0"
                  "0a60b1ce1d7e819d7a431d7c90ea0e5f", 16)),
    "P-521": (int("00c6858e06b70404e9cd9e3ecb662395b4429c648139053fb521f828af606b4d"
                  "3dbaa14b5e77efe75928fe1dc127a2ffa8de3348b3c1856a429bf97e7e31c2e5bd66", 16),
              int("011839296a789a3bc0045c8a5fb42c7d1bd998f54449579b446817afbd17273e"
                  "662c97ee72995ef42640c550b9013fad0761353c7086a272c24088be94769fd16650", 16)),
}
COMB_W = {"P-256": (26, 20), "P-384": (24, 16), "P-521": (20, 16)}   # (generator, key) -- ecdsa.hpp
ALG_OF = {"P-256": "ES256", "P-384": "ES384", "P-521": "ES512"}
SIZE = {"ES256": 32, "ES384": 48, "ES512": 66}
HASH = {"ES256": hashlib.sha256, "ES384": hashlib.sha384, "ES512": hashlib.sha512}
DOCS_TOKEN = ("eyJhbGciOiJSUzI1NiIsInR5cCI6IkpXVCJ9.eyJpc3MiOiJleHBfaXNzIiwiZXhwIjoxNTI2MjM5MDIyfQ."
              "XG1xYJcuPMfgu8xkMzVjkYK2WIUyl4-A1Zq1j4Dfr99-PJUN36ZAgi8Fj08modiexXETrg05MqSxkJAE5Czns1IhqEEypx6xfY"
              "HSINp0SLKxBFHPA4BCi0IW83T-e225JjjVEGFR_Wo8QM6Rc-qQVJ9bqwKD4kcbQeMACkgGFcgNurtNkOM9vtOEs0Pe9tb4nHYw"
              "4ef1stCytTi9GFZwGoHQf0pjpWCpjlxaFIR4vmHQ4YB3w29o_tKN6zqyA2FITnvkzGnaLvdPecJNskRSCPUTRfYcVVNXCOnCvTd"
              "pvwK-c4nCs5yGnw3eeFoT6mhQSp39KYti1MpHNQTYwZrLTA")


# ---------------------------------------------------------------- affine curve arithmetic (a = -3)
def ec_add(crv, P, Q):
    p = CURVES[crv]["p"]
    if P is None:
        return Q
    if Q is None:
        return P
    (x1, y1), (x2, y2) = P, Q
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return None
        lam = (3 * x1 * x1 - 3) * pow(2 * y1, -1, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, p) % p
    x3 = (lam * lam - x1 - x2) % p
    return (x3, (lam * (x1 - x3) - y1) % p)


def ec_mul(crv, k, P):
    R = None
    for bit in bin(k)[2:] if k > 0 else "":
        R = ec_add(crv, R, R)
        if bit == "1":
            R = ec_add(crv, R, P)
    return R


def ec_neg(crv, P):
    return None if P is None else (P[0], (-P[1]) % CURVES[crv]["p"])


def on_curve(crv, P):
    c = CURVES[crv]
    x, y = P
    return (y * y - (x * x * x - 3 * x + c["b"])) % c["p"] == 0


def lift_x(crv, x):
    """A point with this x (even y), or None."""
    c = CURVES[crv]
    p = c["p"]
    rhs = (x * x * x - 3 * x + c["b"]) % p
    if pow(rhs, (p - 1) // 2, p) != 1:
        return None
    if p % 4 == 3:
        y = pow(rhs, (p + 1) // 4, p)
    else:                                    # P-256/P-384/P-521 are all 3 mod 4
        raise ValueError("unsupported prime")
    assert y * y % p == rhs
    return (x, y if y % 2 == 0 else p - y)


def go_verify(crv, alg, Q, sinp: bytes, r, s):
    """crypto/ecdsa.Verify with go-jose's size/hash from the alg (R18-R22)."""
    n = CURVES[crv]["n"]
    if not (1 <= r < n and 1 <= s < n):
        return 0
    h = HASH[alg](sinp).digest()
    nbits = n.bit_length()
    e = int.from_bytes(h, "big")
    if len(h) * 8 > nbits:
        e >>= len(h) * 8 - nbits
    w = pow(s, -1, n)
    R = ec_add(crv, ec_mul(crv, e * w % n, GEN[crv]), ec_mul(crv, r * w % n, Q))
    return 1 if R is not None and R[0] % n == r else 0


def hash_e(crv, alg, sinp):
    n = CURVES[crv]["n"]
    h = HASH[alg](sinp).digest()
    e = int.from_bytes(h, "big")
    if len(h) * 8 > n.bit_length():
        e >>= len(h) * 8 - n.bit_length()
    return e % n


def low_digit(u, W):
    """ecdsa.hip store_digit_rows: the signed W-bit digit of window 0."""
    v = u & ((1 << W) - 1)
    return v - (1 << W) if v >= 1 << (W - 1) else v


def sinput(alg, kid, jti):
    hdr = {"alg": alg, "kid": kid, "typ": "JWT"}
    return (b64u(enc_json(hdr)) + "." + b64u(enc_json(claims(jti)))).encode()


# ---------------------------------------------------------------- accepting-exceptional search
def _search(args):
    """Private key 1 (Q = G), one fixed message, nonces k = k0, k0+1, ...:
    s = (e + r) / k, so u1 = k e / (e + r) and u2 = k r / (e + r); stop when
    the window-0 signed digits of u1 (generator table) and u2 (key table)
    have equal magnitude -- the comb sum then adds +-(the accumulator) to
    itself.  R = kG advances by one affine addition per trial."""
    crv, sinp, k0, limit = args
    alg = ALG_OF[crv]
    n = CURVES[crv]["n"]
    wg, wq = COMB_W[crv]
    e = hash_e(crv, alg, sinp)
    G = GEN[crv]
    R = ec_mul(crv, k0, G)
    k = k0
    for _ in range(limit):
        r = R[0] % n
        inv = pow((e + r) % n, -1, n)
        u1 = k * e % n * inv % n
        u2 = k * r % n * inv % n
        d1, d2 = low_digit(u1, wg), low_digit(u2, wq)
        if d2 != 0 and abs(d1) == abs(d2):
            return k, r, (e + r) * pow(k, -1, n) % n, d1, d2
        R = ec_add(crv, R, G)
        k += 1
    return None


def find_accepting_exceptional(crv, sinp, seed, workers=8, per_round=200_000, rounds=200):
    with mp.Pool(workers) as pool:
        for rd in range(rounds):
            jobs = [(crv, sinp, seed + ((rd * workers + w) << 40), per_round) for w in range(workers)]
            hits = [h for h in pool.map(_search, jobs) if h]
            if hits:
                return min(hits)
    raise RuntimeError("no collision found")


def main():
    keys, toks = [], []

    def key_entry(kid, crv, P):
        assert on_curve(crv, P)
        keys.append(dict(kid=kid, kty="EC", crv=crv, x=format(P[0], "x"), y=format(P[1], "x"), pem=None))

    def tok_entry(name, alg, kid, sinp, r, s, verdict, source, crv, Q, **kw):
        sz = SIZE[alg]
        assert go_verify(crv, alg, Q, sinp, r, s) == verdict, name
        sig = r.to_bytes(sz, "big") + s.to_bytes(sz, "big")
        toks.append(dict(name=name, alg=alg, key=kid, token=sinp.decode() + "." + b64u(sig), verdict=verdict,
                         source=source, **kw))

    for crv in ("P-256", "P-384", "P-521"):
        n = CURVES[crv]["n"]
        G = GEN[crv]
        assert on_curve(crv, G) and ec_mul(crv, n, G) is None
        alg = ALG_OF[crv]
        tag = crv.replace("-", "").lower()
        # 1a. Q = +-G, r = s = e: u1 = u2 = 1
        for nm, Q in ((f"{tag}-G", G), (f"{tag}-negG", ec_neg(crv, G))):
            key_entry(nm, crv, Q)
            sinp = sinput(alg, nm, "u1-eq-u2-eq-1")
            e = hash_e(crv, alg, sinp)
            tok_entry(f"exc-{nm}-r-eq-s-eq-e", alg, nm, sinp, e, e, go_verify(crv, alg, Q, sinp, e, e),
                      "R22 (exceptional: G + " + ("G" if nm.endswith("-G") else "-G") + ")", crv, Q, exceptional=1)
        # 1b. accepting exceptional tokens under Q = G
        sinp = sinput(alg, f"{tag}-G", "exc-accept")
        k, r, s, d1, d2 = find_accepting_exceptional(crv, sinp, 0x5EED)
        tok_entry(f"exc-{tag}-G-accept-d{'eq' if d1 == d2 else 'neg'}", alg, f"{tag}-G", sinp, r, s, 1,
                  f"R22 (window-0 digits {d1} / {d2}: P == {'+' if d1 == d2 else '-'}Q in the comb sum)", crv, G,
                  exceptional=1)
        s2 = s + 1 if s + 1 < n else s - 1
        toks.append(dict(toks[-1], name=toks[-1]["name"] + "-tamper", exceptional=0,
                         token=sinp.decode() + "." + b64u(r.to_bytes(SIZE[alg], "big") + s2.to_bytes(SIZE[alg], "big")),
                         verdict=go_verify(crv, alg, G, sinp, r, s2), source="R22"))
        # 2. x(R) >= n: R0 with x = r + n for the smallest r that lifts
        p = CURVES[crv]["p"]
        r = 1
        while lift_x(crv, r + n) is None:
            r += 1
        assert r + n < p
        R0 = lift_x(crv, r + n)
        nm = f"{tag}-xR-ge-n"
        sinp = sinput(alg, nm, "x-ge-n")
        e = hash_e(crv, alg, sinp)
        Q = ec_mul(crv, pow(r, -1, n), ec_add(crv, R0, ec_neg(crv, ec_mul(crv, e, G))))
        key_entry(nm, crv, Q)
        tok_entry(f"xR-ge-n-{tag}-accept", alg, nm, sinp, r, 1, 1, "R22 (x(R) = r + n)", crv, Q)
        tok_entry(f"xR-ge-n-{tag}-r-plus-1", alg, nm, sinp, r + 1, 1, go_verify(crv, alg, Q, sinp, r + 1, 1),
                  "R22", crv, Q)
    # 2b. ES256 on a P-521 key (R19), r = s = e, Q = R0 - G, x(R0) = e + n
    crv, alg = "P-521", "ES256"
    n = CURVES[crv]["n"]
    for j in range(1000):
        sinp = sinput(alg, "p521-es256-xR-ge-n", f"mismatch-{j}")
        e = hash_e(crv, alg, sinp)
        R0 = lift_x(crv, e + n)
        if R0 is not None:
            break
    Q = ec_add(crv, R0, ec_neg(crv, GEN[crv]))
    key_entry("p521-es256-xR-ge-n", crv, Q)
    tok_entry("xR-ge-n-es256-on-p521", alg, "p521-es256-xR-ge-n", sinp, e, e, 1, "R19/R22 (x(R) = e + n)", crv, Q)
    # 3. the reference's literal example token: no key set here holds its key
    toks.append(dict(name="reference-docs-example-RS256", alg="RS256", key="p256-G", token=DOCS_TOKEN, verdict=0,
                     source="jwt/docs_test.go:35 (unknown key)"))
    with open(os.path.join(HERE, "ec_edge.json"), "w") as f:
        json.dump({"keys": keys, "tokens": toks}, f, indent=1)
    print(f"{len(keys)} keys, {len(toks)} tokens")


if __name__ == "__main__":
    main()
