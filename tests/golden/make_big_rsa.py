"""Generates tests/golden/rsa_big.json: RSA keys above 4096 bits -- 4100 and
4142 (the largest 148-limb RSA-4K+ layout), 6144, 8192 and 8286 (the 296-limb
layout) and 8287, 16384 (the 592-limb layout) -- with RS256 (PKCS#1 v1.5, RFC
8017 EMSA-PKCS1-v1_5) and PS512 (EMSA-PSS, salt = hash length, as go-jose
signs) tokens signed by them, plus a signature-flipped copy of each.  Go's
crypto/rsa verifies keys of any size >= 1024 bits, so the expected verdicts
are accept / reject.  Moduli above 4142 bits are products of several primes
(RSA verification does not depend on how N factors; it keeps generation
fast).  Test infrastructure: run once here, the JSON is committed (sympy
primes, Python big ints)."""
import base64
import hashlib
import json
import os
import random

import sympy

DI = {"RS256": (bytes.fromhex("3031300d060960864801650304020105000420"), hashlib.sha256)}


def b64(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def modulus(bits, rng):
    """N of exactly `bits` bits with known factors: two primes up to 4142 bits,
    else 1024-bit primes and one to fill the length."""
    if bits <= 4142:
        while True:
            p = sympy.randprime(1 << (bits // 2 - 1), 1 << (bits // 2))
            q = sympy.randprime(1 << (bits - bits // 2 - 1), 1 << (bits - bits // 2))
            if (p * q).bit_length() == bits and p != q:
                return p * q, [p, q]
    while True:
        ps = [sympy.randprime(1 << 1023, 1 << 1024) for _ in range(bits // 1024 - 1)]
        P = 1
        for x in ps:
            P *= x
        lo, hi = -(-(1 << (bits - 1)) // P), (1 << bits) // P
        if hi - lo < 1 << 20:
            continue
        last = sympy.randprime(lo, hi)
        if last not in ps and (P * last).bit_length() == bits:
            return P * last, ps + [last]


def mgf1(seed, n, hf):
    out, c = b"", 0
    while len(out) < n:
        out += hf(seed + c.to_bytes(4, "big")).digest()
        c += 1
    return out[:n]


def pss_encode(m, embits, hf, rng):
    hlen = hf().digest_size
    emlen = (embits + 7) // 8
    salt = bytes(rng.getrandbits(8) for _ in range(hlen))
    h = hf(b"\0" * 8 + hf(m).digest() + salt).digest()
    db = b"\0" * (emlen - 2 * hlen - 2) + b"\x01" + salt
    masked = bytearray(x ^ y for x, y in zip(db, mgf1(h, emlen - hlen - 1, hf)))
    masked[0] &= 0xff >> (8 * emlen - embits)
    return bytes(masked) + h + b"\xbc"


def main():
    rng = random.Random(0x5EED)
    out = {"keys": [], "tokens": []}
    for bits in (4100, 4142, 6144, 8192, 8286, 8287, 16384):
        n, primes = modulus(bits, rng)
        e = 65537
        phi = 1
        for p in primes:
            phi *= p - 1
        d = pow(e, -1, phi)
        kid = f"big-{bits}"
        out["keys"].append({"kid": kid, "kty": "RSA", "n": format(n, "x"), "e": e})
        k = (bits + 7) // 8
        algs = ("RS256", "RS512") if bits <= 4142 else ("RS256", "PS512")
        for alg in algs:
            hdr = b64(json.dumps({"alg": alg, "kid": kid, "typ": "JWT"}, separators=(",", ":")).encode())
            pl = b64(json.dumps({"iss": "https://example.com/", "sub": "alice@example.com", "jti": str(rng.getrandbits(32))},
                                separators=(",", ":")).encode())
            si = (hdr + "." + pl).encode()
            if alg == "PS512":
                em = pss_encode(si, bits - 1, hashlib.sha512, rng)
                em = b"\0" * (k - len(em)) + em
            else:
                prefix, hf = DI[alg] if alg in DI else (bytes.fromhex("3051300d060960864801650304020305000440"),
                                                         hashlib.sha512)
                t = prefix + hf(si).digest()
                em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
            s = pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")
            assert pow(int.from_bytes(s, "big"), e, n) == int.from_bytes(em, "big")
            out["tokens"].append({"name": f"valid-{alg}-{kid}", "key": kid, "token": si.decode() + "." + b64(s), "want": 1})
            bad = bytearray(s)
            bad[k // 2] ^= 0x10
            out["tokens"].append({"name": f"tamper-sig-{alg}-{kid}", "key": kid, "token": si.decode() + "." + b64(bytes(bad)),
                                  "want": 0})
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "rsa_big.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
