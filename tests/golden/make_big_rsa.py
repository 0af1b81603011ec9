"""Generates tests/golden/rsa_big.json: RSA keys just above 4096 bits (4100 and
4142, the largest the 148-limb class holds) and RS256 / RS512 tokens signed
with them (PKCS#1 v1.5, RFC 8017 EMSA-PKCS1-v1_5), plus a signature-flipped
copy of each.  Go's crypto/rsa verifies keys of any size >= 1024 bits, so the
expected verdicts are accept / reject.  Test infrastructure: run once here,
the JSON is committed (sympy primes, Python big ints)."""
import base64
import hashlib
import json
import os
import random

import sympy

DI = {"RS256": (bytes.fromhex("3031300d060960864801650304020105000420"), hashlib.sha256),
      "RS512": (bytes.fromhex("3051300d060960864801650304020305000440"), hashlib.sha512)}


def b64(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def main():
    rng = random.Random(0x5EED)
    out = {"keys": [], "tokens": []}
    for bits in (4100, 4142):
        while True:
            p = sympy.randprime(1 << (bits // 2 - 1), 1 << (bits // 2))
            q = sympy.randprime(1 << (bits - bits // 2 - 1), 1 << (bits - bits // 2))
            n = p * q
            if n.bit_length() == bits and p != q:
                break
        e = 65537
        d = pow(e, -1, (p - 1) * (q - 1))
        kid = f"big-{bits}"
        out["keys"].append({"kid": kid, "kty": "RSA", "n": format(n, "x"), "e": e})
        k = (bits + 7) // 8
        for alg in ("RS256", "RS512"):
            prefix, hf = DI[alg]
            hdr = b64(json.dumps({"alg": alg, "kid": kid, "typ": "JWT"}, separators=(",", ":")).encode())
            pl = b64(json.dumps({"iss": "https://example.com/", "sub": "alice@example.com", "jti": str(rng.getrandbits(32))},
                                separators=(",", ":")).encode())
            si = (hdr + "." + pl).encode()
            t = prefix + hf(si).digest()
            em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
            s = pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")
            out["tokens"].append({"name": f"valid-{alg}-{kid}", "key": kid, "token": si.decode() + "." + b64(s), "want": 1})
            bad = bytearray(s)
            bad[k // 2] ^= 0x10
            out["tokens"].append({"name": f"tamper-sig-{alg}-{kid}", "key": kid, "token": si.decode() + "." + b64(bytes(bad)),
                                  "want": 0})
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "rsa_big.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
