#!/usr/bin/env python3
"""Generate the 32-kid key set of BASELINE configs[4] (mixed-alg JWKS: all 10
algs, RS/PS at 2048/3072/4096 bits as jwt/keyset_test.go:79-139, ES on
P-256/384/521, Ed25519) into tools/benchkeys/.  Bench input only; run once here
and committed (RSA-4096 key generation is slow and random).

Each kid is bound to one alg: kids.json lists {kid, alg, pem, jwk}."""
import base64
import json
import os
import re
import subprocess

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchkeys")
PLAN = ([("RS256", 2048)] * 4 + [("RS384", 3072)] * 3 + [("RS512", 4096)] * 3 + [("PS256", 2048)] * 4 +
        [("PS384", 3072)] * 3 + [("PS512", 4096)] * 3 + [("ES256", "prime256v1")] * 4 +
        [("ES384", "secp384r1")] * 3 + [("ES512", "secp521r1")] * 3 + [("EdDSA", None)] * 2)
assert len(PLAN) == 32


def must(args):
    return subprocess.run(args, check=True, capture_output=True).stdout


def b64u(b):
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def hexblock(text, label):
    m = re.search(label + r":\s*\n((?:\s+[0-9a-f:]+\n)+)", text)
    return bytes.fromhex(m.group(1).replace(":", "").replace(" ", "").replace("\n", ""))


def main():
    os.makedirs(HERE, exist_ok=True)
    out = []
    for i, (alg, p) in enumerate(PLAN):
        kid = f"kid-{i:02d}"
        path = os.path.join(HERE, kid + ".pem")
        if not os.path.exists(path):
            if alg[:2] in ("RS", "PS"):
                must(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt", f"rsa_keygen_bits:{p}", "-out", path])
            elif alg == "EdDSA":
                must(["openssl", "genpkey", "-algorithm", "ed25519", "-out", path])
            else:
                must(["openssl", "ecparam", "-name", p, "-genkey", "-noout", "-out", path])
        text = must(["openssl", "pkey", "-in", path, "-text", "-noout"]).decode()
        if alg[:2] in ("RS", "PS"):
            n = hexblock(text, "modulus").lstrip(b"\0")
            e = int(re.search(r"publicExponent: (\d+)", text).group(1))
            jwk = {"kty": "RSA", "kid": kid, "alg": alg, "n": b64u(n), "e": b64u(e.to_bytes(3, "big"))}
        elif alg == "EdDSA":
            jwk = {"kty": "OKP", "kid": kid, "alg": alg, "crv": "Ed25519", "x": b64u(hexblock(text, "pub"))}
        else:
            sz = {"ES256": 32, "ES384": 48, "ES512": 66}[alg]
            pt = hexblock(text, "pub")
            pt = pt[-(2 * sz + 1):]
            jwk = {"kty": "EC", "kid": kid, "alg": alg, "crv": {"ES256": "P-256", "ES384": "P-384", "ES512": "P-521"}[alg],
                   "x": b64u(pt[1:1 + sz]), "y": b64u(pt[1 + sz:])}
        out.append({"kid": kid, "alg": alg, "pem": kid + ".pem", "jwk": jwk})
    json.dump(out, open(os.path.join(HERE, "kids.json"), "w"), indent=1)
    print("wrote", len(out), "keys")


if __name__ == "__main__":
    main()
