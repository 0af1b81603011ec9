#!/usr/bin/env python3
"""Generate the committed golden fixtures for the JWS verify path.

Test infrastructure only (run here, never on the GPU box).  Keys are made and
tokens are signed by the OpenSSL 3 CLI (an implementation independent of both
the oracle and the HIP path); every token's verdict is then re-checked by
`openssl` where OpenSSL can express the check.  Edge cases whose verdict in
the reference differs from OpenSSL's (Go semantics) are
crafted here with the private keys and labelled by rule number.

Token shape follows the reference's own test tokens:
  header  = go-jose signer header, keys sorted: {"alg":..,"kid":..,"typ":"JWT"}
            (oidc/testing.go:38-58 uses "key_id"; both forms are emitted)
  payload = testJWTClaims (jwt/keyset_test.go:666-677), keys sorted like
            encoding/json marshals a map.

Usage: python tests/golden/make_fixtures.py   (rewrites tests/golden/*.json)
"""
import base64
import hashlib
import json
import os
import random
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
KEYDIR = os.path.join(HERE, "keys")

def b64u(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()

def run(args, inp=None):
    r = subprocess.run(args, input=inp, capture_output=True)
    return r.returncode, r.stdout, r.stderr

def must(args, inp=None):
    rc, out, err = run(args, inp)
    if rc != 0:
        raise RuntimeError(f"{args}: {err.decode()}")
    return out

def hexblock(text: str, label: str) -> int:
    m = re.search(label + r":\s*\n((?:\s+[0-9a-f:]+\n)+)", text)
    return int(m.group(1).replace(":", "").replace(" ", "").replace("\n", ""), 16)

# --------------------------------------------------------------------------
# curves (public constants, for crafting edge cases and checking keys)
CURVES = {
    "P-256": dict(
        name="prime256v1", size=32,
        p=0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff,
        n=0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551,
        b=0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b),
    "P-384": dict(
        name="secp384r1", size=48,
        p=int("fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffeffffffff0000000000000000ffffffff", 16),
        n=int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973", 16),
        b=int("b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef", 16)),
    "P-521": dict(
        name="secp521r1", size=66,
        p=(1 << 521) - 1,
        n=int("01fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409", 16),
        b=int("0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf073573df883d2c34f1ef451fd46b503f00", 16)),
}
ES_SIZE = {"ES256": 32, "ES384": 48, "ES512": 66}
HASH = {"256": hashlib.sha256, "384": hashlib.sha384, "512": hashlib.sha512}

# --------------------------------------------------------------------------
# Ed25519 (RFC 8032) in plain Python, only for crafting edge cases
ED_P = 2**255 - 19
ED_L = 2**252 + 27742317777372353535851937790883648493
ED_D = (-121665 * pow(121666, ED_P - 2, ED_P)) % ED_P
ED_I = pow(2, (ED_P - 1) // 4, ED_P)

def ed_recover_x(y, sign):
    xx = (y * y - 1) * pow(ED_D * y * y + 1, ED_P - 2, ED_P) % ED_P
    x = pow(xx, (ED_P + 3) // 8, ED_P)
    if (x * x - xx) % ED_P != 0:
        x = x * ED_I % ED_P
    if (x * x - xx) % ED_P != 0:
        return None
    if x & 1 != sign:
        x = ED_P - x
    return x

ED_BY = 4 * pow(5, ED_P - 2, ED_P) % ED_P
ED_B = (ed_recover_x(ED_BY, 0), ED_BY, 1, ed_recover_x(ED_BY, 0) * ED_BY % ED_P)

def ed_add(P, Q):
    (X1, Y1, Z1, T1), (X2, Y2, Z2, T2) = P, Q
    A = (Y1 - X1) * (Y2 - X2) % ED_P
    B = (Y1 + X1) * (Y2 + X2) % ED_P
    C = T1 * 2 * ED_D * T2 % ED_P
    D = Z1 * 2 * Z2 % ED_P
    E, F, G, H = B - A, D - C, D + C, B + A
    return (E * F % ED_P, G * H % ED_P, F * G % ED_P, E * H % ED_P)

def ed_mul(s, P):
    Q = (0, 1, 1, 0)
    while s > 0:
        if s & 1:
            Q = ed_add(Q, P)
        P = ed_add(P, P)
        s >>= 1
    return Q

def ed_encode(P):
    X, Y, Z, _ = P
    zi = pow(Z, ED_P - 2, ED_P)
    x, y = X * zi % ED_P, Y * zi % ED_P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")

def ed_secret_scalar(seed: bytes):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]

# --------------------------------------------------------------------------
class Keys:
    def __init__(self):
        self.keys = {}   # kid -> dict
        os.makedirs(KEYDIR, exist_ok=True)

    def _pem(self, kid):
        return os.path.join(KEYDIR, kid + ".pem")

    def rsa(self, kid, bits, e=65537):
        path = self._pem(kid)
        if not os.path.exists(path):
            must(["openssl", "genpkey", "-algorithm", "RSA", "-pkeyopt", f"rsa_keygen_bits:{bits}",
                  "-pkeyopt", f"rsa_keygen_pubexp:{e}", "-out", path])
        text = must(["openssl", "pkey", "-in", path, "-text", "-noout"]).decode()
        n = hexblock(text, "modulus")
        d = hexblock(text, "privateExponent")
        e_ = int(re.search(r"publicExponent: (\d+)", text).group(1))
        pub = must(["openssl", "pkey", "-in", path, "-pubout"]).decode()
        self.keys[kid] = dict(kid=kid, kty="RSA", bits=n.bit_length(), n=format(n, "x"), e=e_, pem=pub,
                              _d=d, _path=path)
        return self.keys[kid]

    def ec(self, kid, crv):
        path = self._pem(kid)
        if not os.path.exists(path):
            must(["openssl", "ecparam", "-name", CURVES[crv]["name"], "-genkey", "-noout", "-out", path])
        text = must(["openssl", "pkey", "-in", path, "-text", "-noout"]).decode()
        d = hexblock(text, "priv")
        pt = hexblock(text, "pub")
        sz = CURVES[crv]["size"]
        raw = pt.to_bytes(1 + 2 * sz, "big")
        assert raw[0] == 4
        x, y = int.from_bytes(raw[1:1 + sz], "big"), int.from_bytes(raw[1 + sz:], "big")
        pub = must(["openssl", "pkey", "-in", path, "-pubout"]).decode()
        self.keys[kid] = dict(kid=kid, kty="EC", crv=crv, x=format(x, "x"), y=format(y, "x"), pem=pub,
                              _d=d, _path=path)
        return self.keys[kid]

    def ed(self, kid):
        path = self._pem(kid)
        if not os.path.exists(path):
            must(["openssl", "genpkey", "-algorithm", "ed25519", "-out", path])
        text = must(["openssl", "pkey", "-in", path, "-text", "-noout"]).decode()
        seed = hexblock(text, "priv").to_bytes(32, "big")
        pubb = hexblock(text, "pub").to_bytes(32, "big")
        a, _ = ed_secret_scalar(seed)
        assert ed_encode(ed_mul(a, ED_B)) == pubb
        pub = must(["openssl", "pkey", "-in", path, "-pubout"]).decode()
        self.keys[kid] = dict(kid=kid, kty="OKP", crv="Ed25519", x=pubb.hex(), pem=pub,
                              _seed=seed, _path=path)
        return self.keys[kid]

    def raw_ed(self, kid, pubbytes: bytes):
        """A public-key-only Ed25519 entry (crafted keys, e.g. small-order points)."""
        self.keys[kid] = dict(kid=kid, kty="OKP", crv="Ed25519", x=pubbytes.hex(), pem=None)
        return self.keys[kid]

    def public(self):
        out = []
        for k in self.keys.values():
            out.append({a: b for a, b in k.items() if not a.startswith("_")})
        return out

# --------------------------------------------------------------------------
def claims(jti, t0=1611699344):
    # jwt/keyset_test.go:666-677 shape, keys in encoding/json (sorted) order
    return {"aud": ["www.example.com"], "exp": t0 + 600, "iat": t0, "iss": "https://example.com/",
            "jti": jti, "nbf": t0, "sub": "alice@example.com"}

def enc_json(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":"), sort_keys=True).encode()

def signing_input(alg, kid, payload_obj, kid_field="kid", extra=None):
    hdr = {"alg": alg, "typ": "JWT"}
    if kid is not None:
        hdr[kid_field] = kid
    if extra:
        hdr.update(extra)
    h = enc_json(hdr)
    p = payload_obj if isinstance(payload_obj, bytes) else enc_json(payload_obj)
    return (b64u(h) + "." + b64u(p)).encode()

def ossl_sign(key, alg, msg: bytes, pss_salt="digest"):
    with tempfile.NamedTemporaryFile(delete=False) as f:
        f.write(msg)
        mpath = f.name
    try:
        if alg == "EdDSA":
            return must(["openssl", "pkeyutl", "-sign", "-inkey", key["_path"], "-rawin", "-in", mpath])
        h = "-sha" + alg[2:]
        args = ["openssl", "dgst", h, "-sign", key["_path"]]
        if alg.startswith("PS"):
            args += ["-sigopt", "rsa_padding_mode:pss", "-sigopt", f"rsa_pss_saltlen:{pss_salt}"]
        der = must(args + [mpath])
        if alg.startswith("ES"):
            r, s = der_to_rs(der)
            sz = ES_SIZE[alg]
            return r.to_bytes(sz, "big") + s.to_bytes(sz, "big")
        return der
    finally:
        os.unlink(mpath)

def der_to_rs(der):
    assert der[0] == 0x30
    i = 2 if der[1] < 0x80 else 2 + (der[1] & 0x7f)
    out = []
    for _ in range(2):
        assert der[i] == 2
        ln = der[i + 1]
        out.append(int.from_bytes(der[i + 2:i + 2 + ln], "big"))
        i += 2 + ln
    return out

def der_int(v):
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    return bytes([2, len(b)]) + b

def rs_to_der(r, s):
    body = der_int(r) + der_int(s)
    if len(body) < 128:
        return bytes([0x30, len(body)]) + body
    return bytes([0x30, 0x81, len(body)]) + body

def ossl_verify(key, alg, msg: bytes, sig: bytes, pss_salt="auto"):
    """Independent OpenSSL verdict (1/0) for a standard (non-mismatched) case."""
    with tempfile.TemporaryDirectory() as d:
        mp, sp, kp = os.path.join(d, "m"), os.path.join(d, "s"), os.path.join(d, "k.pem")
        open(mp, "wb").write(msg)
        open(kp, "w").write(key["pem"])
        if alg == "EdDSA":
            open(sp, "wb").write(sig)
            rc, _, _ = run(["openssl", "pkeyutl", "-verify", "-pubin", "-inkey", kp, "-rawin",
                            "-in", mp, "-sigfile", sp])
            return 1 if rc == 0 else 0
        if alg.startswith("ES"):
            sz = ES_SIZE[alg]
            if len(sig) != 2 * sz:
                return 0
            r, s = int.from_bytes(sig[:sz], "big"), int.from_bytes(sig[sz:], "big")
            if r == 0 or s == 0:
                return 0
            sig = rs_to_der(r, s)
        open(sp, "wb").write(sig)
        args = ["openssl", "dgst", "-sha" + alg[2:], "-verify", kp, "-signature", sp]
        if alg.startswith("PS"):
            args += ["-sigopt", "rsa_padding_mode:pss", "-sigopt", f"rsa_pss_saltlen:{pss_salt}"]
        rc, out, _ = run(args + [mp])
        return 1 if (rc == 0 and b"Verified OK" in out) else 0

# --------------------------------------------------------------------------
DIGESTINFO = {
    "256": bytes.fromhex("3031300d060960864801650304020105000420"),
    "384": bytes.fromhex("3041300d060960864801650304020205000430"),
    "512": bytes.fromhex("3051300d060960864801650304020305000440"),
}

def rsa_raw_sign(key, em: bytes) -> bytes:
    n, d = int(key["n"], 16), key["_d"]
    k = (n.bit_length() + 7) // 8
    m = int.from_bytes(em, "big")
    assert m < n
    return pow(m, d, n).to_bytes(k, "big")

def pkcs1_em(key, hbits, msg):
    n = int(key["n"], 16)
    k = (n.bit_length() + 7) // 8
    t = DIGESTINFO[hbits] + HASH[hbits](msg).digest()
    return b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t

def mgf1(seed, ln, h):
    out = b""
    c = 0
    while len(out) < ln:
        out += h(seed + c.to_bytes(4, "big")).digest()
        c += 1
    return out[:ln]

def pss_em(key, hbits, msg, salt: bytes, force_top=False):
    h = HASH[hbits]
    n = int(key["n"], 16)
    embits = n.bit_length() - 1
    emlen = (embits + 7) // 8
    mhash = h(msg).digest()
    hh = h(b"\x00" * 8 + mhash + salt).digest()
    db = b"\x00" * (emlen - len(salt) - len(hh) - 2) + b"\x01" + salt
    masked = bytearray(x ^ y for x, y in zip(db, mgf1(hh, len(db), h)))
    if not force_top:
        masked[0] &= 0xff >> (8 * emlen - embits)
    else:
        masked[0] |= 0x80
    em = bytes(masked) + hh + b"\xbc"
    k = (n.bit_length() + 7) // 8
    return b"\x00" * (k - emlen) + em

def ec_mod_inv(a, n):
    return pow(a, -1, n)

def main():
    random.seed(0x5EED)
    K = Keys()
    K.rsa("rsa2048-a", 2048); K.rsa("rsa2048-b", 2048)
    K.rsa("rsa3072-a", 3072); K.rsa("rsa4096-a", 4096)
    K.rsa("rsa2048-e3", 2048, e=3)
    K.rsa("rsa2047-a", 2047)       # odd size: top two EM bits must be clear (R16)
    K.rsa("rsa2049-a", 2049)       # emLen < k: PSS strips a leading zero byte (R16)
    K.ec("p256-a", "P-256"); K.ec("p256-b", "P-256")
    K.ec("p256-c", "P-256"); K.ec("p256-d", "P-256")     # 4-kid JWKS workload (bench)
    K.ec("p384-a", "P-384"); K.ec("p521-a", "P-521")
    K.ed("ed-a"); K.ed("ed-b")

    toks = []
    def add(name, alg, key, sinp: bytes, sig: bytes, verdict, source, **kw):
        tok = sinp.decode() + "." + b64u(sig)
        toks.append(dict(name=name, alg=alg, key=key["kid"], token=tok, verdict=verdict, source=source, **kw))

    def std(name, alg, key, jti, kid_field="kid", with_kid=True, pss_salt="digest"):
        sinp = signing_input(alg, key["kid"] if with_kid else None, claims(jti), kid_field)
        sig = ossl_sign(key, alg, sinp, pss_salt)
        v = ossl_verify(key, alg, sinp, sig)
        assert v == 1, (name, alg)
        add(name, alg, key, sinp, sig, 1, "openssl")
        return sinp, sig

    # ---- valid tokens: every alg x key size, with / without kid, "key_id" form
    plan = [("RS256", "rsa2048-a"), ("RS384", "rsa3072-a"), ("RS512", "rsa4096-a"),
            ("PS256", "rsa2048-a"), ("PS384", "rsa3072-a"), ("PS512", "rsa4096-a"),
            ("RS256", "rsa4096-a"), ("PS512", "rsa2048-b"), ("RS512", "rsa2048-b"),
            ("ES256", "p256-a"), ("ES384", "p384-a"), ("ES512", "p521-a"),
            ("EdDSA", "ed-a"), ("EdDSA", "ed-b"), ("ES256", "p256-b"),
            ("RS256", "rsa2048-e3"), ("PS256", "rsa2047-a"), ("RS256", "rsa2047-a"),
            ("PS384", "rsa2049-a"), ("RS256", "rsa2049-a")]
    base = {}
    for alg, kid in plan:
        for i in range(4):
            nm = f"valid-{alg}-{kid}-{i}"
            sinp, sig = std(nm, alg, K.keys[kid], f"jti-{alg}-{kid}-{i}",
                            kid_field="key_id" if i == 2 else "kid", with_kid=(i != 3))
            base.setdefault((alg, kid), (sinp, sig))

    # ---- generic tamper cases (signature bit flip, payload flip, header flip, wrong key)
    for (alg, kid), (sinp, sig) in sorted(base.items()):
        key = K.keys[kid]
        s2 = bytearray(sig); s2[len(s2) // 2] ^= 0x01
        add(f"tamper-sig-{alg}-{kid}", alg, key, sinp, bytes(s2), ossl_verify(key, alg, sinp, bytes(s2)), "openssl")
        h, p = sinp.split(b".")
        pj = json.loads(base64.urlsafe_b64decode(p + b"=" * (-len(p) % 4)))
        pj["sub"] = "mallory@example.com"
        sinp2 = h + b"." + b64u(enc_json(pj)).encode()
        add(f"tamper-payload-{alg}-{kid}", alg, key, sinp2, sig, ossl_verify(key, alg, sinp2, sig), "openssl")
        other = {"RSA": "rsa2048-b" if kid != "rsa2048-b" else "rsa2048-a",
                 "EC": "p256-b" if kid != "p256-b" else "p256-a", "OKP": "ed-b" if kid != "ed-b" else "ed-a"}
        ok = K.keys[other[key["kty"]]]
        wrong_v = ossl_verify(ok, alg, sinp, sig) if (key["kty"] != "EC" or ok["crv"] == key["crv"]) else 0
        toks.append(dict(name=f"wrong-key-{alg}-{kid}", alg=alg, key=ok["kid"],
                         token=sinp.decode() + "." + b64u(sig), verdict=wrong_v,
                         source="openssl" if wrong_v == 0 and (key["kty"] != "EC" or ok["crv"] == key["crv"]) else "R19"))

    # header swapped to HS256 (jwt/keyset_test.go:186,458): the verifier rejects (R10/R11)
    sinp, sig = base[("RS256", "rsa2048-a")]
    hs = b"eyJhbGciOiJIUzI1NiIsInR5cCI6IkpXVCJ9." + sinp.split(b".")[1]
    add("hs256-header-swap", "HS256", K.keys["rsa2048-a"], hs, sig, 0, "R10")
    # payload swapped (jwt/keyset_test.go:475)
    sw = sinp.split(b".")[0] + b".eyJzdWIiOiIxMjM0NTY3ODkwIiwibmFtZSI6IkpvaG4gRG9lIiwiaWF0IjoxNTE2MjM5MDIyfQ"
    add("payload-swap-RS256", "RS256", K.keys["rsa2048-a"], sw, sig, 0, "openssl")

    # ---- RSA edge cases (Go crypto/rsa semantics, R12-R17)
    ka = K.keys["rsa2048-a"]
    n = int(ka["n"], 16)
    sinp, sig = base[("RS256", "rsa2048-a")]
    sv = int.from_bytes(sig, "big")
    if sv + n < (1 << 2048):
        add("rsa-sig-plus-n", "RS256", ka, sinp, (sv + n).to_bytes(256, "big"), 0, "R14")
    add("rsa-sig-equals-n", "RS256", ka, sinp, n.to_bytes(256, "big"), 0, "R14")
    add("rsa-sig-zero", "RS256", ka, sinp, bytes(256), 0, "R15")
    add("rsa-sig-one", "RS256", ka, sinp, (1).to_bytes(256, "big"), 0, "R15")
    add("rsa-sig-short-truncated", "RS256", ka, sinp, sig[1:], 0, "R13")
    add("rsa-sig-long", "RS256", ka, sinp, b"\x00" + sig, 0, "R13")
    # a valid signature that starts with a 0x00 byte: accepted at full length, rejected stripped
    for j in range(4000):
        s2 = signing_input("RS256", ka["kid"], claims(f"lead0-{j}"))
        sg = rsa_raw_sign(ka, pkcs1_em(ka, "256", s2))
        if sg[0] == 0:
            add("rsa-leading-zero-sig", "RS256", ka, s2, sg, 1, "R13")
            add("rsa-leading-zero-sig-stripped", "RS256", ka, s2, sg[1:], 0, "R13")
            break
    # bad EM encodings
    s2 = signing_input("RS256", ka["kid"], claims("badem"))
    em = bytearray(pkcs1_em(ka, "256", s2)); em[5] = 0xfe
    add("rsa-em-bad-ff-run", "RS256", ka, s2, rsa_raw_sign(ka, bytes(em)), 0, "R15")
    em = bytearray(pkcs1_em(ka, "256", s2)); em[1] = 0x02
    add("rsa-em-bad-bt", "RS256", ka, s2, rsa_raw_sign(ka, bytes(em)), 0, "R15")
    em = bytearray(pkcs1_em(ka, "256", s2)); em[-33] ^= 0x01   # DigestInfo byte
    add("rsa-em-bad-digestinfo", "RS256", ka, s2, rsa_raw_sign(ka, bytes(em)), 0, "R15")
    em = pkcs1_em(ka, "384", s2)                                  # RS384 EM under RS256 header
    add("rsa-em-wrong-hash", "RS256", ka, s2, rsa_raw_sign(ka, em), 0, "R15")
    em = pkcs1_em(ka, "256", s2)
    add("rsa-em-good-raw", "RS256", ka, s2, rsa_raw_sign(ka, em), 1, "R15")
    # PSS salt lengths (auto-detect, R16)
    for salt in (0, 20, 32, 64, 256 - 32 - 2):
        s2 = signing_input("PS256", ka["kid"], claims(f"pss-salt-{salt}"))
        em = pss_em(ka, "256", s2, os.urandom(salt))
        add(f"pss-salt-{salt}", "PS256", ka, s2, rsa_raw_sign(ka, em), 1, "R16")
    s2 = signing_input("PS256", ka["kid"], claims("pss-salt-openssl-max"))
    sg = ossl_sign(ka, "PS256", s2, pss_salt="max")
    add("pss-salt-openssl-max", "PS256", ka, s2, sg, ossl_verify(ka, "PS256", s2, sg), "openssl")
    s2 = signing_input("PS256", ka["kid"], claims("pss-top-bit"))
    em = pss_em(ka, "256", s2, os.urandom(32), force_top=True)
    if int.from_bytes(em, "big") < n:
        add("pss-top-bit-set", "PS256", ka, s2, rsa_raw_sign(ka, em), 0, "R16")
    em = bytearray(pss_em(ka, "256", s2, os.urandom(32))); em[-1] = 0xbd
    add("pss-bad-trailer", "PS256", ka, s2, rsa_raw_sign(ka, bytes(em)), 0, "R16")
    em = bytearray(pss_em(ka, "256", s2, os.urandom(32))); em[-5] ^= 0x40   # H corrupted
    add("pss-bad-h", "PS256", ka, s2, rsa_raw_sign(ka, bytes(em)), 0, "R16")
    # DB with a non-zero byte before the 0x01 separator: craft DB directly
    h = hashlib.sha256
    mhash = h(s2).digest(); salt = os.urandom(16)
    hh = h(b"\x00" * 8 + mhash + salt).digest()
    db = bytearray(b"\x00" * (255 - 16 - 32 - 2) + b"\x01" + salt); db[3] = 0x02
    masked = bytes(x ^ y for x, y in zip(db, mgf1(hh, len(db), h)))
    masked = bytes([masked[0] & 0x7f]) + masked[1:]
    add("pss-db-bad-ps", "PS256", ka, s2, rsa_raw_sign(ka, masked + hh + b"\xbc"), 0, "R16")
    # PSS accepted under the other PSS hash? (mismatched alg => reject)
    sinp, sig = base[("PS256", "rsa2048-a")]
    sinp384 = sinp.replace(sinp.split(b".")[0], b64u(enc_json({"alg": "PS384", "kid": "rsa2048-a", "typ": "JWT"})).encode())
    add("pss-alg-swap", "PS384", ka, sinp384, sig, 0, "R9")
    # PKCS1 signature under a PS256 header and vice versa
    sinp, sig = base[("RS256", "rsa2048-a")]
    sinpps = sinp.replace(sinp.split(b".")[0], b64u(enc_json({"alg": "PS256", "kid": "rsa2048-a", "typ": "JWT"})).encode())
    add("rs-sig-under-ps-header", "PS256", ka, sinpps, sig, 0, "R16")
    # e=3 key with tamper
    sinp, sig = base[("RS256", "rsa2048-e3")]
    s2b = bytearray(sig); s2b[-1] ^= 1
    add("rsa-e3-tamper", "RS256", K.keys["rsa2048-e3"], sinp, bytes(s2b), 0, "openssl")

    # ---- ECDSA edge cases (R18-R22)
    for alg, kid in (("ES256", "p256-a"), ("ES384", "p384-a"), ("ES512", "p521-a")):
        key = K.keys[kid]
        cv = CURVES[key["crv"]]
        sz = ES_SIZE[alg]
        sinp, sig = base[(alg, kid)]
        r, s = int.from_bytes(sig[:sz], "big"), int.from_bytes(sig[sz:], "big")
        enc = lambda a, b: a.to_bytes(sz, "big") + b.to_bytes(sz, "big")
        add(f"ec-r-zero-{alg}", alg, key, sinp, enc(0, s), 0, "R20")
        add(f"ec-s-zero-{alg}", alg, key, sinp, enc(r, 0), 0, "R20")
        add(f"ec-r-eq-n-{alg}", alg, key, sinp, enc(cv["n"], s), 0, "R20")
        add(f"ec-s-eq-n-{alg}", alg, key, sinp, enc(r, cv["n"]), 0, "R20")
        add(f"ec-r-plus-n-{alg}", alg, key, sinp, enc(r + cv["n"], s) if r + cv["n"] < (1 << (8 * sz)) else enc(cv["n"] + 1, s), 0, "R20")
        add(f"ec-high-s-{alg}", alg, key, sinp, enc(r, cv["n"] - s), 1, "R22")
        add(f"ec-short-sig-{alg}", alg, key, sinp, sig[:-1], 0, "R18")
        add(f"ec-long-sig-{alg}", alg, key, sinp, sig + b"\x00", 0, "R18")
        add(f"ec-swapped-rs-{alg}", alg, key, sinp, enc(s, r), 0, "openssl")
    # alg/curve mismatches: hash and sig size from the alg, curve from the key (R19/R21)
    for alg, kid in (("ES384", "p256-a"), ("ES512", "p256-a"), ("ES512", "p384-a"), ("ES256", "p521-a"),
                     ("ES384", "p521-a")):
        key = K.keys[kid]
        sinp = signing_input(alg, kid, claims(f"mismatch-{alg}-{kid}"))
        cv = CURVES[key["crv"]]
        # openssl signs the (truncated) digest with the key's curve
        with tempfile.NamedTemporaryFile(delete=False) as f:
            f.write(sinp); mp = f.name
        der = must(["openssl", "dgst", "-sha" + alg[2:], "-sign", key["_path"], mp]); os.unlink(mp)
        r, s = der_to_rs(der)
        sz = ES_SIZE[alg]
        if r < (1 << (8 * sz)) and s < (1 << (8 * sz)):
            sig = r.to_bytes(sz, "big") + s.to_bytes(sz, "big")
            add(f"ec-mismatch-{alg}-{kid}", alg, key, sinp, sig, 1, "R19")
            s2b = bytearray(sig); s2b[-1] ^= 1
            add(f"ec-mismatch-tamper-{alg}-{kid}", alg, key, sinp, bytes(s2b), 0, "R19")
        else:
            # r or s does not fit the alg's field: no valid token exists; a real-size sig is rejected
            sig = (r % (1 << (8 * sz))).to_bytes(sz, "big") + (s % (1 << (8 * sz))).to_bytes(sz, "big")
            add(f"ec-mismatch-{alg}-{kid}", alg, key, sinp, sig, 0, "R19")
    # ES256 signature checked with an RSA / Ed key: wrong key type (R10)
    sinp, sig = base[("ES256", "p256-a")]
    toks.append(dict(name="ec-token-rsa-key", alg="ES256", key="rsa2048-a", token=sinp.decode() + "." + b64u(sig),
                     verdict=0, source="R10"))
    toks.append(dict(name="ec-token-ed-key", alg="ES256", key="ed-a", token=sinp.decode() + "." + b64u(sig),
                     verdict=0, source="R10"))
    sinp, sig = base[("RS256", "rsa2048-a")]
    toks.append(dict(name="rsa-token-ec-key", alg="RS256", key="p256-a", token=sinp.decode() + "." + b64u(sig),
                     verdict=0, source="R10"))

    # ---- Ed25519 edge cases (R23-R26)
    ke = K.keys["ed-a"]
    a, prefix = ed_secret_scalar(ke["_seed"])
    A = bytes.fromhex(ke["x"])
    def ed_sign_with(Rb: bytes, r: int, msg: bytes, Ab: bytes, a_: int):
        k = int.from_bytes(hashlib.sha512(Rb + Ab + msg).digest(), "little") % ED_L
        return (r + k * a_) % ED_L
    sinp, sig = base[("EdDSA", "ed-a")]
    s = int.from_bytes(sig[32:], "little")
    add("ed-s-plus-L", "EdDSA", ke, sinp, sig[:32] + (s + ED_L).to_bytes(32, "little"), 0, "R25")
    add("ed-s-eq-L", "EdDSA", ke, sinp, sig[:32] + ED_L.to_bytes(32, "little"), 0, "R25")
    hb = bytearray(sig); hb[63] |= 0x20
    add("ed-sig63-high-bits", "EdDSA", ke, sinp, bytes(hb), 0, "R25")
    add("ed-short-sig", "EdDSA", ke, sinp, sig[:63], 0, "R23")
    # R = identity via r = 0: canonical encoding verifies, non-canonical (y = p + 1) does not
    ident = (1).to_bytes(32, "little")
    sinp = signing_input("EdDSA", "ed-a", claims("ed-r-identity"))
    S = ed_sign_with(ident, 0, sinp, A, a)
    add("ed-R-identity-canonical", "EdDSA", ke, sinp, ident + S.to_bytes(32, "little"), 1, "R26")
    nc = (ED_P + 1).to_bytes(32, "little")
    S = ed_sign_with(nc, 0, sinp, A, a)
    add("ed-R-identity-noncanonical", "EdDSA", ke, sinp, nc + S.to_bytes(32, "little"), 0, "R26")
    # R with x = 0 but sign bit set (encodes the identity only non-canonically)
    nz = bytearray(ident); nz[31] |= 0x80
    S = ed_sign_with(bytes(nz), 0, sinp, A, a)
    add("ed-R-negzero", "EdDSA", ke, sinp, bytes(nz) + S.to_bytes(32, "little"), 0, "R26")
    # small-order / non-canonical public keys (accepted by Go: cofactorless, SetBytes allows y >= p)
    ident_nc = K.raw_ed("ed-A-identity-noncanon", (ED_P + 1).to_bytes(32, "little"))
    ident_c = K.raw_ed("ed-A-identity", ident)
    for kk in (ident_nc, ident_c):
        sinp = signing_input("EdDSA", kk["kid"], claims("small-order-" + kk["kid"]))
        r = random.randrange(1, ED_L)
        Rb = ed_encode(ed_mul(r, ED_B))
        add(f"ed-small-order-A-{kk['kid']}", "EdDSA", kk, sinp, Rb + r.to_bytes(32, "little"), 1, "R24/R26")
    # order-4 point (x = sqrt(-1), y = 0); encoded with y = p (non-canonical, sign 0) and y = 0
    for enc_y, nm in ((ED_P, "ed-A-order4-noncanon"), (0, "ed-A-order4")):
        kk = K.raw_ed(nm, enc_y.to_bytes(32, "little"))
        Ab = bytes.fromhex(kk["x"])
        x0 = ed_recover_x(0, 0)
        P4 = (x0, 0, 1, 0)
        got = {0: 0, 1: 0}
        for j in range(64):
            sinp = signing_input("EdDSA", nm, claims(f"{nm}-{j}"))
            r = random.randrange(1, ED_L)
            Rb = ed_encode(ed_mul(r, ED_B))
            k = int.from_bytes(hashlib.sha512(Rb + Ab + sinp).digest(), "little") % ED_L
            # [r]B - [k]A == [r]B  iff  [k]A == identity iff k % 4 == 0 (cofactorless check)
            v = 1 if ed_encode(ed_add(ed_mul(r, ED_B), ed_mul((-k) % 4, P4))) == Rb else 0
            assert v == (1 if k % 4 == 0 else 0)
            if got[v] < 2:
                add(f"{nm}-k{k % 4}-{j}", "EdDSA", kk, sinp, Rb + r.to_bytes(32, "little"), v, "R26")
                got[v] += 1
            if got[0] >= 2 and got[1] >= 2:
                break
    # an invalid public key encoding (not on the curve) rejects every token (R24)
    for y in range(2, 200):
        if ed_recover_x(y, 0) is None:
            bad = K.raw_ed("ed-A-invalid", y.to_bytes(32, "little"))
            break
    sinp, sig = base[("EdDSA", "ed-a")]
    add("ed-invalid-A", "EdDSA", bad, sinp, sig, 0, "R24")

    # ---- parse-level cases (R1-R8), verdicts per go-jose semantics
    sinp, sig = base[("ES256", "p256-a")]
    kp = K.keys["p256-a"]
    tok = sinp.decode() + "." + b64u(sig)
    h, p, sgs = tok.split(".")
    def addraw(name, token, verdict, src, alg="ES256", key=kp):
        toks.append(dict(name=name, alg=alg, key=key["kid"], token=token, verdict=verdict, source=src))
    addraw("parse-two-parts", h + "." + p, 0, "R2")
    addraw("parse-four-parts", tok + ".x", 0, "R2")
    addraw("parse-one-part", "eyJhbGciOiJFUzI1NiJ9", 0, "R2")
    addraw("parse-empty-sig", h + "." + p + ".", 0, "R5")
    addraw("parse-whitespace-inside", h[:5] + " \n\t" + h[5:] + "." + p + ".\r\n" + sgs, 1, "R1")
    addraw("parse-pad-equals", h + "." + p + "." + sgs + "==", 1, "R3")
    addraw("parse-bad-b64-char", h + "." + p + "." + sgs[:-2] + "*" + sgs[-1], 0, "R3")
    addraw("parse-std-b64-alphabet", h + "." + p + "." + sgs.replace("-", "+").replace("_", "/"),
           1 if ("-" not in sgs and "_" not in sgs) else 0, "R3")
    # non-zero trailing bits in the payload segment: go-jose hashes the canonical re-encoding (R6)
    # -> the literal bytes differ from the signed bytes only if the last char carries spare bits
    if len(p) % 4 in (2, 3):
        alphabet = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
        last = alphabet.index(p[-1])
        spare = 0x0f if len(p) % 4 == 2 else 0x03
        if (last & spare) == 0:
            p_nc = p[:-1] + alphabet[last | 1]
            addraw("parse-noncanonical-trailing-bits", h + "." + p_nc + "." + sgs, 1, "R6")
    # header not JSON / alg missing / alg not a string / crit / b64
    def hdr_tok(hdr_bytes, name, verdict, src, payload_raw=None, key=kp, alg="ES256"):
        hb = b64u(hdr_bytes)
        if payload_raw is None:
            sinp2 = (hb + "." + p).encode()
        else:
            sinp2 = (hb + ".").encode() + payload_raw
        sg = ossl_sign(key, alg, sinp2)
        tokp = p if payload_raw is None else b64u(payload_raw)
        addraw(name, hb + "." + tokp + "." + b64u(sg), verdict, src, alg=alg, key=key)
    hdr_tok(b'{"alg":"ES256","crit":["exp"],"exp":5}', "parse-crit-unknown", 0, "R7")
    hdr_tok(b'not json', "parse-header-not-json", 0, "R4")
    hdr_tok(b'{"typ":"JWT"}', "parse-alg-missing", 0, "R8")
    hdr_tok(b'{"alg":256}', "parse-alg-not-string", 0, "R4")
    hdr_tok(b'{"alg":"ES256","kid":7}', "parse-kid-not-string", 0, "R4")
    hdr_tok(b'{"alg":"ES256","alg":"RS256"}', "parse-dup-alg-last-wins", 0, "R4")
    hdr_tok(b'{"alg":"RS256","alg":"ES256"}', "parse-dup-alg-last-wins-ok", 1, "R4")
    hdr_tok(b'{"alg":"ES256","x-extra":{"a":[1,2,{"b":null}]},"typ":"JWT"}', "parse-extra-header", 1, "R4")
    hdr_tok(b'{"alg":"ES256","b64":true,"crit":["b64"]}', "parse-b64-true-crit", 1, "R7")
    hdr_tok(b'{"alg":"none"}', "parse-alg-none", 0, "R11", alg="ES256")
    # b64:false -> signing input has the RAW payload; compact-form payload segment is then
    # base64 of the raw bytes for go-jose's parser, but hashed raw (R7)
    raw_payload = enc_json(claims("b64-false"))
    hb = b64u(b'{"alg":"ES256","b64":false,"crit":["b64"]}')
    sinp2 = (hb + ".").encode() + raw_payload
    sg = ossl_sign(kp, "ES256", sinp2)
    addraw("parse-b64-false", hb + "." + b64u(raw_payload) + "." + b64u(sg), 1, "R7")
    # payload edge cases (R33/R35): signature valid, payload null / not JSON / not an object
    for nm, praw, v in (("payload-null", b"null", 1), ("payload-not-json", b"not json", 0),
                        ("payload-array", b"[1,2]", 0), ("payload-empty", b"", 0),
                        ("payload-string", b'"x"', 0), ("payload-dup-keys", b'{"a":1,"a":2}', 1)):
        hb = b64u(enc_json({"alg": "ES256", "kid": "p256-a", "typ": "JWT"}))
        sinp2 = (hb + "." + b64u(praw)).encode()
        sg = ossl_sign(kp, "ES256", sinp2)
        toks.append(dict(name=nm, alg="ES256", key="p256-a", token=sinp2.decode() + "." + b64u(sg),
                         verdict=1, source="openssl", keyset_verdict=v))
    # JSON (flattened) serialization is accepted by go-jose's ParseSigned (R1)
    sinp, sig = base[("ES256", "p256-a")]
    h, p = sinp.decode().split(".")
    js = json.dumps({"protected": h, "payload": p, "signature": b64u(sig)})
    addraw("parse-json-serialization", js, 1, "R1")

    pub = K.public()
    with open(os.path.join(HERE, "keys.json"), "w") as f:
        json.dump(pub, f, indent=1)
    with open(os.path.join(HERE, "tokens.json"), "w") as f:
        json.dump(toks, f, indent=1)
    print(f"{len(pub)} keys, {len(toks)} tokens "
          f"({sum(t['verdict'] for t in toks)} accept / {sum(1 - t['verdict'] for t in toks)} reject)")

if __name__ == "__main__":
    main()
