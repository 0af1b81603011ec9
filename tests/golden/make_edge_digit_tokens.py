"""Make tests/golden/edge_digit_tokens.json: valid tokens whose signed comb
digits hit the last table entry (|digit| = 2^(W-1)) -- the one entry of each
window the common case never reads.  Tokens are signed by tools/tokgen
(OpenSSL) with bench kids; u1 = e/s, u2 = r/s mod n (ECDSA) or S and
k = SHA-512(R || A || M) mod L (Ed25519) are recoded exactly as
kernels/ecdsa_impl.hpp store_digit_rows (digits in [-2^(W-1), 2^(W-1))) and
kernels/ed25519.hip recode (digits in (-2^(W-1), 2^(W-1)]) do, and tokens with
an edge digit kept.  usage: python tests/golden/make_edge_digit_tokens.py"""
import base64
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

ORDER = {"ES384": int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973", 16),
         "ES512": int("01fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409", 16)}
HASH = {"ES384": (hashlib.sha384, 48, 384), "ES512": (hashlib.sha512, 66, 521)}
ED_L = 2 ** 252 + 27742317777372353535851937790883648493


def digits(u, w, nwin, ed):
    out, c = [], 0
    for i in range(nwin):
        v = ((u >> (w * i)) & ((1 << w) - 1)) + c
        c = 1 if (v > (1 << (w - 1)) if ed else v >= (1 << (w - 1))) else 0
        out.append(v - (c << w))
    return out


def edges(ds, w):
    return [i for i, x in enumerate(ds) if abs(x) == 1 << (w - 1)]


def scan_ec(alg, kid, n, wg, wq, meta, threads):
    toks = bench.gen_tokens(alg, n, [meta[kid][2]], threads, "edge")
    h, cb, bits = HASH[alg]
    nn = ORDER[alg]
    hits = []
    for i, t in enumerate(toks):
        d = t.rfind(b".")
        sig = base64.urlsafe_b64decode(t[d + 1:] + b"=" * (-len(t[d + 1:]) % 4))
        r, s = int.from_bytes(sig[:cb], "big"), int.from_bytes(sig[cb:], "big")
        hv = h(t[:d]).digest()
        e = int.from_bytes(hv, "big") >> max(0, len(hv) * 8 - bits)
        w = pow(s, -1, nn)
        e1 = edges(digits(e * w % nn, wg, -(-(bits + 1) // wg), False), wg)
        e2 = edges(digits(r * w % nn, wq, -(-(bits + 1) // wq), False), wq)
        if e1 or e2:
            hits.append((toks[i].decode(), e1, e2))
    return hits


def scan_ed(kid, n, wb, wa, meta, threads):
    x = meta[kid][4]["x"]
    a = base64.urlsafe_b64decode(x + "=" * (-len(x) % 4))
    toks = bench.gen_tokens("EdDSA", n, [meta[kid][2]], threads, "edge")
    hits = []
    for t in toks:
        d = t.rfind(b".")
        sig = base64.urlsafe_b64decode(t[d + 1:] + b"=" * (-len(t[d + 1:]) % 4))
        s = int.from_bytes(sig[32:], "little")
        k = int.from_bytes(hashlib.sha512(sig[:32] + a + t[:d]).digest(), "little") % ED_L
        e1 = edges(digits(s, wb, -(-254 // wb), True), wb)
        e2 = edges(digits(k, wa, -(-254 // wa), True), wa)
        if e1 or e2:
            hits.append((t.decode(), e1, e2))
    return hits


def scan_p521_top_carry(kid, n, meta, threads):
    """ES512 tokens whose u2, recoded at W = 18 over 29 windows (round 3's
    window count), carries out of the top window (tests/test_gpu_tables.py)."""
    toks = bench.gen_tokens("ES512", n, [meta[kid][2]], threads, "topcarry")
    nn = ORDER["ES512"]
    hits = []
    for t in toks:
        d = t.rfind(b".")
        sig = base64.urlsafe_b64decode(t[d + 1:] + b"=" * (-len(t[d + 1:]) % 4))
        r, s = int.from_bytes(sig[:66], "big"), int.from_bytes(sig[66:], "big")
        u2 = r * pow(s, -1, nn) % nn
        c = 0
        for w in range(29):
            v = ((u2 >> (18 * w)) & ((1 << 18) - 1)) + c
            c = 1 if v >= (1 << 17) else 0
        if c:
            hits.append(t.decode())
    return hits


def main():
    meta = {m[0]: m for m in bench.bench_keys()}
    threads = os.cpu_count() or 1
    sets = []
    for alg, kid, n, wg, wq in (("ES384", "kid-24", 200000, 20, 24), ("ES512", "kid-27", 100000, 20, 20)):
        h = scan_ec(alg, kid, n, wg, wq, meta, threads)
        sets.append({"alg": alg, "kid": kid, "wg": wg, "wq": wq, "tokens": [x[0] for x in h],
                     "hits": [[i, x[1], x[2]] for i, x in enumerate(h)]})
    h = scan_ed("kid-30", 1000000, 24, 24, meta, threads)
    sets.append({"alg": "EdDSA", "kid": "kid-30", "wg": 24, "wq": 24, "tokens": [x[0] for x in h],
                 "hits": [[i, x[1], x[2]] for i, x in enumerate(h)]})
    sets.append({"name": "p521_w18_top_carry", "alg": "ES512", "kid": "kid-27", "wg": 20, "wq": 18,
                 "tokens": scan_p521_top_carry("kid-27", 200000, meta, threads),
                 "hits": "u2's top W = 18 window all ones with a carry in (lost over 29 windows; 30 hold it)"})
    json.dump({"note": "valid tokens whose comb digits hit the last table entry; made by make_edge_digit_tokens.py",
               "sets": sets}, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "edge_digit_tokens.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
