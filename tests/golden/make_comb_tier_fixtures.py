#!/usr/bin/env python3
"""Comb-boundary fixtures for every key-table width tier the runtime can pick.

Test infrastructure only (run here; writes tests/golden/comb_tiers.json).

The point kernels sum one table entry per comb window (kernels/ecdsa_impl.hpp,
kernels/ed25519.hip).  Random tokens reach a window's last entry
(|digit| = 2^(W-1)) with probability ~2^-W, a carry into the top window about
as rarely, so a wrong table entry or a lost carry at one width tier can pass
a random-token suite: round 3's P-521 W = 18 lost carry did (2 false rejects in
1.19 M bench tokens, none in the parity tests).  This file builds the digit
patterns directly.

ECDSA (crypto/ecdsa.Verify behind /root/reference/jwt/keyset.go:163, R18-R22):
the scalars are u1 = e/s (generator table, width wg) and u2 = r/s (key table,
width wq).  For chosen u1, u2 and a message with hash e: s = e/u1, r = u2 s;
lift a point R0 with x(R0) = r; the key is Q = u2^-1 (R0 - u1 G).  Then
u1 G + u2 Q = R0 and Go accepts.  One key per token; for every tier
(P-256 wq 26/24/22/20 with wg 26; P-384 wq 24/20/18/16 with wg 24 (20 before
round 6); P-521 wq 20/18/16 with wg 20) six tokens:
  edge-first-mid  digit -2^(W-1) (the last entry) in window 0 and a middle window
  edge-every      digit -2^(W-1) in every window below the top one
  top-carry       u = n - 1 - x: the top window all ones with a carry in
  zeros           zero digits in windows 0, 1 / the middle / the second highest
  sparse          u1 non-zero in window 0 only; u2 non-zero in the highest window
                  that u < n lets hold a digit only
  max-pos         u1 alternating +-1, u2 = 2^(W-1) - 1 in every window
each for u1 and u2 at once, plus a copy with s + 1 (rejects).  Digits follow
ecdsa_impl.hpp store_digit_rows: d in [-2^(W-1), 2^(W-1)), ceil((bits+2)/W)
windows (ecdsa.hpp ec_windows_w).  Verdicts: the Go rule in affine big-integer
arithmetic below.

Ed25519 (ed25519.Verify behind keyset.go:127/163, R23-R26): k = SHA-512(R || A
|| M) mod L is a hash, so it is scanned: one key (secret scalar a, fixed nonce
R = rB), messages M varied by their jti, s = r + k a mod L.  Digits follow
ed25519.hip recode: d in (-2^(W-1), 2^(W-1)], ceil(254/W) windows.  Kept:
tokens whose k has the last-entry digit +2^(W-1) in window 0, a middle window
or the highest window that can hold it, at each key tier W = 24/22/20/18/16,
and tokens whose s has it in window 0 or a middle window of the base-point
table (W = 24).  Verdicts: encode([s]B - [k]A) == R (cofactorless), plus an
s + 1 copy of each.

Usage: python tests/golden/make_comb_tier_fixtures.py [--only CURVE]
  --only P-384: rebuild that curve's EC tiers (its own RNG stream) and keep
  every other entry of the committed comb_tiers.json (the Ed25519 scan is slow)
"""
import hashlib
import json
import multiprocessing as mp
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_fixtures import CURVES, claims, enc_json, b64u, ED_L, ED_B, ed_add, ed_mul, ed_encode  # noqa: E402
from make_ec_edge_fixtures import GEN, ec_add, ec_mul, ec_neg, on_curve, lift_x, go_verify, hash_e  # noqa: E402

EC_TIERS = {"P-256": (26, (26, 24, 22, 20)), "P-384": (24, (24, 20, 18, 16)), "P-521": (20, (20, 18, 16))}
ED_WB, ED_TIERS = 24, (24, 22, 20, 18, 16)
ALG_OF = {"P-256": "ES256", "P-384": "ES384", "P-521": "ES512"}
SIZE = {"ES256": 32, "ES384": 48, "ES512": 66}
BITS = {"P-256": 256, "P-384": 384, "P-521": 521}


def sinput(alg, kid, jti):
    hdr = {"alg": alg, "kid": kid, "typ": "JWT"}
    return (b64u(enc_json(hdr)) + "." + b64u(enc_json(claims(jti)))).encode()


# ---------------------------------------------------------------- ECDSA digits
def ec_nwin(bits, w):
    return -(-(bits + 2) // w)


def ec_recode(u, w, nw):
    """ecdsa_impl.hpp store_digit_rows: d in [-2^(W-1), 2^(W-1)), carry out when v >= 2^(W-1)."""
    out, c = [], 0
    for i in range(nw):
        v = ((u >> (w * i)) & ((1 << w) - 1)) + c
        c = 1 if v >= 1 << (w - 1) else 0
        out.append(v - (c << w))
    assert c == 0, "carry out of the top window"
    return out


def from_digits(ds, w):
    return sum(d << (w * i) for i, d in enumerate(ds))


def scalar(kind, n, bits, w, rng, role):
    """A scalar 0 < u < n with the digit pattern `kind` (see the module doc);
    returns (u, digits).  Lower windows random where the pattern leaves them free."""
    nw = ec_nwin(bits, w)
    half = 1 << (w - 1)
    mid = nw // 2
    for _ in range(10000):
        rnd = [rng.randrange(-half, half) for _ in range(nw - 1)]
        if kind == "top-carry":
            u = n - 1 - rng.randrange(1 << (w * max(1, nw - 3)))
        else:
            ds = list(rnd)
            if kind == "edge-first-mid":
                ds[0] = ds[mid] = -half
            elif kind == "edge-every":
                ds = [-half] * (nw - 1)
            elif kind == "zeros":
                for i in ((0, 1, mid) if role == 1 else (0, mid, nw - 2)):
                    ds[i] = 0
            elif kind == "sparse":
                ds = [0] * (nw - 1)
                if role == 1:
                    ds[0] = rng.randrange(1, half)
                elif (n - 1) >> (w * (nw - 1)) == 0:
                    ds[nw - 2] = rng.randrange(1, half)    # u < n leaves the top window empty (P-384 at W = 24)
            elif kind == "max-pos":
                ds = [1 if i % 2 == 0 else -1 for i in range(nw - 1)] if role == 1 else [half - 1] * (nw - 1)
            else:
                raise ValueError(kind)
            low = from_digits(ds, w)
            top_max = (n - 1 - low) >> (w * (nw - 1))
            if kind == "sparse" and (role == 1 or ds[-1]):
                top = 0
            else:
                lo_top = 1 if low <= 0 else 0
                if top_max < lo_top:
                    continue
                top = rng.randrange(lo_top, top_max + 1)
            u = low + (top << (w * (nw - 1)))
        if not 0 < u < n:
            continue
        ds = ec_recode(u, w, nw)
        if kind == "top-carry":
            raw_top = u >> (w * (nw - 1))
            if ds[-1] != raw_top + 1:                 # no carry into the top window
                continue
        return u, ds
    raise RuntimeError(f"no scalar for {kind}")


def craft_ec(crv, wg, wq, kind, idx, rng):
    alg = ALG_OF[crv]
    c = CURVES[crv]
    n, bits = c["n"], BITS[crv]
    u1, d1 = scalar(kind, n, bits, wg, rng, 1)
    u2, d2 = scalar(kind, n, bits, wq, rng, 2)
    kid = f"{crv.replace('-', '').lower()}-w{wq}-{kind}"
    for j in range(1000):
        sinp = sinput(alg, kid, f"{kind}-{j}")
        e = hash_e(crv, alg, sinp)
        if e == 0:
            continue
        s = e * pow(u1, -1, n) % n
        r = u2 * s % n
        if r == 0:
            continue
        R0 = lift_x(crv, r)
        if R0 is None:
            continue
        T = ec_add(crv, R0, ec_neg(crv, ec_mul(crv, u1, GEN[crv])))
        if T is None:
            continue
        Q = ec_mul(crv, pow(u2, -1, n), T)
        break
    else:
        raise RuntimeError("no liftable r")
    assert on_curve(crv, Q)
    w = pow(s, -1, n)
    assert e * w % n == u1 and r * w % n == u2
    sz = SIZE[alg]
    key = dict(kid=kid, kty="EC", crv=crv, x=format(Q[0], "x"), y=format(Q[1], "x"))
    toks = []
    for name, ss in ((kind, s), (kind + "-s-plus-1", (s + 1) % n or 1)):
        verdict = go_verify(crv, alg, Q, sinp, r, ss)
        if ss == s:
            assert verdict == 1, (crv, wq, kind)
        sig = r.to_bytes(sz, "big") + ss.to_bytes(sz, "big")
        toks.append(dict(name=f"{kid}-{name}", alg=alg, key=kid, token=sinp.decode() + "." + b64u(sig),
                         verdict=verdict))
    toks[0]["u1_digits"], toks[0]["u2_digits"] = d1, d2
    return key, toks


# ---------------------------------------------------------------- Ed25519 scan
def ed_nwin(w):
    return -(-254 // w)


def ed_recode(u, w):
    """ed25519.hip recode: d in (-2^(W-1), 2^(W-1)], carry out when v > 2^(W-1)."""
    out, c = [], 0
    for i in range(ed_nwin(w)):
        v = ((u >> (w * i)) & ((1 << w) - 1)) + c
        c = 1 if v > 1 << (w - 1) else 0
        out.append(v - (c << w))
    assert c == 0
    return out


def ed_targets():
    """(scalar, W, window) triples wanted: k at every key tier, s at the base width."""
    t = []
    for w in ED_TIERS:
        nw = ed_nwin(w)
        # highest window that can reach 2^(W-1): the top one only if it holds W - 1 bits of k < 2^253
        top = nw - 1 if 253 - w * (nw - 1) >= w - 1 else nw - 2
        for win in sorted({0, nw // 2, top}):
            t.append(("k", w, win))
    for win in (0, ed_nwin(ED_WB) // 2):
        t.append(("s", ED_WB, win))
    return t


ED_KID = "ed25519-tiers"
ED_ALG = "EdDSA"


def _ed_sinput_parts():
    """The scan's signing input is hdr.b64(payload(jti)); jti = tier-scan-<j>."""
    mark = "@@JTI@@"
    pre, post = enc_json(claims(mark)).decode().split(mark)
    hdr = sinput(ED_ALG, ED_KID, "x").split(b".")[0] + b"."
    return hdr, pre, post


def _ed_scan(args):
    import base64
    a, r, Rb, Ab, start, count, targets = args
    hdr, pre, post = _ed_sinput_parts()
    h0 = hashlib.sha512(Rb + Ab + hdr)
    by_u = {}
    for (which, w, win) in targets:
        by_u.setdefault((which, w), []).append(win)
    hits = {}
    for j in range(start, start + count):
        pay = base64.urlsafe_b64encode(f"{pre}tier-scan-{j}{post}".encode()).rstrip(b"=")
        h = h0.copy()
        h.update(pay)
        k = int.from_bytes(h.digest(), "little") % ED_L
        s = (r + k * a) % ED_L
        for (which, w), wins in by_u.items():
            u = k if which == "k" else s
            half = 1 << (w - 1)
            mask = (1 << w) - 1
            # cheap filter on the raw windows (value + carry == 2^(W-1)) before the exact recode
            cand = [win for win in wins if (which, w, win) not in hits and
                    ((u >> (w * win)) & mask) in (half, half - 1)]
            if not cand:
                continue
            ds = ed_recode(u, w)
            for win in cand:
                if ds[win] == half:
                    hits[(which, w, win)] = j
    return hits


def scan_ed(workers=8, chunk=400_000, max_rounds=60):
    rng = random.Random(0x5EED25519)
    a = rng.randrange(1, ED_L)
    r = rng.randrange(1, ED_L)
    A, R = ed_mul(a, ED_B), ed_mul(r, ED_B)
    Ab, Rb = ed_encode(A), ed_encode(R)
    targets = ed_targets()
    found = {}
    with mp.Pool(workers) as pool:
        for rd in range(max_rounds):
            todo = [t for t in targets if t not in found]
            if not todo:
                break
            jobs = [(a, r, Rb, Ab, (rd * workers + i) * chunk, chunk, todo) for i in range(workers)]
            for h in pool.map(_ed_scan, jobs):
                for t, j in h.items():
                    found.setdefault(t, j)
            print(f"ed scan round {rd}: {len(found)}/{len(targets)}", flush=True)
    missing = [t for t in targets if t not in found]
    if missing:
        raise RuntimeError(f"Ed25519 targets not found: {missing}")
    key = dict(kid=ED_KID, kty="OKP", crv="Ed25519", x=Ab.hex())
    toks = []
    negA = (-A[0] % (2**255 - 19), A[1], A[2], -A[3] % (2**255 - 19))
    for (which, w, win), j in sorted(found.items(), key=lambda kv: kv[1]):
        sinp = sinput(ED_ALG, ED_KID, f"tier-scan-{j}")
        k = int.from_bytes(hashlib.sha512(Rb + Ab + sinp).digest(), "little") % ED_L
        s = (r + k * a) % ED_L
        for name, ss in (("", s), ("-s-plus-1", (s + 1) % ED_L)):
            verdict = int(ed_encode(ed_add(ed_mul(ss, ED_B), ed_mul(k, negA))) == Rb)
            if not name:
                assert verdict == 1
            sig = Rb + ss.to_bytes(32, "little")
            toks.append(dict(name=f"ed25519-{which}-w{w}-win{win}{name}", alg=ED_ALG, key=ED_KID,
                             token=sinp.decode() + "." + b64u(sig), verdict=verdict,
                             edge=dict(scalar=which, w=w, window=win)))
    return key, toks


def hash_seed(name):
    return int.from_bytes(hashlib.sha256(name.encode()).digest()[:4], "big")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        only = sys.argv[2]
        path = os.path.join(HERE, "comb_tiers.json")
        out = json.load(open(path))
        rng = random.Random(0xC0B ^ hash_seed(only))
        wg, tiers = EC_TIERS[only]
        fresh = []
        for wq in tiers:
            keys, toks = [], []
            for i, kind in enumerate(("edge-first-mid", "edge-every", "top-carry", "zeros", "sparse", "max-pos")):
                k, t = craft_ec(only, wg, wq, kind, i, rng)
                keys.append(k)
                toks += t
            fresh.append(dict(crv=only, wg=wg, wq=wq, keys=keys, tokens=toks))
            print(f"{only} wq={wq}: {len(keys)} keys, {len(toks)} tokens", flush=True)
        it = iter(fresh)
        out["ec"] = [next(it) if e["crv"] == only else e for e in out["ec"]]
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return
    rng = random.Random(0xC0B)
    out = {"note": "comb-boundary fixtures per key-table width tier; made by make_comb_tier_fixtures.py",
           "ec": [], "ed25519": None}
    for crv, (wg, tiers) in EC_TIERS.items():
        for wq in tiers:
            keys, toks = [], []
            for i, kind in enumerate(("edge-first-mid", "edge-every", "top-carry", "zeros", "sparse", "max-pos")):
                k, t = craft_ec(crv, wg, wq, kind, i, rng)
                keys.append(k)
                toks += t
            out["ec"].append(dict(crv=crv, wg=wg, wq=wq, keys=keys, tokens=toks))
            print(f"{crv} wq={wq}: {len(keys)} keys, {len(toks)} tokens", flush=True)
    key, toks = scan_ed()
    out["ed25519"] = dict(wb=ED_WB, tiers=list(ED_TIERS), keys=[key], tokens=toks)
    print(f"Ed25519: {len(toks)} tokens")
    with open(os.path.join(HERE, "comb_tiers.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
