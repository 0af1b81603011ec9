"""GPU parity: the HIP path through the C ABI (libcapjwt.so) against the
golden fixtures (OpenSSL-signed, Go-semantics labelled) and the CPU oracle."""
import os

import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from cap_amd import _lib
    keys, _ = H.golden()
    c = _lib.Context()
    c.load_keys([H.abi_key(k) for k in keys])
    yield c
    c.close()


def test_golden_vectors(ctx):
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    out = ctx.verify(arena)
    bad = []
    for t, s in zip(toks, slots):
        got = 0 if s is None else out[s]
        if got != t["verdict"]:
            bad.append((t["name"], got, t["verdict"], t["source"]))
    assert not bad, bad


def test_device_base64_decoder_edges(ctx):
    """The device base64url decoder (prep.hip: word-at-a-time fast path, and the
    byte-serial fallback for P-521 and odd-length RSA signatures) against Go's
    base64.RawURLEncoding after go-jose's '=' trim (R3): a byte outside the
    alphabet anywhere rejects, non-zero unused tail bits are accepted (Go's
    decoder is not strict), a 4k+1 length rejects -- at every arena alignment."""
    from cap_amd import _lib
    from oracle import jws
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    names = ["valid-RS256-rsa2048-a-0", "valid-PS512-rsa4096-a-1", "valid-ES256-p256-a-0", "valid-ES384-p384-a-0",
             "valid-ES512-p521-a-0", "valid-EdDSA-ed-a-0", "valid-RS256-rsa2049-a-0"]
    by = {t["name"]: t for t in toks}
    arena = _lib.Arena()
    want = []
    for name in names:
        t = by[name]
        p = jws.parse_jws(t["token"])
        sig = jws.b64url_encode(p.signature)
        n = len(sig)
        variants = [(sig, 1)]
        for pos in sorted({0, 1, 2, 3, 15, 16, 63, 64, 127, 128, 129, 255, 256, n // 2, n - 2, n - 1}):
            if pos < n:
                for bad in "*=+/. \x7f":
                    variants.append((sig[:pos] + bad + sig[pos + 1:], 0))
        variants.append((sig + "A", 0))                          # one character too many
        if n % 4 in (2, 3):                                     # flip the unused low bits of the last char
            unused = 4 if n % 4 == 2 else 2
            last = alpha.index(sig[-1]) ^ ((1 << unused) - 1)
            variants.append((sig[:-1] + alpha[last], 1))
        variants.append((sig[:-1] + alpha[(alpha.index(sig[-1]) + 32) % 64], 0))  # a used bit flips
        for vi, (s, w) in enumerate(variants):
            arena.buf += b"#" * (vi % 4)                        # every alignment of the segment
            arena.add(p.signing_input, s.encode(), p.alg, kid_index[t["key"]])
            want.append(w)
    out = ctx.verify(arena)
    bad = [i for i, w in enumerate(want) if out[i] != w]
    assert not bad, (len(bad), [(i, want[i]) for i in bad[:20]])


def test_cross_product_every_token_every_key(ctx):
    """Every golden token against every loaded key in ONE batch (mixed classes,
    signatures longer than the key, wrong families): each verdict equals the
    oracle's.  Pins the per-class scratch bounds and the class bucketing."""
    from oracle import jws
    keys, toks = H.golden()
    okeys = [jws.Key.from_fixture(k) for k in keys]
    from cap_amd import _lib
    arena = _lib.Arena()
    want = []
    for t in toks:
        p = jws.parse_jws(t["token"])
        if p is None or not p.crit_ok:
            continue
        sig_b64 = jws.b64url_encode(p.signature).encode()
        for ki, k in enumerate(okeys):
            arena.add(p.signing_input, sig_b64, p.alg, ki)
            want.append(int(jws.verify_sig(p, k)))
    out = ctx.verify(arena)
    bad = [i for i, w in enumerate(want) if out[i] != w]
    assert not bad, (len(bad), bad[:20])
    assert sum(want) > 150


def test_contexts_share_fixed_base_tables():
    """The generator / base-point tables are one copy per device shared by every
    jg_ctx (jg_runtime.cpp shared_table): a second context verifies with them,
    and keeps verifying after the context that built them is destroyed."""
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    pick = [t for t in toks if t["name"].startswith(("valid-ES256", "valid-ES384", "valid-ES512", "valid-EdDSA",
                                                     "tamper-sig-ES", "tamper-sig-EdDSA"))]
    a = _lib.Context()
    a.load_keys([H.abi_key(k) for k in keys])
    arena, slots = H.jobs_from_tokens(pick, kid_index)
    want = [t["verdict"] for t in pick]
    assert [a.verify(arena)[s] for s in slots] == want
    b = _lib.Context()
    b.load_keys([H.abi_key(k) for k in keys])
    assert [b.verify(arena)[s] for s in slots] == want
    a.close()
    arena2, slots2 = H.jobs_from_tokens(pick, kid_index)
    assert [b.verify(arena2)[s] for s in slots2] == want
    b.close()


def test_timed_and_streamed_runs_agree(ctx):
    """jg_batch_run (classes in sequence, per-kernel events) and
    jg_batch_enqueue (every class on its own stream) give identical verdicts on
    a batch mixing all seven kernel classes, run after run."""
    from cap_amd import _lib
    from oracle import jws
    keys, toks = H.golden()
    okeys = [jws.Key.from_fixture(k) for k in keys]
    arena = _lib.Arena()
    want = []
    for t in toks:
        p = jws.parse_jws(t["token"])
        if p is None or not p.crit_ok:
            continue
        sig_b64 = jws.b64url_encode(p.signature).encode()
        for ki, k in enumerate(okeys):
            arena.add(p.signing_input, sig_b64, p.alg, ki)
            want.append(int(jws.verify_sig(p, k)))
    b = ctx.stage(arena)
    timed = b.run(want_verdicts=True)
    assert list(timed) == want
    assert {n.split("_")[0] for n, _ in b.kernel_times()} >= {"rsa2048", "p256", "p384", "p521", "ed25519"}
    pinned = _lib.PinnedBuffer(len(want))
    for _ in range(3):
        b.enqueue(pinned)
    b.sync()
    assert list(pinned.bytes()[:len(want)]) == want
    pinned.free()
    b.free()


def _fresh_p256_key():
    """A P-256 public key no earlier test loaded (comb tables are cached per
    device by key content, across contexts): Q = k G for a random k."""
    import secrets
    from tests.test_gpu_mp import ec_mul
    c = {"p": 2**256 - 2**224 + 2**192 + 2**96 - 1}
    G = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
         0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)
    Q = ec_mul(c, 1 + secrets.randbelow(2**255), G)
    return {"kty": "EC", "crv": "P-256", "kid": "fresh-p256", "x": f"{Q[0]:064x}", "y": f"{Q[1]:064x}"}


def test_key_reload_reuses_tables():
    """jg_keys_load keeps the comb tables of keys it already had (copied by
    content into the new key blob) and builds only new ones: reloading the
    golden key set in reverse order, then a subset, verifies every golden token
    exactly as a fresh load does.  The first load holds a key no earlier test
    loaded, so it builds at least that key's table; a reload of the key set
    the context holds (in any order) builds none (jg_debug_tables_built, a
    counter: no wall-clock comparison).  The subset may build wider tables
    (fewer keys share the budget), and the full set after it rebuilds the
    tables the subset released."""
    from cap_amd import _lib
    keys, toks = H.golden()
    keys = keys + [_fresh_p256_key()]
    c = _lib.Context()
    c.load_keys([H.abi_key(k) for k in keys])
    c.wait_tables()
    built = c.tables_built()
    assert built >= 1                 # the fresh key's table at least
    held = {k["kid"] for k in keys}
    for order in (keys[::-1], keys[::2], keys, keys[::-1]):
        c.load_keys([H.abi_key(k) for k in order])
        kid_index = {k["kid"]: i for i, k in enumerate(order)}
        sel = [t for t in toks if t["key"] in kid_index]
        arena, slots = H.jobs_from_tokens(sel, kid_index)
        out = c.verify(arena)
        bad = [(t["name"], out[s] if s is not None else 0, t["verdict"]) for t, s in zip(sel, slots)
               if (0 if s is None else out[s]) != t["verdict"]]
        assert not bad, bad
        c.wait_tables()
        if {k["kid"] for k in order} == held:
            assert c.tables_built() == built, (len(order), c.tables_built(), built)
        held = {k["kid"] for k in order}
        built = c.tables_built()
    c.close()


def test_rsa_keys_above_4096_bits():
    """RSA moduli of 4100 to 16384 bits -- every layout of the RSA-4K+ class
    (148 limbs up to 4142 bits, 296 up to 8286, 592 above; signatures of 513 to
    2048 bytes, PKCS#1 v1.5 and PSS): the GPU verdicts equal the oracle's and
    the fixture's (tests/golden/rsa_big.json, made by make_big_rsa.py)."""
    import json
    from oracle import jws
    d = json.load(open(os.path.join(H.ROOT, "tests", "golden", "rsa_big.json")))
    from cap_amd import _lib
    kid_index = {k["kid"]: i for i, k in enumerate(d["keys"])}
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in d["keys"]])
    arena, slots = H.jobs_from_tokens(d["tokens"], kid_index)
    out = ctx.verify(arena)
    ctx.close()
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in d["keys"]}
    for t, s in zip(d["tokens"], slots):
        want = int(jws.verify_sig(jws.parse_jws(t["token"]), okeys[t["key"]]))
        assert want == t["want"], t["name"]
        assert out[s] == want, t["name"]


@pytest.mark.parametrize("tier", [26, 24, 22, 20])
def test_p256_key_table_widths(tier):
    """The P-256 key comb width follows the table budget (jg_set_table_budget,
    one total over every curve, jg_runtime.cpp key_widths): W = 26 / 24 / 22 /
    20 give the same verdicts as the oracle on every golden token against every
    key, and the library reports the width the budget buys (bench.key_widths)."""
    import bench
    from cap_amd import _lib
    from oracle import jws
    keys, toks = H.golden()
    crv = {"P-256": "p256", "P-384": "p384", "P-521": "p521"}
    cls = [crv.get(k.get("crv")) if k.get("kty") == "EC" else ("ed25519" if k.get("kty") == "OKP" else None)
           for k in keys]
    counts = {c: cls.count(c) for c in ("p256", "p384", "p521", "ed25519")}
    assert counts["p256"] >= 2
    narrow = sum(n * bench.table_bytes(c, bench.WIDTH_TIERS[c][-1]) for c, n in counts.items())
    budget = narrow + counts["p256"] * (bench.table_bytes("p256", tier) - bench.table_bytes("p256", 20))
    assert bench.key_widths(counts, budget)["p256"] == tier
    ctx = _lib.Context()
    ctx.set_table_budget(budget)
    ctx.load_keys([H.abi_key(k) for k in keys])
    widths = ctx.table_widths()
    want_w = bench.key_widths(counts, budget)
    for k, c, w in zip(keys, cls, widths):
        if c is not None and w:
            assert w == want_w[c], (k["kid"], w, want_w[c])
    assert [w for c, w in zip(cls, widths) if c == "p256"] == [tier] * counts["p256"]
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in keys}
    sel = [t for t in toks if t["alg"] in ("ES256", "ES384", "ES512")]
    cross = [dict(t, key=k["kid"]) for t in sel for k in keys if k.get("kty") == "EC"]
    arena, slots = H.jobs_from_tokens(cross, kid_index)
    out = ctx.verify(arena)
    ctx.close()
    bad = []
    for t, s in zip(cross, slots):
        p = jws.parse_jws(t["token"])
        want = int(jws.verify_sig(p, okeys[t["key"]])) if p is not None else 0
        if (0 if s is None else out[s]) != want:
            bad.append((t["name"], t["key"]))
    assert not bad, bad[:10]


@pytest.mark.parametrize("tier", [24, 22, 20, 18, 16])
def test_ed25519_key_table_widths(tier):
    """Every Ed25519 key comb width (ed25519.hpp ED_WA, picked by the table
    budget) against the oracle: the golden Ed25519 keys alone in a context
    whose budget buys `tier`, every EdDSA golden token against every one of
    them (small-order and non-canonical keys included)."""
    import bench
    from cap_amd import _lib
    from oracle import jws
    keys, toks = H.golden()
    ed = [k for k in keys if k.get("kty") == "OKP"]
    n = len(ed)
    budget = n * bench.table_bytes("ed25519", tier)
    assert bench.key_widths({"ed25519": n}, budget)["ed25519"] == tier
    ctx = _lib.Context()
    ctx.set_table_budget(budget)
    ctx.load_keys([H.abi_key(k) for k in ed])
    widths = ctx.table_widths()
    assert {w for w in widths if w} == {tier}, widths
    kid_index = {k["kid"]: i for i, k in enumerate(ed)}
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in ed}
    cross = [dict(t, key=k["kid"]) for t in toks if t["alg"] == "EdDSA" for k in ed]
    arena, slots = H.jobs_from_tokens(cross, kid_index)
    out = ctx.verify(arena)
    ctx.close()
    bad = []
    for t, s in zip(cross, slots):
        p = jws.parse_jws(t["token"])
        want = int(jws.verify_sig(p, okeys[t["key"]])) if p is not None else 0
        if (0 if s is None else out[s]) != want:
            bad.append((t["name"], t["key"]))
    assert not bad, bad[:10]
