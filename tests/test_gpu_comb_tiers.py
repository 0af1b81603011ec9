"""Comb-boundary parity at every key-table width tier (GPU).

tests/golden/comb_tiers.json (make_comb_tier_fixtures.py) holds, per
(curve, key width) tier, ECDSA tokens crafted on their own keys so that u1
(generator table) and u2 (key table) take chosen signed-digit patterns: the
last table entry in the first / a middle / every window, a carry into an
all-ones top window, zero windows, a lone digit, the largest positive digit;
plus an s + 1 copy of each.  For Ed25519 one key and scanned tokens whose k
(key table) hits the last entry at each key tier and whose s hits it in the
base-point table.  Each tier is loaded through jg_set_table_budget, the width
the runtime picked is asserted, and every verdict must equal the fixture's
(the Go rule in big-integer arithmetic) and the C oracle's -- through the
streaming jg_verify_batch and a resident batch.  The reference behaviour is
crypto/ecdsa.Verify / ed25519.Verify reached from
/root/reference/jwt/keyset.go:127,163.

A last test holds one class at two widths (jg_debug_max_upgrades) with
exceptional tokens in both width runs, so the second run's k_ec_exact appends
to the class's exception list (jg_runtime.cpp width_runs)."""
import json
import os

import pytest

from oracle import jws
from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu

TAB = {"P-256": "p256", "P-384": "p384", "P-521": "p521"}


def fixtures():
    return json.load(open(os.path.join(H.ROOT, "tests", "golden", "comb_tiers.json")))


def _check(ctx, keys, toks):
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in keys}
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    assert None not in slots
    out = ctx.verify(arena)
    b = ctx.stage(arena)
    res = b.run(want_verdicts=True)
    b.free()
    for t, s in zip(toks, slots):
        want = int(jws.verify_sig(jws.parse_jws(t["token"]), okeys[t["key"]]))
        assert want == t["verdict"], ("oracle", t["name"])
        assert out[s] == t["verdict"], ("stream", t["name"])
        assert res[s] == t["verdict"], ("resident", t["name"])
    assert sum(t["verdict"] for t in toks) == len(toks) // 2


def _ec_tiers():
    return [(s["crv"], s["wq"]) for s in fixtures()["ec"]]


@pytest.mark.parametrize("crv,wq", _ec_tiers())
def test_ecdsa_comb_tier(crv, wq):
    import bench
    from cap_amd import _lib
    s = next(x for x in fixtures()["ec"] if x["crv"] == crv and x["wq"] == wq)
    keys = s["keys"]
    ctx = _lib.Context()
    try:
        # exactly this tier for every key of the load (bench.key_widths mirrors the runtime)
        budget = len(keys) * bench.table_bytes(TAB[crv], wq)
        assert bench.key_widths({TAB[crv]: len(keys)}, budget)[TAB[crv]] == wq
        ctx.set_table_budget(budget)
        ctx.load_keys([H.abi_key(k) for k in keys])
        assert ctx.table_widths() == [wq] * len(keys)
        _check(ctx, keys, s["tokens"])
    finally:
        ctx.close()


@pytest.mark.parametrize("n", [40000, 140000])
@pytest.mark.parametrize("crv,wq", _ec_tiers())
def test_ecdsa_comb_tier_mid_launch(crv, wq, n):
    """The same tokens tiled to ~40 k and ~140 k jobs, so the class launch is
    past the 4-lane split's 16 k: P-256 runs the two-lane prefetching split
    (k_ec_point_split<CV, 2, true>, up to 128 k tokens) and then the one-lane
    prefetching chain (<CV, 1, true>, up to 256 k), P-384 the one-lane chain,
    P-521 the one-lane chain at 40 k and k_ec_point at 140 k (ecdsa_impl.hpp
    launch_chain).  Every verdict equals the fixture's."""
    import bench
    from cap_amd import _lib
    s = next(x for x in fixtures()["ec"] if x["crv"] == crv and x["wq"] == wq)
    keys = s["keys"]
    reps = n // len(s["tokens"]) + 1
    toks = s["tokens"] * reps
    assert len(toks) > 16384 * 2
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    ctx = _lib.Context()
    try:
        budget = len(keys) * bench.table_bytes(TAB[crv], wq)
        ctx.set_table_budget(budget)
        ctx.load_keys([H.abi_key(k) for k in keys])
        assert ctx.table_widths() == [wq] * len(keys)
        arena, slots = H.jobs_from_tokens(toks, kid_index)
        out = ctx.verify(arena)
        b = ctx.stage(arena)
        res = b.run(want_verdicts=True)
        b.free()
        bad = [t["name"] for t, sl in zip(toks, slots) if out[sl] != t["verdict"] or res[sl] != t["verdict"]]
        assert not bad, bad[:10]
    finally:
        ctx.close()


@pytest.mark.parametrize("wa", [24, 22, 20, 18, 16])
def test_ed25519_comb_tier(wa):
    import bench
    from cap_amd import _lib
    s = fixtures()["ed25519"]
    # every scanned edge tier is present, and this tier's tokens among them
    assert {t["edge"]["w"] for t in s["tokens"] if t["edge"]["scalar"] == "k"} == set(s["tiers"])
    assert any(t["edge"]["scalar"] == "s" for t in s["tokens"])
    ctx = _lib.Context()
    try:
        ctx.set_table_budget(bench.table_bytes("ed25519", wa))
        ctx.load_keys([H.abi_key(k) for k in s["keys"]])
        assert ctx.table_widths() == [wa]
        _check(ctx, s["keys"], s["tokens"])
    finally:
        ctx.close()


def test_mixed_width_class_with_exceptions_in_both_runs():
    """P-256 keys [Q = G, six W = 24 tier keys, Q = -G]: with two upgrades
    allowed the first two keys widen to 24 and the rest stay at 20, so the
    class runs as two width chains.  Q = +-G with r = s = e (u1 = u2 = 1) meets
    P == +-Q in window 0 at any width: one exceptional token per chain, the
    second chain's k_ec_exact appending to the first's list."""
    import bench
    from cap_amd import _lib
    edge = json.load(open(os.path.join(H.ROOT, "tests", "golden", "ec_edge.json")))
    ekeys = {k["kid"]: k for k in edge["keys"]}
    tier = next(x for x in fixtures()["ec"] if x["crv"] == "P-256" and x["wq"] == 24)
    keys = [ekeys["p256-G"]] + tier["keys"] + [ekeys["p256-negG"]]
    exc = [t for t in edge["tokens"] if t["name"] in ("exc-p256-G-r-eq-s-eq-e", "exc-p256-negG-r-eq-s-eq-e")]
    assert len(exc) == 2
    toks = tier["tokens"] + exc
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in keys}
    ctx = _lib.Context()
    try:
        ctx.set_table_budget(len(keys) * bench.table_bytes("p256", 24))
        ctx.debug_max_upgrades(2)
        ctx.load_keys([H.abi_key(k) for k in keys])
        w = ctx.table_widths()
        assert w == [24, 24] + [20] * (len(keys) - 2), w
        arena, slots = H.jobs_from_tokens(toks, kid_index)
        b = ctx.stage(arena)
        res = b.run(want_verdicts=True)
        assert b.exceptions()[4] == 2                 # CLS_P256: both exceptional tokens, once each
        b.free()
        out = ctx.verify(arena)
        for t, s in zip(toks, slots):
            want = int(jws.verify_sig(jws.parse_jws(t["token"]), okeys[t["key"]]))
            assert want == t["verdict"], t["name"]
            assert res[s] == want and out[s] == want, t["name"]
        # lifting the cap lets the upgrader finish: one width again, same verdicts
        ctx.debug_max_upgrades(-1)
        ctx.wait_tables()
        assert ctx.table_widths() == [24] * len(keys)
        out2 = ctx.verify(arena)
        assert out2 == out
    finally:
        ctx.close()


@pytest.mark.parametrize("n", [20000, 140000])
@pytest.mark.parametrize("wa", [24, 20, 16])
def test_ed25519_comb_tier_large_launch(wa, n):
    """The tier's edge tokens tiled past 16 k jobs, so the class launch runs
    one lane per token instead of the 4-lane k_ed_point_split that every
    smaller launch takes: k_ed_point_pf (entries prefetched) up to 128 k
    tokens, k_ed_point above (ed25519.hip launch_ed)."""
    import bench
    from cap_amd import _lib
    s = fixtures()["ed25519"]
    reps = n // len(s["tokens"]) + 1
    toks = s["tokens"] * reps
    assert len(toks) > 16384
    kid_index = {k["kid"]: i for i, k in enumerate(s["keys"])}
    ctx = _lib.Context()
    try:
        ctx.set_table_budget(bench.table_bytes("ed25519", wa))
        ctx.load_keys([H.abi_key(k) for k in s["keys"]])
        assert ctx.table_widths() == [wa]
        arena, slots = H.jobs_from_tokens(toks, kid_index)
        out = ctx.verify(arena)
        bad = [t["name"] for t, sl in zip(toks, slots)
               if (0 if sl is None else out[sl]) != t["verdict"]]
        assert not bad, bad[:10]
    finally:
        ctx.close()
