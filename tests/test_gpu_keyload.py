"""GPU checks of key loading as a JWKS refresh exercises it (jg_keys_load,
jg_runtime.cpp stage_device / upgrade_one; go-oidc RemoteKeySet updateKeys
behind /root/reference/jwt/keyset.go:127):

- an identical key list is a no-op (no device work, staged batches stay valid);
- a load that fails on the device (an allocation failure injected with
  jg_debug_fail_alloc) keeps the previous table in force, as go-oidc keeps its
  cached keys when updateKeys fails;
- a new key verifies at once on a narrow comb table and gives the same
  verdicts after its wide table is swapped in;
- a batch queued before a reload runs against the table it was submitted with;
- a bad job in a later pipeline chunk fails jg_wait with -1 (include/jg.h).

Every verdict is compared with the oracle's."""

import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


def _oracle_verdicts(keys, toks, kid_index):
    from oracle import jws
    okeys = {k["kid"]: jws.Key.from_fixture(k) for k in keys}
    out = []
    for t in toks:
        p = jws.parse_jws(t["token"])
        out.append(int(jws.verify_sig(p, okeys[t["key"]])) if p is not None and p.crit_ok else 0)
    return out


def _ec_ed_cross(keys, toks):
    """every EC / EdDSA golden token against every EC / Ed25519 key"""
    sel = [t for t in toks if t["alg"] in ("ES256", "ES384", "ES512", "EdDSA")]
    return [dict(t, key=k["kid"]) for t in sel for k in keys if k.get("kty") in ("EC", "OKP")]


def _verify(ctx, toks, kid_index):
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    out = ctx.verify(arena)
    return [0 if s is None else out[s] for s in slots]


def test_identical_reload_is_a_no_op():
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    ctx = _lib.Context()
    abi = [H.abi_key(k) for k in keys]
    ctx.load_keys(abi)
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    b = ctx.stage(arena)
    before = b.run(want_verdicts=True)
    ctx.wait_tables()
    built = ctx.tables_built()
    for _ in range(20):
        ctx.load_keys(abi, wait_tables=False)
    ctx.wait_tables()
    assert ctx.tables_built() == built                       # host-only: no table build (a counter, not a clock)
    assert b.run(want_verdicts=True) == before               # the staged batch is still valid (same epoch)
    assert [0 if s is None else before[s] for s in slots] == [t["verdict"] for t in toks]
    # a different budget is a different load: the batch's plan stays valid only
    # while the key list is unchanged, so it must now be re-staged
    ctx.set_table_budget(0)
    ctx.load_keys(abi)
    with pytest.raises(_lib.JgError, match="reloaded"):
        b.run(want_verdicts=True)
    b.free()
    assert _verify(ctx, toks, kid_index) == [t["verdict"] for t in toks]
    ctx.close()


@pytest.mark.parametrize("nth", [1, 2, 3, 4, 5])
def test_device_failure_keeps_previous_table(nth):
    """The nth device allocation of a load fails: jg_keys_load returns -2, the
    previous key list keeps verifying (same verdicts as before the attempt),
    and the next load succeeds."""
    from cap_amd import _lib
    keys, toks = H.golden()
    half = [k for k in keys if k["kid"] in ("rsa2048-a", "p256-a", "p384-a", "ed-a")]
    kid_a = {k["kid"]: i for i, k in enumerate(half)}
    sel = [t for t in toks if t["key"] in kid_a]
    ctx = _lib.Context()
    ctx.set_table_budget(0)
    ctx.load_keys([H.abi_key(k) for k in half])
    before = _verify(ctx, sel, kid_a)
    assert before == _oracle_verdicts(half, sel, kid_a)
    assert any(before)
    ctx.debug_fail_alloc(nth)
    with pytest.raises(_lib.JgError, match="out of memory"):
        ctx.load_keys([H.abi_key(k) for k in keys[::-1]])
    ctx.debug_fail_alloc(0)
    assert _verify(ctx, sel, kid_a) == before                 # old keys, old indices
    order = keys[::-1]
    kid_b = {k["kid"]: i for i, k in enumerate(order)}
    ctx.load_keys([H.abi_key(k) for k in order])
    assert _verify(ctx, toks, kid_b) == [t["verdict"] for t in toks]
    ctx.close()


def test_new_key_verifies_narrow_then_wide():
    """A P-256 key budgeted for W = 24 verifies as soon as jg_keys_load returns
    (on its narrow W = 20 table, or already the wide one), and the verdicts do
    not change when the wide table is swapped in -- on a resident batch staged
    before the swap as well."""
    import bench
    from cap_amd import _lib
    keys, toks = H.golden()
    ec = [k for k in keys if k.get("kty") in ("EC", "OKP")]
    kid_index = {k["kid"]: i for i, k in enumerate(ec)}
    cross = _ec_ed_cross(ec, toks)
    want = _oracle_verdicts(ec, cross, kid_index)
    counts = {"p256": 4, "p384": 1, "p521": 1, "ed25519": 7}
    narrow = sum(n * bench.table_bytes(c, bench.WIDTH_TIERS[c][-1]) for c, n in counts.items())
    budget = narrow + 4 * (bench.table_bytes("p256", 24) - bench.table_bytes("p256", 20))
    ctx = _lib.Context()
    ctx.set_table_budget(budget)
    ctx.load_keys([H.abi_key(k) for k in ec], wait_tables=False)
    first = ctx.table_widths()
    p256 = [i for i, k in enumerate(ec) if k.get("crv") == "P-256"]
    assert all(first[i] in (20, 24) for i in p256), first
    arena, slots = H.jobs_from_tokens(cross, kid_index)
    b = ctx.stage(arena)
    got = b.run(want_verdicts=True)
    assert [0 if s is None else got[s] for s in slots] == want
    assert ctx.wait_tables()
    assert [ctx.table_widths()[i] for i in p256] == [24] * 4
    got = b.run(want_verdicts=True)                            # same batch, wide tables
    assert [0 if s is None else got[s] for s in slots] == want
    b.free()
    assert _verify(ctx, cross, kid_index) == want
    # reloading the same keys in another order reuses every table (no build):
    # the widths are right at once
    order = ec[::-1]
    ctx.load_keys([H.abi_key(k) for k in order], wait_tables=False)
    w2 = ctx.table_widths()
    assert [w2[len(ec) - 1 - i] for i in p256] == [24] * 4
    kid2 = {k["kid"]: i for i, k in enumerate(order)}
    assert _verify(ctx, cross, kid2) == want
    ctx.close()


def test_batch_queued_across_a_reload_uses_its_table():
    """Submissions made before a jg_keys_load finish against the key table of
    their submit time; submissions after it use the new one."""
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_a = {k["kid"]: i for i, k in enumerate(keys)}
    order = keys[::-1]
    kid_b = {k["kid"]: i for i, k in enumerate(order)}
    ctx = _lib.Context()
    ctx.set_table_budget(0)
    ctx.load_keys([H.abi_key(k) for k in keys])
    ctx.set_chunk(64)
    arena_a, slots_a = H.jobs_from_tokens(toks * 8, kid_a)
    pend = [ctx.submit(arena_a) for _ in range(3)]
    ctx.load_keys([H.abi_key(k) for k in order])              # no drain: the queued batches keep table A
    arena_b, slots_b = H.jobs_from_tokens(toks, kid_b)
    pb = ctx.submit(arena_b)
    want = [t["verdict"] for t in toks] * 8
    for p in pend:
        out = p.wait()
        assert [0 if s is None else out[s] for s in slots_a] == want
    out = pb.wait()
    assert [0 if s is None else out[s] for s in slots_b] == [t["verdict"] for t in toks]
    ctx.close()


def test_bad_job_in_a_later_chunk_fails_the_wait():
    """include/jg.h: jobs are validated per chunk by the device workers; a bad
    key_idx in a later chunk makes jg_wait return -1 (jg_submit returned 0)."""
    import ctypes
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    ctx.set_chunk(64)
    arena, slots = H.jobs_from_tokens(toks * 4, kid_index)
    ta = arena.tok_array()
    n = len(arena.toks)
    assert n > 640
    ta[n - 5].key_idx = len(keys) + 3
    out = (ctypes.c_uint8 * n)()
    L = _lib.lib()
    t = ctypes.c_void_p()
    buf = bytes(arena.buf)
    assert L.jg_submit(ctx.h, buf, len(buf), ta, n, out, ctypes.byref(t)) == 0
    assert L.jg_wait(ctx.h, t) == -1
    assert "key_idx" in ctx.error()
    # the chunks before the bad one were verified
    good = [t["verdict"] for t in toks * 4]
    first = [0 if s is None else out[s] for s in slots[:256]]
    assert first == good[:256]
    ctx.close()
