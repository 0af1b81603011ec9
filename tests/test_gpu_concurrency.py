"""The single-token drop-in path and the degraded path, on the GPU.

* Concurrent single-token calls (VerifySignature / Validate from many threads,
  the goroutine-per-request pattern of an unchanged cap caller,
  /root/reference/jwt/jwt.go:97 and jwt/keyset.go:27-32) are coalesced into
  device batches (KeySet coalescer): every result equals the same token's
  VerifySignatureBatch / ValidateBatch result and the oracle's.
* A device failure (jg_debug_fail_verify: the n-th submission fails as a fault
  would and the context stays unusable, like a sticky HIP error): the call that
  carried it gets "capjwt: signature verification unavailable: ..." for every
  token that needed the device, the key set recreates its context and
  re-stages its keys (Engine::recover), the next call's results equal the
  oracle's, and a JWKS key set fetches nothing (SURVEY §5 failure row).
"""
import concurrent.futures as cf
import json

import pytest

from oracle import jws
from tests.test_gpu_edges import CountingJWKS, _c5_pool

pytestmark = pytest.mark.gpu

UNAVAILABLE = "capjwt: signature verification unavailable: "


@pytest.fixture(scope="module")
def c5():
    meta, pool, tampered, okeys = _c5_pool(per_kid=24, seed=5)
    pool = pool + ["not-a-jwt", pool[0] + "x"]
    return meta, pool, okeys


def oracle_jwks(tok, okeys):
    try:
        return jws.jwks_keyset_verify(tok, okeys), None
    except jws.ErrNoKey as e:
        return None, str(e)


def same(got, want):
    """got == the oracle's (claims, err); the oracle's "oidc: malformed jwt"
    stands for the whole go-jose parse error after it (the parse error text
    itself is pinned by tests/test_host_cpu.py)"""
    got, want = tuple(got), tuple(want)
    if want[1] and want[1].endswith("oidc: malformed jwt"):
        return got[0] is None and got[1] is not None and got[1].startswith(want[1] + ": ")
    return got == want


def test_concurrent_single_calls_equal_batch_and_oracle(c5):
    from cap_amd import jwt
    meta, pool, okeys = c5
    fetch = CountingJWKS({"keys": [m[4] for m in meta]}, max_age=3600)
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "", fetch)
    assert err is None
    batch = ks.VerifySignatureBatch(pool)
    for inflight in (1, 4):
        ks.SetCoalescing(max_inflight=inflight, window_us=200 if inflight == 1 else 0)
        with cf.ThreadPoolExecutor(48) as ex:
            single = list(ex.map(ks.VerifySignature, pool))
        assert single == batch
    st = ks.CoalescingStats()
    assert st["calls"] == 2 * len(pool) and st["batches"] <= st["calls"]
    for tok, g in zip(pool, batch):
        assert same(g, oracle_jwks(tok, okeys)), (tok, g)
    # Validator.Validate from many threads == ValidateBatch == the oracle
    v, _ = jwt.NewValidator(ks)
    algs = sorted({m[1] for m in meta})
    e = jwt.Expected(SigningAlgorithms=algs, Issuer="https://example.com/", Audiences=["www.example.com"],
                     Now=lambda: 1611699344 + 60)
    vb = v.ValidateBatch(pool, e)
    with cf.ThreadPoolExecutor(48) as ex:
        vs = list(ex.map(lambda t: v.Validate(t, e), pool))
    assert vs == vb
    now_ns = (1611699344 + 60) * jws.SECOND
    exp = dict(SigningAlgorithms=algs, Issuer="https://example.com/", Audiences=["www.example.com"])
    for tok, g in zip(pool, vb):
        assert same(g, jws.validate(tok, lambda t: jws.jwks_keyset_verify(t, okeys), exp, now_ns)), (tok, g)
    assert fetch.calls == 1


def test_native_concurrent_callers_accept_exactly(c5):
    """The bench's measurement helper: C++ threads calling Validator::Validate
    per token (no GIL); accepts == the batch's accepts over the same tokens."""
    from cap_amd import jwt
    meta, pool, okeys = c5
    fetch = CountingJWKS({"keys": [m[4] for m in meta]}, max_age=3600)
    ks, _ = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "", fetch)
    v, _ = jwt.NewValidator(ks)
    algs = sorted({m[1] for m in meta})
    e = jwt.Expected(SigningAlgorithms=algs, Now=lambda: 1611699344 + 60)
    want = sum(g[1] is None for g in v.ValidateBatch(pool, e))
    blob = "\n".join(pool).encode()
    for callers in (1, 16, 128):
        r = v._impl._concurrent_validate(blob, e._native(), callers, 2 * len(pool))
        assert r["calls"] == 2 * len(pool)
        assert r["accepted"] == 2 * want, (callers, r)
        assert 0 < r["p50_us"] <= r["p99_us"] <= r["max_us"]


@pytest.mark.parametrize("single", [False, True])
def test_device_failure_then_recovery_jwks(c5, single):
    from cap_amd import jwt
    meta, pool, okeys = c5
    fetch = CountingJWKS({"keys": [m[4] for m in meta]}, max_age=0)     # expired at once: misses would refetch
    ks, _ = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "", fetch)
    good = [t for t in pool if oracle_jwks(t, okeys)[1] is None][:64]
    assert ks.VerifySignatureBatch(good) == [oracle_jwks(t, okeys) for t in good]
    calls0 = fetch.calls
    assert ks.DeviceStatus() == "" and ks.DeviceRecoveries() == 0
    ks._impl._debug_fail_verify(1)
    toks = good + ["not-a-jwt"]
    if single:
        with cf.ThreadPoolExecutor(16) as ex:
            got = list(ex.map(ks.VerifySignature, toks))
    else:
        got = ks.VerifySignatureBatch(toks)
    # the failed call: every token that reached the device carries the device
    # error (single calls: those coalesced into the failing batch); the parse
    # error stays a parse error; nothing was refetched
    failed = [i for i, (c, err) in enumerate(got) if err and err.startswith(UNAVAILABLE)]
    assert failed and all(i < len(good) for i in failed)
    assert "injected device failure" in got[failed[0]][1]
    assert got[-1][0] is None and got[-1][1].startswith("oidc: malformed jwt: ")
    for i, g in enumerate(got[:-1]):
        if i not in failed:
            assert same(g, oracle_jwks(toks[i], okeys))
    assert fetch.calls == calls0
    # recovered: a new context with the same key list, verdicts exact again
    assert ks.DeviceRecoveries() == 1 and ks.DeviceStatus() == ""
    assert all(same(g, oracle_jwks(t, okeys)) for t, g in zip(pool, ks.VerifySignatureBatch(pool)))
    assert [ks.VerifySignature(t) for t in good[:8]] == [oracle_jwks(t, okeys) for t in good[:8]]
    assert fetch.calls == calls0 + 1                # the pool's tampered tokens miss: one refresh (max_age 0)


def test_device_failure_then_recovery_static_validator():
    from cap_amd import jwt
    import bench
    kids = ["p256-a", "p256-b"]
    pool = [t.decode() for t in bench.gen_tokens("ES256", 96, bench.golden_keypaths(kids), 4, "recov")]
    from tests import gpu_helpers as H
    keys, _ = H.golden()
    by = {k["kid"]: k for k in keys}
    nat = [jwt.PublicKey.ec("P-256", int(by[k]["x"], 16).to_bytes(32, "big"), int(by[k]["y"], 16).to_bytes(32, "big"))
           for k in kids]
    ks, _ = jwt.NewStaticKeySet(nat)
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(SigningAlgorithms=["ES256"], Now=lambda: 1611699344 + 60)
    ok = v.ValidateBatch(pool, e)
    assert all(err is None for _, err in ok)
    ks._impl._debug_fail_verify(1)
    bad = v.ValidateBatch(pool, e)
    assert all(c is None and err.startswith("error verifying token signature: " + UNAVAILABLE) for c, err in bad)
    assert ks.DeviceRecoveries() == 1
    assert v.ValidateBatch(pool, e) == ok
    assert [v.Validate(t, e) for t in pool[:4]] == ok[:4]
