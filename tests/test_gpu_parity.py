"""GPU parity: the HIP path through the C ABI (libcapjwt.so) against the
golden fixtures (OpenSSL-signed, Go-semantics labelled) and the CPU oracle."""
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
