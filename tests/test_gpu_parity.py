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
