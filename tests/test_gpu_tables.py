"""Comb tables: edge digits and background widening (GPU).

- tests/golden/edge_digit_tokens.json: valid ES384 / ES512 / EdDSA tokens whose
  signed comb digits select the LAST entry of a window (|d| = 2^(W-1)), which
  uniformly random digits reach with probability ~2^-W per window; every one
  must verify at the fixture's key widths.
- A table widened by the background upgrader equals the table a synchronous
  build gives (jg_debug_table_digest), key by key, for the golden keys.
"""
import json
import os

import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


def test_edge_digit_tokens_verify():
    import bench
    from cap_amd import _lib
    d = json.load(open(os.path.join(H.ROOT, "tests", "golden", "edge_digit_tokens.json")))
    meta = {m[0]: m for m in bench.bench_keys()}
    kids = sorted({s["kid"] for s in d["sets"] if s.get("name") != "p521_w18_top_carry"})
    ctx = _lib.Context()
    ctx.set_table_budget(40 << 30)                     # P-384 W = 24, Ed25519 W = 24, P-521 W = 20
    ctx.load_keys([meta[k][3] for k in kids])
    widths = dict(zip(kids, ctx.table_widths()))
    arena = _lib.Arena()
    slots = []
    for s in d["sets"]:
        if s.get("name") == "p521_w18_top_carry":
            continue                                    # its own width: test_p521_w18_top_window_carry
        assert widths[s["kid"]] == s["wq"], (s["kid"], widths[s["kid"]], s["wq"])
        for t in s["tokens"]:
            b = t.encode()
            dot = b.rfind(b".")
            slots.append((s["alg"], arena.add(b[:dot], b[dot + 1:], s["alg"], kids.index(s["kid"]))))
    assert len(slots) >= 5
    out = ctx.verify(arena)
    ctx.close()
    assert [out[i] for _, i in slots] == [1] * len(slots)


def test_background_widening_matches_sync_build():
    """Context A widens its tables while golden-token batches run against it;
    context B widens the same keys with nothing else running."""
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    arena, slots = H.jobs_from_tokens(toks, kid_index)
    want = [t["verdict"] for t in toks]
    a = _lib.Context()
    a.load_keys([H.abi_key(k) for k in keys], wait_tables=False)
    for _ in range(6):                                  # verification beside the upgrades
        out = a.verify(arena)
        assert [0 if s is None else out[s] for s in slots] == want
    a.wait_tables()
    da = [a.table_digest(i) for i in range(len(keys))]
    wa = a.table_widths()
    # closed first: key tables are shared per physical device between live
    # contexts (jg_runtime.cpp phys_tables), and B must build its own
    a.close()
    b = _lib.Context()
    b.load_keys([H.abi_key(k) for k in keys])
    db = [b.table_digest(i) for i in range(len(keys))]
    assert wa == b.table_widths()
    b.close()
    assert any(da)
    assert da == db


def test_p521_w18_top_window_carry():
    """Valid ES512 tokens whose u2 has bits 504..520 all ones and a carry into
    its top W = 18 window: with 29 windows (522 bits) the signed recoding lost
    that carry and rejected them; ecdsa.hpp ec_windows_w now gives 30."""
    import bench
    from cap_amd import _lib
    d = json.load(open(os.path.join(H.ROOT, "tests", "golden", "edge_digit_tokens.json")))
    s = next(x for x in d["sets"] if x.get("name") == "p521_w18_top_carry")
    meta = {m[0]: m for m in bench.bench_keys()}
    ctx = _lib.Context()
    ctx.set_table_budget(bench.table_bytes("p521", 18))      # one P-521 key at W = 18
    ctx.load_keys([meta[s["kid"]][3]])
    assert ctx.table_widths() == [18]
    arena = _lib.Arena()
    slots = []
    for t in s["tokens"]:
        b = t.encode()
        dot = b.rfind(b".")
        slots.append(arena.add(b[:dot], b[dot + 1:], "ES512", 0))
    out = ctx.verify(arena)
    ctx.close()
    assert len(slots) >= 2
    assert [out[i] for i in slots] == [1] * len(slots)
