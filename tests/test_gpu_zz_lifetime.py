"""Key-memory lifetime under reloads (GPU; jg_runtime.cpp UseLog).

The runtime frees a key generation's device memory (records, blob, comb
tables) through a reaper thread once the last holder drops it; the rule is
that no queued or running launch can still read it then.  hipFree's
device-wide synchronisation would mask a violation, so the check records an
event on every stream that launches against a generation (lanes, class-group
lanes, the chunk control stream, plan fill) and queries them all when the
generation is released.  This module runs after every other GPU module of the
suite (the conftest turns the check on for -m gpu sessions): it drives the
reload patterns that once faulted with stream-ordered allocation
(tools/diag_reload.py: reverse / subset / full reloads), with pipelined
submissions, resident batches and background comb-table upgrades in flight
across each reload, and then requires zero violations over everything checked
so far."""
import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


def test_reloads_with_work_in_flight_release_only_finished_generations():
    from cap_amd import _lib
    _lib.lifetime_check(1)
    bad0, chk0 = _lib.lifetime_check()
    keys, toks = H.golden()
    ctx = _lib.Context()
    ctx.set_chunk(64)
    try:
        ctx.load_keys([H.abi_key(k) for k in keys], wait_tables=False)     # upgrades publish generations meanwhile
        cur = keys
        for name, order in (("reverse", keys[::-1]), ("subset", keys[::2]), ("full", keys)):
            kid_cur = {k["kid"]: i for i, k in enumerate(cur)}
            sel = [t for t in toks if t["key"] in kid_cur]
            arena, slots = H.jobs_from_tokens(sel * 4, kid_cur)
            pend = [ctx.submit(arena) for _ in range(3)]                     # pipelined, not waited
            b = ctx.stage(arena)
            pinned = _lib.PinnedBuffer(len(arena.toks))
            b.enqueue(pinned)                                                # resident, not waited
            ctx.load_keys([H.abi_key(k) for k in order], wait_tables=False)  # reload with all of it in flight
            cur = order
            want = [t["verdict"] for t in sel] * 4
            for p in pend:
                out = p.wait()
                assert [0 if s is None else out[s] for s in slots] == want, name
            b.sync()
            got = pinned.bytes()
            assert [0 if s is None else got[s] for s in slots] == want, name
            pinned.free()
            b.free()
        ctx.wait_tables()
    finally:
        ctx.close()
    bad, chk = _lib.lifetime_check()
    assert chk > chk0                       # generations were released and their uses checked
    assert bad == bad0 == 0, f"{bad} lifetime violations (stderr names the streams)"
