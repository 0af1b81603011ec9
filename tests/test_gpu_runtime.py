"""GPU checks of the runtime behind the C ABI (jg_runtime.cpp): argument and
bounds errors, key-load failure handling, the chunked streaming pipeline
(jg_submit / jg_wait), and the in-process multi-device split -- every verdict
against the oracle."""
import ctypes

import pytest

from tests import gpu_helpers as H

pytestmark = pytest.mark.gpu


def _mixed_arena(keys, toks, reps=1):
    """Every golden token against every key (all seven kernel classes, wrong
    families, bad signatures), `reps` times; returns (arena, oracle verdicts)."""
    from cap_amd import _lib
    from oracle import jws
    okeys = [jws.Key.from_fixture(k) for k in keys]
    arena = _lib.Arena()
    want = []
    cache = {}
    for _ in range(reps):
        for t in toks:
            p = jws.parse_jws(t["token"])
            if p is None or not p.crit_ok:
                continue
            sig_b64 = jws.b64url_encode(p.signature).encode()
            for ki, k in enumerate(okeys):
                arena.add(p.signing_input, sig_b64, p.alg, ki)
                key = (t["name"], ki)
                if key not in cache:
                    cache[key] = int(jws.verify_sig(p, k))
                want.append(cache[key])
    return arena, want


def test_abi_return_codes_zero_jobs_zero_keys():
    """jg_verify_batch with zero jobs, with zero keys loaded, and with jobs
    whose key or spans are out of range (SURVEY §8b error conventions)."""
    from cap_amd import _lib
    L = _lib.lib()
    ctx = _lib.Context()
    out = (ctypes.c_uint8 * 4)()
    # no keys loaded yet, zero jobs: OK, nothing written
    assert L.jg_verify_batch(ctx.h, None, 0, None, 0, None) == 0
    assert L.jg_keys_load(ctx.h, None, 0) == 0                 # an empty key table is legal
    assert L.jg_verify_batch(ctx.h, None, 0, None, 0, None) == 0
    # a job naming key 0 of an empty table: bad argument
    arena = b"a.b" + b"\0" * 8
    tok = (_lib.JgTok * 1)()
    tok[0].off, tok[0].sig_in_len, tok[0].sig_rel_off, tok[0].sig_b64_len, tok[0].key_idx, tok[0].alg = 0, 1, 2, 1, 0, 7
    assert L.jg_verify_batch(ctx.h, arena, len(arena), tok, 1, out) == -1
    assert "key_idx" in ctx.error()
    keys, _ = H.golden()
    ctx.load_keys([H.abi_key(k) for k in keys])
    assert L.jg_verify_batch(ctx.h, arena, len(arena), tok, 1, out) == 0
    assert out[0] == 0
    # spans past the arena: rejected on the host before any upload
    for fld, val in (("off", len(arena) + 1), ("sig_in_len", len(arena) + 1), ("sig_b64_len", len(arena)),
                     ("sig_rel_off", 1 << 31)):
        bad = (_lib.JgTok * 1)()
        ctypes.memmove(bad, tok, ctypes.sizeof(bad))
        setattr(bad[0], fld, val)
        assert L.jg_verify_batch(ctx.h, arena, len(arena), bad, 1, out) == -1, fld
        assert "past the arena" in ctx.error()
        h = ctypes.c_void_p()
        assert L.jg_batch_stage(ctx.h, 0, arena, len(arena), bad, 1, ctypes.byref(h)) == -1, fld
    # null context / pointers
    assert L.jg_verify_batch(None, arena, len(arena), tok, 1, out) == -1
    assert L.jg_verify_batch(ctx.h, arena, len(arena), tok, 1, None) == -1
    assert L.jg_keys_load(None, None, 0) == -1
    assert L.jg_set_chunk(ctx.h, 8) == -1
    ctx.close()


def test_key_load_failure_keeps_table_and_does_not_hang():
    """More P-256 keys than a comb-table budget allows: jg_keys_load returns -2,
    the previous table stays in force (verification neither hangs nor changes)."""
    from cap_amd import _lib
    keys, toks = H.golden()
    kid_index = {k["kid"]: i for i, k in enumerate(keys)}
    sel = [t for t in toks if t["name"].startswith(("valid-ES256", "tamper-sig-ES256", "valid-RS256"))]
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    arena, slots = H.jobs_from_tokens(sel, kid_index)
    before = ctx.verify(arena)
    p256 = next(k for k in keys if k["kid"] == "p256-a")
    with pytest.raises(_lib.JgError, match="at most 256 keys"):
        ctx.load_keys([H.abi_key(p256)] * 257)
    assert ctx.verify(arena) == before                        # same table, no deadlock
    assert [before[s] for s in slots] == [t["verdict"] for t in sel]
    ctx.load_keys([H.abi_key(k) for k in keys])                # and a later load works
    assert ctx.verify(arena) == before
    ctx.close()


def test_streaming_pipeline_chunks_and_overlapping_submits():
    """jg_submit with small pipeline chunks (many chunks per device, all
    NSLOT slots in flight) and several submissions in flight at once: every
    verdict equals the oracle's and the synchronous path's."""
    from cap_amd import _lib
    keys, toks = H.golden()
    arena, want = _mixed_arena(keys, toks)
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    ref = ctx.verify(arena)
    assert list(ref) == want
    for chunk in (64, 1000, 4096):
        ctx.set_chunk(chunk)
        pend = [ctx.submit(arena) for _ in range(3)]
        for p in pend:
            assert p.wait() == ref, chunk
    ctx.close()


def test_streaming_from_pinned_and_scattered_arenas():
    """The pipeline's three arena routes: direct DMA from a pinned arena,
    copy of a compact pageable span, and per-job repacking when the jobs of a
    chunk are scattered far apart in the arena."""
    from cap_amd import _lib
    keys, toks = H.golden()
    arena, want = _mixed_arena(keys, toks)
    L = _lib.lib()
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    ctx.set_chunk(512)
    n = len(arena.toks)
    ta = arena.tok_array()
    out = (ctypes.c_uint8 * n)()
    # pinned
    pa = _lib.PinnedBuffer(len(arena.buf))
    ctypes.memmove(pa.ptr, bytes(arena.buf), len(arena.buf))
    assert L.jg_verify_batch(ctx.h, pa.ptr, len(arena.buf), ta, n, out) == 0
    assert list(out) == want
    pa.free()
    # scattered: every job's bytes on its own 4 KiB page (span >> bytes needed)
    gap = 4096
    buf = bytearray()
    spread = (_lib.JgTok * n)()
    for i in range(n):
        t = ta[i]
        end = max(t.off + t.sig_in_len, t.off + t.sig_rel_off + t.sig_b64_len)
        buf += b"\0" * (gap - len(buf) % gap if len(buf) % gap else 0)
        spread[i] = t
        spread[i].off = len(buf)
        buf += bytes(arena.buf[t.off:end])
    out2 = (ctypes.c_uint8 * n)()
    assert L.jg_verify_batch(ctx.h, bytes(buf), len(buf), spread, n, out2) == 0
    assert list(out2) == want
    ctx.close()


def test_multi_device_split_on_two_slots():
    """A context with two device slots on the same GPU ({0, 0}): the batch is
    split by the cost model, each slot stages only its share's arena span
    (rebased), and the verdicts equal the oracle's -- the in-process
    multi-device path without a second GPU."""
    from cap_amd import _lib
    keys, toks = H.golden()
    arena, want = _mixed_arena(keys, toks, reps=3)
    ctx = _lib.Context([0, 0])
    ctx.load_keys([H.abi_key(k) for k in keys])
    assert list(ctx.verify(arena)) == want
    ctx.set_chunk(700)
    pend = [ctx.submit(arena) for _ in range(2)]
    for p in pend:
        assert list(p.wait()) == want
    # a key reload between batches reaches both slots
    order = keys[::-1]
    ctx.load_keys([H.abi_key(k) for k in order])
    kid_index = {k["kid"]: i for i, k in enumerate(order)}
    arena2, slots = H.jobs_from_tokens(toks, kid_index)
    out = ctx.verify(arena2)
    assert [0 if s is None else out[s] for s in slots] == [t["verdict"] for t in toks]
    ctx.close()


def _pinned_copy(arena, tail=0):
    """The arena's bytes in a PinnedBuffer sized exactly to them (+ `tail`
    spare bytes), so the last token ends at the block's end."""
    from cap_amd import _lib
    pa = _lib.PinnedBuffer(len(arena.buf) + tail)
    ctypes.memmove(pa.ptr, bytes(arena.buf), len(arena.buf))
    return pa


def test_zero_copy_class_major_plans():
    """Mixed batches from jg_host_alloc memory run as class-major zero-copy
    plans (jg_set_zero_copy: per class, k_zc_gather copies the class's token
    bytes from the pinned arena over PCIe into a per-key strided device arena,
    then the class's prep and arithmetic run on it): verdicts equal the
    oracle's and the chunked DMA path's -- whole-item plans,
    items cut into several plans, several submissions in flight across both
    zero-copy slots, the last token ending exactly at the block's end, and a
    two-slot context whose items each read their own share in place."""
    from cap_amd import _lib
    keys, toks = H.golden()
    arena, want = _mixed_arena(keys, toks, reps=2)
    L = _lib.lib()
    n = len(arena.toks)
    ta = arena.tok_array()
    for slots in ([0], [0, 0]):
        ctx = _lib.Context(slots)
        ctx.load_keys([H.abi_key(k) for k in keys])
        pa = _pinned_copy(arena)
        for zc, zmax in ((False, 0), (True, 1 << 21), (True, 640), (True, 64)):
            ctx.set_zero_copy(zc, zmax)
            out = (ctypes.c_uint8 * n)()
            assert L.jg_verify_batch(ctx.h, pa.ptr, len(arena.buf), ta, n, out) == 0
            assert list(out) == want, (slots, zc, zmax)
        # overlapping submissions (more than the two zero-copy slots in flight)
        ctx.set_zero_copy(True, 1000)
        outs, tickets = [], []
        for _ in range(5):
            o = (ctypes.c_uint8 * n)()
            t = ctypes.c_void_p()
            assert L.jg_submit(ctx.h, pa.ptr, len(arena.buf), ta, n, o, ctypes.byref(t)) == 0
            outs.append(o)
            tickets.append(t)
        for t, o in zip(tickets, outs):
            assert L.jg_wait(ctx.h, t) == 0
            assert list(o) == want
        pa.free()
        with pytest.raises(_lib.JgError):
            ctx.set_zero_copy(True, 8)
        ctx.close()


def test_zero_copy_only_inside_host_alloc_blocks():
    """An arena that is pinned but reaches past its jg_host_alloc block's
    usable bytes, or sits in pageable memory, takes the chunked path: the
    verdicts are the same either way (the prep kernels never read outside
    the caller's block plus its slack)."""
    from cap_amd import _lib
    keys, toks = H.golden()
    arena, want = _mixed_arena(keys, toks)
    L = _lib.lib()
    n = len(arena.toks)
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    ctx.set_zero_copy(True, 0)
    # arena at an offset inside a larger block, ending 1 byte before its end
    big = _lib.PinnedBuffer(len(arena.buf) + 4097)
    ctypes.memmove(big.ptr + 4096, bytes(arena.buf), len(arena.buf))
    ta = arena.tok_array()
    out = (ctypes.c_uint8 * n)()
    assert L.jg_verify_batch(ctx.h, big.ptr + 4096, len(arena.buf), ta, n, out) == 0
    assert list(out) == want
    # arena_len claims one byte past the block (not eligible; the spans are in bounds)
    out2 = (ctypes.c_uint8 * n)()
    assert L.jg_verify_batch(ctx.h, big.ptr + 4096, len(arena.buf) + 2, ta, n, out2) == 0
    assert list(out2) == want
    big.free()
    out3 = (ctypes.c_uint8 * n)()
    assert L.jg_verify_batch(ctx.h, bytes(arena.buf), len(arena.buf), ta, n, out3) == 0
    assert list(out3) == want
    ctx.close()


def test_zero_copy_gather_layout_edges():
    """k_zc_gather's layout edges: an arena base that is 16-byte
    but not 256-byte aligned inside a jg_host_alloc block, and the tokens of
    one key with different lengths, so that key's longest span sets its
    device stride -- the short tokens' slots carry slack, the long ones fill
    them exactly.  Verdicts == the oracle's and the chunked path's."""
    from cap_amd import _lib
    from oracle import jws
    keys, toks = H.golden()
    okeys = [jws.Key.from_fixture(k) for k in keys]
    L = _lib.lib()
    arena = _lib.Arena()
    want = []
    for t in toks:
        p = jws.parse_jws(t["token"])
        if p is None or not p.crit_ok:
            continue
        sig_b64 = jws.b64url_encode(p.signature).encode()
        for ki, k in enumerate(okeys):
            # each token twice: as signed, and with one more signing-input
            # byte (a reject) -- every key sees several span lengths
            arena.add(p.signing_input, sig_b64, p.alg, ki)
            want.append(int(jws.verify_sig(p, k)))
            arena.add(p.signing_input + b"A", sig_b64, p.alg, ki)
            # a reject, except where any message verifies (the golden set's
            # small-order Ed25519 key with S = 0): the oracle decides
            want.append(int(jws.verify_alg_sig(p.alg, k, p.signing_input + b"A", p.signature)))
    lens = {}
    for off, si, rel, sb, ki, alg in arena.toks:
        lens.setdefault(ki, set()).add(rel + sb)
    assert any(len(v) > 2 for v in lens.values())        # mixed lengths on one key
    n = len(arena.toks)
    ta = arena.tok_array()
    ctx = _lib.Context()
    ctx.load_keys([H.abi_key(k) for k in keys])
    big = _lib.PinnedBuffer(len(arena.buf) + 16 + 512)
    ctypes.memmove(big.ptr + 16, bytes(arena.buf), len(arena.buf))     # base == 16 (mod 256)
    for zc in (True, False):
        ctx.set_zero_copy(zc, 1 << 21)
        out = (ctypes.c_uint8 * n)()
        assert L.jg_verify_batch(ctx.h, big.ptr + 16, len(arena.buf), ta, n, out) == 0
        assert list(out) == want, zc
    big.free()
    ctx.close()
