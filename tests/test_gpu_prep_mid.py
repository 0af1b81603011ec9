"""GPU parity of the prep kernel's shared block 0 (kernels/prep.hip k_prep_mid):
the first wave of each key run records its first token's SHA-256 block 0 and
midstate, and a wave whose every live lane has that same block starts from the
midstate.  Every case below is checked token by token against the oracle
(oracle/jws.py verify_sig), through the C ABI.

Each scenario is its own key run (the same key material loaded under several
key indices; the plan sorts jobs by key, keeping submission order inside a run):
  * all lanes share block 0 (the skip path) -- ES256 and RS256;
  * one lane of a wave tampered inside block 0 (that wave hashes normally);
  * the run's FIRST token tampered inside block 0, so the recorded block is the
    tampered one (the valid tokens mismatch it and hash normally);
  * a whole wave sharing one tampered block 0 (skip path from the tampered
    midstate: every token must still reject);
  * RS256 and PS512 interleaved under one RSA key (mixed SHA families)."""
import pytest

from oracle import jws

pytestmark = pytest.mark.gpu

ALPHA = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"


def _flip_block0(tok, pos=3):
    """flip one payload character inside the first 64 signing-input bytes"""
    h, p, s = tok.split(".")
    assert len(h) + 1 + pos < 64
    p = p[:pos] + ALPHA[ALPHA.index(p[pos]) ^ 1] + p[pos + 1:]
    return ".".join((h, p, s))


def test_shared_block0_midstate_vs_oracle():
    import bench
    from cap_amd import _lib
    meta = {m[0]: m for m in bench.bench_keys()}
    es_kid, rs_kid, ps_kid = "kid-20", "kid-00", "kid-17"
    es = [t.decode() for t in bench.gen_tokens("ES256", 320, [meta[es_kid][2]], 4, "midtest", kid_base=20)]
    rs = [t.decode() for t in bench.gen_tokens("RS256", 160, [meta[rs_kid][2]], 4, "midtest", kid_base=0)]
    # a PS512 token signed by the RS256 kid's key (same RSA key, other hash family)
    ps = [t.decode() for t in bench.gen_tokens("PS512", 32, [meta[rs_kid][2]], 4, "midtest", kid_base=0)]
    runs = []                                      # (key material kid, [tokens])
    runs.append((es_kid, es[0:192]))               # k0: 3 waves, all shared
    k1 = list(es[192:320])
    k1[70] = _flip_block0(k1[70])                  # k1: one mismatching lane in wave 1
    runs.append((es_kid, k1))
    k2 = [_flip_block0(es[0])] + es[1:128]         # k2: the recorded block is a tampered one
    runs.append((es_kid, k2))
    runs.append((es_kid, [_flip_block0(t) for t in es[128:192]]))   # k3: shared tampered block 0
    runs.append((rs_kid, rs[0:128]))               # k4: RSA class, all shared
    k5 = []
    for i in range(64):                            # k5: RS256 / PS512 interleaved
        k5.append(rs[128 + i % 32] if i % 2 == 0 else ps[i // 2])
    runs.append((rs_kid, k5))

    ctx = _lib.Context()
    try:
        ctx.load_keys([meta[kid][3] for kid, _ in runs])
        okeys = {kid: jws.jwk_decode(meta[kid][4]) for kid, _ in runs}
        arena = _lib.Arena()
        slots, want = [], []
        for ki, (kid, toks) in enumerate(runs):
            for t in toks:
                p = jws.parse_jws(t)
                assert p is not None and p.crit_ok
                slots.append(arena.add(p.signing_input, jws.b64url_encode(p.signature).encode(), p.alg, ki))
                want.append(int(jws.verify_sig(p, okeys[kid])))
        out = ctx.verify(arena)
        got = [out[s] for s in slots]
    finally:
        ctx.close()
    assert got == want
    # every scenario has both outcomes where it should
    assert sum(want[:192]) == 192 and want[192 + 70] == 0 and sum(want[192:320]) == 127
    assert want[320] == 0 and sum(want[320:448]) == 127
    assert sum(want[448:512]) == 0
    assert sum(want[512:640]) == 128 and sum(want[640:704]) == 64
