"""Run the golden vectors through the GPU and print every mismatch."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cap_amd import _lib
from tests import gpu_helpers as H
keys, toks = H.golden()
kid_index = {k["kid"]: i for i, k in enumerate(keys)}
ctx = _lib.Context()
ctx.load_keys([H.abi_key(k) for k in keys])
arena, slots = H.jobs_from_tokens(toks, kid_index)
out = ctx.verify(arena)
bad = 0
by = {}
for t, s in zip(toks, slots):
    got = 0 if s is None else out[s]
    ok = got == t["verdict"]
    by.setdefault(t["alg"], [0, 0])[0 if ok else 1] += 1
    if not ok:
        bad += 1
        print("MISMATCH", t["name"], "gpu", got, "want", t["verdict"], t["source"])
print("per-alg [ok, bad]:", by)
print("mismatches:", bad, "of", len(toks))
