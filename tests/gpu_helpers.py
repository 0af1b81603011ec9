"""Shared helpers for the GPU parity tests: golden fixtures -> C-ABI jobs."""
import json
import os

from cap_amd import _lib
from oracle import jws

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def abi_key(d):
    """tests/golden/keys.json entry -> _lib.Key"""
    if d["kty"] == "RSA":
        n = int(d["n"], 16)
        return _lib.Key.rsa(n.to_bytes((n.bit_length() + 7) // 8, "big"), int(d["e"]))
    if d["kty"] == "EC":
        sz = {"P-256": 32, "P-384": 48, "P-521": 66}[d["crv"]]
        return _lib.Key.ec(d["crv"], int(d["x"], 16).to_bytes(sz, "big"), int(d["y"], 16).to_bytes(sz, "big"))
    return _lib.Key.ed25519(bytes.fromhex(d["x"]))


def golden():
    d = os.path.join(ROOT, "tests", "golden")
    return json.load(open(os.path.join(d, "keys.json"))), json.load(open(os.path.join(d, "tokens.json")))


def jobs_from_tokens(tokens, kid_index):
    """Parse each token the way go-jose does (oracle restatement) and pack the
    signature job; tokens that fail to parse get no job (verdict 0 upstream)."""
    arena = _lib.Arena()
    slots = []
    parsed = {}                     # tiled fixtures repeat tokens: parse each once
    for t in tokens:
        if t["token"] not in parsed:
            p = jws.parse_jws(t["token"])
            parsed[t["token"]] = None if p is None or not p.crit_ok else \
                (p.signing_input, jws.b64url_encode(p.signature).encode(), p.alg)
        job = parsed[t["token"]]
        if job is None:
            slots.append(None)
            continue
        slots.append(arena.add(job[0], job[1], job[2], kid_index[t["key"]]))
    return arena, slots
