"""Per-class device cost of one verification on MI355X, for the multi-device
cost model (jg_runtime.cpp cls_cost, cap_amd/shard.py ALG_COST; SURVEY §8e
"weighted by per-alg cost").  Each class runs alone as a resident batch large
enough to fill the chip; the cost is the summed kernel time of its chain
(prep + arithmetic + pad / finish) per token, relative to ES256.  RSA moduli
above 4096 bits (no private keys here) use tokens with random signature
values < n: the modexp and pad run in full and reject, which costs the same.

usage: python tools/class_costs.py out.json [label,label,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402

# (label, alg, golden kid or rsa_big kid, tokens per batch)
CASES = [("p256", "ES256", "p256-a", 1 << 20), ("ed25519", "EdDSA", "ed-a", 1 << 20),
         ("p384", "ES384", "p384-a", 1 << 19), ("p521", "ES512", "p521-a", 1 << 18),
         ("rsa2048", "RS256", "rsa2048-a", 1 << 19), ("rsa2048_pss", "PS256", "rsa2048-a", 1 << 19),
         ("rsa3072", "RS384", "rsa3072-a", 1 << 18), ("rsa4096", "RS512", "rsa4096-a", 1 << 17),
         ("rsa4096_pss", "PS512", "rsa4096-a", 1 << 17), ("rsa8192", "RS256", "big-8192", 1 << 15),
         ("rsa16384", "RS256", "big-16384", 1 << 13)]


def big_rsa_tokens(kid, count, template):
    """RS256-shaped tokens whose signature is a random value below the modulus
    of rsa_big.json's `kid` (the verify arithmetic runs in full and rejects)."""
    import base64
    d = next(k for k in json.load(open(os.path.join(ROOT, "tests", "golden", "rsa_big.json")))["keys"]
             if k["kid"] == kid)
    n = int(d["n"], 16)
    from cap_amd import _lib
    key = _lib.Key.rsa(n.to_bytes((n.bit_length() + 7) // 8, "big"), int(d["e"]))
    k = (n.bit_length() + 7) // 8
    rng = np.random.default_rng(7)
    si = template[:template.rfind(b".")]
    out = []
    for _ in range(count):
        s = int.from_bytes(rng.bytes(k), "big") % n
        out.append(si + b"." + base64.urlsafe_b64encode(s.to_bytes(k, "big")).rstrip(b"="))
    return key, out


def main(dst, only=None):
    from cap_amd import _lib
    th = bench.cpu_info()["cores_used"]
    ctx = _lib.Context([0])
    res = {}
    template = bench.gen_tokens("RS256", 1, bench.golden_keypaths(["rsa2048-a"]), 1, "cc")[0]
    for label, alg, kid, ntok in CASES:
        if only and label not in only and label != "p256":
            continue
        if kid.startswith("big-"):
            key, pool = big_rsa_tokens(kid, min(ntok, 4096), template)
            ctx.load_keys([key])
        else:
            ctx.load_keys(bench.abi_keys([kid]))
            pool = bench.gen_tokens(alg, min(ntok, 1 << 18), bench.golden_keypaths([kid]), th, "cc")
        arena, toks = bench.pack(pool, [bench.ALG_IDS[alg]] * len(pool), [0] * len(pool), ntok)
        el, acc, kms, _ = bench.measure(ctx, arena, toks, 6, 2, False)
        kern = sum(v for k, v in kms.items() if k != "scatter")
        res[label] = {"alg": alg, "key": kid, "tokens": ntok, "accepted": acc, "kernel_ms": kms,
                      "ns_per_token_kernels": kern * 1e6 / ntok, "ns_per_token_step": el / 6 * 1e9 / ntok}
        print(label, round(kern * 1e6 / ntok, 3), "ns/token", flush=True)
    base = res["p256"]["ns_per_token_kernels"]
    for v in res.values():
        v["cost_vs_es256"] = v["ns_per_token_kernels"] / base
    ctx.close()
    json.dump({"source": "tools/class_costs.py: each class alone as a resident batch filling the chip; summed "
                         "kernel time (HIP events) per token", "classes": res}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "class_costs.json",
         sys.argv[2].split(",") if len(sys.argv) > 2 else None)
