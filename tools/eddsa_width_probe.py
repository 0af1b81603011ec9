"""configs[3] (EdDSA + ES384, 1 M unique tokens) at several key-table
budgets: is a narrower comb tier (fewer, smaller tables: fewer TLB / cache
misses per entry, more additions per token) faster in absolute time than the
widest one the default budget gives?  Prints widths, batch rate and the
point kernels' ms per budget.
usage: python tools/eddsa_width_probe.py [out.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    from cap_amd import _lib
    ctx = _lib.Context()
    n = 1 << 19
    pe = bench.gen_tokens("EdDSA", n, bench.golden_keypaths(["ed-a"]), 16, "wp")
    p3 = bench.gen_tokens("ES384", n, bench.golden_keypaths(["p384-a"]), 16, "wp", kid_base=1)
    pool = [t for pair in zip(pe, p3) for t in pair]
    algs = [bench.ALG_IDS["EdDSA"], bench.ALG_IDS["ES384"]] * len(pe)
    res = []
    for gb in (110, 24, 12, 6, 3):
        ctx.set_table_budget(int(gb * (1 << 30)))
        ctx.load_keys(bench.abi_keys(["ed-a", "p384-a"]))
        w = ctx.table_widths()
        kern = {"p384_point": bench.p384_point_mads_per_token(w[1]),
                "ed25519_point": bench.ed25519_point_mads_per_token(w[0])}
        line = bench.config_line(ctx, "eddsa_es384_mixed", "width probe", pool, algs, [0, 1] * len(pe),
                                 bench.np.ones(len(pool), bool), 1 << 20, 5, 1, False, 1, kernels=kern)
        r = {"budget_GiB": gb, "widths": w, "value": line["value"],
             "p384_point_ms": line["kernel_ms"]["p384_point"], "ed25519_point_ms": line["kernel_ms"]["ed25519_point"],
             "frac": {k: v["frac"] for k, v in line["roofline"].items()}}
        print(json.dumps(r), flush=True)
        res.append(r)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
