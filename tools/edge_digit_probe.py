"""Verify tests/golden/edge_digit_tokens.json (valid ES384 / ES512 tokens whose
comb digits hit -2^(W-1)) through the C ABI with the 32 bench kids loaded
under bench.py's C5 table budget, printing each verdict."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    from cap_amd import _lib
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "edge_digit_tokens.json")))
    meta = bench.bench_keys()
    kid_index = {m[0]: i for i, m in enumerate(meta)}
    for budget in (160, 32):
        ctx = _lib.Context()
        ctx.set_table_budget(budget << 30)
        ctx.load_keys([m[3] for m in meta])
        w = ctx.table_widths()
        for s in d["sets"]:
            arena = _lib.Arena()
            for t in s["tokens"]:
                b = t.encode()
                dot = b.rfind(b".")
                arena.add(b[:dot], b[dot + 1:], s["alg"], kid_index[s["kid"]])
            out = ctx.verify(arena)
            print(f"budget {budget} GiB {s['alg']} key W {w[kid_index[s['kid']]]}: verdicts {list(out)[:len(s['tokens'])]} "
                  f"hits {s['hits']}", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
