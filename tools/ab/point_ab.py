"""A/B of a point kernel on a configs[3]-size launch: 1 M unique EdDSA (or,
with AB_ALG=ES384, ES384) tokens on one key (32 GiB budget: W = 24 tables),
per-kernel times of synchronous runs (bench.measure), one child process per
library variant (CAPJWT_LIB), the variants alternated 3 times.
usage: [AB_ALG=ES384|ES256|ES512] python tools/ab/ed_point_ab.py out.json name=lib.so [name=lib.so ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


ALGS = {"EdDSA": ("ed-a", "ed25519_point", "ed25519_point_mads_per_token"),
        "ES256": ("p256-a", "p256_point", "p256_point_mads_per_token"),
        "ES512": ("p521-a", "p521_point", "p521_point_mads_per_token"),
        "ES384": ("p384-a", "p384_point", "p384_point_mads_per_token")}


def child():
    import bench
    from cap_amd import _lib
    alg = os.environ.get("AB_ALG", "EdDSA")
    kid, mark, madf = ALGS[alg]
    n = int(os.environ.get("AB_N", 1 << 20))              # AB_N: tokens per launch
    pool = bench.gen_tokens(alg, n, bench.golden_keypaths([kid]), 16, "ab" + alg)
    ctx = _lib.Context()
    ctx.set_table_budget(32 << 30)
    ctx.load_keys(bench.abi_keys([kid]))
    w = ctx.table_widths()[0]
    arena, toks = bench.pack(pool, [bench.ALG_IDS[alg]] * n, [0] * n, n)
    el, acc, kms, _ = bench.measure(ctx, arena, toks, 6, 5, False)
    mads = getattr(bench, madf)(w) * n
    pt = kms[mark]
    print(json.dumps({"w": w, "accepted": acc, "value": n * 6 / el, "kernel_ms": kms, "mark": mark,
                      "frac": mads / (pt * 1e-3) / 1e12 / bench.MAD_PEAK_T}))


def main():
    if sys.argv[1] == "--child":
        return child()
    out, specs = sys.argv[1], [a.split("=", 1) for a in sys.argv[2:]]
    res = {}
    for rep in range(int(os.environ.get("AB_REPS", 3))):
        for name, lib in specs:
            env = dict(os.environ, CAPJWT_LIB=os.path.join(ROOT, lib))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                print(name, "FAILED", r.stderr[-1500:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(name, []).append(d)
            print(name, rep, d["accepted"], round(d["kernel_ms"][d["mark"]], 4), "frac", round(d["frac"], 4),
                  flush=True)
            json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
