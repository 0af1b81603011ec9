"""A/B of the Ed25519 point kernel on a configs[3]-size launch: 1 M unique
EdDSA tokens (one key, W = 24 tables), per-kernel times of synchronous runs
(bench.measure), one child process per library variant (CAPJWT_LIB), the
variants alternated `reps` times.
usage: python tools/ab/ed_point_ab.py out.json name=lib.so [name=lib.so ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child():
    import bench
    from cap_amd import _lib
    n = 1 << 20
    pool = bench.gen_tokens("EdDSA", n, bench.golden_keypaths(["ed-a"]), 16, "edab")
    ctx = _lib.Context()
    ctx.set_table_budget(32 << 30)
    ctx.load_keys(bench.abi_keys(["ed-a"]))
    w = ctx.table_widths()[0]
    arena, toks = bench.pack(pool, [bench.ALG_IDS["EdDSA"]] * n, [0] * n, n)
    el, acc, kms, _ = bench.measure(ctx, arena, toks, 6, 5, False)
    mads = bench.ed25519_point_mads_per_token(w) * n
    pt = kms["ed25519_point"]
    print(json.dumps({"w": w, "accepted": acc, "value": n * 6 / el, "kernel_ms": kms,
                      "frac": mads / (pt * 1e-3) / 1e12 / bench.MAD_PEAK_T}))


def main():
    if sys.argv[1] == "--child":
        return child()
    out, specs = sys.argv[1], [a.split("=", 1) for a in sys.argv[2:]]
    res = {}
    for rep in range(3):
        for name, lib in specs:
            env = dict(os.environ, CAPJWT_LIB=os.path.join(ROOT, lib))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                print(name, "FAILED", r.stderr[-1500:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(name, []).append(d)
            print(name, rep, d["accepted"], round(d["kernel_ms"]["ed25519_point"], 4), "frac", round(d["frac"], 4),
                  flush=True)
            json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
