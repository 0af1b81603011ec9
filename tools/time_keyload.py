"""Time engine creation and key loading (fixed-base table builds) on the GPU.

    python tools/time_keyload.py      (on the GPU box)

Prints one JSON line: jg_create seconds, then jg_keys_load seconds for the
bench key sets (ES256 x4, all 32 bench kids), each twice (the second load of
the same kids rebuilds the tables too: there is no cross-call table cache).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from cap_amd import _lib
    keys = bench.bench_keys()
    out = {}
    t = time.perf_counter()
    ctx = _lib.Context()
    out["create_s"] = time.perf_counter() - t
    es = [k[3] for k in keys if k[1] == "ES256"][:4]
    for name, ks in (("es256x4", es), ("all32", [k[3] for k in keys])):
        for rep in range(2):
            t = time.perf_counter()
            ctx.load_keys(ks)
            out[f"{name}_load_s_{rep}"] = time.perf_counter() - t
    print(json.dumps(out))


if __name__ == "__main__":
    main()
