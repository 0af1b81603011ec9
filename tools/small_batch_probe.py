"""Latency of small jg_verify_batch calls (the coalesced single-token path's
device round trip): ES256 tokens of the 4 bench kids, batch sizes 1 ... 4096,
pinned host arena, p50 / p90 of many calls per size; optionally several
threads submitting concurrently (pipelining on the device worker).
usage: python tools/small_batch_probe.py [out.json] [threads] [ES256|ES384|ES512|EdDSA|RS256|PS256]
(SBP_SIZES=1,64 picks the batch sizes)"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    nthr = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    from cap_amd import _lib
    L = _lib.lib()
    alg = sys.argv[3] if len(sys.argv) > 3 else "ES256"
    kids = {"EdDSA": ["ed-a"], "RS256": ["rsa2048-a", "rsa2048-b"], "PS256": ["rsa2048-a", "rsa2048-b"],
            "ES384": ["p384-a"], "ES512": ["p521-a"]}.get(alg, ["p256-a", "p256-b", "p256-c", "p256-d"])
    ctx = _lib.Context()
    ctx.load_keys(bench.abi_keys(kids))
    ctx.wait_tables()
    pool = bench.gen_tokens(alg, 8192, bench.golden_keypaths(kids), 8, "sbp")
    arena, toks = bench.pack(pool, [bench.ALG_IDS[alg]] * len(pool), np.arange(len(pool)) % len(kids), len(pool))
    pa = _lib.PinnedBuffer(len(arena))
    ctypes.memmove(pa.ptr, arena, len(arena))
    res = {"threads": nthr, "sizes": {}}
    sizes = [int(x) for x in os.environ.get("SBP_SIZES", "1,8,64,256,1024,4096").split(",")]
    for n in sizes:
        reps = 400 if n <= 256 else 100
        lat = [[] for _ in range(nthr)]

        def worker(t):
            vout = (ctypes.c_uint8 * n)()
            for r in range(reps):
                lo = ((r * nthr + t) * n) % (len(toks) - n)
                tp = toks[lo:lo + n].ctypes.data_as(ctypes.POINTER(_lib.JgTok))
                t0 = time.perf_counter()
                if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, n, vout) != 0:
                    raise RuntimeError(ctx.error())
                lat[t].append((time.perf_counter() - t0) * 1e6)
                if sum(vout) != n:
                    raise RuntimeError(f"accepted {sum(vout)} of {n}")
        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthr)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        a = np.sort(np.concatenate([np.asarray(x[10:]) for x in lat]))
        res["sizes"][n] = {"p50_us": float(np.percentile(a, 50)), "p90_us": float(np.percentile(a, 90)),
                           "min_us": float(a[0]), "tokens_per_s": n * reps * nthr / wall}
        print(n, {k: round(v, 1) for k, v in res["sizes"][n].items()}, flush=True)
    pa.free()
    ctx.close()
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
