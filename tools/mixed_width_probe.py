"""Mixed comb widths inside one class (the window while the background
upgrader widens a class's keys one by one), made deterministic with
CAPJWT_DEBUG_MAX_UPGRADES: the 32 bench kids at the default table budget,
upgrades stopped after n, then the C5 pool's tokens of every class verified
through jg_verify_batch against the expected verdicts.
usage: CAPJWT_DEBUG_MAX_UPGRADES=n python tools/mixed_width_probe.py [chunk]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    from cap_amd import _lib
    cpu = bench.cpu_info()
    ctx = _lib.Context([0])
    meta = bench.bench_keys()
    ctx.load_keys([m[3] for m in meta])          # waits for the (limited) upgrades
    print("widths", ctx.table_widths(), flush=True)
    pool, algs, keyidx, good = bench.c5_pool(meta, 10_000_000 // 8, cpu["cores_used"], 0)
    arena, toks = bench.pack(pool, algs, keyidx, len(pool))
    L = _lib.lib()
    out = (ctypes.c_uint8 * len(toks))()
    ctx.set_chunk(chunk)
    want = np.asarray(good)
    for it in range(2):
        if L.jg_verify_batch(ctx.h, arena, len(arena), toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok)), len(toks),
                             out) != 0:
            raise RuntimeError(ctx.error())
        got = np.frombuffer(out, dtype=np.uint8).astype(bool)
        bad = np.nonzero(got != want)[0]
        print(f"pass {it}: mismatches {len(bad)}", [(int(j), int(algs[j]), int(keyidx[j]), bool(want[j])) for j in bad[:10]],
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
