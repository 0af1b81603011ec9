"""configs[4]'s stream leg as bench.py builds it (bench.c5_pool: unique EC /
Ed25519 tokens, 5 % tampered, the 32 bench kids under bench.py's C5 table
budget), timed over several passes per chunk size: the A/B harness of the
pipeline's chunk scheduling (run once per CAPJWT_* setting).
usage: python tools/c5_stream_probe.py out.json [passes] [mode ...]
mode: a chunk size (chunked DMA pipeline, zero-copy plans off), or zN:
zero-copy class-major plans of at most N jobs (z0: the library default)"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out = sys.argv[1]
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    chunks = sys.argv[3:] or ["524288", "z0"]
    from cap_amd import _lib
    cpu = bench.cpu_info()
    ctx = _lib.Context([0])
    ctx.set_table_budget(int(160 * (1 << 30)))
    meta = bench.bench_keys()
    ctx.load_keys([m[3] for m in meta])
    pool, algs, keyidx, good = bench.c5_pool(meta, 10_000_000 // 8, cpu["cores_used"], 0)
    arena, toks = bench.pack(pool, algs, keyidx, len(pool))
    L = _lib.lib()
    pa = _lib.PinnedBuffer(len(arena))
    ctypes.memmove(pa.ptr, arena, len(arena))
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("CAPJWT_")}, "tokens": len(toks),
           "expected_accepted": int(np.asarray(good).sum()), "ms": {}}
    vout = (ctypes.c_uint8 * len(toks))()
    tp = toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok))
    for ch in chunks:
        if ch.startswith("z"):
            ctx.set_zero_copy(True, int(ch[1:]))
        else:
            ctx.set_zero_copy(False)
            ctx.set_chunk(int(ch))
        ms = []
        for _ in range(passes + 1):
            t0 = time.perf_counter()
            if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, len(toks), vout) != 0:
                raise RuntimeError(ctx.error())
            ms.append((time.perf_counter() - t0) * 1e3)
        acc = int(np.frombuffer(vout, dtype=np.uint8).sum())
        res["ms"][ch] = ms[1:]
        print(ch, "accepted", acc, "ms", [round(x, 1) for x in ms], "best M/s", round(len(toks) / min(ms[1:]) / 1e3, 1),
              flush=True)
        if acc != res["expected_accepted"]:
            raise RuntimeError(f"accepted {acc} != {res['expected_accepted']}")
    pa.free()
    ctx.close()
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
