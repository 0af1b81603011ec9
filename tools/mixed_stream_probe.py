"""The configs[4] stream leg alone (all 10 algs, 32 kids, 5 % tampered,
1.25 M tokens through jg_verify_batch from pinned memory), for tracing the
pipeline under rocprofv3.  usage: python tools/mixed_stream_probe.py [chunk]"""
import ctypes
import os
import sys
import time

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
    ctx.load_keys([m[3] for m in meta])
    pool, algs, keyidx = [], [], []
    for ki, (kid, alg, pem, _, _) in enumerate(meta):
        n = 512 if alg in ("RS512", "PS512") else 1024
        toks = bench.gen_tokens(alg, n, [pem], cpu["cores_used"], "msp", kid_base=ki)
        pool += toks
        algs += [bench.ALG_IDS[alg]] * n
        keyidx += [ki] * n
    order = np.random.default_rng(1).permutation(len(pool))
    pool = [pool[i] for i in order]
    algs = [algs[i] for i in order]
    keyidx = [keyidx[i] for i in order]
    pool, algs, keyidx, good = bench.tamper(pool, algs, keyidx, meta, 0.05)
    arena, toks = bench.pack(pool, algs, keyidx, 10_000_000 // 8)
    L = _lib.lib()
    pa = _lib.PinnedBuffer(len(arena))
    ctypes.memmove(pa.ptr, arena, len(arena))
    out = (ctypes.c_uint8 * len(toks))()
    tp = toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok))
    ctx.set_chunk(chunk)
    for it in range(3):
        t0 = time.perf_counter()
        if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, len(toks), out) != 0:
            raise RuntimeError(ctx.error())
        print(f"chunk {chunk}: {1e3 * (time.perf_counter() - t0):.1f} ms, accepted {sum(out)}", flush=True)
    pa.free()
    ctx.close()


if __name__ == "__main__":
    main()
