import sys, os, ctypes, time
sys.path.insert(0, os.getcwd())
import numpy as np
import bench
from cap_amd import _lib
ctx = _lib.Context([0])
kids = ["p256-a", "p256-b", "p256-c", "p256-d"]
ctx.load_keys(bench.abi_keys(kids))
pool = bench.gen_tokens("ES256", 1 << 15, bench.golden_keypaths(kids), 16, "pp")
arena, toks = bench.pack(pool, [7] * len(pool), np.arange(len(pool)) % 4, 1 << 20)
L = _lib.lib()
pa = _lib.PinnedBuffer(len(arena)); ctypes.memmove(pa.ptr, arena, len(arena))
out = (ctypes.c_uint8 * len(toks))()
tp = toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok))
for ch in [int(x) for x in sys.argv[1:]]:
    ctx.set_chunk(ch)
    for it in range(3):
        t0 = time.perf_counter()
        assert L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, len(toks), out) == 0
        print(f"chunk {ch} iter {it}: {1e3*(time.perf_counter()-t0):.2f} ms, accepted {sum(out)}", file=sys.stderr, flush=True)
