"""Phase trace of JWKS key loads on the GPU box (CAPJWT_LOAD_TRACE=1 prints
jg_keys_load's phases):

1. a new-key rotation (bench.measure_refresh's load): the 32 bench kids loaded
   at the configs[4] budget, then the same set plus one new P-256 key;
2. the multi-slot load: the 32 kids loaded cold
   (no key table built yet) on a one-slot context and on a two-slot context of
   the same GPU, where the slots stage on their own threads and the second
   slot reuses the first's tables (jg_runtime.cpp per_device, phys_tables).

usage: python tools/keyload_trace.py"""
import json
import os
import sys
import time

os.environ["CAPJWT_LOAD_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed_load(ctx, keys, **kw):
    t = time.perf_counter()
    ctx.load_keys(keys, **kw)
    return (time.perf_counter() - t) * 1e3


def main():
    import bench
    from cap_amd import _lib
    from tests import gpu_helpers as H
    meta = bench.bench_keys()
    keys = [m[3] for m in meta]
    out = {}
    ctx = _lib.Context()
    ctx.set_table_budget(160 << 30)
    ms = timed_load(ctx, keys)
    print(f"first load (32 kids, waits for wide tables): {ms:.1f} ms", flush=True)
    gk, _ = H.golden()
    newk = next(k for k in gk if k["kid"] == "p256-a")
    ctx.set_table_budget(200 << 30)
    for rep in range(2):
        ms = timed_load(ctx, keys + [H.abi_key(newk)] if rep == 0 else keys, wait_tables=False)
        print(f"rotation {rep}: jg_keys_load {ms:.1f} ms, widths {ctx.table_widths()[-3:]}", flush=True)
        t = time.perf_counter()
        ctx.wait_tables()
        print(f"  wait_tables {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    ctx.close()
    # cold loads (every context closed before the next: no key table cached;
    # the generator tables are process-wide and already built above)
    for slots in ([0], [0, 0], [0], [0, 0]):
        c = _lib.Context(slots)
        ms = timed_load(c, keys, wait_tables=False)
        t = time.perf_counter()
        c.wait_tables()
        wide = (time.perf_counter() - t) * 1e3
        print(f"cold load on slots {slots}: jg_keys_load {ms:.1f} ms, wide tables after {wide:.1f} ms", flush=True)
        out.setdefault(str(len(slots)), []).append({"load_ms": ms, "wide_ms": wide})
        c.close()
    one = min(x["load_ms"] for x in out["1"])
    two = min(x["load_ms"] for x in out["2"])
    print(json.dumps({"multi_slot_load": out, "ratio_2_over_1": two / one}), flush=True)


if __name__ == "__main__":
    main()
