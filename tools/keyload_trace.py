"""Phase trace of a JWKS key rotation on the GPU box (bench.measure_refresh's
new-key load): the 32 bench kids loaded at the configs[4] budget, then the
same set plus one new P-256 key, with CAPJWT_LOAD_TRACE=1 printing
jg_keys_load's phases.  usage: python tools/keyload_trace.py"""
import os
import sys
import time

os.environ["CAPJWT_LOAD_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from cap_amd import _lib
    from tests import gpu_helpers as H
    meta = bench.bench_keys()
    keys = [m[3] for m in meta]
    ctx = _lib.Context()
    ctx.set_table_budget(160 << 30)
    t = time.perf_counter()
    ctx.load_keys(keys)
    print(f"first load (32 kids, waits for wide tables): {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    gk, _ = H.golden()
    newk = next(k for k in gk if k["kid"] == "p256-a")
    ctx.set_table_budget(200 << 30)
    for rep in range(2):
        t = time.perf_counter()
        ctx.load_keys(keys + [H.abi_key(newk)] if rep == 0 else keys, wait_tables=False)
        print(f"rotation {rep}: jg_keys_load {(time.perf_counter() - t) * 1e3:.1f} ms, widths {ctx.table_widths()[-3:]}",
              flush=True)
        t = time.perf_counter()
        ctx.wait_tables()
        print(f"  wait_tables {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
