"""The coalesced single-token path (bench.py `single`) under several
coalescer settings: Validator.Validate per token from N C++ threads on the
configs[1] pool, per (max_inflight, window_us) and N.
usage: python tools/single_probe.py [out.json] [inflight,window ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    settings = [tuple(int(x) for x in s.split(",")) for s in sys.argv[2:]] or [(4, 0), (2, 0), (8, 0), (4, 100)]
    from cap_amd import jwt
    cpu = bench.cpu_info()
    kids = ["p256-a", "p256-b", "p256-c", "p256-d"]
    # PROBE_POOL_N / PROBE_TOTAL: pool size and calls per point (the bench's
    # single line: 262144 unique tokens, each called once)
    pool = bench.gen_tokens("ES256", int(os.environ.get("PROBE_POOL_N", 1 << 16)), bench.golden_keypaths(kids),
                            cpu["cores_used"], "single")
    total = int(os.environ.get("PROBE_TOTAL", 1 << 17))
    jwk = [{"kty": "EC", "kid": f"kid-{i:02d}", "crv": "P-256", **xy} for i, xy in enumerate(bench.p256_jwk_xy(kids))]
    jwks = json.dumps({"keys": jwk}).encode()
    # PROBE_DEVICES: the key set's device slots ("0,0": two submission pipelines on one GPU)
    devs = [int(x) for x in os.environ.get("PROBE_DEVICES", "").split(",") if x]
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                   lambda url, ca: {"status": 200, "body": jwks, "max_age": 3600}, devices=devs)
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=["ES256"],
                     Now=lambda: 1611699344 + 60)
    blob = b"\n".join(pool)
    pre = os.environ.get("PROBE_PRE")        # "e2e": a 1M-token ValidateBatch on another key set first (the bench's order);
    #                                          "headline": the bench's headline context (W = 26 tables) first, closed
    keep = None
    if pre == "e2e":
        ks2, _ = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                      lambda url, ca: {"status": 200, "body": jwks, "max_age": 3600})
        v2, _ = jwt.NewValidator(ks2)
        big = b"\n".join((pool * 16)[:1 << 20])
        v2.ValidateBlob(big[:1 << 20], e)
        ks2.WaitTables()
        for _ in range(2):
            v2.ValidateBlob(big, e)
        keep = (ks2, v2) if os.environ.get("PROBE_PRE_KEEP") else None
        del big, v2, ks2
    if pre == "headline":
        # the bench's headline leg first: the 4 kids' W = 26 tables under a
        # 110 GiB budget (~86 GB), a 1 M-token batch, then the context closed
        import ctypes
        from cap_amd import _lib
        ctx = _lib.Context()
        ctx.set_table_budget(110 << 30)
        ctx.load_keys(bench.abi_keys(kids))
        ctx.wait_tables()
        big = (pool * 16)[:1 << 20]
        arena, toks = bench.pack(big, [bench.ALG_IDS["ES256"]] * len(big), [i % 4 for i in range(len(big))], len(big))
        out_v = (ctypes.c_uint8 * len(toks))()
        L = _lib.lib()
        for _ in range(3):
            assert L.jg_verify_batch(ctx.h, ctypes.c_char_p(arena), len(arena), toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok)),
                                     len(toks), out_v) == 0, ctx.error()
        ctx.close()
        del arena, toks, big
    v.ValidateBlob(blob, e)
    ks.WaitTables()
    res = {"cpu": cpu, "pre": pre, "runs": []}
    for inflight, window in settings:
        ks.SetCoalescing(max_inflight=inflight, window_us=window)
        callers = os.environ.get("PROBE_CALLERS")
        for c in ([int(x) for x in callers.split(",")] if callers else (cpu["cores_used"], 64, 256, 1024)):
            v._impl._concurrent_validate(blob, e._native(), c, 1 << 14)
            s0 = ks.CoalescingStats()
            h0 = bench.host_snapshot()
            r = dict(v._impl._concurrent_validate(blob, e._native(), c, total))
            hd = bench.host_delta(h0, bench.host_snapshot())
            s1 = ks.CoalescingStats()
            r["host"] = {k: hd[k] for k in ("utime", "stime", "minflt", "nvcsw", "nivcsw", "cg_nr_throttled", "cg_throttled_usec",
                                           "cpu_by_thread_name")}
            r.update(inflight=inflight, window_us=window, callers=c, value=r["calls"] / r["wall_s"],
                     mean_batch=r["calls"] / max(1, s1["batches"] - s0["batches"]))
            res["runs"].append(r)
            print(f"inflight {inflight} window {window} callers {c}: {r['value'] / 1e6:.3f} M/s p50 {r['p50_us']:.0f} "
                  f"p99 {r['p99_us']:.0f} us, mean batch {r['mean_batch']:.1f}, accepted {r['accepted']}/{r['calls']}; "
                  f"cpu {r['host']['utime']:.2f}u {r['host']['stime']:.2f}s throttled {r['host']['cg_throttled_usec'] / 1e3:.0f} ms minflt {r['host']['minflt']} "
                  f"cs {r['host']['nvcsw']}/{r['host']['nivcsw']} "
                  f"top {list(r['host']['cpu_by_thread_name'].items())[:3]}",
                  flush=True)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
