"""Print the headline fields of a bench.py JSON line (GPU-run summaries)."""
import json
import sys
d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json"))
print("es256 %.1f M/s  point %.3f ms frac %.3f" % (d["value"] / 1e6, d["kernel_ms"]["p256_point"], d["roofline"]["frac"]))
print("pcie", {k: (round(v / 1e6, 1) if k == "value" else v) for k, v in d["pcie"].items() if k in ("value", "ms_by_chunk", "raw_h2d_GBps", "h2d_bound")})
print("pool_ab", d.get("pool_ab", {}).get("value", 0) / 1e6, d.get("pool_ab", {}).get("kernel_ms", {}).get("p256_point"))
print("rs256 %.1f M/s frac %.3f" % (d["rs256"]["value"] / 1e6, d["rs256"]["roofline"]["frac"]))
for k, v in d["configs"].items():
    print(k, round(v["value"] / 1e6, 1), {a: round(b["frac"], 3) for a, b in v.get("roofline", {}).items()}, v.get("error"))
print("e2e %.2f M/s" % (d["e2e"]["value"] / 1e6), "cpu_baseline", d["cpu_baseline"]["value"], d["cpu_baseline"].get("label", "")[:20],
      "port", d.get("cpu_baseline_port", {}).get("value"), "openssl", {k: v["value"] for k, v in d.get("cpu_baseline_openssl", {}).items()})
if "cpu_baseline_rs256_port" in d:
    print("cpu rs256 port", d["cpu_baseline_rs256_port"]["value"])
for k, v in d.get("configs", {}).items():
    for sub in ("stream", "jwks_e2e", "refresh"):
        if sub in v:
            print(k, sub, {a: b for a, b in v[sub].items() if not isinstance(b, (dict, list, str))})
print("speedup", d["speedup_vs_cpu"])
e = d["e2e"]
fr = e.get("fresh_child", e.get("in_bench_process", {}))
print("e2e %.2f M/s (other process %.2f)" % (e["value"] / 1e6, fr.get("value", 0) / 1e6),
      "flt", {k: v for k, v in e.get("phases_ms_last_pass", {}).items() if "flt" in k})
if "single" in d:
    for c, r in d["single"]["by_callers"].items():
        print("single callers %5s: %.3f M/s p50 %.0f us p99 %.0f us mean batch %.1f %s" % (
            c, r["value"] / 1e6, r["p50_us"], r["p99_us"], r["mean_batch"], r.get("error", "")))
