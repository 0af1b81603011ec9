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
print("e2e %.2f M/s" % (d["e2e"]["value"] / 1e6), "cpu port", d["cpu_baseline"]["value"], "openssl", {k: v["value"] for k, v in d["cpu_baseline_openssl"].items()})
print("cpu rs256 port", d["cpu_baseline_rs256"]["value"], d["cpu_baseline_rs256"]["sample"][:80])
print("speedup", d["speedup_vs_cpu"])
