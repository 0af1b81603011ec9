# round-2 full check: GPU parity suite, then the benchmark (all legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("es256 %.1f M/s  point %.3f ms frac %.3f" % (d["value"] / 1e6, d["kernel_ms"]["p256_point"], d["roofline"]["frac"]))
print("pcie", {k: (round(v / 1e6, 1) if k == "value" else v) for k, v in d["pcie"].items() if k in ("value", "ms_by_chunk", "raw_h2d_GBps", "h2d_bound")})
print("pool_ab", d.get("pool_ab", {}).get("value", 0) / 1e6, d.get("pool_ab", {}).get("kernel_ms", {}).get("p256_point"))
print("rs256 %.1f M/s frac %.3f" % (d["rs256"]["value"] / 1e6, d["rs256"]["roofline"]["frac"]))
for k, v in d["configs"].items():
    print(k, round(v["value"] / 1e6, 1), {a: round(b["frac"], 3) for a, b in v.get("roofline", {}).items()}, v.get("error"))
print("e2e %.2f M/s" % (d["e2e"]["value"] / 1e6), "cpu port", d["cpu_baseline"]["value"], "openssl", {k: v["value"] for k, v in d["cpu_baseline_openssl"].items()})
print("cpu rs256 port", d["cpu_baseline_rs256"]["value"], d["cpu_baseline_rs256"]["sample"][:80])
print("speedup", d["speedup_vs_cpu"])
PY
