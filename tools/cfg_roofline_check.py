"""Recompute bench.py's per-config roofline fractions from rocprofv3 output
(VERDICT r02 item 1): for every `configs.<name>.roofline.<mark>` of the bench
line, the launches of that mark's kernel(s) inside the config's
`trace_window` (bench.py measure(): CLOCK_BOOTTIME, the clock of rocprofv3's
timestamps, around the `runs` synchronous runs of the resident batch whose
HIP-event times bench.py's config rooflines use) give

  rocprof ms per run  = summed kernel-trace durations / runs
  rocprof frac        = bench frac x bench ms / rocprof ms   (same work per run)
  HBM bytes per run   = (2 x FETCH_SIZE + WRITE_SIZE) / runs  (the guide's x2
                        FETCH correction on gfx950, calibrated for this repo's
                        gather pattern in profiles/r02_s13_pmc_traffic.json)
  SQ split            = VALU-active / issue-stalled / parked share of wave
                        cycles (tools/sq_summary.py's definitions)

Inputs are the files tools/gpu_profile_cfg.sh writes under gpurun_out/<tag>:
bench.json (the un-profiled run whose fractions are checked), kt.json +
kt/*_kernel_trace.csv, fetch.json + fetch/*counter_collection.csv,
write.json + write/..., sq.json + sq/....  Each profiled pass is its own
process, so each is windowed by its own bench line.

usage: python tools/cfg_roofline_check.py gpurun_out/<tag> profiles/<out>.json
"""
import collections
import csv
import glob
import json
import os
import sys

# bench.py roofline mark -> kernel symbol prefixes (one mark may launch
# several instantiations, e.g. one per comb width, or the split kernels that
# launch_chain / launch_ed pick for launches of at most 16384 / 131072 tokens)
MARKS = {
    "p256_point": ["void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP256W<",
                   "void (anonymous namespace)::k_ec_point_split<(anonymous namespace)::CurveP256W<"],
    "p384_point": ["void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP384W<",
                   "void (anonymous namespace)::k_ec_point_split<(anonymous namespace)::CurveP384W<"],
    "p521_point": ["void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP521W<",
                   "void (anonymous namespace)::k_ec_point_split<(anonymous namespace)::CurveP521W<"],
    "ed25519_point": ["void (anonymous namespace)::k_ed_point<", "void (anonymous namespace)::k_ed_point_split<",
                      "void (anonymous namespace)::k_ed_point_pf<"],
    "ed25519_prep": ["(anonymous namespace)::k_prep_ed("],
    "ed25519_finish": ["(anonymous namespace)::k_ed_finish("],
    "p384_prep": ["void (anonymous namespace)::k_prep<4, "],
    "rsa2048_modexp": ["void (anonymous namespace)::k_rsa_modexp<37, 2, 8>"],
    "rsa3072_modexp": ["void (anonymous namespace)::k_rsa_modexp<56, 2, 8>", "void (anonymous namespace)::k_rsa_modexp<28, 4, 8>"],
    "rsa4096_modexp": ["void (anonymous namespace)::k_rsa_modexp<37, 4, 8>"],
    "rsa4096_prep": ["void (anonymous namespace)::k_prep<1, ", "(anonymous namespace)::k_prep_mid("],
    "rsa4096_pad": ["void (anonymous namespace)::k_rsa_pad<"],
}
# marks reported beside the roofline ones (no roofline in bench.py)
EXTRA = {"eddsa_es384_mixed": ["ed25519_finish"], "ps512_rsa4096": ["rsa4096_pad"]}


def bench_line(path):
    """The bench result of a run's stdout file: the full result from the
    line's `detail` file (bench.py since round 6: the stdout line is compact),
    looked up beside `path` first, or the line itself."""
    with open(path) as f:
        line = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    det = line.get("detail")
    if det:
        for cand in (os.path.join(os.path.dirname(path), os.path.basename(det)), det):
            if os.path.exists(cand):
                return json.load(open(cand))
    return line


def one_csv(d, pattern):
    hits = glob.glob(os.path.join(d, pattern))
    if len(hits) != 1:
        raise SystemExit(f"expected one {pattern} under {d}, found {hits}")
    return hits[0]


def matches(name, mark):
    return any(name.startswith(p) for p in MARKS[mark])


def in_window(r, w):
    return w[0] <= int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= w[1]


def trace_ms(rows, window, mark):
    hit = [r for r in rows if matches(r["Kernel_Name"], mark) and in_window(r, window["boottime_ns"])]
    total = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in hit) * 1e-6
    return total / window["runs"], len(hit)


def counter_sum(rows, window, mark, counter):
    vals = collections.defaultdict(float)
    for r in rows:
        if r["Counter_Name"] == counter and matches(r["Kernel_Name"], mark) and in_window(r, window["boottime_ns"]):
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / window["runs"], len(vals)


def sq_split(rows, window, mark):
    c = collections.defaultdict(float)
    for r in rows:
        if matches(r["Kernel_Name"], mark) and in_window(r, window["boottime_ns"]):
            c[r["Counter_Name"]] += float(r["Counter_Value"])
    if not c.get("SQ_WAVE_CYCLES"):
        return None
    wc = c["SQ_WAVE_CYCLES"]
    return {"valu_active": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "issue_stalled": c.get("SQ_WAIT_INST_ANY", 0) / wc,
            "parked": c.get("SQ_WAIT_ANY", 0) / wc,
            "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / max(1.0, c.get("SQ_WAVES", 1))}


def main(d, out):
    kt = bench_line(os.path.join(d, "kt.json"))["configs"]
    # bench.json: an un-profiled run; without one the traced run's own HIP-event
    # fractions are checked.  No counter passes: trace only.
    bp = os.path.join(d, "bench.json")
    bench = bench_line(bp)["configs"] if os.path.exists(bp) else kt
    counters = os.path.exists(os.path.join(d, "fetch.json"))
    kt_rows = list(csv.DictReader(open(one_csv(d, "kt/*kernel_trace.csv"))))
    if counters:
        fe = bench_line(os.path.join(d, "fetch.json"))["configs"]
        wr = bench_line(os.path.join(d, "write.json"))["configs"]
        sq = bench_line(os.path.join(d, "sq.json"))["configs"]
        fe_rows = list(csv.DictReader(open(one_csv(d, "fetch/*counter_collection.csv"))))
        wr_rows = list(csv.DictReader(open(one_csv(d, "write/*counter_collection.csv"))))
        sq_rows = list(csv.DictReader(open(one_csv(d, "sq/*counter_collection.csv"))))
    res = {}
    for cfg, line in bench.items():
        marks = list(line.get("roofline", {})) + EXTRA.get(cfg, [])
        rc = {}
        for mark in marks:
            if mark not in MARKS or mark not in line["kernel_ms"]:
                continue
            ms, n = trace_ms(kt_rows, kt[cfg]["trace_window"], mark)
            e = {"bench_ms": line["kernel_ms"][mark], "rocprof_ms_per_run": ms, "launches": n,
                 "runs": kt[cfg]["trace_window"]["runs"], "symbols": MARKS[mark]}
            rl = line.get("roofline", {}).get(mark)
            if rl and ms > 0:
                e.update({"bench_frac": rl["frac"], "rocprof_frac": rl["frac"] * line["kernel_ms"][mark] / ms,
                          "bound": rl["bound"], "unit": rl["unit"]})
                e["agree"] = abs(e["rocprof_frac"] / rl["frac"] - 1) <= 0.10
            if not counters:
                rc[mark] = e
                continue
            f, nf = counter_sum(fe_rows, fe[cfg]["trace_window"], mark, "FETCH_SIZE")
            w, nw = counter_sum(wr_rows, wr[cfg]["trace_window"], mark, "WRITE_SIZE")
            e["hbm_bytes_per_run"] = (2 * f + w) * 1024          # FETCH/WRITE_SIZE are KiB
            e["fetch_kib_raw_per_run"], e["write_kib_per_run"] = f, w
            if rl and rl["bound"] == "hbm" and ms > 0:
                e["hbm_frac_by_counters"] = e["hbm_bytes_per_run"] / (ms * 1e-3) / (rl["peak"] * 1e9)
            e["sq"] = sq_split(sq_rows, sq[cfg]["trace_window"], mark)
            rc[mark] = e
        res[cfg] = rc
    json.dump({"source": "tools/cfg_roofline_check.py over " + d.rstrip("/") + " (tools/gpu_profile_cfg.sh)",
               "method": __doc__.split("\n\n")[0], "configs": res}, open(out, "w"), indent=1)
    for cfg, rc in res.items():
        for mark, e in rc.items():
            fr = (f"frac bench {e['bench_frac']:.3f} rocprof {e['rocprof_frac']:.3f}" if "bench_frac" in e
                  else "(no roofline)")
            sqs = e.get("sq") or {}
            print(f"{cfg:18s} {mark:16s} ms {e['bench_ms']:.3f}/{e['rocprof_ms_per_run']:.3f} {fr}  "
                  f"hbm {e.get('hbm_bytes_per_run', 0) / 1e6:8.1f} MB  valu {sqs.get('valu_active', 0):.2f} "
                  f"stall {sqs.get('issue_stalled', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
