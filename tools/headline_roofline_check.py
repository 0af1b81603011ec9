"""Recompute the headline rooflines of a bench line from rocprofv3 output:
the ES256 line's k_ec_point<P256> and the rs256 line's RSA-2048 modexp.
Each roofline carries the CLOCK_BOOTTIME `trace_window` of the synchronous
runs its HIP-event time comes from (bench.py measure()); the kernel-trace
launches of that kernel inside the window give

  rocprof ms per run = summed kernel-trace durations / runs
  rocprof frac       = bench frac x bench ms / rocprof ms   (same work per run)

and, when FETCH_SIZE / WRITE_SIZE passes are given, the HBM bytes per run
(2 x FETCH_SIZE + WRITE_SIZE, the guide's x2 FETCH correction on gfx950).
Input: a directory written by tools/gpu_profile_r04.sh (kt.json +
kt/*kernel_trace.csv; fetch.json + fetch/*counter_collection.csv and
write.json + write/... optional).

usage: python tools/headline_roofline_check.py gpurun_out/<tag> profiles/<out>.json
"""
import csv
import glob
import json
import os
import sys

SYMS = {"p256_point": "void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP256W<",
        "rsa2048_modexp": "void (anonymous namespace)::k_rsa_modexp<37, 2, 8>"}


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


def rows_of(d, pattern):
    hits = glob.glob(os.path.join(d, pattern))
    return list(csv.DictReader(open(hits[0]))) if len(hits) == 1 else None


def in_window(r, w):
    return w[0] <= int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= w[1]


def lines(b):
    """(mark, roofline dict, bench kernel ms) of the two headline rooflines."""
    out = [("p256_point", b["roofline"], b["kernel_ms"]["p256_point"])]
    if "rs256" in b:
        out.append(("rsa2048_modexp", b["rs256"]["roofline"], b["rs256"]["kernel_ms"]["rsa2048_modexp"]))
    return out


def main(d, out):
    kt = bench_line(os.path.join(d, "kt.json"))
    ktr = rows_of(d, "kt/*kernel_trace.csv")
    fe = rows_of(d, "fetch/*counter_collection.csv")
    wr = rows_of(d, "write/*counter_collection.csv")
    fej = bench_line(os.path.join(d, "fetch.json")) if fe else None
    wrj = bench_line(os.path.join(d, "write.json")) if wr else None
    res = {}
    for i, (mark, rl, bms) in enumerate(lines(kt)):
        w = rl.get("trace_window")
        if not w:
            continue
        hit = [r for r in ktr if r["Kernel_Name"].startswith(SYMS[mark]) and in_window(r, w["boottime_ns"])]
        ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in hit) * 1e-6 / w["runs"]
        e = {"bench_hip_event_ms": bms, "rocprof_ms_per_run": ms, "launches": len(hit), "runs": w["runs"],
             "launch_ms": [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in hit],
             "frac_bench": rl["frac"], "frac_rocprof": rl["frac"] * bms / ms if ms else None,
             "symbol": SYMS[mark]}
        for name, rows, j in (("FETCH_SIZE", fe, fej), ("WRITE_SIZE", wr, wrj)):
            if not rows:
                continue
            wj = lines(j)[i][1]["trace_window"]
            tot = sum(float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == name
                      and r["Kernel_Name"].startswith(SYMS[mark]) and in_window(r, wj["boottime_ns"]))
            e[name.lower() + "_kib_per_run"] = tot / wj["runs"]
        if "fetch_size_kib_per_run" in e and "write_size_kib_per_run" in e:
            e["hbm_bytes_per_run"] = (2 * e["fetch_size_kib_per_run"] + e["write_size_kib_per_run"]) * 1024
        res[mark] = e
        print(f"{mark:16s} bench {bms:.3f} ms / rocprof {ms:.3f} ms over {len(hit)} launches; frac bench "
              f"{rl['frac']:.3f} rocprof {e['frac_rocprof']:.3f}"
              + (f"; HBM {e['hbm_bytes_per_run'] / 1e9:.2f} GB per run" if "hbm_bytes_per_run" in e else ""))
    json.dump({"source": "tools/headline_roofline_check.py over " + d.rstrip("/"), "method": __doc__.split("\n\n")[0],
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
