"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; counter_collection.csv) -> profiles/*_pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md
(HBM section) FETCH_SIZE reports half the bytes of wide coalesced streaming
reads on gfx950; other access patterns are uncalibrated there, so the third
input calibrates the point kernel's own pattern: tools/ubench/gather_cal
(random 80-byte comb-table entries, 16-B aligned, 5 x dwordx4 per entry, a
7.97 GB table) and a 16-B/lane stream, each with a known requested byte count,
under rocprofv3 --pmc FETCH_SIZE.  Measured on MI355X: stream FETCH = 0.500 x
requested (the guide's x2), gather FETCH = 1.20 x requested = 96 B per 80-B
entry = half of the 1.5 128-B lines an entry touches on average -- so the x2
correction also gives line traffic for the gathers.  Only the launches of the
largest grid (the resident 1,048,576-token batch) are used; the bench's
pipelined chunks launch the same kernels on smaller grids.

usage: python tools/pmc_traffic.py fetch.csv write.csv cal.csv cal.json out.json
"""
import collections
import csv
import json
import sys

ALIASES = {  # bench.py mark name -> kernel symbol prefix
    "p256_point": "void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP256W<",
    "p256_prep": "void (anonymous namespace)::k_prep<4, ",
    "p256_scalar": "void (anonymous namespace)::k_ec_scalar_batch<(anonymous namespace)::CurveP256W<",
    "rsa2048_modexp": "void (anonymous namespace)::k_rsa_modexp<37, 2, 8>",
    "rsa2048_prep": "void (anonymous namespace)::k_prep<1, ",
    "rsa2048_pad": "(anonymous namespace)::k_rsa_pad",
}


def load(fn):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fn)):
        agg[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return agg


def biggest(agg, sym):
    ks = [k for k in agg if k[0].startswith(sym)]
    if not ks:
        return None, None
    k = max(ks, key=lambda k: k[1])
    v = agg[k]
    return k[1], (sum(v) / len(v) * 1024, len(v))


def calibration(cal_csv, cal_json):
    req = json.load(open(cal_json))
    agg = load(cal_csv)
    out = {}
    for (name, _), v in agg.items():
        for tag, key in (("gather", "gather_requested_bytes"), ("gather64", "gather64_requested_bytes"),
                         ("stream", "stream_requested_bytes")):
            if name.startswith("k_" + tag + "(") and key in req:
                out[tag] = {"fetch_bytes": sum(v) * 1024, "requested_bytes": req[key],
                            "fetch_per_requested_byte": sum(v) * 1024 / req[key]}
    out["gather"]["fetch_bytes_per_80B_entry"] = out["gather"]["fetch_per_requested_byte"] * 80
    if "gather64" in out:
        out["gather64"]["fetch_bytes_per_64B_entry"] = out["gather64"]["fetch_per_requested_byte"] * 64
    return out


def main(fetch_csv, write_csv, cal_csv, cal_json, out):
    f, w = load(fetch_csv), load(write_csv)
    res = {}
    for alias, sym in ALIASES.items():
        grid, fv = biggest(f, sym)
        _, wv = biggest(w, sym)
        if not fv or not wv:
            continue
        fetch, write = fv[0], wv[0]
        res[alias] = {"symbol": sym, "grid": grid, "launches": fv[1], "fetch_bytes_raw": fetch, "write_bytes": write,
                      "hbm_bytes_per_launch": 2 * fetch + write, "hbm_bytes_per_launch_undoubled": fetch + write}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes over a short bench.py run "
                         "(tools/gpu_profile_r03.sh; round 2: tools/gpu_profile_r02.sh)",
               "correction": "FETCH_SIZE x2: the guide's streaming-read calibration; `calibration` below measures "
                             "this repo's patterns with known byte counts (tools/ubench/gather_cal): streaming 0.5 "
                             "FETCH per requested byte, 80-B entries 1.2 (x2 = the 1.5 128-B lines an entry "
                             "touches), 64-B-aligned entries (P-256's packed tables since round 3) 1.0 (x2 = the "
                             "128-B line holding the entry)",
               "calibration": calibration(cal_csv, cal_json),
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:16s} grid {v['grid']:8d} fetch {v['fetch_bytes_raw'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:9.1f} MB")


if __name__ == "__main__":
    main(*sys.argv[1:6])
