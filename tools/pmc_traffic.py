"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; counter_collection.csv) -> profiles/*_pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md
(HBM section) FETCH_SIZE reports half the bytes of wide coalesced streaming
reads on gfx950, so it is doubled here; WRITE_SIZE is taken as is.  The gathers
of these kernels are not wide streaming reads, so the doubled figure is an
upper estimate (the undoubled one is kept beside it).

usage: python tools/pmc_traffic.py fetch.csv write.csv out.json
"""
import collections
import csv
import json
import sys

ALIASES = {  # bench.py mark name -> kernel symbol prefix
    "p256_point": "void (anonymous namespace)::k_ec_point<(anonymous namespace)::CurveP256>",
    "p256_prep": "void (anonymous namespace)::k_prep<4, ",
    "p256_scalar": "void (anonymous namespace)::k_ec_scalar_batch<(anonymous namespace)::CurveP256>",
    "rsa2048_modexp": "void (anonymous namespace)::k_rsa_modexp<37, 2, 8>",
    "rsa2048_prep": "void (anonymous namespace)::k_prep<1, ",
    "rsa2048_pad": "(anonymous namespace)::k_rsa_pad",
}


def load(fn):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fn)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(fetch_csv, write_csv, out):
    f, w = load(fetch_csv), load(write_csv)
    res = {}
    for alias, sym in ALIASES.items():
        fk = [v for k, v in f.items() if k.startswith(sym)]
        wk = [v for k, v in w.items() if k.startswith(sym)]
        if not fk or not wk:
            continue
        fetch = sum(fk[0]) / len(fk[0]) * 1024
        write = sum(wk[0]) / len(wk[0]) * 1024
        res[alias] = {"symbol": sym, "launches": len(fk[0]), "fetch_bytes_raw": fetch, "write_bytes": write,
                      "hbm_bytes_per_launch": 2 * fetch + write, "hbm_bytes_per_launch_undoubled": fetch + write}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes over "
                         "`bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-configs` (tools/gpu_profile.sh)",
               "correction": "FETCH_SIZE x2 (gfx950 streaming-read calibration, MI355X_MICROARCH.md HBM section)",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:16s} fetch {v['fetch_bytes_raw'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:9.1f} MB")


if __name__ == "__main__":
    main(*sys.argv[1:4])
