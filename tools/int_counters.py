"""Summarise the integer-instruction / LDS counter passes (tools/gpu_pmc_int.sh)
per kernel: SQ_INSTS_VALU_INT32 / _INT64 share of SQ_INSTS_VALU,
instructions per wave, LDS instructions and SQ_LDS_BANK_CONFLICT as a fraction
of SQ_LDS_IDX_ACTIVE (the guide: conflict = extra LDS cycles, IDX_ACTIVE = all
LDS-array cycles).  Only launches of the verification kernels on batches of
>= 2^17 padded jobs are kept (table builds and small probes are excluded).
usage: python tools/int_counters.py out.json csv [csv ...]"""
import collections
import csv
import json
import re
import sys

KEEP = re.compile(r"k_prep|k_ec_point|k_ec_scalar|k_ed_point|k_ed_finish|k_rsa_modexp|k_rsa_pad|k_prep_ed")


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(PrepArgs\)|\(RsaArgs\)|\(EcArgs\)|\(EdArgs\)", "", name)
    return name.replace("void ", "").strip()


def main(out, files):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not KEEP.search(k) or int(r["Grid_Size"]) < (1 << 17):
                continue
            s = short(k)
            agg[s][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[s].add((f, r["Dispatch_Id"]))
    res = {}
    for s, c in sorted(agg.items()):
        waves = c.get("SQ_WAVES", 0) or 1
        valu = c.get("SQ_INSTS_VALU", 0) or 1
        lds_act = c.get("SQ_LDS_IDX_ACTIVE", 0)
        res[s] = {"launches": len(launches[s]), "waves": c.get("SQ_WAVES", 0),
                  "valu_per_wave": valu / waves,
                  "int32_share": c.get("SQ_INSTS_VALU_INT32", 0) / valu,
                  "int64_share": c.get("SQ_INSTS_VALU_INT64", 0) / valu,
                  "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0) / waves,
                  "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT", 0),
                  "lds_idx_active_cycles": lds_act,
                  "lds_conflict_frac": (c.get("SQ_LDS_BANK_CONFLICT", 0) / lds_act) if lds_act else None}
        print(f"{s[:60]:60s} n={len(launches[s]):3d} valu/wave={res[s]['valu_per_wave']:9.0f} "
              f"int32={res[s]['int32_share']:.3f} int64={res[s]['int64_share']:.3f} "
              f"lds/wave={res[s]['lds_insts_per_wave']:7.1f} conflict={res[s]['lds_conflict_frac']}")
    json.dump({"source": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 "
                         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS over bench.py (tools/gpu_pmc_int.sh)",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
