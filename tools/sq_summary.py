"""Summarise a rocprofv3 --pmc SQ pass (counter_collection.csv) per kernel:
wave cycles split into VALU-active / other-active / issue-stalled / parked,
VALU instructions, waves.  usage: python tools/sq_summary.py in.csv out.json"""
import collections
import csv
import json
import sys


def main(src, out):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(src)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, v in agg.items():
        if any(s in k for s in ("rocclr", "table", "keyprep")):
            continue
        m = {c: sum(x) / len(x) for c, x in v.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        res[k] = {"launches": len(next(iter(v.values()))), "waves": m.get("SQ_WAVES"),
                  "valu_insts": m.get("SQ_INSTS_VALU"), "wave_cycles": m.get("SQ_WAVE_CYCLES"),
                  "frac_valu_active": m.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                  "frac_any_active": m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                  "frac_issue_stall": m.get("SQ_WAIT_INST_ANY", 0) / wc,
                  "frac_parked": m.get("SQ_WAIT_ANY", 0) / wc}
    json.dump({"source": "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                         "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU over bench.py (tools/gpu_pmc_sq.sh)",
               "kernels": res}, open(out, "w"), indent=1)
    for k, r in res.items():
        print(f"{k[:70]:70s} valu {r['frac_valu_active']:.2f} stall {r['frac_issue_stall']:.2f} parked {r['frac_parked']:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
