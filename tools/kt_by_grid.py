"""rocprofv3 --kernel-trace CSV -> per (kernel, grid size) call count and
average / min / max duration (ms): the resident 1M-token launches of bench.py
separated from its pipelined-chunk launches of the same kernels.
usage: python tools/kt_by_grid.py kernel_trace.csv out.csv"""
import collections
import csv
import sys


def main(src, out):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)
        agg[(r["Kernel_Name"], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid", "calls", "avg_ms", "min_ms", "max_ms", "total_ms"])
        for (k, g), v in rows:
            w.writerow([k, g, len(v), f"{sum(v) / len(v):.4f}", f"{min(v):.4f}", f"{max(v):.4f}", f"{sum(v):.3f}"])
    for (k, g), v in rows[:12]:
        print(f"{k[:64]:64s} {g:9d} {len(v):4d} {sum(v) / len(v):9.4f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
