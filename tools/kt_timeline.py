"""Per-queue kernel timeline of one pass out of a rocprofv3 kernel trace:
the launches from the n-th k_plan_fill whose grid is >= min_grid up to the
next k_plan_fill of such a size (or the end), start / end relative to that
plan fill, queue id and grid.  usage:
  python tools/kt_timeline.py kt_kernel_trace.csv [nth] [min_grid] [--to-next-big]"""
import csv
import re
import sys


def main(path, nth=0, min_grid=0, min_ms=0.0):
    rows = list(csv.DictReader(open(path)))
    fills = [i for i, r in enumerate(rows) if "k_plan_fill" in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= min_grid]
    i0 = fills[nth]
    end = fills[nth + 1] if nth + 1 < len(fills) else len(rows)
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:end]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e6
        e = (int(r["End_Timestamp"]) - t0) / 1e6
        if e - s < min_ms:
            continue
        k = re.sub(r"\(.*\)$", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))
        print(f"q{r['Queue_Id']:>2} {s:8.3f} {e:8.3f} {e - s:7.3f}  {k[:44]:44s} grid {r['Grid_Size_X']}")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]) if len(a) > 1 else 0, int(a[2]) if len(a) > 2 else 0, float(a[3]) if len(a) > 3 else 0.0)
