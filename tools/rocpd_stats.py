"""Summarise a rocprofv3 SQLite (rocpd) result into a kernel-stats CSV
(name, calls, total_ns, avg_ns, min_ns, max_ns, pct, vgpr, sgpr, lds, scratch)."""
import csv
import sqlite3
import sys


def main(db_path, out_csv):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                      "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) "
                      "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage",
                    "arch_vgpr", "accum_vgpr", "sgpr", "lds_bytes", "scratch_bytes"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / tot, 2)] + list(r[6:]))
    for r in rows[:12]:
        print(f"{r[1]:5d} {r[3] / 1e6:9.3f} ms avg  {100.0 * r[2] / tot:5.1f}%  {r[0][:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
