"""Summarise a rocprofv3 rocpd database (kernel dispatches): per-kernel count and
median duration, then a window of consecutive dispatches (timeline).
usage: python tools/rocpd_summary.py results.db [start_fraction] [count]"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
    cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(c.execute("select name,start,end,stream_id,grid_x,workgroup_x,vgpr_count from kernels order by start"))
    st = collections.defaultdict(list)
    for n, s, e, *_ in rows:
        st[n[:90]].append(e - s)
    print(f"{len(rows)} dispatches")
    for k, v in sorted(st.items(), key=lambda x: -sum(x[1]))[:25]:
        v.sort()
        print(f"{len(v):6d} med {v[len(v) // 2] / 1000:9.1f} us  {k}")
    mid = int(len(rows) * frac)
    t0 = rows[mid][1]
    for n, s, e, sid, g, wg, vg in rows[mid:mid + cnt]:
        print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} s{sid} grid {g:7d}/{wg:4d} v{vg:3d} {n[:80]}")


if __name__ == "__main__":
    main()
