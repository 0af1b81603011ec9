"""Print every bench kid's comb-table width and digest (jg_debug_table_digest)
after a load at the given table budget: run it once with CAPJWT_TABLES_SYNC=1
(every table built inside jg_keys_load) and once without (narrow tables, then
the background upgrader) and compare the two outputs.
usage: python tools/table_digest_dump.py [budget_gib]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    budget = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    from cap_amd import _lib
    meta = bench.bench_keys()
    ctx = _lib.Context()
    ctx.set_table_budget(budget << 30)
    ctx.load_keys([m[3] for m in meta])
    w = ctx.table_widths()
    print(json.dumps({m[0]: [w[i], ctx.table_digest(i)] for i, m in enumerate(meta) if w[i]}))
    ctx.close()


if __name__ == "__main__":
    main()
