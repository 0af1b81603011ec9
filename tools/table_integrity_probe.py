"""Comb tables widened in the background while verification runs must equal
tables built with the device idle.  Context A loads the 32 bench kids
(narrow-first) and streams the C5 pool through jg_verify_batch until every
upgrade has landed; context B loads the same keys with nothing else running.
Every key's table digest (jg_debug_table_digest) and every pass's verdicts are
compared.  usage: python tools/table_integrity_probe.py [chunk]"""
import ctypes
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    from cap_amd import _lib
    cpu = bench.cpu_info()
    meta = bench.bench_keys()
    pool, algs, keyidx, good = bench.c5_pool(meta, 10_000_000 // 8, cpu["cores_used"], 0)
    arena, toks = bench.pack(pool, algs, keyidx, len(pool))
    want = np.asarray(good)
    L = _lib.lib()
    out = (ctypes.c_uint8 * len(toks))()
    tp = toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok))

    a = _lib.Context([0])
    a.set_chunk(chunk)
    a.load_keys([m[3] for m in meta], wait_tables=False)
    done = threading.Event()
    threading.Thread(target=lambda: (a.wait_tables(), done.set()), daemon=True).start()
    npass = 0
    while not done.is_set() or npass < 2:
        if L.jg_verify_batch(a.h, arena, len(arena), tp, len(toks), out) != 0:
            raise RuntimeError(a.error())
        got = np.frombuffer(out, dtype=np.uint8).astype(bool)
        bad = np.nonzero(got != want)[0]
        print(f"A pass {npass} widths {a.table_widths()[20:]} mismatches {len(bad)} "
              f"{[(int(j), int(algs[j]), int(keyidx[j])) for j in bad[:6]]}", flush=True)
        npass += 1
    da = [a.table_digest(k) for k in range(len(meta))]
    wa = a.table_widths()

    b = _lib.Context([0])
    b.load_keys([m[3] for m in meta])               # built with the device otherwise idle
    db = [b.table_digest(k) for k in range(len(meta))]
    wb = b.table_widths()
    diff = [(m[0], wa[k], wb[k]) for k, m in enumerate(meta) if da[k] != db[k]]
    print("widths equal", wa == wb, "table digests differing:", diff, flush=True)
    a.close()
    b.close()
    sys.exit(1 if diff else 0)


if __name__ == "__main__":
    main()
