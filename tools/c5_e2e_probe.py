"""configs[4]'s JWKS end-to-end leg (bench.measure_jwks_e2e's flow: a
NewJSONWebKeySet with max_age 0 over the 32 bench kids, ValidateBatch over the
5 %-tampered 1.25 M-token share) repeated, printing the accept count of every
pass against the expected count: the check of the pipeline's verdict
delivery under the host layer.  usage: python tools/c5_e2e_probe.py [passes]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    from cap_amd import jwt
    cpu = bench.cpu_info()
    meta = bench.bench_keys()
    pool, algs, keyidx, good = bench.c5_pool(meta, 10_000_000 // 8, cpu["cores_used"], 0)
    jwks = json.dumps({"keys": [m[4] for m in meta]}).encode()
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                   lambda url, ca: {"status": 200, "body": jwks, "max_age": 0})
    assert err is None, err
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=list(bench.ALG_IDS),
                     Now=lambda: 1611699344 + 60)
    blob = b"\n".join(pool)
    want = np.asarray(good)
    bad_total = 0
    for i in range(passes):
        t0 = time.perf_counter()
        ok = np.frombuffer(v.ValidateBlob(blob, e), dtype=np.uint8).astype(bool)
        el = time.perf_counter() - t0
        diff = np.nonzero(ok != want)[0]
        bad_total += len(diff)
        print(f"pass {i}: {el * 1e3:.0f} ms accepted {int(ok.sum())} expected {int(want.sum())} "
              f"mismatches {len(diff)} {[(int(j), int(algs[j]), int(keyidx[j]), bool(want[j])) for j in diff[:8]]}",
              flush=True)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
