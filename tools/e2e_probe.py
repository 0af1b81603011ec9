"""Phase breakdown of the end-to-end Validator.ValidateBlob path (bench.py's
`e2e` line) on the GPU box: CAPJWT_TRACE=1 makes the C++ host layer print
per-phase wall times to stderr.  usage: python tools/e2e_probe.py [tokens]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CAPJWT_TRACE"] = "1"

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    cpu = bench.cpu_info()
    kids = ["p256-a", "p256-b", "p256-c", "p256-d"]
    pool = bench.gen_tokens("ES256", n, bench.golden_keypaths(kids), cpu["cores_used"], "probe")
    jwk = [{"kty": "EC", "kid": f"kid-{i:02d}", "crv": "P-256", **xy} for i, xy in enumerate(bench.p256_jwk_xy(kids))]
    t0 = time.perf_counter()
    r = bench.measure_e2e(pool, jwk, n, cpu["cores_used"])
    print(r, "cpu", cpu, "wall %.2f s" % (time.perf_counter() - t0))


if __name__ == "__main__":
    main()
