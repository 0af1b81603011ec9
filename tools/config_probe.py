"""One BASELINE config line alone, measured as bench.py measures it -- for
kernel A/Bs through CAPJWT_LIB.  usage: python tools/config_probe.py ps512|eddsa_es384|rs256_3072"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    from cap_amd import _lib
    which = sys.argv[1] if len(sys.argv) > 1 else "ps512"
    cpu = bench.cpu_info()
    th = cpu["cores_used"]
    ctx = _lib.Context([0])
    if which == "ps512":
        ctx.load_keys(bench.abi_keys(["rsa4096-a"]))
        pool = bench.gen_tokens("PS512", 4096, bench.golden_keypaths(["rsa4096-a"]), th, "probe")
        line = bench.config_line(ctx, "ps512_rsa4096", "PS512 RSA-4096 probe", pool,
                                 [bench.ALG_IDS["PS512"]] * len(pool), [0] * len(pool), np.ones(len(pool), bool),
                                 131072, 10, 3, False, 1,
                                 kernels={"rsa4096_modexp": bench.rsa_modexp_mads_per_token(148, 4)})
    elif which == "rs256_3072":        # the RSA-3K class alone (configs[4] holds RSA-3072 kids)
        ctx.load_keys(bench.abi_keys(["rsa3072-a"]))
        pool = bench.gen_tokens("RS256", 4096, bench.golden_keypaths(["rsa3072-a"]), th, "probe")
        line = bench.config_line(ctx, "rs256_3072", "RS256 RSA-3072 probe", pool,
                                 [bench.ALG_IDS["RS256"]] * len(pool), [0] * len(pool), np.ones(len(pool), bool),
                                 1 << 19, 10, 3, False, 1,
                                 kernels={"rsa3072_modexp": bench.rsa_modexp_mads_per_token(112, 4)})
    else:
        ctx.load_keys(bench.abi_keys(["ed-a", "p384-a"]))
        pe = bench.gen_tokens("EdDSA", 8192, bench.golden_keypaths(["ed-a"]), th, "probe")
        p3 = bench.gen_tokens("ES384", 8192, bench.golden_keypaths(["p384-a"]), th, "probe", kid_base=1)
        pool = [t for pair in zip(pe, p3) for t in pair]
        algs = [bench.ALG_IDS["EdDSA"], bench.ALG_IDS["ES384"]] * len(pe)
        line = bench.config_line(ctx, "eddsa_es384_mixed", "EdDSA + ES384 probe", pool, algs, [0, 1] * len(pe),
                                 np.ones(len(pool), bool), 1 << 20, 10, 3, False, 1,
                                 kernels={"ed25519_point": bench.ed25519_point_mads_per_token()})
    print(json.dumps({"value": line["value"], "kernel_ms": line["kernel_ms"]}))


if __name__ == "__main__":
    main()
