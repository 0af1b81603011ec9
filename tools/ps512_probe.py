"""BASELINE configs[2] alone (PS512 RSA-4096, 131072 tokens per GPU), as
bench.py measures it -- for A/Bs of the RSA-4K+ kernels through CAPJWT_LIB.
usage: python tools/ps512_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    from cap_amd import _lib
    cpu = bench.cpu_info()
    ctx = _lib.Context([0])
    ctx.load_keys(bench.abi_keys(["rsa4096-a"]))
    pool = bench.gen_tokens("PS512", 4096, bench.golden_keypaths(["rsa4096-a"]), cpu["cores_used"], "ps512probe")
    line = bench.config_line(ctx, "ps512_rsa4096", "PS512 RSA-4096 probe", pool, [bench.ALG_IDS["PS512"]] * len(pool),
                             [0] * len(pool), np.ones(len(pool), bool), 131072, 10, 3, False, 1,
                             kernels={"rsa4096_modexp": bench.rsa_modexp_mads_per_token(148, 4)})
    print(json.dumps({"value": line["value"], "kernel_ms": line["kernel_ms"],
                      "frac": line["roofline"]["rsa4096_modexp"]["frac"]}))


if __name__ == "__main__":
    main()
