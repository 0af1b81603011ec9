"""Run bench.py's ES256 line (or another bench.py argument set) once per
variant -- an environment (library build via CAPJWT_LIB, runtime knobs) --
and collect value + per-kernel times into one JSON: the A/B driver of the
profiles/*_ab.json files.

usage: python tools/ab_run.py out.json 'name:ENV=V,ENV2=V2' ... [-- bench args]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["--no-rs256", "--no-configs", "--no-e2e", "--no-cpu", "--no-ab", "--steps", "10", "--warmup", "3"]


def main():
    out, rest = sys.argv[1], sys.argv[2:]
    args = DEFAULT
    if "--" in rest:
        i = rest.index("--")
        rest, args = rest[:i], rest[i + 1:]
    res = {"bench_args": args, "variants": {}}
    for spec in rest:
        name, _, envs = spec.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v if k != "CAPJWT_LIB" else os.path.join(ROOT, v)
        t0 = time.time()
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            res["variants"][name] = {"env": envs, "error": r.stderr[-2000:]}
            print(name, "FAILED", r.stderr[-500:], flush=True)
            json.dump(res, open(out, "w"), indent=1)
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        line = d if "value" in d else d.get("configs", {})
        res["variants"][name] = {"env": envs, "value": d.get("value"), "kernel_ms": d.get("kernel_ms"),
                                 "ms_per_step": d.get("ms_per_step"), "accepted": d.get("accepted"),
                                 "error": d.get("error"), "configs": {k: {"value": v.get("value"),
                                                                           "kernel_ms": v.get("kernel_ms")}
                                                                       for k, v in d.get("configs", {}).items()},
                                 "wall_s": time.time() - t0}
        print(name, round((d.get("value") or 0) / 1e6, 1), {k: round(v, 3) for k, v in (d.get("kernel_ms") or {}).items()},
              flush=True)
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
