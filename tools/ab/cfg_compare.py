"""Side-by-side of `bench.py --configs-only` lines: value and per-kernel
frac / ms per config.  usage: python tools/ab/cfg_compare.py name=file.json ..."""
import json
import sys

runs = [(a.split("=", 1)[0], json.load(open(a.split("=", 1)[1]))["configs"]) for a in sys.argv[1:]]
for cfg in runs[0][1]:
    print(cfg)
    for name, c in runs:
        line = c[cfg]
        fr = {k: round(v["frac"], 3) for k, v in (line.get("roofline") or {}).items() if "frac" in v}
        extra = f" stream {line['stream']['value'] / 1e6:.1f}M" if "stream" in line else ""
        print(f"  {name:6s} value {line['value'] / 1e6:8.2f}M{extra}  {fr}")
