"""CPU checks of bench.py's accounting (no GPU): the key comb width it assumes
for the roofline's MAD count must be the one the library picks for the same
table budget (kernels/ecdsa.hpp ec_key_w / include/jg.h jg_set_table_budget),
and the MAD counts must follow the additions per token."""
import os
import re

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GiB = 1 << 30


def _header_tiers():
    src = open(os.path.join(ROOT, "cap_amd", "csrc", "kernels", "ecdsa.hpp")).read()
    m = re.search(r"EC_P256_WQ\[\d+\]\s*=\s*\{([^}]*)\}", src)
    return [int(x) for x in m.group(1).split(",")]


def test_p256_width_tiers_match_the_library():
    assert _header_tiers() == [26, 24, 22, 20]
    # the documented cut-offs (jg.h)
    # 64-B packed entries (ecdsa.hpp JG_EC_PACK64): W = 26 is 21.5 GB per key
    assert bench.table_bytes("p256", 26) == 10 * (1 << 25) * 64
    assert bench.p256_key_w(5, 110 * GiB) == 26
    assert bench.p256_key_w(6, 110 * GiB) == 24
    assert bench.p256_key_w(4, 32 * GiB) == 24
    assert bench.p256_key_w(21, 32 * GiB) == 22
    assert bench.p256_key_w(22, 32 * GiB) == 20
    assert bench.p256_key_w(1, 0) == 20


def test_p384_width_tiers_match_the_library():
    src = open(os.path.join(ROOT, "cap_amd", "csrc", "kernels", "ecdsa.hpp")).read()
    m = re.search(r"EC_P384_WQ\[\d+\]\s*=\s*\{([^}]*)\}", src)
    assert [int(x) for x in m.group(1).split(",")] == [24, 20, 18, 16]
    assert bench.p384_key_w(1, 32 * GiB) == 24          # configs[3]: one P-384 key
    assert bench.p384_key_w(3, 110 * GiB) == 24         # configs[4]: three, at the bench's budget
    assert bench.p384_key_w(3, 32 * GiB) == 20
    assert bench.p384_key_w(1, 0) == 16


def test_point_mads_follow_the_window_count():
    # one fewer key window (one fewer mixed addition) per step of the tiers
    m = {w: bench.p256_point_mads_per_token(w) for w in (20, 22, 24, 26)}
    assert m[20] > m[22] > m[24] > m[26]
    per_add = m[24] - m[26]
    assert abs((m[22] - m[24]) - per_add) < 1 and abs((m[20] - m[22]) - per_add) < 1
    # a mixed addition: 8 mul + 3 sqr (L = 10) under 10 reductions of 4 L MADs
    assert abs(per_add - (8 * 100 + 3 * 55 + 10 * 40)) < 1


def test_p521_point_mads():
    src = open(os.path.join(ROOT, "cap_amd", "csrc", "kernels", "ecdsa.hpp")).read()
    m = re.search(r"EC_P521_WQ\[\d+\]\s*=\s*\{([^}]*)\}", src)
    assert [int(x) for x in m.group(1).split(",")] == [20, 18, 16]
    assert bench.p521_key_w(3, 32 * GiB) == 20
    assert bench.p521_key_w(1, 0) == 16
    m = {w: bench.p521_point_mads_per_token(w) for w in (16, 18, 20)}
    # windows ceil(523 / W): 27 at 20, 30 at 18, 33 at 16 -- three mixed additions per step
    per_add = (m[18] - m[20]) / 3
    assert abs((m[16] - m[18]) / 3 - per_add) < 1
    # a mixed addition: 8 mul + 3 sqr (L = 20) under 10 one-constant reductions + one fold MAD
    assert abs(per_add - (8 * 400 + 3 * 210 + 10 * 20 + 1)) < 1


def test_rsa_modexp_layouts_match_the_library():
    """bench.py prices each RSA class's modexp on the lanes per token the
    library launches it with (kernels/rsa.hpp: RSA-2048 2 lanes, RSA-3072
    JG_RSA3K_G lanes, RSA-4096 4): a squaring's partial products depend on it."""
    src = open(os.path.join(ROOT, "cap_amd", "csrc", "kernels", "rsa.hpp")).read()
    g3k = int(re.search(r"#define JG_RSA3K_G (\d+)", src).group(1))
    g2k = int(re.search(r"#define JG_RSA2K_G (\d+)", src).group(1))
    bsrc = open(os.path.join(ROOT, "bench.py")).read()
    assert f'"rsa3072_modexp": rsa_modexp_mads_per_token(112, {g3k})' in bsrc
    assert f'"rsa2048_modexp": rsa_modexp_mads_per_token(74, {g2k})' in bsrc
    # e = 65537: 2 full products (2 L^2 each) + 16 squarings (lanes^2 H(H+1)/2 + L^2)
    h = 112 // g3k
    assert bench.rsa_modexp_mads_per_token(112, g3k) == 4 * 112 * 112 + 16 * (g3k * g3k * h * (h + 1) // 2 + 112 * 112)


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _full_result():
    """A complete bench result (round 5's full line, the largest the bench has
    printed: 22.9 KB) as the stub the line builder compacts."""
    import json
    path = os.path.join(ROOT, "profiles", "r05_s9", "bench_full.json")
    return json.loads(open(path).read().strip().splitlines()[-1])


def test_compact_line_fits_and_keeps_the_contract_keys(tmp_path):
    import json
    full = _full_result()
    assert len(json.dumps(full)) > bench.LINE_MAX_BYTES           # the stub is the over-size line
    full["multi_device"] = {"value": 1.0e9, "devices": [0, 0], "verify_batch": {"value": 5e8},
                            "validate_batch": {"value": 2e7}, "accepted": 10, "expected_accepted": 10,
                            "per_device": [{"dev": 0, "kernel_ms": {"x": 1.0}}] * 8}
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_MAX_BYTES // 2, len(text)
    for k in REQUIRED:
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    assert 0 < line["roofline"]["frac"] < 1
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["detail"] == "gpurun_out/bench_detail.json"
    for name, c in line["configs"].items():
        assert c["accepted"] == c["expected"], name
        assert c["frac"], name
    assert line["multi_device"]["verify_batch"] == 5e8


def test_emit_line_writes_the_detail_file(tmp_path, capsys):
    import json
    full = _full_result()
    path = str(tmp_path / "detail.json")
    bench.emit_line(full, path)
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    line = json.loads(out[0])
    assert line["detail"] == path
    assert json.load(open(path)) == full
