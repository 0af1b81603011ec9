"""Static check of the gfx950 assembly of the RSA kernels (CPU only).

The RSA modexp spreads each token over 2 or 4 lanes and moves carries, borrows
and limbs between them with DPP.  A DPP read placed inside an EXEC-masked
region reads the masked-off source lanes as 0: written as `lane0 ? 0 : dpp(x)`,
LLVM turned the select into a branch and sank the DPP under it, so the final
subtraction lost lane 0's borrow whenever s^e mod n = n - 1 (found by
tests/test_gpu_rsa.py; fixed with opaque lane masks, rsa.hip opaque_mask).
This test keeps every k_rsa_modexp instantiation free of that shape."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cap_amd", "csrc")
ASM = os.path.join(CSRC, "build", "rsa.s")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def rsa_asm():
    src = os.path.join(CSRC, "kernels", "rsa.hip")
    if not os.path.exists(ASM) or os.path.getmtime(ASM) < os.path.getmtime(src):
        if not os.path.exists(HIPCC):
            pytest.skip("hipcc not available and build/rsa.s not built")
        subprocess.run(["make", "-s", "-C", CSRC, "build/rsa.s"], check=True, timeout=900)
    return open(ASM).read().split("\n")


def functions(lines, prefix):
    out, cur = {}, None
    for ln in lines:
        m = re.match(r"^(_Z\S+):", ln)
        if m and prefix in m.group(1):
            cur = m.group(1)
            out[cur] = []
            continue
        if ln.startswith(".Lfunc_end"):
            cur = None
        if cur:
            out[cur].append(ln.strip())
    return out


def dpp_in_masked_region(body):
    """DPP instructions between an EXEC narrowing and the next EXEC restore."""
    masked, bad = False, []
    for ins in body:
        if re.match(r"s_(and_saveexec|andn2_saveexec|or_saveexec)_b64|s_(mov|and|andn2)_b64 exec,", ins):
            masked = True
        elif re.match(r"s_or_b64 exec, exec", ins):
            masked = False
        elif "_dpp" in ins and masked:
            bad.append(ins)
    return bad


def test_rsa_modexp_has_no_dpp_under_exec_mask(rsa_asm):
    fns = functions(rsa_asm, "k_rsa_modexp")
    assert len(fns) >= 3, sorted(fns)
    for name, body in fns.items():
        assert sum("_dpp" in i for i in body) > 0, name
        bad = dpp_in_masked_region(body)
        assert not bad, (name, bad[:4])
