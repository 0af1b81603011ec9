"""The host layer (JSON, base64url, JWS parse, JWK / JWKS / PEM / DER, claims)
under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 sanitizer row):
tools/sanitize/run.sh builds an instrumented copy of the host extension and
runs the host CPU tests -- golden vectors, edge cases and the mutation fuzzers
-- through it.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_layer_under_asan_ubsan():
    if not shutil.which("gcc") or not os.path.exists(
            subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()):
        pytest.skip("no ASan runtime")
    env = dict(os.environ, CAPJWT_FUZZ_SCALE="2")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "run.sh"), "-x"], capture_output=True,
                       text=True, env=env, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout and "failed" not in r.stdout
