"""Degraded path on a device failure (SURVEY §5 failure row; VERDICT r03
"missing" 5): when jg_verify_batch fails -- a HIP error, a lost device -- the
key sets do not throw out of the batch and do not verify on the CPU.  Every
token that needed the device gets "capjwt: signature verification
unavailable: <the runtime's error>" as its own error (Go's VerifySignature /
Validate return an error per token, jwt/keyset.go:127,163, jwt/jwt.go:95);
parse errors and no-key misses keep their own errors, and a JWKS key set does
not refetch for a token whose device call failed (it is no miss,
go-oidc remoteKeySet.verify).

The host layer is built here against tests/host_faults/fault_stub.cpp, a
stand-in C ABI whose verify call always fails.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "cap_amd", "csrc", "host")
HERE = os.path.join(ROOT, "tests", "host_faults")


def test_device_failure_becomes_per_token_errors(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path / "degraded")
    srcs = [os.path.join(HERE, "degraded.cpp"), os.path.join(HERE, "fault_stub.cpp")] + [
        os.path.join(HOST, f) for f in ("hostmem.cpp", "json.cpp", "jose.cpp", "cap_jwt.cpp")]
    b = subprocess.run(["g++", "-O0", "-std=c++17", "-pthread", "-o", exe] + srcs,
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "degraded: ok" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
