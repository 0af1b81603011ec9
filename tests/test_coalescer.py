"""The single-token coalescer (host/cap_jwt.cpp Coalescer: lock-free
submission stack, dispatcher threads, tree wake-up) as a C++ unit test, under
ASan + UBSan and under TSan: 96 threads x 400 calls, batches that throw,
dispatcher count and batch cap changed while calls are in flight.  CPU only;
the host layer links against the fault stub ABI (no device)."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "cap_amd", "csrc", "host")

SAN = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


@pytest.mark.parametrize("san", sorted(SAN))
def test_coalescer_under_sanitizer(san):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "coalescer_test")
        srcs = [os.path.join(ROOT, "tests", "host_unit", "coalescer_test.cpp"),
                os.path.join(ROOT, "tests", "host_faults", "fault_stub.cpp")] + [
            os.path.join(HOST, f) for f in ("hostmem.cpp", "json.cpp", "jose.cpp", "cap_jwt.cpp")]
        r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-pthread", "-fno-omit-frame-pointer"] + SAN[san] +
                           ["-o", exe] + srcs, capture_output=True, text=True, timeout=600)
        if san == "tsan" and r.returncode != 0 and "tsan" in r.stderr.lower():
            pytest.skip("no TSan runtime: " + r.stderr[-300:])
        assert r.returncode == 0, r.stderr[-3000:]
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1",
                   TSAN_OPTIONS="halt_on_error=1")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
        assert "coalescer test ok" in r.stdout
