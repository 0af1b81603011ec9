"""Batch arenas of the claims trees (host/json.hpp Vec / Arena, host/hostmem.hpp),
as a C++ unit test under ASan + UBSan: trees moved out of their batch survive
the arena's release, moves inside a batch stay shallow, heap vectors stay on
the heap, the pools honour their retention cap.  CPU only."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "cap_amd", "csrc", "host")


def test_json_arena_under_asan():
    if not shutil.which("g++"):
        pytest.skip("no g++")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "json_arena_test")
        srcs = [os.path.join(ROOT, "tests", "host_unit", "json_arena_test.cpp")] + [
            os.path.join(HOST, f) for f in ("hostmem.cpp", "json.cpp")]
        r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                            "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-o", exe] + srcs,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
        assert "json arena test ok" in r.stdout
