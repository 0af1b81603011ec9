"""The device SHA-256 / SHA-384 / SHA-512 code (cap_amd/csrc/kernels/sha2.hpp:
compression, padding, the Ed25519 R || A prefix) compiled for the CPU with
the AMDGPU builtins emulated (tests/host_kernels), against hashlib -- a CPU
check of the hash arithmetic every prep kernel runs.  (The GPU parity tests
cover the kernels themselves.)"""
import ctypes
import hashlib
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HK = os.path.join(ROOT, "tests", "host_kernels")


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sha2") / "libsha2host.so")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-I", HK, "-o", out,
                    os.path.join(HK, "sha2_host.cpp")], check=True)
    L = ctypes.CDLL(out)
    L.sha2_host.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p]
    return L


@pytest.mark.parametrize("bits", [256, 384, 512])
def test_sha2_matches_hashlib(lib, bits):
    rnd = random.Random(bits)
    for n in list(range(0, 300)) + [rnd.randrange(300, 3000) for _ in range(40)]:
        m = bytes(rnd.randrange(256) for _ in range(n))
        out = ctypes.create_string_buffer(64)
        k = lib.sha2_host(bits, m, len(m), None, out)
        assert out.raw[:k] == getattr(hashlib, f"sha{bits}")(m).digest(), (bits, n)


def test_sha512_with_ed25519_prefix(lib):
    rnd = random.Random(5)
    for n in (0, 1, 47, 48, 63, 64, 111, 112, 255, 1000):
        pre = bytes(rnd.randrange(256) for _ in range(64))
        m = bytes(rnd.randrange(256) for _ in range(n))
        out = ctypes.create_string_buffer(64)
        lib.sha2_host(512, m, len(m), pre, out)
        assert out.raw == hashlib.sha512(pre + m).digest(), n
