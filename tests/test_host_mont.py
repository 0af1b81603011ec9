"""RSA key constants computed on the host at key staging (cap_amd/csrc/
host_mont.hpp, used by jg_runtime.cpp build_keys): R^2 mod n for the device
radix R = 2^(28 L) and n' = -n^-1 mod 2^28, against Python big integers, for
every RSA layout size (L = 74 / 112 / 148 / 296 / 592 limbs) and moduli of
1024 .. 16574 bits, including the bit lengths at the layout edges."""
import ctypes
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HK = os.path.join(ROOT, "tests", "host_kernels")


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("hm") / "libhostmont.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", out,
                    os.path.join(HK, "host_mont_test.cpp")], check=True)
    L = ctypes.CDLL(out)
    L.host_rsa_key_constants.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return L


def test_rr_and_nprime_match_big_integers(lib):
    rng = random.Random(28)
    cases = []
    for L, bits_list in ((74, (1024, 2047, 2048, 2070)), (112, (2071, 3072, 3134)), (148, (3135, 4096, 4142)),
                         (296, (4143, 8192, 8286)), (592, (8287, 16384, 16574))):
        for bits in bits_list:
            for _ in range(2):
                n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
                cases.append((L, n))
        cases.append((L, (1 << bits_list[-1]) - 1))        # all ones
        cases.append((L, (1 << (bits_list[0] - 1)) + 1))   # smallest of the size
    for L, n in cases:
        limbs = [(n >> (28 * i)) & 0x0fffffff for i in range(L)]
        N = (ctypes.c_uint32 * L)(*limbs)
        RR = (ctypes.c_uint32 * L)()
        NP = ctypes.c_uint32()
        lib.host_rsa_key_constants(N, L, RR, ctypes.byref(NP))
        rr = sum(v << (28 * i) for i, v in enumerate(RR))
        assert rr == pow(2, 56 * L, n), (L, n.bit_length())
        assert (NP.value * n) % (1 << 28) == (1 << 28) - 1, (L, n.bit_length())
