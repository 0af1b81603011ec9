"""Device check of kernels/fe25519.hpp (the radix-2^25.5 field of the
Ed25519 point loop) through the test library's tk_fe25519 hook: fe::mul and
fe::canon must equal the bit-exact Python model of tools/fe25519_bounds.py
(which tests/test_fe25519_model.py holds to big-integer arithmetic), limb for
limb, on random inputs up to the Niels addition's operand maxima and on the
extremes."""
import ctypes
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import fe25519_bounds as B  # noqa: E402

pytestmark = pytest.mark.gpu


def _run(tk, op, xs, ys):
    n = len(xs)
    A = (ctypes.c_uint32 * (n * B.L))(*[l for v in xs for l in v])
    Bv = (ctypes.c_uint32 * (n * B.L))(*[l for v in ys for l in v])
    O = (ctypes.c_uint32 * (n * B.L))()
    assert tk.tk_fe25519(op, A, Bv, O, n) == 0
    return [list(O[i * B.L:(i + 1) * B.L]) for i in range(n)]


def test_fe25519_mul_and_canon_match_the_model():
    tk = ctypes.CDLL(os.path.join(ROOT, "cap_amd", "libcapjwt_tk.so"))
    tk.tk_fe25519.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    rng = random.Random(255)
    norm = B.niels_addition_bounds()
    big_f = B.mx_sub(B.mx_add(norm, norm), norm)
    big_g = B.mx_sub(norm, norm)
    xs = [[rng.randrange(m + 1) for m in big_f] for _ in range(4000)] + [big_f, list(B.MASK), B.to_limbs(B.P - 1)]
    ys = [[rng.randrange(m + 1) for m in big_g] for _ in range(4000)] + [big_g, list(B.MASK), B.to_limbs(B.P - 1)]
    out = _run(tk, 0, xs, ys)
    for x, y, o in zip(xs, ys, out):
        assert o == B.model_mul(x, y)
        assert B.value(o) % B.P == B.value(x) * B.value(y) % B.P
    lz = [[rng.randrange(1 << 31) for _ in range(B.L)] for _ in range(2000)]
    lz += [B.to_limbs(v) for v in (0, 1, B.P - 1, B.P, B.P + 18, 2**255 - 1)]
    out = _run(tk, 1, lz, lz)
    for x, o in zip(lz, out):
        assert o == B.model_canon(x)
        assert B.value(o) == B.value(x) % B.P
