"""Exact parity of the RSA public operation y = s^e mod n (kernels/rsa.hip
k_rsa_modexp: mont_mul, the mont_sqr squaring rows, the lane carries and the
final canonical subtraction) against Python's pow(), word for word, through the
test hook tk_rsa_modexp (cap_amd/csrc/tests/tk_rsa.hip).  The product path
(jg_verify_batch) only exposes accept/reject; this checks the integer itself
for random and edge signatures, every RSA class (2048/3072/4096-bit layouts and
the odd sizes that share them), e = 65537 (squarings + one multiply) and other
exponents (the generic square-and-multiply path), ragged batch sizes, and the
s >= n rejection of Go >= 1.20."""
import ctypes
import os
import random

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLS_RSA2K, CLS_RSA3K, CLS_RSA4K = 1, 2, 3
# modulus bit lengths per class (limits 28 L - 2 bits: 2070 / 3134; the RSA-4K+
# class picks 148 / 296 / 592 limbs by key size: up to 4142 / 8286 / 16574 bits)
SIZES = [(CLS_RSA2K, 2048), (CLS_RSA2K, 2049), (CLS_RSA2K, 2070), (CLS_RSA3K, 3072), (CLS_RSA3K, 2071),
         (CLS_RSA4K, 4096), (CLS_RSA4K, 3135), (CLS_RSA4K, 4142)]
BIG_SIZES = [(CLS_RSA4K, 4143), (CLS_RSA4K, 8192), (CLS_RSA4K, 8286), (CLS_RSA4K, 8287), (CLS_RSA4K, 16384),
             (CLS_RSA4K, 16574)]


@pytest.fixture(scope="module")
def tk():
    L = ctypes.CDLL(os.path.join(ROOT, "cap_amd", "libcapjwt_tk.so"))
    L.tk_rsa_modexp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.tk_rsa_modexp.restype = ctypes.c_int
    return L


def words(v, n):
    return [(v >> (32 * i)) & 0xffffffff for i in range(n)]


def modexp(tk, cls, n, e, sigs):
    nw = (n.bit_length() + 31) // 32
    N = (ctypes.c_uint32 * nw)(*words(n, nw))
    S = (ctypes.c_uint32 * (nw * len(sigs)))(*[w for s in sigs for w in words(s, nw)])
    Y = (ctypes.c_uint32 * (nw * len(sigs)))()
    OK = (ctypes.c_uint8 * len(sigs))()
    assert tk.tk_rsa_modexp(cls, N, nw, e, S, len(sigs), Y, OK) == 0
    ys = [sum(Y[i * nw + q] << (32 * q) for q in range(nw)) for i in range(len(sigs))]
    return ys, list(OK)


def edge_sigs(n, rng, count):
    bits = n.bit_length()
    edges = [0, 1, 2, 3, n - 1, n - 2, (n - 1) // 2, 1 << (bits - 1), (1 << (bits - 1)) - 1,
             (1 << 28) - 1, 1 << 28, (1 << (28 * 37)) - 1, n >> 1, n - (1 << 28)]
    edges = [s for s in edges if 0 <= s < n]
    return edges + [rng.randrange(n) for _ in range(count - len(edges))]


@pytest.mark.parametrize("cls,bits", SIZES)
@pytest.mark.parametrize("e", [65537, 3, 17, 2**31 - 1])
def test_modexp_exact(tk, cls, bits, e):
    rng = random.Random(bits * 1000003 + e)
    n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    sigs = edge_sigs(n, rng, 200)          # ragged: not a whole number of waves
    ys, ok = modexp(tk, cls, n, e, sigs)
    bad = [i for i, (s, y) in enumerate(zip(sigs, ys)) if not ok[i] or y != pow(s, e, n)]
    assert not bad, (len(bad), bad[:8])


@pytest.mark.parametrize("cls,bits", BIG_SIZES)
@pytest.mark.parametrize("e", [65537, 3, 2**31 - 1])
def test_modexp_exact_big_layouts(tk, cls, bits, e):
    """The 296- and 592-limb layouts (8 and 16 lanes per token: DPP row shifts
    and ds_swizzle broadcasts, column normalisation every 80 / 74 rows)."""
    rng = random.Random(bits * 1000003 + e)
    n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    sigs = edge_sigs(n, rng, 70)
    ys, ok = modexp(tk, cls, n, e, sigs)
    bad = [i for i, (s, y) in enumerate(zip(sigs, ys)) if not ok[i] or y != pow(s, e, n)]
    assert not bad, (len(bad), bad[:8])


@pytest.mark.parametrize("cls,bits", [(CLS_RSA2K, 2048), (CLS_RSA4K, 4096), (CLS_RSA4K, 8192), (CLS_RSA4K, 16384)])
def test_modexp_rejects_sig_not_below_modulus(tk, cls, bits):
    rng = random.Random(bits)
    n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    top = (1 << (32 * ((bits + 31) // 32))) - 1
    sigs = [n, n + 1, n + (1 << 28), top, 5, n - 1]
    ys, ok = modexp(tk, cls, n, 65537, sigs)
    assert ok == [0, 0, 0, 0, 1, 1]
    assert ys[4] == pow(5, 65537, n) and ys[5] == n - 1


def test_modexp_many_tokens_one_key(tk):
    """A full-occupancy launch (4096 tokens = 64 waves x 2 lanes) of the RS256
    layout: the squaring's LDS operand rows and limb shifts across all wave slots."""
    rng = random.Random(7)
    n = rng.getrandbits(2048) | (1 << 2047) | 1
    sigs = [rng.randrange(n) for _ in range(4096)]
    ys, ok = modexp(tk, CLS_RSA2K, n, 65537, sigs)
    assert all(ok)
    assert all(y == pow(s, 65537, n) for s, y in zip(sigs, ys))
