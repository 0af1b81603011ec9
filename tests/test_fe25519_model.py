"""CPU checks of kernels/fe25519.hpp, the radix-2^25.5 field of the Ed25519
point loop: the limb-maxima analysis of the Niels addition
(tools/fe25519_bounds.py: every 64-bit product column and 32-bit limb fits),
and the bit-exact Python model of mul / canon against big-integer arithmetic
mod p = 2^255 - 19 on random and extreme (limb-maximal) inputs.  The GPU test
tests/test_gpu_fe25519.py holds the device code to the same model."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import fe25519_bounds as B  # noqa: E402


def test_niels_addition_bounds():
    norm = B.niels_addition_bounds()
    assert all(n < (1 << 31) for n in norm)


def _rand_limbs(rng, maxima):
    return [rng.randrange(m + 1) for m in maxima]


def test_model_mul_and_canon():
    rng = random.Random(25519)
    norm = B.niels_addition_bounds()
    big_f = B.mx_sub(B.mx_add(norm, norm), norm)      # ~4 units: F = D - C
    big_g = B.mx_sub(norm, norm)                      # ~3 units: E = B - A
    cases = []
    for _ in range(3000):
        cases.append((_rand_limbs(rng, big_f), _rand_limbs(rng, big_g)))
    cases.append((big_f, big_g))                      # every limb at its maximum
    cases.append((list(B.MASK), list(B.MASK)))
    cases.append((B.to_limbs(B.P - 1), B.to_limbs(B.P - 1)))
    cases.append((B.to_limbs(0), big_g))
    for f, g in cases:
        r = B.model_mul(f, g)
        assert all(x <= n for x, n in zip(r, norm))
        assert B.value(r) % B.P == B.value(f) * B.value(g) % B.P
        c = B.model_canon(r)
        assert B.value(c) == B.value(f) * B.value(g) % B.P
    # canon of lazy sums (limbs < 2^31) and of values in [p, 2^255)
    for v in [B.P, B.P + 1, 2**255 - 1, 0, 1, B.P - 1]:
        assert B.value(B.model_canon(B.to_limbs(v % 2**255) if v < 2**255 else B.to_limbs(v))) == v % B.P
    for _ in range(2000):
        x = [rng.randrange(1 << 31) for _ in range(B.L)]
        assert B.value(B.model_canon(x)) == B.value(x) % B.P
