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


def test_extended_addition_bounds():
    # k_ed_point_split's lane combine (ed25519.hip add_ext): its products fit
    # and its outputs stay within the Niels addition's normalized maxima
    out = B.extended_addition_bounds()
    assert all(n < (1 << 31) for n in out)


def test_add_ext_model():
    """add_ext restated with the bit-exact model: random points of the curve's
    group in extended coordinates (scaled by random Z), their sum equals the
    affine Edwards sum -- the formula and its constant 2d are right."""
    p = B.P
    d = (-121665 * pow(121666, p - 2, p)) % p
    D2 = [0x2b2f159, 0x1a6e509, 0x22add7a, 0x0d4141d, 0x0038052, 0x0f3d130, 0x3407977, 0x19ce331, 0x1c56dff, 0x0901b67]
    assert B.value(D2) == 2 * d % p

    def recover_x(y, sign):
        x2 = (y * y - 1) * pow(d * y * y + 1, p - 2, p) % p
        x = pow(x2, (p + 3) // 8, p)
        if (x * x - x2) % p:
            x = x * pow(2, (p - 1) // 4, p) % p
        if (x * x - x2) % p:
            return None
        return p - x if (x & 1) != sign else x

    def ext(x, y, z):
        lim = lambda v: B.to_limbs(v % p)
        return [lim(x * z), lim(y * z), lim(z), lim(x * y * z)]     # X = xZ, Y = yZ, Z, T = xyZ

    def sub(a, b):
        return [x + q - y for x, y, q in zip(a, b, B.P2)]

    def add(a, b):
        return [x + y for x, y in zip(a, b)]

    def add_ext(P_, Q_):
        X1, Y1, Z1, T1 = P_
        X2, Y2, Z2, T2 = Q_
        t = B.model_mul(T2, D2)
        C = B.model_mul(t, T1)
        t = B.model_mul(Z1, Z2)
        Dd = add(t, t)
        F, G = sub(Dd, C), add(Dd, C)
        A = B.model_mul(sub(Y2, X2), sub(Y1, X1))
        Bb = B.model_mul(add(Y2, X2), add(Y1, X1))
        E, H = sub(Bb, A), add(Bb, A)
        return [B.model_mul(F, E), B.model_mul(H, G), B.model_mul(F, G), B.model_mul(H, E)]   # X, Y, Z, T

    rng = random.Random(2)
    done = 0
    while done < 40:
        y1, y2 = rng.randrange(p), rng.randrange(p)
        x1, x2 = recover_x(y1, rng.randrange(2)), recover_x(y2, rng.randrange(2))
        if x1 is None or x2 is None:
            continue
        z1, z2 = rng.randrange(1, p), rng.randrange(1, p)
        X3, Y3, Z3, T3 = (B.value(v) % p for v in add_ext(ext(x1, y1, z1), ext(x2, y2, z2)))
        # affine twisted Edwards addition, a = -1
        den = d * x1 * x2 * y1 * y2 % p
        x3 = (x1 * y2 + y1 * x2) * pow(1 + den, p - 2, p) % p
        y3 = (y1 * y2 + x1 * x2) * pow(1 - den, p - 2, p) % p
        zi = pow(Z3, p - 2, p)
        assert X3 * zi % p == x3 and Y3 * zi % p == y3
        assert T3 * Z3 % p == X3 * Y3 % p
        done += 1


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
