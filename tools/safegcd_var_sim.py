"""Model of the variable-time safegcd inversion in kernels/mp.hpp
(sg_divsteps28_var / inv_plain_var): 28-divstep batches on the low 32 bits,
Wuille's var-time divsteps (trailing zeros in one step, up to 6 / 4 bits of g
cancelled per odd step), the batch matrix applied to the full-width f, g and to
d, e.  Checks a * a^-1 == 1 and reports batches and odd steps per inversion.
usage: python tools/safegcd_var_sim.py [count]"""
import random
import statistics
import sys

ORDERS = {
    "P-256 n": 0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551,
    "P-384 n": int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf"
                   "581a0db248b0a77aecec196accc52973", 16),
    "P-521 n": int("01ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff"
                   "fa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409", 16),
}
M32 = (1 << 32) - 1


def divsteps28_var(eta, f, g):
    """one batch; f, g are the low 32 bits (mod 2^32 arithmetic as on the GPU)"""
    u, v, q, r = 1, 0, 0, 1
    i, odd = 28, 0
    f &= M32
    g &= M32
    while True:
        x = g | ((M32 << i) & M32)
        zeros = (x & -x).bit_length() - 1
        g >>= zeros
        u <<= zeros
        v <<= zeros
        eta -= zeros
        i -= zeros
        if i == 0:
            break
        odd += 1
        if eta < 0:
            eta = -eta
            f, g = g, (-f) & M32
            u, q = q, -u
            v, r = r, -v
            limit = min(eta + 1, i)
            m = (M32 >> (32 - limit)) & 63
            w = (f * g * (f * f - 2)) & m
        else:
            limit = min(eta + 1, i)
            m = (M32 >> (32 - limit)) & 15
            w = f + (((f + 1) & 4) << 1)
            w = (-w * g) & m
        g = (g + f * w) & M32
        q += u * w
        r += v * w
    for x in (u, v, q, r):
        assert abs(x) <= 1 << 28
    return eta, (u, v, q, r), odd


def inv_var(a, m, max_batches):
    f, g, d, e, eta = m, a, 0, 1, -1
    batches = odd = 0
    inv28 = pow(2, -28, m)
    while g != 0:
        assert batches < max_batches
        eta, (u, v, q, r), k = divsteps28_var(eta, f, g)
        odd += k
        batches += 1
        f, g = (u * f + v * g), (q * f + r * g)
        assert f % (1 << 28) == 0 and g % (1 << 28) == 0     # the shift is exact
        f >>= 28
        g >>= 28
        d, e = (u * d + v * e) * inv28 % m, (q * d + r * e) * inv28 % m
    assert f in (1, -1)
    return (d if f == 1 else -d) % m, batches, odd


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    rng = random.Random(7)
    out = {}
    for name, m in ORDERS.items():
        bits = m.bit_length()
        ct_batches = ((45907 * bits + 26313) // 19929 + 1 + 27) // 28
        B, O = [], []
        for a in [1, 2, m - 1, m - 2] + [rng.randrange(1, m) for _ in range(count)]:
            x, b, o = inv_var(a, m, 2 * ct_batches)
            assert x * a % m == 1
            B.append(b)
            O.append(o)
        out[name] = {"const_time_batches": ct_batches, "batches_mean": statistics.mean(B), "batches_max": max(B),
                     "odd_steps_mean": statistics.mean(O)}
        print(name, out[name])
    return out


if __name__ == "__main__":
    main()
