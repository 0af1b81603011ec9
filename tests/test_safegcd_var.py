"""The variable-time safegcd of the one-launch small paths (kernels/mp.hpp
sg_divsteps28_var / inv_plain_var4: s^-1 mod n of a public signature scalar,
Z^-1 mod p of a public point) restated in Python by tools/safegcd_var_sim.py:
28-divstep batches on the low 32 bits with the var-time elimination of up to
6 / 4 bits per odd step, the batch matrix applied to the full f, g, d, e.
Here (CPU): the model inverts every order it is used with, its transition
matrices stay within 2^28 (the int32 limb updates' bound), every batch divides
f, g exactly, and it ends within twice the constant-time batch bound (the
kernel's loop cap)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import safegcd_var_sim as S  # noqa: E402

ED25519_P = (1 << 255) - 19


def test_var_time_inverse_matches_pow():
    rng = random.Random(11)
    for name, m in list(S.ORDERS.items()) + [("Ed25519 p", ED25519_P)]:
        bits = m.bit_length()
        cap = 2 * (((45907 * bits + 26313) // 19929 + 1 + 27) // 28)
        for a in [1, 2, 3, m - 1, m - 2, (m + 1) // 2] + [rng.randrange(1, m) for _ in range(60)]:
            x, batches, _ = S.inv_var(a, m, cap)
            assert x == pow(a, -1, m), (name, a)
            assert batches <= cap


def test_batch_matrix_bound_and_exact_division():
    rng = random.Random(5)
    m = S.ORDERS["P-256 n"]
    for _ in range(200):
        f, g = m, rng.randrange(1, m)
        eta = -1
        while g:
            eta, (u, v, q, r), _ = S.divsteps28_var(eta, f, g)
            assert max(abs(u) + abs(v), abs(q) + abs(r)) <= 1 << 28
            nf, ng = u * f + v * g, q * f + r * g
            assert nf % (1 << 28) == 0 and ng % (1 << 28) == 0
            f, g = nf >> 28, ng >> 28
        assert f in (1, -1)
