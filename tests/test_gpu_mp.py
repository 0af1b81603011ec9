"""Device unit tests of the lazy 28-bit-limb Montgomery core (mp.hpp) and the
EC point primitives, against Python big-integer arithmetic (exact)."""
import ctypes
import os
import random

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, MASK = 28, (1 << 28) - 1

P256 = 0xffffffff00000001000000000000000000000000ffffffffffffffffffffffff
N256 = 0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551
P384 = 2**384 - 2**128 - 2**96 + 2**32 - 1
N384 = int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf581a0db248b0a77aecec196accc52973", 16)
P521 = 2**521 - 1
N521 = int("01fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffa51868783bf2f966b7fcc0148f709a5d03bb5c9b8899c47aebb6fb71e91386409", 16)
P25519 = 2**255 - 19
L25519 = 2**252 + 27742317777372353535851937790883648493
# field id -> (modulus, limbs, fold bit)
FIELDS = {0: (P256, 10, 256), 1: (N256, 10, None), 2: (P384, 15, 384), 3: (N384, 15, None),
          4: (P521, 20, 521), 5: (N521, 20, None), 6: (P25519, 10, 255), 7: (L25519, 10, None)}
CURVES = {
    1: dict(p=P256, n=N256, L=10, b=0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b,
            gx=0x6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296,
            gy=0x4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5),
    2: dict(p=P384, n=N384, L=15,
            b=int("b3312fa7e23ee7e4988e056be3f82d19181d9c6efe8141120314088f5013875ac656398d8a2ed19d2a85c8edd3ec2aef", 16),
            gx=int("aa87ca22be8b05378eb1c71ef320ad746e1d3b628ba79b9859f741e082542a385502f25dbf55296c3a545e3872760ab7", 16),
            gy=int("3617de4a96262c6f5d9e98bf9292dc29f8f41dbd289a147ce9da3113b5f0b8c00a60b1ce1d7e819d7a431d7c90ea0e5f", 16)),
    3: dict(p=P521, n=N521, L=20,
            b=int("0051953eb9618e1c9a1f929a21a0b68540eea2da725b99b315f3b8b489918ef109e156193951ec7e937b1652c0bd3bb1bf073573df883d2c34f1ef451fd46b503f00", 16),
            gx=int("00c6858e06b70404e9cd9e3ecb662395b4429c648139053fb521f828af606b4d3dbaa14b5e77efe75928fe1dc127a2ffa8de3348b3c1856a429bf97e7e31c2e5bd66", 16),
            gy=int("011839296a789a3bc0045c8a5fb42c7d1bd998f54449579b446817afbd17273e662c97ee72995ef42640c550b9013fad0761353c7086a272c24088be94769fd16650", 16)),
}


@pytest.fixture(scope="module")
def tk():
    path = os.path.join(ROOT, "cap_amd", "libcapjwt_tk.so")
    L = ctypes.CDLL(path)
    L.tk_field_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.tk_ec.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                        ctypes.c_int]
    return L


def to_limbs(v, L):
    out = []
    for _ in range(L):
        out.append(v & MASK)
        v >>= W
    assert v == 0
    return out


def from_limbs(ls):
    return sum(x << (W * i) for i, x in enumerate(ls))


def run_field(tk, fid, op, xs, ys):
    m, L, _ = FIELDS[fid]
    n = len(xs)
    A = (ctypes.c_uint32 * (n * L))(*[l for v in xs for l in to_limbs(v, L)])
    B = (ctypes.c_uint32 * (n * L))(*[l for v in ys for l in to_limbs(v, L)])
    O = (ctypes.c_uint32 * (n * L))()
    assert tk.tk_field_op(fid, op, A, B, O, n) == 0
    return [list(O[i * L:(i + 1) * L]) for i in range(n)]


@pytest.mark.parametrize("fid", sorted(FIELDS))
def test_mont_mul_sqr_inv(tk, fid):
    m, L, _ = FIELDS[fid]
    R = 1 << (W * L)
    Ri = pow(R, -1, m)
    rng = random.Random(fid)
    xs = [rng.randrange(m) for _ in range(200)] + [0, 1, m - 1, m - 2]
    ys = [rng.randrange(m) for _ in range(200)] + [m - 1, m - 1, m - 1, 1]
    # lazy inputs: values up to 2m with normalized limbs are legal too
    xs = [x + (m if i % 3 == 0 and x + m < R else 0) for i, x in enumerate(xs)]
    for op, fn in ((0, lambda x, y: x * y * Ri), (1, lambda x, y: x * x * Ri)):
        out = run_field(tk, fid, op, xs, ys)
        for x, y, o in zip(xs, ys, out):
            assert max(o) <= MASK
            v = from_limbs(o)
            assert v < 2 * m and v % m == fn(x, y) % m, (op, x, y)
    # mulf / sqrf (the point loop's products; P-384 uses its special-form
    # signed reduction): one operand with 28-bit limbs, the other lazy up to
    # the sub bound (a + KSUB - b); squares of normalized values
    lz = [x + (2 * m if i % 2 and x + 2 * m < R else 0) for i, x in enumerate(ys)]
    xn = [x % m + (m if i % 3 == 0 else 0) for i, x in enumerate(xs)]
    for op, a_, b_, fn in ((7, xn, lz, lambda x, y: x * y * Ri), (7, lz, xn, lambda x, y: x * y * Ri),
                           (8, xn, xn, lambda x, y: x * x * Ri)):
        out = run_field(tk, fid, op, a_, b_)
        for x, y, o in zip(a_, b_, out):
            assert max(o) <= MASK
            v = from_limbs(o)
            assert v < 2 * m and v % m == fn(x, y) % m, (op, x, y)
    # inverse of Montgomery-form values
    # (safegcd: random values plus the small / near-m / power-of-two / lazy
    # inputs that stress the divstep sign handling and the final normalisation)
    specials = [1, 2, 3, m - 1, m - 2, (m + 1) // 2, m // 3]
    specials += [1 << k for k in range(1, m.bit_length() - 1, 37)]
    specials += [m - (1 << k) for k in range(1, m.bit_length() - 1, 41)]
    xs2 = [rng.randrange(1, m) for _ in range(1024)]
    xm = [x * R % m for x in xs2] + [s * R % m for s in specials]
    xs2 += specials
    xm = [v + (m if i % 5 == 0 and v + m < R else 0) for i, v in enumerate(xm)]
    out = run_field(tk, fid, 2, xm, xm)
    for x, o in zip(xs2, out):
        assert from_limbs(o) % m == pow(x, -1, m) * R % m, x
    out = run_field(tk, fid, 2, [0], [0])
    assert from_limbs(out[0]) % m == 0
    xs2 = xs2[:64]
    xm = [x * R % m for x in xs2]
    # to / from Montgomery
    out = run_field(tk, fid, 3, xs2, xs2)
    assert all(from_limbs(o) % m == x * R % m for x, o in zip(xs2, out))
    out = run_field(tk, fid, 4, xm, xm)
    assert all(from_limbs(o) == x for x, o in zip(xs2, out))


@pytest.mark.parametrize("fid", [0, 2, 4, 6])
def test_freduce_canon(tk, fid):
    m, L, fold = FIELDS[fid]
    rng = random.Random(7 + fid)
    # lazy values: limbs up to 2^30, value below 2^(fold + 20)
    xs, lz = [], []
    for i in range(300):
        v = rng.randrange(1 << (fold + 20)) if i % 2 else rng.randrange(16 * m)
        xs.append(v)
    A = (ctypes.c_uint32 * (len(xs) * L))()
    for i, v in enumerate(xs):
        ls = to_limbs(v, L)
        # de-normalize: move 2 units of each limb down into the next as 2^29
        for j in range(L - 1):
            if ls[j + 1] >= 2:
                ls[j + 1] -= 2
                ls[j] += 2 << W
        for j in range(L):
            A[i * L + j] = ls[j]
    for canon in (0, 1):
        O = (ctypes.c_uint32 * (len(xs) * L))()
        assert tk.tk_field_op(fid, 100 + canon, A, A, O, len(xs)) == 0
        for i, v in enumerate(xs):
            o = list(O[i * L:(i + 1) * L])
            assert max(o) <= MASK
            r = from_limbs(o)
            assert r % m == v % m
            assert r < (m if canon else 2 * m)


def ec_add(c, P, Q):
    p = c["p"]
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0]:
        if (P[1] + Q[1]) % p == 0:
            return None
        lam = (3 * P[0] * P[0] - 3) * pow(2 * P[1], -1, p) % p
    else:
        lam = (Q[1] - P[1]) * pow(Q[0] - P[0], -1, p) % p
    x = (lam * lam - P[0] - Q[0]) % p
    return (x, (lam * (P[0] - x) - P[1]) % p)


def ec_mul(c, k, P):
    R = None
    while k:
        if k & 1:
            R = ec_add(c, R, P)
        P = ec_add(c, P, P)
        k >>= 1
    return R


# value bound of madd's X3 per curve id: P-256 subtracts inside r^2's columns
# (X3 < 8p + p + r^2/R, ecdsa.hip x3_from); P-384 / P-521 fold to < 2p
X3_BOUND = {1: 10, 2: 2, 3: 2}

@pytest.mark.parametrize("cid", [1, 2, 3])
def test_madd_z1_matches_affine_add(tk, cid):
    """madd_z1: the accumulator holds one affine table entry (Z = Montgomery 1)."""
    c = CURVES[cid]
    p, L = c["p"], c["L"]
    R = 1 << (W * L)
    G = (c["gx"], c["gy"])
    rng = random.Random(100 + cid)
    ins, want, N = [], [], 128
    for i in range(N):
        P1 = ec_mul(c, rng.randrange(1, c["n"]), G)
        P2 = ec_mul(c, rng.randrange(1, c["n"]), G)
        vals = [P1[0] * R % p, P1[1] * R % p, R % p, P2[0] * R % p, P2[1] * R % p]
        if i % 2:
            vals[1] = vals[1] + p if vals[1] + p < R else vals[1]
        ins += [l for v in vals for l in to_limbs(v, L)]
        want.append(ec_add(c, P1, P2))
    A = (ctypes.c_uint32 * len(ins))(*ins)
    O = (ctypes.c_uint32 * (N * 3 * L))()
    assert tk.tk_ec(cid, 2, A, ctypes.sizeof(A), O, ctypes.sizeof(O), N) == 0
    Ri = pow(R, -1, p)
    for i, w in enumerate(want):
        ls = [O[(3 * i + k) * L:(3 * i + k + 1) * L] for k in range(3)]
        assert all(max(l) <= MASK for l in ls)
        assert from_limbs(ls[0]) < X3_BOUND[cid] * p and from_limbs(ls[1]) < 2 * p
        X, Y, Z = (from_limbs(l) * Ri % p for l in ls)
        zi = pow(Z, -1, p)
        assert (X * zi * zi % p, Y * zi * zi * zi % p) == w


@pytest.mark.parametrize("cid", [1, 2, 3])
def test_madd_matches_affine_add(tk, cid):
    c = CURVES[cid]
    p, L = c["p"], c["L"]
    R = 1 << (W * L)
    G = (c["gx"], c["gy"])
    rng = random.Random(cid)
    ins, want = [], []
    N = 256
    for i in range(N):
        P1 = ec_mul(c, rng.randrange(1, c["n"]), G)
        P2 = ec_mul(c, rng.randrange(1, c["n"]), G)
        z = rng.randrange(1, p)
        X, Y, Z = P1[0] * z * z % p, P1[1] * z * z * z % p, z
        vals = [X * R % p, Y * R % p, Z * R % p, P2[0] * R % p, P2[1] * R % p]
        if i % 2:                           # lazy Jacobian inputs: values in [p, 2p) where they fit
            vals[:3] = [v + p if v + p < (1 << (W * L)) else v for v in vals[:3]]
            if i % 4 == 1:                  # X as a previous X3 may be: up to X3_BOUND p
                vals[0] += (X3_BOUND[cid] - 2) * p
        ins += [l for v in vals for l in to_limbs(v, L)]
        want.append(ec_add(c, P1, P2))
    A = (ctypes.c_uint32 * len(ins))(*ins)
    O = (ctypes.c_uint32 * (N * 3 * L))()
    assert tk.tk_ec(cid, 0, A, ctypes.sizeof(A), O, ctypes.sizeof(O), N) == 0
    Ri = pow(R, -1, p)
    for i, w in enumerate(want):
        for k in range(3):                  # outputs keep the normalized invariant: limbs < 2^28, value < 2p
            ls = O[(3 * i + k) * L:(3 * i + k + 1) * L]      # (X3 < 10p where r^2's columns subtract, ecdsa.hip x3_from)
            assert max(ls) <= MASK and from_limbs(ls) < (X3_BOUND[cid] if k == 0 else 2) * p
        X, Y, Z = (from_limbs(O[(3 * i + k) * L:(3 * i + k + 1) * L]) * Ri % p for k in range(3))
        zi = pow(Z, -1, p)
        assert (X * zi * zi % p, Y * zi * zi * zi % p) == w


@pytest.mark.parametrize("cid", [1, 2, 3])
def test_generator_table_entries(tk, cid):
    c = CURVES[cid]
    p, L = c["p"], c["L"]
    R = 1 << (W * L)
    G = (c["gx"], c["gy"])
    cw = {1: 26, 2: 24, 3: 20}[cid]                 # ecdsa.hpp ec_comb_w(cls, gen=true)
    nwin = -(-(c["n"].bit_length() + 1) // cw)
    ne = 1 << (cw - 1)
    wd = [(0, 1), (0, 2), (0, ne), (1, 1), (1, ne - 1), (5, 64), (nwin - 1, 1), (nwin - 1, ne), (nwin // 2, 77)]
    A = (ctypes.c_int * (2 * len(wd)))(*[v for t in wd for v in t])
    O = (ctypes.c_uint32 * (len(wd) * 2 * L))()
    assert tk.tk_ec(cid, 1, A, ctypes.sizeof(A), O, ctypes.sizeof(O), len(wd)) == 0
    for i, (w, d) in enumerate(wd):
        want = ec_mul(c, d << (cw * w), G)
        x = from_limbs(O[2 * i * L:(2 * i + 1) * L])
        y = from_limbs(O[(2 * i + 1) * L:(2 * i + 2) * L])
        assert (x, y) == (want[0] * R % p, want[1] * R % p), (w, d)
