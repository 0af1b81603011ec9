"""Bound check and bit-exact model of kernels/fe25519.hpp (radix 2^25.5
arithmetic mod p = 2^255 - 19) as k_ed_point's Niels addition uses it.

`limb maxima` are propagated through add / sub / neg / mul exactly as the
device code computes them; every 64-bit product column and every 32-bit limb
(including 19 g_j) must stay below its register width.  `model_*` are
bit-exact Python restatements used by tests/test_fe25519_model.py.
usage: python tools/fe25519_bounds.py"""
P = 2**255 - 19
L = 10
WID = [26 if i % 2 == 0 else 25 for i in range(L)]
OFF = [(51 * i + 1) // 2 for i in range(L)]
MASK = [(1 << w) - 1 for w in WID]
P2 = [(1 << 27) - 38] + [(1 << (WID[i] + 1)) - 2 for i in range(1, L)]
U32, U64 = 1 << 32, 1 << 64


# ---------------------------------------------------------------- limb-maxima propagation
def mx_add(a, b):
    return [x + y for x, y in zip(a, b)]


def mx_sub(a, b):
    assert all(bi <= p for bi, p in zip(b, P2)), "sub: subtrahend limb above 2p's limb"
    return [x + p for x, p in zip(a, P2)]


def mx_neg(b):
    assert all(bi <= p for bi, p in zip(b, P2))
    return list(P2)


def mx_mul(f, g):
    """maxima of the product columns; returns the output maxima (normalized)"""
    g19 = [19 * x for x in g]
    assert max(g19[1:]) < U32 and max(f) < U32 and max(g) < U32, "limb or 19 g_j above 32 bits"
    f2 = [2 * x if i % 2 else x for i, x in enumerate(f)]
    assert max(f2) < U32
    h = [0] * L
    for i in range(L):
        for j in range(L):
            a = f2[i] if (i % 2 and j % 2) else f[i]
            b = g19[j] if i + j >= L else g[j]
            h[(i + j) % L] += a * b
    assert max(h) < U64, f"product column overflows 64 bits: {max(h).bit_length()} bits"
    # carry chain 0 -> 9 (each column grows by the carry in)
    for i in range(L - 1):
        h[i + 1] += h[i] >> WID[i]
        assert h[i + 1] < U64
    c = h[L - 1] >> 25
    t = MASK[0] + 19 * c
    assert t < U64
    out = list(MASK)
    out[1] = MASK[1] + (t >> 26)
    return out


NORM = None     # filled below: the normalized output maxima


def niels_addition_bounds():
    """k_ed_point add_niels on normalized X, Y, Z, T and a canonical (or
    negated) table entry; returns the largest column size in bits."""
    global NORM
    canon = list(MASK)
    negd = mx_neg(canon)                     # -2dxy = 2p - t2d (limbs up to 2p's)
    ent = [max(a, b) for a, b in zip(canon, negd)]
    # a fixed point: outputs of the addition feed the next one
    norm = mx_mul(canon, canon)
    for _ in range(3):
        X = Y = Z = T = norm
        t1 = mx_sub(Y, X)
        t2 = mx_add(Y, X)
        A = mx_mul(canon, t1)                # f = table entry, g = point side (ed25519.hip add_niels)
        B = mx_mul(canon, t2)
        C = mx_mul(ent, T)
        D = mx_add(Z, Z)
        E = mx_sub(B, A)
        F = mx_sub(D, C)
        G = mx_add(D, C)
        H = mx_add(B, A)
        outs = [mx_mul(F, E), mx_mul(H, G), mx_mul(H, E), mx_mul(F, G)]   # X3, Y3, T3, Z3
        new = [max(v) for v in zip(*outs)]
        if new == norm:
            break
        norm = [max(a, b) for a, b in zip(norm, new)]
    NORM = norm
    return norm


def extended_addition_bounds():
    """ed25519.hip add_ext (k_ed_point_split's lane combine): extended +
    extended on the normalized outputs of the Niels additions, k = 2d canonical"""
    norm = NORM if NORM is not None else niels_addition_bounds()
    canon = list(MASK)
    P_ = Q_ = norm
    t = mx_mul(Q_, canon)                    # 2d T2 (f = T2, g = the constant)
    C = mx_mul(t, P_)
    D = mx_add(mx_mul(P_, Q_), mx_mul(P_, Q_))
    F = mx_sub(D, C)
    G = mx_add(D, C)
    A = mx_mul(mx_sub(Q_, Q_), mx_sub(P_, P_))   # (Y2 - X2)(Y1 - X1)
    B = mx_mul(mx_add(Q_, Q_), mx_add(P_, P_))   # (Y2 + X2)(Y1 + X1)
    E = mx_sub(B, A)
    H = mx_add(B, A)
    outs = [mx_mul(F, E), mx_mul(H, G), mx_mul(H, E), mx_mul(F, G)]
    new = [max(v) for v in zip(*outs)]
    assert all(a <= b for a, b in zip(new, norm)), "add_ext outputs above the normalized maxima"
    return new


# ---------------------------------------------------------------- bit-exact model
def to_limbs(v):
    return [(v >> OFF[i]) & MASK[i] for i in range(L)]


def value(r):
    return sum(x << OFF[i] for i, x in enumerate(r))


def model_mul(f, g):
    g19 = [(19 * x) % U32 for x in g]
    f2 = [(2 * x) % U32 if i % 2 else x for i, x in enumerate(f)]
    h = [0] * L
    for i in range(L):
        for j in range(L):
            a = f2[i] if (i % 2 and j % 2) else f[i]
            b = g19[j] if i + j >= L else g[j]
            h[(i + j) % L] = (h[(i + j) % L] + a * b) % U64
    r = [0] * L
    for i in range(L - 1):
        h[i + 1] = (h[i + 1] + (h[i] >> WID[i])) % U64
        r[i] = h[i] & MASK[i]
    c = h[L - 1] >> 25
    r[L - 1] = h[L - 1] & MASK[L - 1]
    t = (r[0] + c * 19) % U64
    r[0] = t & MASK[0]
    r[1] = (r[1] + (t >> 26)) % U32
    return r


def model_canon(r):
    r = list(r)
    for _ in range(2):
        c = 0
        for i in range(L):
            v = (r[i] + c) % U32
            r[i] = v & MASK[i]
            c = v >> WID[i]
        r[0] = (r[0] + 19 * c) % U32
    c0 = r[0] >> 26
    r[0] &= MASK[0]
    r[1] += c0
    q = (r[0] + 19) >> 26
    for i in range(1, L):
        q = (r[i] + q) >> WID[i]
    r[0] += 19 * q
    c = 0
    for i in range(L):
        v = r[i] + c
        r[i] = v & MASK[i]
        c = v >> WID[i]
    return r


def main():
    norm = niels_addition_bounds()
    print("normalized limb maxima:", [hex(x) for x in norm])
    extended_addition_bounds()
    print("ok: every product column of the Niels addition and of add_ext fits 64 bits, every limb and 19 g_j 32 bits")


if __name__ == "__main__":
    main()
