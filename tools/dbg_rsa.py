# debug helper (test infrastructure): RSA modexp mismatches by position / value
import sys, random
sys.path.insert(0, '.')
from tests.test_gpu_rsa import modexp, edge_sigs, CLS_RSA2K, CLS_RSA4K
import ctypes, os
L = ctypes.CDLL(os.path.join('cap_amd', sys.argv[1] if len(sys.argv) > 1 else 'libcapjwt_tk.so'))
L.tk_rsa_modexp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
for bits, cls in ((2048, CLS_RSA2K),):
    e = 65537
    rng = random.Random(bits * 1000003 + e)
    n = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    for name, sigs in (("edge", edge_sigs(n, rng, 200)), ("nm1-first", [n - 1] + [5] * 9), ("nm1-at4", [0, 1, 2, 3, n - 1, 7]),
                       ("nm1-at4-nz", [9, 1, 2, 3, n - 1, 7]), ("zero-first", [0, 5, 6]), ("rand", [rng.randrange(n) for _ in range(64)])):
        ys, ok = modexp(L, cls, n, e, sigs)
        bad = [(i, ok[i], ((ys[i] - pow(s, e, n)) % n).bit_length(), ys[i] == pow(s, e, n) + n, ((ys[i] - pow(s, e, n)) % n) == (1 << 2072) % n) for i, s in enumerate(sigs) if ys[i] != pow(s, e, n)]
        print(bits, name, len(sigs), 'bad', len(bad), bad[:6])
