"""ctypes binding of the C ABI in include/jg.h (libcapjwt.so).

This is plumbing for tests / bench / the Python mirror of cap's jwt package;
the product is the shared library.  There is deliberately no CPU fallback:
if libcapjwt.so is missing or no HIP device is present, every entry point
raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CAPJWT_LIB") or os.path.join(HERE, "libcapjwt.so")

# jwt/algs.go:12-21
ALG_IDS = {"RS256": 1, "RS384": 2, "RS512": 3, "PS256": 4, "PS384": 5, "PS512": 6,
           "ES256": 7, "ES384": 8, "ES512": 9, "EdDSA": 10}
KEY_RSA, KEY_EC, KEY_ED25519 = 1, 2, 3
CURVE_IDS = {"P-256": 1, "P-384": 2, "P-521": 3}

# every symbol include/jg.h declares
EXPORTS = ["jg_create", "jg_destroy", "jg_keys_load", "jg_verify_batch", "jg_last_error",
           "jg_host_alloc", "jg_host_free", "jg_batch_stage", "jg_batch_run", "jg_batch_enqueue", "jg_batch_sync",
           "jg_batch_free", "jg_batch_kernel_times", "jg_batch_exceptions", "jg_hash_batch", "jg_version",
           "jg_submit", "jg_wait", "jg_set_chunk", "jg_set_zero_copy", "jg_set_table_budget", "jg_keys_wait_tables",
           "jg_keys_table_widths", "jg_debug_fail_alloc", "jg_debug_table_digest",
           "jg_debug_max_upgrades", "jg_debug_lifetime_check", "jg_debug_fail_verify", "jg_debug_tables_built",
           "jg_debug_small_path"]


class JgKey(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("curve", ctypes.c_int32),
                ("n", ctypes.c_void_p), ("n_len", ctypes.c_int32), ("e", ctypes.c_uint64),
                ("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("coord_len", ctypes.c_int32)]


class JgTok(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("sig_in_len", ctypes.c_uint32), ("sig_rel_off", ctypes.c_uint32),
                ("sig_b64_len", ctypes.c_uint32), ("key_idx", ctypes.c_uint16), ("alg", ctypes.c_uint8),
                ("flags", ctypes.c_uint8)]


assert ctypes.sizeof(JgTok) == 24

_lib = None


class JgError(RuntimeError):
    pass


def lib():
    """Load libcapjwt.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise JgError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.jg_create.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.jg_create.restype = vp
        L.jg_destroy.argtypes = [vp]
        L.jg_keys_load.argtypes = [vp, ctypes.POINTER(JgKey), ctypes.c_int]
        L.jg_verify_batch.argtypes = [vp, vp, sz, ctypes.POINTER(JgTok), sz, vp]
        L.jg_last_error.argtypes = [vp]
        L.jg_last_error.restype = ctypes.c_char_p
        L.jg_host_alloc.argtypes = [sz]
        L.jg_host_alloc.restype = vp
        L.jg_host_free.argtypes = [vp]
        L.jg_batch_stage.argtypes = [vp, ctypes.c_int, vp, sz, ctypes.POINTER(JgTok), sz, ctypes.POINTER(vp)]
        L.jg_batch_run.argtypes = [vp, vp, vp]
        L.jg_batch_enqueue.argtypes = [vp, vp, vp]
        L.jg_batch_sync.argtypes = [vp, vp]
        L.jg_batch_free.argtypes = [vp, vp]
        L.jg_batch_kernel_times.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float),
                                            ctypes.c_int]
        L.jg_batch_exceptions.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        L.jg_submit.argtypes = [vp, vp, sz, ctypes.POINTER(JgTok), sz, vp, ctypes.POINTER(vp)]
        L.jg_wait.argtypes = [vp, vp]
        L.jg_set_chunk.argtypes = [vp, sz]
        L.jg_set_zero_copy.argtypes = [vp, ctypes.c_int, sz]
        L.jg_set_table_budget.argtypes = [vp, ctypes.c_uint64]
        L.jg_hash_batch.argtypes = [vp, vp, sz, vp, sz, vp]
        L.jg_keys_wait_tables.argtypes = [vp]
        L.jg_keys_table_widths.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.jg_debug_fail_alloc.argtypes = [vp, ctypes.c_int]
        L.jg_debug_max_upgrades.argtypes = [vp, ctypes.c_int]
        L.jg_debug_fail_verify.argtypes = [vp, ctypes.c_int]
        L.jg_debug_lifetime_check.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                              ctypes.POINTER(ctypes.c_uint64)]
        L.jg_debug_table_digest.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.jg_debug_tables_built.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.jg_debug_small_path.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        L.jg_version.restype = ctypes.c_char_p
        _lib = L
    return _lib


def lifetime_check(enable=-1):
    """jg_debug_lifetime_check: 1 / 0 turns the key-memory lifetime check on /
    off (-1 leaves it); returns (violations, events checked) so far."""
    bad, chk = ctypes.c_uint64(), ctypes.c_uint64()
    lib().jg_debug_lifetime_check(int(enable), ctypes.byref(bad), ctypes.byref(chk))
    return bad.value, chk.value


class Key:
    """A public key handed to jg_keys_load (bytes are big-endian; Ed25519: raw 32 bytes)."""

    def __init__(self, kind, n=b"", e=0, curve=0, x=b"", y=b""):
        self.kind, self.n, self.e, self.curve, self.x, self.y = kind, n, e, curve, x, y

    @staticmethod
    def rsa(n: bytes, e: int):
        return Key(KEY_RSA, n=n, e=e)

    @staticmethod
    def ec(curve: str, x: bytes, y: bytes):
        return Key(KEY_EC, curve=CURVE_IDS[curve], x=x, y=y)

    @staticmethod
    def ed25519(pub: bytes):
        return Key(KEY_ED25519, x=pub)


class Arena:
    """Packed job list: signing inputs and base64url signatures in one buffer."""

    def __init__(self):
        self.buf = bytearray()
        self.toks = []

    def add(self, signing_input: bytes, sig_b64: bytes, alg: str, key_idx: int):
        sig_b64 = sig_b64.rstrip(b"=")
        off = len(self.buf)
        self.buf += signing_input + b"." + sig_b64
        self.toks.append((off, len(signing_input), len(signing_input) + 1, len(sig_b64), key_idx,
                          ALG_IDS.get(alg, 0)))
        return len(self.toks) - 1

    def tok_array(self):
        arr = (JgTok * max(1, len(self.toks)))()
        for i, t in enumerate(self.toks):
            arr[i].off, arr[i].sig_in_len, arr[i].sig_rel_off, arr[i].sig_b64_len, arr[i].key_idx, arr[i].alg = t
        return arr


class Context:
    """Owns a jg_ctx on the given HIP devices."""

    def __init__(self, devices=None):
        L = lib()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            self.h = L.jg_create(arr, len(devices))
        else:
            self.h = L.jg_create(None, 0)
        if not self.h:
            raise JgError("jg_create failed: " + (L.jg_last_error(None) or b"").decode())
        self._keep = []

    def close(self):
        if self.h:
            lib().jg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self):
        return (lib().jg_last_error(self.h) or b"").decode()

    def load_keys(self, keys, wait_tables=True):
        """jg_keys_load; with wait_tables (default) also jg_keys_wait_tables, so
        every key runs at its budgeted comb width when this returns."""
        arr = (JgKey * max(1, len(keys)))()
        keep = []
        for i, k in enumerate(keys):
            arr[i].kind = k.kind
            arr[i].curve = k.curve
            for fld in ("n", "x", "y"):
                b = getattr(k, fld)
                if b:
                    cb = ctypes.create_string_buffer(bytes(b), len(b))
                    keep.append(cb)
                    setattr(arr[i], fld, ctypes.cast(cb, ctypes.c_void_p))
            arr[i].n_len = len(k.n)
            arr[i].e = k.e
            arr[i].coord_len = len(k.x) if k.kind != KEY_RSA else 0
        rc = lib().jg_keys_load(self.h, arr, len(keys))
        if rc != 0:
            raise JgError(f"jg_keys_load rc={rc}: {self.error()}")
        if wait_tables:
            self.wait_tables()

    def wait_tables(self):
        """jg_keys_wait_tables: True when every table reached its budgeted width."""
        rc = lib().jg_keys_wait_tables(self.h)
        if rc < 0:
            raise JgError(f"jg_keys_wait_tables rc={rc}")
        return rc == 0

    def table_widths(self):
        """jg_keys_table_widths: comb width per loaded key (0 = none)."""
        n = lib().jg_keys_table_widths(self.h, None, 0)
        arr = (ctypes.c_int * max(1, n))()
        lib().jg_keys_table_widths(self.h, arr, n)
        return list(arr[:n])

    def table_digest(self, key):
        """jg_debug_table_digest: 64-bit digest of key `key`'s comb table (0 = none)."""
        v = ctypes.c_uint64()
        if lib().jg_debug_table_digest(self.h, int(key), ctypes.byref(v)) != 0:
            raise JgError(f"jg_debug_table_digest: {self.error()}")
        return v.value

    def tables_built(self):
        """jg_debug_tables_built: comb tables this context has built (cache reuses excluded)."""
        v = ctypes.c_uint64()
        if lib().jg_debug_tables_built(self.h, ctypes.byref(v)) != 0:
            raise JgError(f"jg_debug_tables_built: {self.error()}")
        return v.value

    def debug_max_upgrades(self, n):
        """jg_debug_max_upgrades: the background upgrader widens at most n more tables (-1 = no limit)."""
        if lib().jg_debug_max_upgrades(self.h, int(n)) != 0:
            raise JgError("jg_debug_max_upgrades failed")

    def debug_small_path(self, enable=None):
        """jg_debug_small_path: small ECDSA submissions as one launch per curve (True, the
        default) or through the batch chain (False; None leaves it); returns the
        number of one-launch verifications enqueued so far.  Verdicts are identical."""
        v = ctypes.c_uint64()
        if lib().jg_debug_small_path(self.h, -1 if enable is None else (1 if enable else 0), ctypes.byref(v)) != 0:
            raise JgError("jg_debug_small_path failed")
        return v.value

    def debug_fail_alloc(self, n):
        """jg_debug_fail_alloc: the n-th device allocation of later key loads fails (0 = off)."""
        if lib().jg_debug_fail_alloc(self.h, int(n)) != 0:
            raise JgError("jg_debug_fail_alloc failed")

    def debug_fail_verify(self, n):
        """jg_debug_fail_verify: the n-th later submission fails as a device fault and the
        context stays unusable (0 = off)."""
        if lib().jg_debug_fail_verify(self.h, int(n)) != 0:
            raise JgError("jg_debug_fail_verify failed")

    def verify(self, arena: Arena):
        n = len(arena.toks)
        out = (ctypes.c_uint8 * max(1, n))()
        buf = bytes(arena.buf) or b"\0"
        rc = lib().jg_verify_batch(self.h, buf, len(arena.buf), arena.tok_array(), n, out)
        if rc != 0:
            raise JgError(f"jg_verify_batch rc={rc}: {self.error()}")
        return bytes(out[:n])

    def set_chunk(self, jobs):
        if lib().jg_set_chunk(self.h, jobs) != 0:
            raise JgError("jg_set_chunk: chunk must be >= 64 jobs")

    def set_zero_copy(self, enable, max_jobs=0):
        """jg_set_zero_copy: class-major zero-copy plans for mixed batches whose
        arena is a PinnedBuffer (off by default), and the jobs per plan."""
        if lib().jg_set_zero_copy(self.h, 1 if enable else 0, max_jobs) != 0:
            raise JgError("jg_set_zero_copy: max_jobs must be 0 or >= 64")

    def set_table_budget(self, nbytes):
        """jg_set_table_budget: HBM for all key comb tables (applies at the next load_keys)."""
        if lib().jg_set_table_budget(self.h, int(nbytes)) != 0:
            raise JgError("jg_set_table_budget failed")

    def submit(self, arena: Arena):
        """jg_submit; returns a Pending whose wait() gives the verdict bytes."""
        return Pending(self, arena)

    # ---- device-resident batches (bench)
    def stage(self, arena: Arena, slot=0):
        h = ctypes.c_void_p()
        buf = bytes(arena.buf) or b"\0"
        rc = lib().jg_batch_stage(self.h, slot, buf, len(arena.buf), arena.tok_array(), len(arena.toks),
                                  ctypes.byref(h))
        if rc != 0:
            raise JgError(f"jg_batch_stage rc={rc}: {self.error()}")
        return Batch(self, h, len(arena.toks))


class Pending:
    """One jg_submit in flight (buffers kept alive until wait())."""

    def __init__(self, ctx, arena):
        self.ctx = ctx
        self.n = len(arena.toks)
        self.buf = ctypes.create_string_buffer(bytes(arena.buf) or b"\0", max(1, len(arena.buf)))
        self.toks = arena.tok_array()
        self.out = (ctypes.c_uint8 * max(1, self.n))()
        self.t = ctypes.c_void_p()
        rc = lib().jg_submit(ctx.h, self.buf, len(arena.buf), self.toks, self.n, self.out, ctypes.byref(self.t))
        if rc != 0:
            raise JgError(f"jg_submit rc={rc}: {ctx.error()}")

    def wait(self):
        rc = lib().jg_wait(self.ctx.h, self.t)
        self.t = None
        if rc != 0:
            raise JgError(f"jg_wait rc={rc}: {self.ctx.error()}")
        return bytes(self.out[:self.n])


class PinnedBuffer:
    """Page-locked host memory from jg_host_alloc (hipHostMalloc)."""

    def __init__(self, nbytes):
        self.n = nbytes
        self.ptr = lib().jg_host_alloc(max(1, nbytes))
        if not self.ptr:
            raise JgError("jg_host_alloc failed")

    def bytes(self):
        return ctypes.string_at(self.ptr, self.n)

    def free(self):
        if self.ptr:
            lib().jg_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Batch:
    def __init__(self, ctx, h, n):
        self.ctx, self.h, self.n = ctx, h, n

    def run(self, want_verdicts=False):
        out = (ctypes.c_uint8 * max(1, self.n))() if want_verdicts else None
        rc = lib().jg_batch_run(self.ctx.h, self.h, out)
        if rc != 0:
            raise JgError(f"jg_batch_run rc={rc}: {self.ctx.error()}")
        return bytes(out[:self.n]) if want_verdicts else None

    def enqueue(self, pinned_verdicts=None):
        """Enqueue one run without waiting; verdicts land in `pinned_verdicts`
        (a PinnedBuffer) once sync() returns."""
        ptr = pinned_verdicts.ptr if pinned_verdicts is not None else None
        rc = lib().jg_batch_enqueue(self.ctx.h, self.h, ptr)
        if rc != 0:
            raise JgError(f"jg_batch_enqueue rc={rc}: {self.ctx.error()}")

    def sync(self):
        rc = lib().jg_batch_sync(self.ctx.h, self.h)
        if rc != 0:
            raise JgError(f"jg_batch_sync rc={rc}: {self.ctx.error()}")

    def exceptions(self):
        """Per-class count of tokens the last run sent down the exact ECDSA path."""
        c = (ctypes.c_uint32 * 8)()
        n = lib().jg_batch_exceptions(self.h, c, 8)
        if n < 0:
            raise JgError(f"jg_batch_exceptions rc={n}: {self.ctx.error()}")
        return list(c)

    def kernel_times(self):
        names = (ctypes.c_char_p * 64)()
        ms = (ctypes.c_float * 64)()
        n = lib().jg_batch_kernel_times(self.h, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(min(n, 64))]

    def free(self):
        if self.h:
            lib().jg_batch_free(self.ctx.h, self.h)
            self.h = None
