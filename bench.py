#!/usr/bin/env python3
"""Throughput benchmark for the MI355X batched JWS verifier (BASELINE.json metric).

A "step" = one pass of the verify hot path (libcapjwt.so: base64url + SHA-2 +
signature arithmetic + verdict scatter, then the verdict bytes copied to the
host) over one batch of synthetic signed tokens already resident in HBM.

Headline workload (BASELINE.json configs[1]): ES256, P-256 JWKS with 4 kids,
1,048,576 tokens per GPU.  Second half of the metric: RS256 RSA-2048 on the same
batch size (reported under "rs256").  The other BASELINE configs are reported
under "configs" (per-GPU share of each, same timing rules), the end-to-end
Validator.ValidateBatch rate (host parse + GPU + claims) under "e2e".  Tokens
are signed by OpenSSL (tools/tokgen) from a unique pool replicated to the batch
size; verdicts are never cached, and every line checks its accept count.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, weak scaling)
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

KEYDIR = os.path.join(ROOT, "tests", "golden", "keys")
BENCHKEYS = os.path.join(ROOT, "tools", "benchkeys")
TOKGEN = os.path.join(ROOT, "tools", "tokgen", "tokgen")
TRAFFIC = os.path.join(ROOT, "profiles", "r06_s12_pmc_traffic.json")
COLL_DEVICE = "cuda"            # device of the timing all-reduce (RCCL); "cpu" under gloo

# measured v_mad_u64_u32 issue rate, chip-wide: the integer multiply-add
# roofline denominator.  36.98 T lane-MAD/s = 8 waves/SIMD, 8 MADs per asm
# statement (no hazard padding), profiles/r01_int_rates2.json -- i.e. one
# wave64 VALU instruction per 4 cycles per SIMD, the chip's full VALU issue rate.
MAD_PEAK_T = 36.98
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)

JG_TOK = np.dtype([("off", "<u8"), ("sig_in_len", "<u4"), ("sig_rel_off", "<u4"), ("sig_b64_len", "<u4"),
                   ("key_idx", "<u2"), ("alg", "u1"), ("flags", "u1")])
assert JG_TOK.itemsize == 24
ALG_IDS = {"RS256": 1, "RS384": 2, "RS512": 3, "PS256": 4, "PS384": 5, "PS512": 6,
           "ES256": 7, "ES384": 8, "ES512": 9, "EdDSA": 10}


# ---------------------------------------------------------------- algorithmic work
P256_WQ = 24          # key comb width of the run (main() sets it from the table budget)


def p256_point_mads_per_token(wq=None):
    """Algorithmic multiply-accumulates (v_mad_u64_u32 on 28-bit limbs) the P-256 comb kernel
    (k_ec_point) issues per token: 28-bit limbs, L = 10; a product is L^2 (mul)
    or L(L+1)/2 (sqr) partial products, a Montgomery reduction L * 4 (p + 1 has
    4 non-zero limbs above limb 0, mp.hpp).  Mixed addition = 8 mul + 3 sqr
    under 10 reductions (Y3 = r t - Y1 hhh sums two products under one,
    ecdsa.hip y3_from; X3's subtractions ride in r^2's columns, x3_from, so no
    value fold).  The carry MADs of the unmasked reduction rows (hi32 * 16,
    mp.hpp mont_reduce) and the column adds of x3_from are carries / additions,
    not partial products, and are not counted.
    Signed comb digits (ecdsa.hpp ec_comb_w / ec_key_w): 10 windows of 26
    bits for u1 (generator table) and ceil(257 / wq) for u2 (key table: W = 26
    for the bench's 4 kids under its 110 GiB table budget, 10 windows),
    each non-zero w.p. 1 - 2^-W, the first addition an assignment and the
    second onto Z == 1 (madd_z1: 4 mul + 2 sqr under 5 reductions); final check
    1 sqr + 2 mul."""
    return ec_point_mads_per_token(10, 4, 0, 26, wq or P256_WQ, 256, 10 * 4, merged=True)


# key comb-table width tiers, widest first (kernels/ecdsa.hpp EC_*_WQ, ed25519.hpp ED_WA)
WIDTH_TIERS = {"p256": (26, 24, 22, 20), "p384": (24, 20, 18, 16), "ed25519": (24, 22, 20, 18, 16), "p521": (20, 18, 16)}
# (bits + 2 for EC / 254 for Ed25519, entry bytes): ceil(that / W) windows
# (ecdsa.hpp ec_windows_w, ed25519.hpp ed_windows_w); P-256 entries are packed
# to 64 B (ecdsa.hpp JG_EC_PACK64)
_TAB = {"p256": (258, 64), "p384": (386, 128), "p521": (523, 160), "ed25519": (254, 128)}


def table_bytes(cls, w):
    """Bytes of one key comb table: ceil((bits + 2) / W) windows x 2^(W-1) entries."""
    bits, entry = _TAB[cls]
    return -(-bits // w) * (1 << (w - 1)) * entry


def key_widths(counts, budget):
    """jg_runtime.cpp key_widths: one budget over all curves' key tables.  Every
    key starts at its curve's narrowest width; then P-256, P-384, Ed25519,
    P-521 in that order each take the widest tier that still fits."""
    w = {c: t[-1] for c, t in WIDTH_TIERS.items()}
    used = sum(counts.get(c, 0) * table_bytes(c, w[c]) for c in w)
    for c in ("p256", "p384", "ed25519", "p521"):
        n = counts.get(c, 0)
        if not n:
            continue
        for t in WIDTH_TIERS[c]:
            extra = n * (table_bytes(c, t) - table_bytes(c, w[c]))
            if used + extra <= budget:
                w[c] = t
                used += extra
                break
    return w


def p256_key_w(nkeys, budget):
    """The P-256 key comb width of a load holding `nkeys` P-256 keys and
    nothing else (W = 26 / 24 / 22 / 20)."""
    return key_widths({"p256": nkeys}, budget)["p256"]


def ec_point_mads_per_token(L, red_row, fold, wg, wq, bits, red_generic, merged):
    """Algorithmic multiply-accumulates of a comb point kernel (k_ec_point) per
    token: products are L^2 (mul) or L(L+1)/2 (sqr) partial products, a
    reduction is L rows x `red_row` non-zero reduction constants; a mixed
    addition is 8 mul + 3 sqr under 11 reductions and 2 value folds (`fold`
    MADs each), or under 10 reductions and 1 fold where Y3's two products share
    one reduction (`merged`, ecdsa.hip sum_ok; fold = 0 where X3 needs none);
    the first addition is an
    assignment, the second lands on Z == 1 (4 mul + 2 sqr); the final check is
    1 sqr + 2 mul with the generic reduction."""
    red = L * red_row
    nred, nfold = (10, 1) if merged else (11, 2)
    madd = 8 * L * L + 3 * L * (L + 1) // 2 + nred * red + nfold * fold
    madd_z1 = 4 * L * L + 2 * L * (L + 1) // 2 + (nred - 5) * red + nfold * fold
    ng, nq = (bits + 2 + wg - 1) // wg, (bits + 2 + wq - 1) // wq
    adds = ng * (1 - 2.0 ** -wg) + nq * (1 - 2.0 ** -wq) - 1
    gmul, gsqr = L * L + red_generic, L * (L + 1) // 2 + red_generic
    return (adds - 1) * madd + madd_z1 + gsqr + 2 * gmul


def p384_key_w(nkeys, budget):
    """The P-384 key comb width of a load holding `nkeys` P-384 keys and
    nothing else (W = 24 / 20 / 18 / 16)."""
    return key_widths({"p384": nkeys}, budget)["p384"]


P384_BUDGET = 32 << 30    # main() sets the run's table budget


def p384_point_mads_per_token(wq=None, nkeys=1):
    """P-384 (ecdsa.hpp: L = 15 28-bit limbs, G W = 24 (20 before round 6), key W = 24 / 20 / 18 / 16
    by the table budget -- 24 for config 3's single key): the hot loop's mulf /
    sqrf use the special-form reduction, 4 signed MADs per row (mp.hpp
    mont_reduce_p384); value folds through freduce (5 non-zero constants of
    2^384 mod p); final check with m+1's 12 non-zero limbs."""
    return ec_point_mads_per_token(15, 4, 5, 24, wq or p384_key_w(nkeys, P384_BUDGET), 384, 15 * 12, merged=False)


def p521_key_w(nkeys, budget):
    """The P-521 key comb width of a load holding `nkeys` P-521 keys and
    nothing else (W = 20 / 18 / 16)."""
    return key_widths({"p521": nkeys}, budget)["p521"]


def p521_point_mads_per_token(wq=None, nkeys=1):
    """P-521 (ecdsa.hpp: L = 20 28-bit limbs, G W = 20, key W = 20 / 18 / 16
    by the table budget): p = 2^521 - 1, so m + 1 = 2^521 has ONE non-zero
    28-bit limb (M1[18] = 2^17, field_consts.hpp P521P) and a Montgomery
    reduction row is one constant MAD (the unmasked rows' hi32 * 16 carry MADs
    are carries, not counted); Y3's two products share one reduction
    (ecdsa_impl.hpp y3_from, sum_ok), X3 = r^2 - hhh - 2v is one value fold
    through freduce (2^521 = 1 mod p: FOLDC = 1, one MAD); the final check's
    generic reduction is the same one-constant row."""
    return ec_point_mads_per_token(20, 1, 1, 20, wq or p521_key_w(nkeys, P384_BUDGET), 521, 20 * 1, merged=True)


def ed25519_point_mads_per_token(wa=24):
    """k_ed_point: 11 comb windows of the base point (W = 24) + ceil(254 / wa)
    of the key (ed25519.hpp ED_WA: W = 24 / 22 / 20 / 18 / 16 by the table
    budget), each a Niels addition of 7 field products (ed25519.hip
    add_niels) in radix 2^25.5 (kernels/fe25519.hpp): 100 partial products
    and the one MAD that folds the carry out of the top limb (x 19) -- no
    reduction rows.  Plus k = H mod L (one Montgomery reduction + one product
    mod L, 28-bit limbs: 220)."""
    L = 10
    mul = L * L + 1
    adds = 11 * (1 - 2.0 ** -24) + -(-254 // wa) * (1 - 2.0 ** -wa)
    return adds * 7 * mul + 220


def rsa_modexp_mads_per_token(limbs, lanes):
    """k_rsa_modexp (e = 65537): 18 Montgomery products on L 28-bit limbs held
    by `lanes` lanes per token (H = L / lanes each; RSA-2048: L = 74 on 2 lanes,
    RSA-3072: 112 on 2 (rsa.hpp RSA3K_G), RSA-4096: 148 on 4).  To-Montgomery and the final
    multiply (mont_mul) are 2 L^2 multiply-accumulates each; the 16 squarings
    (mont_sqr) issue each limb product once -- lanes^2 * H(H+1)/2 for the
    square (L(L+1)/2 plus the diagonal blocks' duplicated diagonal) + L^2 for
    the reduction."""
    h = limbs // lanes
    sqr = lanes * lanes * h * (h + 1) // 2 + limbs * limbs
    return 2 * 2 * limbs * limbs + 16 * sqr


def prep_bytes_per_token(token_bytes, sig_rows):
    """Algorithmic HBM bytes of k_prep per token: the token's signing input and
    signature read once, the 24-B job + 4-B plan entry, the decoded signature
    rows (4 B each), 16 digest words, status + signature length."""
    return token_bytes + 28 + 4 * sig_rows + 64 + 3


# ---------------------------------------------------------------- inputs
def ensure_tokgen():
    if not os.path.exists(TOKGEN):
        subprocess.run(["make", "-s", "-C", os.path.dirname(TOKGEN)], check=True)


def gen_tokens(alg, count, keypaths, threads, tag, kid_base=0):
    ensure_tokgen()
    out = os.path.join("/tmp", f"capjwt_{tag}_{alg}_{count}_{kid_base}_{os.getpid()}.txt")
    env = dict(os.environ, TOKGEN_KID_BASE=str(kid_base))
    subprocess.run([TOKGEN, alg, str(count), str(threads), out] + list(keypaths), check=True, env=env)
    with open(out, "rb") as f:
        toks = f.read().split(b"\n")[:count]
    os.unlink(out)
    return toks


def golden_keypaths(kids):
    return [os.path.join(KEYDIR, k + ".pem") for k in kids]


def pack(pool, algs, keyidx, total):
    """Pack a unique token pool (with per-token alg id and key index) into
    (arena bytes, jg_tok array), replicated to `total` jobs."""
    lens = np.fromiter((len(t) for t in pool), dtype=np.int64, count=len(pool))
    dots = np.fromiter((t.rfind(b".") for t in pool), dtype=np.int64, count=len(pool))
    offs = np.zeros(len(pool), dtype=np.int64)
    offs[1:] = np.cumsum(lens)[:-1]
    blob = b"".join(pool)
    reps = (total + len(pool) - 1) // len(pool)
    arena = blob * reps
    idx = np.arange(reps * len(pool)) % len(pool)
    toks = np.zeros(reps * len(pool), dtype=JG_TOK)
    toks["off"] = offs[idx] + (np.arange(reps * len(pool)) // len(pool)) * len(blob)
    toks["sig_in_len"] = dots[idx]
    toks["sig_rel_off"] = dots[idx] + 1
    toks["sig_b64_len"] = (lens - dots - 1)[idx]
    toks["key_idx"] = np.asarray(keyidx)[idx]
    toks["alg"] = np.asarray(algs)[idx]
    return arena, toks[:total]


def abi_keys(names):
    from tests import gpu_helpers as H
    keys, _ = H.golden()
    by = {k["kid"]: k for k in keys}
    return [H.abi_key(by[n]) for n in names]


def bench_keys():
    """tools/benchkeys/kids.json -> [(kid, alg, pem path, _lib.Key, jwk)]"""
    import base64
    from cap_amd import _lib
    def d(s):
        return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))
    out = []
    for k in json.load(open(os.path.join(BENCHKEYS, "kids.json"))):
        j = k["jwk"]
        if j["kty"] == "RSA":
            key = _lib.Key.rsa(d(j["n"]), int.from_bytes(d(j["e"]), "big"))
        elif j["kty"] == "EC":
            key = _lib.Key.ec(j["crv"], d(j["x"]), d(j["y"]))
        else:
            key = _lib.Key.ed25519(d(j["x"]))
        out.append((k["kid"], k["alg"], os.path.join(BENCHKEYS, k["pem"]), key, j))
    return out


# ---------------------------------------------------------------- measurement
def measure(ctx, arena, toks, steps, warmup, dist, second=None):
    """Stage the batch (and a second one: `second` = (arena, toks), default a
    copy of the first) and time `steps` steps enqueued back to back,
    alternating between the two staged batches.  The runtime puts consecutive
    resident batches on two lanes on different hardware queues, so one step's
    front kernels overlap the previous step's point kernel (jg_runtime.cpp
    batch_lanes); each step is a complete pass over its own 1 x `len(toks)`
    jobs (its own device arena copy and scratch, verdicts copied back every
    step).  BENCH_ONE_BATCH=1 times one staged batch alone (round-2 layout)."""
    from cap_amd import _lib
    from cap_amd.shard import max_over_ranks
    global LAST_WINDOW, LAST_SYNC_MS
    L = _lib.lib()

    def stage(ar, tk):
        h = ctypes.c_void_p()
        if L.jg_batch_stage(ctx.h, 0, ar, len(ar), tk.ctypes.data_as(ctypes.POINTER(_lib.JgTok)), len(tk),
                            ctypes.byref(h)) != 0:
            raise RuntimeError(ctx.error())
        return _lib.Batch(ctx, h, len(tk))
    b = stage(arena, toks)
    v = np.frombuffer(b.run(want_verdicts=True), dtype=np.uint8)
    accepted = int(v.sum())
    pinned = _lib.PinnedBuffer(len(toks))
    batches = [(b, pinned, accepted)]
    if os.environ.get("BENCH_ONE_BATCH") != "1":
        a2, t2 = second if second is not None else (arena, toks)
        if len(t2) != len(toks):
            raise ValueError("the second batch must have as many jobs as the first")
        b2 = stage(a2, t2)
        acc2 = int(np.frombuffer(b2.run(want_verdicts=True), dtype=np.uint8).sum())
        batches.append((b2, _lib.PinnedBuffer(len(t2)), acc2))
    # per-kernel device times: average over synchronous runs (the warmup)
    times = {}
    w0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    for _ in range(max(1, warmup)):
        b.run(want_verdicts=True)
        for name, ms in b.kernel_times():
            times.setdefault(name, []).append(ms)
    w1 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    LAST_SYNC_MS = {k: float(np.mean(x)) for k, x in times.items()}
    if dist:
        import torch
        import torch.distributed as td
        torch.cuda.synchronize()
        td.barrier()
    # timed region: K steps streamed back to back (kernels + verdict D2H into
    # pinned memory each step), alternating batches, one synchronisation per batch at the end
    t0 = time.perf_counter()
    for i in range(steps):
        bb, pb, _ = batches[i % len(batches)]
        bb.enqueue(pb)
    for bb, _, _ in batches:
        bb.sync()
    elapsed = time.perf_counter() - t0
    for bb, pb, acc in batches[:min(steps, len(batches))]:
        if int(np.frombuffer(pb.bytes(), dtype=np.uint8).sum()) != acc:
            raise RuntimeError("verdicts changed between runs")
    if len(batches) > 1 and batches[1][2] != accepted and second is None:
        raise RuntimeError("the two copies of the batch disagree")
    for bb, pb, _ in batches:
        pb.free()
    if dist:
        import torch
        torch.cuda.synchronize()
        elapsed = max_over_ranks(elapsed, device=COLL_DEVICE)
    for bb, _, _ in batches:
        bb.free()
    kms = {k: float(np.mean(x)) for k, x in times.items()}
    # the synchronous runs' launches, for tools/cfg_roofline_check.py: every
    # kernel of this batch ran `runs` times inside [start, end] (CLOCK_BOOTTIME,
    # the clock of rocprofv3's timestamps)
    LAST_WINDOW = {"boottime_ns": [w0, w1], "runs": max(1, warmup)}
    global LAST_ACCEPTED2
    LAST_ACCEPTED2 = batches[1][2] if len(batches) > 1 else None
    return elapsed, accepted, kms, v


LAST_WINDOW = None
LAST_SYNC_MS = None
LAST_ACCEPTED2 = None       # accepted count of measure()'s second staged batch


def h2d_bandwidth(nbytes, iters=5):
    """Raw pinned host -> device copy bandwidth (bytes/s), best of `iters`,
    measured in the same process through the HIP runtime libcapjwt.so uses
    (ctypes on libamdhip64; torch bundles a different HIP runtime)."""
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    h, d = ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipHostMalloc(ctypes.byref(h), nbytes, 0) or hip.hipMalloc(ctypes.byref(d), nbytes):
        raise RuntimeError("hip allocation failed")
    ctypes.memset(h, 1, nbytes)
    best = float("inf")
    for _ in range(iters + 1):
        t0 = time.perf_counter()
        if hip.hipMemcpy(d, h, nbytes, 1):                  # hipMemcpyHostToDevice (synchronous)
            raise RuntimeError("hipMemcpy failed")
        best = min(best, time.perf_counter() - t0)
    hip.hipFree(d)
    hip.hipHostFree(h)
    return nbytes / best


def measure_pcie(ctx, arena, toks, iters=5, chunks=(32768, 65536, 131072), warm=1):
    """jg_verify_batch end to end from PINNED host buffers: H2D of arena + jobs
    (chunked, copies overlapping the previous chunk's kernels), planning,
    kernels, verdict D2H.  `warm` untimed passes per chunk size, then the best
    of `iters`.  A chunk entry "zc" runs the library's class-major zero-copy
    plans (jg_set_zero_copy: mixed batches only; per-class gathers from the
    pinned arena instead of chunk DMAs); integer entries run the chunked DMA
    pipeline with zero-copy plans off.  Reported beside `value`, never as it."""
    from cap_amd import _lib
    L = _lib.lib()
    pa = _lib.PinnedBuffer(len(arena))
    ctypes.memmove(pa.ptr, arena, len(arena))
    out = (ctypes.c_uint8 * len(toks))()
    tp = toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok))
    per_chunk = {}
    for ch in chunks:
        if ch == "zc":
            ctx.set_zero_copy(True)
        else:
            ctx.set_zero_copy(False)
            ctx.set_chunk(ch)
        best = float("inf")
        # untimed passes first: the pipeline slots size their device and
        # pinned buffers once per process (a long-running stream never pays
        # that again); a mixed 1.25 M-token pass reaches its steady state
        # after ~3 (profiles/r03_s12_c5_stream_ab.json)
        for _ in range(warm):
            if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, len(toks), out) != 0:
                raise RuntimeError(ctx.error())
        for _ in range(iters):
            t0 = time.perf_counter()
            if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), tp, len(toks), out) != 0:
                raise RuntimeError(ctx.error())
            best = min(best, time.perf_counter() - t0)
        per_chunk[ch] = best
    ctx.set_chunk(65536)
    ctx.set_zero_copy(False)
    pa.free()
    ch, best = min(per_chunk.items(), key=lambda kv: kv[1])
    bw = h2d_bandwidth(len(arena))
    bytes_per_tok = (len(arena) + 24 * len(toks)) / len(toks)       # arena + the 24-B job read by k_plan_fill
    return {"value": len(toks) / best, "unit": "verified JWTs/s", "ms_per_batch": best * 1e3,
            "chunk": ch, "ms_by_chunk": {str(k): v * 1e3 for k, v in per_chunk.items()},
            "arena_bytes": len(arena), "h2d_bytes_per_token": bytes_per_tok,
            "raw_h2d_GBps": bw / 1e9, "h2d_bound": bw / bytes_per_tok,
            "note": "jg_verify_batch from pinned host memory (chunked H2D overlapping kernels + plan + D2H, or "
                    "\"zc\": class-major zero-copy plans with per-class gathers over PCIe), "
                    f"best of {iters} after {warm} warm-up pass(es); h2d_bound = raw pinned H2D bandwidth / bytes per token; "
                    "not the headline"}


def host_snapshot():
    """Process-level host counters around an e2e pass:
    cgroup v2 CPU throttling, rusage (page faults, context switches, CPU time)
    and CPU time per thread name.  Linux only; missing files are skipped."""
    import resource
    snap = {"t": time.perf_counter()}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            snap["cg"] = {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
    except OSError:
        snap["cg"] = {}
    ru = resource.getrusage(resource.RUSAGE_SELF)
    snap["ru"] = {"minflt": ru.ru_minflt, "majflt": ru.ru_majflt, "nvcsw": ru.ru_nvcsw, "nivcsw": ru.ru_nivcsw,
                  "utime": ru.ru_utime, "stime": ru.ru_stime}
    thr = {}
    tick = os.sysconf("SC_CLK_TCK")
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                with open(f"/proc/self/task/{tid}/stat") as f:
                    s = f.read()
                name = s[s.index("(") + 1:s.rindex(")")]
                fields = s[s.rindex(")") + 2:].split()
                thr[tid] = (name, (int(fields[11]) + int(fields[12])) / tick)
            except (OSError, ValueError, IndexError):
                pass
    except OSError:
        pass
    snap["thr"] = thr
    return snap


def host_delta(a, b):
    """What changed between two host_snapshot()s: wall, CPU, faults, throttling
    and the threads that used the most CPU in between (by name)."""
    d = {"wall_s": b["t"] - a["t"]}
    d.update({k: b["ru"][k] - a["ru"][k] for k in a["ru"]})
    d.update({"cg_" + k: b["cg"].get(k, 0) - a["cg"].get(k, 0) for k in ("nr_throttled", "throttled_usec",
                                                                       "usage_usec", "nr_periods")})
    by_name = {}
    for tid, (name, cpu) in b["thr"].items():
        used = cpu - a["thr"].get(tid, (name, 0.0))[1]
        if used > 0:
            by_name[name] = by_name.get(name, 0.0) + used
    d["threads_now"] = len(b["thr"])
    counts = {}
    for name, _ in b["thr"].values():
        counts[name] = counts.get(name, 0) + 1
    d["threads_by_name"] = dict(sorted(counts.items(), key=lambda kv: -kv[1])[:10])
    d["cpu_by_thread_name"] = dict(sorted(by_name.items(), key=lambda kv: -kv[1])[:8])
    return d


def measure_e2e(pool, kids_jwk, total, threads):
    """Validator.ValidateBatch through the C++ host mirror (JWKS key set, host
    parse + kid routing + one GPU batch + claims validation), tokens handed
    over as one newline-separated host blob.  Not the headline value."""
    from cap_amd import jwt
    jwks = json.dumps({"keys": kids_jwk}).encode()
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                   lambda url, ca: {"status": 200, "body": jwks, "max_age": 3600})
    assert err is None, err
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=["ES256"],
                     Now=lambda: 1611699344 + 60)
    reps = (total + len(pool) - 1) // len(pool)
    blob = b"\n".join((pool * reps)[:total])
    v.ValidateBlob(b"\n".join(pool[:4096]), e)          # warm: JWKS fetch + key staging
    # steady state: the key set's comb tables widened in the background after
    # the first fetch (narrow tables first, jg_runtime.cpp upgrade_one); timed
    # passes that overlap those ~1 s of table builds measure the load, not the
    # validation rate (round 3's e2e line did)
    ks.WaitTables()
    best, acc, diag = float("inf"), 0, []
    for _ in range(2):
        s0 = host_snapshot()
        t0 = time.perf_counter()
        ok = v.ValidateBlob(blob, e)
        dt = time.perf_counter() - t0
        diag.append(host_delta(s0, host_snapshot()))
        best = min(best, dt)
        acc = sum(ok)
    if acc != total:
        raise RuntimeError(f"e2e accepted {acc}/{total}")
    from cap_amd import _capjwt_host
    return {"value": total / best, "unit": "validated JWTs/s", "ms_per_batch": best * 1e3, "tokens": total,
            "host_threads": _capjwt_host.host_threads(), "host_diag": diag,
            "note": "Validator.ValidateBatch (jwt/jwt.go:95 semantics) end to end: host parse/kid routing/claims "
                    "on host_threads cores + one jg_verify_batch (H2D included); not the headline value"}


def md_devices(spec):
    """--md-devices: "auto" = every visible GPU, or a one-GPU rehearsal [0, 0]
    (two device slots on one card: the runtime's split, workers and completers
    run as on two GPUs); else a comma list of device ids."""
    if spec != "auto":
        return [int(x) for x in spec.split(",")]
    import torch
    n = torch.cuda.device_count()              # does not initialise the GPU
    return list(range(n)) if n > 1 else [0, 0]


def measure_multi_device(pool, kids, kids_jwk, devices, per_dev, threads):
    """The deployment shape of SURVEY §8(e): ONE process, one jg_ctx spanning
    `devices`, the runtime's cost-weighted host-side split across them (per
    device worker + completer, jg_runtime.cpp per_device), no collective.
    (a) jg_verify_batch of len(devices) x per_dev ES256 tokens from pinned
    host memory (H2D, plan, kernels, D2H on every device), best of 3;
    (b) Validator.ValidateBatch over the same tokens through a JWKS key set on
    the same devices (host parse, kid routing, claims on `threads` cores).
    Accept counts are checked exactly."""
    from cap_amd import _lib, jwt
    total = len(devices) * per_dev
    ctx = _lib.Context(devices)
    ctx.load_keys(abi_keys(kids))
    arena, toks = pack(pool, [ALG_IDS["ES256"]] * len(pool), np.arange(len(pool)) % len(kids), total)
    vb = measure_pcie(ctx, arena, toks, iters=3, chunks=(262144,), warm=1)
    L = _lib.lib()
    out = (ctypes.c_uint8 * len(toks))()
    pa = _lib.PinnedBuffer(len(arena))
    ctypes.memmove(pa.ptr, arena, len(arena))
    if L.jg_verify_batch(ctx.h, pa.ptr, len(arena), toks.ctypes.data_as(ctypes.POINTER(_lib.JgTok)), len(toks),
                         out) != 0:
        raise RuntimeError(ctx.error())
    acc_vb = int(np.frombuffer(out, dtype=np.uint8).sum())
    pa.free()
    ctx.close()
    del arena, toks
    jwks = json.dumps({"keys": kids_jwk}).encode()
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                   lambda url, ca: {"status": 200, "body": jwks, "max_age": 3600}, devices=devices)
    assert err is None, err
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=["ES256"],
                     Now=lambda: 1611699344 + 60)
    reps = (total + len(pool) - 1) // len(pool)
    blob = b"\n".join((pool * reps)[:total])
    v.ValidateBlob(b"\n".join(pool[:4096]), e)
    ks.WaitTables()
    best, acc_v = float("inf"), 0
    for _ in range(2):
        t0 = time.perf_counter()
        ok = v.ValidateBlob(blob, e)
        best = min(best, time.perf_counter() - t0)
        acc_v = sum(ok)
    del blob
    res = {"value": vb["value"], "unit": "verified JWTs/s", "devices": devices, "tokens": total,
           "accepted": acc_vb, "expected_accepted": total,
           "verify_batch": {"value": vb["value"], "ms_per_batch": vb["ms_per_batch"], "accepted": acc_vb,
                            "h2d_bytes_per_token": vb["h2d_bytes_per_token"], "raw_h2d_GBps": vb["raw_h2d_GBps"]},
           "validate_batch": {"value": total / best, "ms_per_batch": best * 1e3, "accepted": acc_v,
                              "host_threads": threads},
           "note": "one process, one jg_ctx over `devices` (the runtime's host-side split, per-device streams, no "
                   "RCCL): jg_verify_batch from pinned host memory and Validator.ValidateBatch over the same "
                   "ES256 tokens" + ("; [0, 0] = a one-GPU rehearsal: two device slots on one card"
                                     if len(set(devices)) < len(devices) else "")}
    if acc_vb != total or acc_v != total:
        res["error"] = f"accepted {acc_vb} (verify_batch) / {acc_v} (ValidateBatch) of {total}"
    return res


def measure_single(pool, kids_jwk, threads, callers_list=None, total=1 << 18):
    """The drop-in path of an unchanged cap caller: C++
    threads, each calling Validator.Validate once per token -- Go's
    goroutine-per-request pattern -- on the configs[1] pool (ES256, 4-kid
    JWKS).  The key set coalesces concurrent calls into device batches
    (KeySet coalescer, default settings).  Per-call latency percentiles and
    the aggregate rate for host_threads callers (the headline of this line)
    and for more concurrent requests."""
    from cap_amd import jwt
    jwks = json.dumps({"keys": kids_jwk}).encode()
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "",
                                   lambda url, ca: {"status": 200, "body": jwks, "max_age": 3600})
    assert err is None, err
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=["ES256"],
                     Now=lambda: 1611699344 + 60)
    blob = b"\n".join(pool[:1 << 18])
    v.ValidateBlob(blob[:1 << 20], e)                # first fetch + key staging
    ks.WaitTables()
    out = {}
    for c in callers_list or (threads, 64, 256, 1024):
        v._impl._concurrent_validate(blob, e._native(), c, min(total, 1 << 15))      # warm the callers' path
        st0 = ks.CoalescingStats()
        h0 = host_snapshot()
        r = dict(v._impl._concurrent_validate(blob, e._native(), c, total))
        hd = host_delta(h0, host_snapshot())
        st1 = ks.CoalescingStats()
        batches = st1["batches"] - st0["batches"]
        # CPU the process spent per call, and whether the cgroup quota throttled it
        r["host"] = {"cpu_us_per_call": (hd["utime"] + hd["stime"]) / max(1, r["calls"]) * 1e6,
                     "stime_s": hd["stime"], "cg_throttled_ms": hd["cg_throttled_usec"] / 1e3,
                     "voluntary_cs": hd["nvcsw"],
                     "cpu_s_by_thread_name": dict(list(hd.get("cpu_by_thread_name", {}).items())[:6]),
                     "threads_by_name": hd.get("threads_by_name")}
        r["value"] = r["calls"] / r["wall_s"]
        r["mean_batch"] = r["calls"] / max(1, batches)
        if r["accepted"] != r["calls"]:
            r["error"] = f"accepted {r['accepted']} of {r['calls']}"
        out[str(c)] = r
    # the most callers again with every caller thread on host_threads CPUs (the
    # box shows the process all its CPUs under a host_threads-CPU quota; a Go
    # service runs its goroutines on GOMAXPROCS threads)
    c = max(int(k) for k in out)
    st0 = ks.CoalescingStats()
    h0 = host_snapshot()
    r = dict(v._impl._concurrent_validate(blob, e._native(), c, total, threads))
    hd = host_delta(h0, host_snapshot())
    st1 = ks.CoalescingStats()
    r["value"] = r["calls"] / r["wall_s"]
    r["mean_batch"] = r["calls"] / max(1, st1["batches"] - st0["batches"])
    r["host"] = {"cpu_us_per_call": (hd["utime"] + hd["stime"]) / max(1, r["calls"]) * 1e6,
                 "stime_s": hd["stime"], "cg_throttled_ms": hd["cg_throttled_usec"] / 1e3}
    if r["accepted"] != r["calls"]:
        r["error"] = f"accepted {r['accepted']} of {r['calls']}"
    out[f"{c}_callers_on_{threads}_cpus"] = r
    head = out[str(threads)]
    return {"value": head["value"], "unit": "validated JWTs/s", "callers": threads, "p50_us": head["p50_us"],
            "p99_us": head["p99_us"], "by_callers": out,
            "note": "Validator.Validate per token from N concurrent host threads (one call per token, as Go callers "
                    "do), coalesced into device batches by the key set; value/p50/p99 at N = host_threads; "
                    "by_callers: the same at more concurrent requests (host: CPU per call, cgroup throttling; "
                    "the process sees every CPU of the box under a 16-CPU quota). Not the headline."}


E2E_KIDS = ["p256-a", "p256-b", "p256-c", "p256-d"]


def e2e_child_main(tokfile, total):
    """--e2e-child: measure_e2e over the tokens in `tokfile` (newline-separated)
    in this fresh process, CAPJWT_TRACE phase times of the best pass included;
    one JSON line on stdout."""
    os.environ["CAPJWT_TRACE"] = "1"
    pool = open(tokfile, "rb").read().split(b"\n")
    jwk = [{"kty": "EC", "kid": f"kid-{i:02d}", "crv": "P-256", **xy} for i, xy in enumerate(p256_jwk_xy(E2E_KIDS))]
    cpu = cpu_info()
    print(json.dumps(measure_e2e(pool, jwk, total, cpu["cores_used"])))


def measure_e2e_fresh(pool, total):
    """measure_e2e in a child process (bench.py --e2e-child), so the line
    measures Validator.ValidateBatch as a fresh service process runs it and
    not this bench process's accumulated state; the child's CAPJWT_TRACE
    phase times of its last pass ride along."""
    import tempfile
    fd, path = tempfile.mkstemp(prefix="capjwt_e2e_", suffix=".txt")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(b"\n".join(pool))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--e2e-child", path, "--tokens", str(total)],
                           capture_output=True, text=True, timeout=600)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        raise RuntimeError(f"e2e child failed: {r.stderr[-2000:]}")
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["phases_ms_last_pass"] = trace_phases(r.stderr)
    out["process"] = "fresh child process (bench.py --e2e-child)"
    return out


def trace_phases(text):
    """CAPJWT_TRACE phase lines -> {phase: ms} (and {phase + " flt": minor
    page faults} where the line carries them); the last pass's phases win."""
    import re
    pat = re.compile(r"^\[capjwt\] (.+?)\s+(?:(-?\d+) flt\s+)?(-?[\d.]+) ms\s*$")
    phases = {}
    for line in text.splitlines():
        m = pat.match(line)
        if m:
            name = " ".join(m.group(1).split())
            phases[name] = float(m.group(3))
            if m.group(2) is not None:
                phases[name + " flt"] = int(m.group(2))
    return phases


def with_trace_phases(fn):
    """Run fn() in this process with CAPJWT_TRACE=1 and fd 2 sent to a temp
    file; returns (fn's result, its last pass's phase times)."""
    import tempfile
    sys.stderr.flush()
    saved = os.dup(2)
    old = os.environ.get("CAPJWT_TRACE")
    with tempfile.TemporaryFile() as tf:
        os.dup2(tf.fileno(), 2)
        os.environ["CAPJWT_TRACE"] = "1"
        try:
            res = fn()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
            if old is None:
                os.environ.pop("CAPJWT_TRACE", None)
            else:
                os.environ["CAPJWT_TRACE"] = old
        tf.seek(0)
        text = tf.read().decode(errors="replace")
    return res, trace_phases(text)


def cpu_info():
    """The host CPUs this process may use: nproc (cgroup-aware), the affinity
    mask, the cgroup v2 CPU quota, and the lscpu model."""
    import math
    info = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        info["nproc"] = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        info["nproc"] = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        info["model"] = next((ln.split(":", 1)[1].strip() for ln in out.splitlines() if ln.startswith("Model name")), None)
    except OSError:
        info["model"] = None
    info["cores_used"] = max(1, min(info["affinity"], math.ceil(quota) if quota else info["affinity"]))
    return info


def cpu_baseline(pool, alg, okeys, threads, seconds, keyidx=None, max_tokens=None, cpu=None):
    """The C oracle (oracle/jws_oracle.c) on the host's cores over a bounded
    sample (the whole pool when max_tokens is given and fits)."""
    from oracle import jws
    L = jws.lib()

    class Job(ctypes.Structure):
        _fields_ = [("alg", ctypes.c_int), ("key_kind", ctypes.c_int), ("curve", ctypes.c_int),
                    ("n", ctypes.c_void_p), ("x", ctypes.c_void_p), ("y", ctypes.c_void_p),
                    ("nlen", ctypes.c_size_t), ("coord_len", ctypes.c_size_t), ("e", ctypes.c_uint64),
                    ("msg", ctypes.c_void_p), ("mlen", ctypes.c_size_t), ("sig", ctypes.c_void_p),
                    ("slen", ctypes.c_size_t)]
    L.or_verify_many.argtypes = [ctypes.POINTER(Job), ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    keep = []

    def buf(b):
        c = ctypes.create_string_buffer(b, len(b))
        keep.append(c)
        return ctypes.cast(c, ctypes.c_void_p)

    def make_jobs(n):
        jobs = (Job * n)()
        for i in range(n):
            t = pool[i % len(pool)]
            d = t.rfind(b".")
            sig = jws.b64url_decode(t[d + 1:].decode())
            k = okeys[(keyidx[i % len(pool)] if keyidx is not None else i % len(okeys))]
            j = jobs[i]
            j.alg = jws.ALGS[alg if isinstance(alg, str) else alg[i % len(pool)]]
            j.msg, j.mlen = buf(t[:d]), d
            j.sig, j.slen = buf(sig), len(sig)
            if k.kty == "RSA":
                j.key_kind, j.n, j.nlen, j.e = 0, buf(k.n), len(k.n), k.e
            elif k.kty == "EC":
                j.key_kind, j.curve = 1, jws.CURVES[k.crv]
                j.x, j.y, j.coord_len = buf(k.x), buf(k.y), len(k.x)
            else:
                j.key_kind, j.x = 2, buf(k.x)
        return jobs
    if max_tokens:
        n = max_tokens
    else:
        # calibrate on 64 tokens single-threaded, then size the sample for `seconds` of wall time
        probe = make_jobs(64)
        out = (ctypes.c_uint8 * 64)()
        t0 = time.perf_counter()
        L.or_verify_many(probe, 64, 1, out)
        per = (time.perf_counter() - t0) / 64
        n = int(max(256, min(len(pool), seconds * threads / per)))
    jobs = make_jobs(n)
    out = (ctypes.c_uint8 * n)()
    t0 = time.perf_counter()
    L.or_verify_many(jobs, n, threads, out)
    el = time.perf_counter() - t0
    ok = sum(out)
    name = alg if isinstance(alg, str) else "mixed"
    res = {"value": n / el, "unit": "verified JWTs/s", "cores": threads, "kind": "port",
           "sample": f"{n} {name} tokens from the benchmark pool verified by the C oracle "
                     f"(oracle/jws_oracle.c, a restatement of Go crypto/*, not Go itself) "
                     f"on {threads} host threads (all cores available to the process); {ok}/{n} accepted; "
                     f"{el:.2f} s wall", "accepted": ok, "tokens": n}
    if cpu:
        res["cpu"] = cpu
    return res


CPUVERIFY = os.path.join(ROOT, "tools", "cpuverify", "cpuverify")


def openssl_baseline(pool, alg, keypaths, threads, seconds):
    """All-core OpenSSL libcrypto verification of the same tokens
    (tools/cpuverify): a closer stand-in for Go's assembly-backed crypto than
    the clarity-first C oracle.  Token i is verified with key i % len(keypaths),
    as tools/tokgen signed it."""
    if not os.path.exists(CPUVERIFY):
        subprocess.run(["make", "-s", "-C", os.path.dirname(CPUVERIFY)], check=True)
    path = os.path.join("/tmp", f"capjwt_cpuverify_{alg}_{os.getpid()}.txt")
    with open(path, "wb") as f:
        f.write(b"\n".join(pool) + b"\n")
    try:
        r = subprocess.run([CPUVERIFY, alg, str(threads), str(seconds), path] + list(keypaths),
                           capture_output=True, text=True, check=True)
    finally:
        os.unlink(path)
    d = json.loads(r.stdout)
    return {"value": d["per_second"], "unit": "verified JWTs/s", "cores": threads, "kind": "openssl",
            "sample": f"{d['tokens']} {alg} tokens (the benchmark pool) verified {d['verified']} times in total "
                      f"by {d['openssl']} (tools/cpuverify, EVP_DigestVerify) on {threads} threads for "
                      f"{d['seconds']:.1f} s; {d['accepted']}/{d['verified']} accepted. Not Go.",
            "accepted": d["accepted"], "verified": d["verified"]}


def golden_oracle_keys(kids):
    from oracle import jws
    from tests import gpu_helpers as H
    kd = {k["kid"]: k for k in H.golden()[0]}
    return [jws.Key.from_fixture(kd[k]) for k in kids]


# ---------------------------------------------------------------- other BASELINE configs
def _set_header(tok, **kv):
    """Rewrite members of a compact token's protected header (the signature is
    left as it is, so the token no longer verifies)."""
    import base64
    h, rest = tok.split(b".", 1)
    hd = json.loads(base64.urlsafe_b64decode(h + b"=" * (-len(h) % 4)))
    hd.update(kv)
    h2 = base64.urlsafe_b64encode(json.dumps(hd, separators=(",", ":")).encode()).rstrip(b"=")
    return h2 + b"." + rest


def tamper(pool, algs, keyidx, keys_meta, frac, seed=1):
    """5 % tampered tokens: sig bit-flip, payload char flip, kid
    swap, alg swap in equal parts.  The kid and alg swaps rewrite the token's
    header (and its job's key / alg with it), so a host-side parse routes the
    token exactly as the job list does.  Returns new (pool, algs, keyidx, expected)."""
    rng = np.random.default_rng(seed)
    pool, algs, keyidx = list(pool), np.array(algs), np.array(keyidx)
    good = np.ones(len(pool), dtype=bool)
    sel = rng.choice(len(pool), int(len(pool) * frac), replace=False)
    b64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"
    fam = {a: a[:2] if a != "EdDSA" else "Ed" for a in ALG_IDS}
    by_id = {v: k for k, v in ALG_IDS.items()}
    for j, i in enumerate(sel):
        t = bytearray(pool[i])
        mode = j % 4
        if mode == 0:                                   # signature bit flip (first sig char)
            d = t.rfind(b".") + 1
            t[d] = b64[(b64.index(t[d]) ^ 1)]
        elif mode == 1:                                 # payload character flip
            d = t.index(b".") + 5
            t[d] = b64[(b64.index(t[d]) ^ 2)]
        else:
            a = by_id[int(algs[i])]
            alts = [x for x in ALG_IDS if fam[x] == fam[a] and x != a]
            if mode == 3 and alts:                      # alg swap within the family (RS<->PS ...)
                algs[i] = ALG_IDS[alts[j % len(alts)]]
                t = bytearray(_set_header(bytes(t), alg=alts[j % len(alts)]))
            else:                                       # kid swap: the header names another kid
                keyidx[i] = (keyidx[i] + 1) % len(keys_meta)
                t = bytearray(_set_header(bytes(t), kid=keys_meta[keyidx[i]][0]))
        pool[i] = bytes(t)
        good[i] = False
    return pool, algs, keyidx, good


RSA_ALGS = ("RS256", "RS384", "RS512", "PS256", "PS384", "PS512")


def c5_pool(meta, total, threads, rank, ec_unique=True):
    """configs[4]'s token list for one GPU: `total` tokens, every kid 1/32 of
    them, in a fixed random order, 5 % tampered.  EC and Ed25519 tokens are all
    unique (their comb-entry gathers would otherwise hit the Infinity Cache for
    repeated tokens); RSA tokens cycle a per-kid pool of 1024 (512 for the
    4096-bit kids), since the modexp reads only the token's own signature and
    the key's modulus -- a repeat costs exactly what a new token costs.
    ec_unique=False is round 2's layout (1024 per kid for every alg)."""
    per = -(-total // len(meta))
    pool, algs, keyidx = [], [], []
    for ki, (kid, alg, pem, _, _) in enumerate(meta):
        n = (512 if alg in ("RS512", "PS512") else 1024) if (alg in RSA_ALGS or not ec_unique) else per
        toks = gen_tokens(alg, n, [pem], threads, f"c4r{rank}", kid_base=ki)
        pool += [toks[i % n] for i in range(per)]
        algs += [ALG_IDS[alg]] * per
        keyidx += [ki] * per
    order = np.random.default_rng(1).permutation(len(pool))[:total]
    pool = [pool[i] for i in order]
    algs = [algs[i] for i in order]
    keyidx = [keyidx[i] for i in order]
    return tamper(pool, algs, keyidx, meta, 0.05)


def c5_pool_note(ec_unique):
    if ec_unique:
        return ("every EC / Ed25519 token unique over the 1,250,000-token share (the resident steps alternate "
                "between its first two --c5-chunk chunks); RSA tokens cycle 1024 (512 for 4096-bit kids) per kid: the modexp has no data-dependent "
                "gathers, so repeats cost the same")
    return "1024 (512) unique tokens per kid replicated (round-2 layout)"


def roofline_line(kernel_ms, per_gpu, kernels):
    """{kernel: roofline} for each (key, mads-per-token | ('hbm', bytes-per-token))."""
    out = {}
    for key, work in kernels.items():
        if key not in kernel_ms:
            continue
        sec = kernel_ms[key] * 1e-3
        if isinstance(work, tuple):               # ("hbm", bytes per token)
            ach = work[1] * per_gpu / sec / 1e9
            out[key] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBPS, "bytes_per_token": work[1]}
        else:
            ach = work * per_gpu / sec / 1e12
            out[key] = {"bound": "valu", "achieved": ach, "peak": MAD_PEAK_T, "unit": "TMAD/s",
                        "frac": ach / MAD_PEAK_T, "mads_per_token": work}
    return out


def config_line(ctx, name, workload, pool, algs, keyidx, expected_good, per_gpu, steps, warmup, dist, world,
                kernels=None, class_of_key=None, second=None):
    """One BASELINE config measured like the headline.  `kernels`: roofline
    work per token of the class kernels to report; a kernel sees only its
    class's tokens -- by alg family, or by `class_of_key[key index]` (kernel
    class name per key) where keys of one family fall into several classes.
    `second` = (pool, algs, keyidx, expected_good) of measure()'s second
    staged batch (default: a copy of the first)."""
    arena, toks = pack(pool, algs, keyidx, per_gpu)
    sec = pack(*second[:3], per_gpu) if second is not None else None
    el, acc, _, v = measure(ctx, arena, toks, steps, warmup, dist, second=sec)
    acc2 = LAST_ACCEPTED2
    del sec
    # per-class kernel times from the synchronous runs of the batch: in the
    # timed region steps are pipelined, so a class kernel there shares the
    # chip with the previous step's kernels and its duration is no roofline
    # time (round 3: C5's P-256 point ran 0.12 ms alone, 0.37-0.50 ms
    # overlapped -- profiles/r03_s5_cfg_roofline_check.json)
    kms = LAST_SYNC_MS
    reps = (per_gpu + len(pool) - 1) // len(pool)
    want = int(np.tile(expected_good, reps)[:per_gpu].sum())
    line = {"workload": workload, "value": world * per_gpu * steps / el, "unit": "verified JWTs/s",
            "ms_per_step": el * 1000.0 / steps, "tokens_per_gpu": per_gpu, "unique_pool": len(pool),
            "accepted": acc, "expected_accepted": want, "kernel_ms": kms,
            "kernel_ms_from": "synchronous runs of the batch (bench warmup), one at a time", "trace_window": LAST_WINDOW}
    want2 = want
    if second is not None:
        reps2 = (per_gpu + len(second[0]) - 1) // len(second[0])
        want2 = int(np.tile(second[3], reps2)[:per_gpu].sum())
    if acc != want or acc2 not in (None, want2):
        line["error"] = f"accepted {acc} (second batch {acc2}) != expected {want} ({want2})"
    if kernels:
        # per-class token counts: a mixed batch's class kernels see only their share
        share = {}
        for key in kernels:
            cls = key.split("_")[0]
            share[key] = cls
        counts = {}
        aid = np.asarray(algs)
        kcls = np.asarray([class_of_key[k] for k in keyidx]) if class_of_key else None
        for key, cls in share.items():
            if kcls is not None:
                counts[key] = float((kcls == cls).mean())
                continue
            fam = {"p256": (7,), "p384": (8,), "p521": (9,), "ed25519": (10,), "rsa2048": (1, 2, 3, 4, 5, 6),
                   "rsa3072": (1, 2, 3, 4, 5, 6), "rsa4096": (1, 2, 3, 4, 5, 6)}[cls]
            frac = float(np.isin(aid, fam).mean()) if cls not in ("rsa2048", "rsa3072", "rsa4096") else None
            counts[key] = frac
        rl = {}
        for key, work in kernels.items():
            frac = counts[key]
            n = per_gpu * (frac if frac is not None else 1.0)
            rl.update(roofline_line(kms, n, {key: work}))
        line["roofline"] = rl
    return line


def run_configs(ctx, args, threads, rank, world, dist):
    out = {}
    # configs[2]: PS512 RSA-4096, 1M tokens sharded across 8 GPUs -> 131072 per GPU
    ctx.load_keys(abi_keys(["rsa4096-a"]))
    pool = gen_tokens("PS512", 4096, golden_keypaths(["rsa4096-a"]), threads, f"c2r{rank}")
    out["ps512_rsa4096"] = config_line(
        ctx, "ps512_rsa4096", "PS512 RSA-4096 (PSS/MGF1-SHA512), 1M tokens / 8 GPUs = 131072 per GPU (configs[2]); "
        "a 4096-token signed pool replicated 32x (the modexp has no data-dependent gathers)",
        pool, [ALG_IDS["PS512"]] * len(pool), [0] * len(pool), np.ones(len(pool), bool), 131072,
        max(1, args.steps // 2), 1, dist, world,
        kernels={"rsa4096_modexp": rsa_modexp_mads_per_token(148, 4),
                 "rsa4096_prep": ("hbm", prep_bytes_per_token(939, 132))})
    # configs[3]: EdDSA Ed25519 + ES384 P-384 mixed, 1M tokens per GPU, every
    # token unique (a replicated pool lets repeated comb-entry gathers hit the
    # 256 MiB Infinity Cache; `pool_ab` measures the old 16384-token pool beside it)
    ctx.load_keys(abi_keys(["ed-a", "p384-a"]))
    c4w = ctx.table_widths()                  # [Ed25519 key, P-384 key]
    c4n = args.c4_pool // 2
    pe = gen_tokens("EdDSA", c4n, golden_keypaths(["ed-a"]), threads, f"c3r{rank}")
    p3 = gen_tokens("ES384", c4n, golden_keypaths(["p384-a"]), threads, f"c3r{rank}", kid_base=1)
    pool = [t for pair in zip(pe, p3) for t in pair]
    algs = [ALG_IDS["EdDSA"], ALG_IDS["ES384"]] * len(pe)
    c4_kernels = {"p384_point": p384_point_mads_per_token(c4w[1]), "ed25519_point": ed25519_point_mads_per_token(c4w[0]),
                  "p384_prep": ("hbm", prep_bytes_per_token(384, 49)),
                  "ed25519_prep": ("hbm", prep_bytes_per_token(342, 16))}
    line = config_line(
        ctx, "eddsa_es384_mixed", "EdDSA Ed25519 + ES384 P-384 50/50 mixed batch, 1M tokens per GPU (configs[3])",
        pool, algs, [0, 1] * len(pe), np.ones(len(pool), bool), 1 << 20, max(1, args.steps // 2), 1, dist, world,
        kernels=c4_kernels)
    if not args.no_ab and len(pool) > 16384:
        sub = 16384
        ab = config_line(ctx, "eddsa_es384_mixed_ab", "pool A/B", pool[:sub], algs[:sub], [0, 1] * (sub // 2),
                         np.ones(sub, bool), 1 << 20, max(1, args.steps // 2), 1, dist, world, kernels=c4_kernels)
        line["pool_ab"] = {"replicated_pool": sub, "value": ab["value"], "kernel_ms": ab["kernel_ms"],
                           "roofline": ab.get("roofline"),
                           "note": "same 1M-token batch from a 16384-token pool replicated 64x (round-2 layout); "
                                   "`value` above uses unique tokens"}
    out["eddsa_es384_mixed"] = line
    del pool, pe, p3
    # configs[4]: all 10 algs, 32 kids, ~5 % tampered; the 10M stream in 256k-token chunks (one chunk per step)
    meta = bench_keys()
    # one table budget over every curve (jg_set_table_budget): enough for the
    # 32 kids' widest tiers (P-256 W = 26, P-384 24, Ed25519 24, P-521 20: 171.0 GB of 171.8)
    ctx.set_table_budget(int(args.c5_table_budget_gb * (1 << 30)))
    ctx.load_keys([m[3] for m in meta])
    c5w = ctx.table_widths()
    pool, algs, keyidx, good = c5_pool(meta, 10_000_000 // 8, threads, rank, args.c5_unique)
    # kernel class of each kid's key (ecdsa/rsa/ed25519 classes of the runtime)
    def key_class(jwk):
        if jwk["kty"] == "RSA":
            import base64
            bits = int.from_bytes(base64.urlsafe_b64decode(jwk["n"] + "=" * (-len(jwk["n"]) % 4)), "big").bit_length()
            return "rsa2048" if bits <= 2070 else "rsa3072" if bits <= 3134 else "rsa4096"
        if jwk["kty"] == "EC":
            return {"P-256": "p256", "P-384": "p384", "P-521": "p521"}[jwk["crv"]]
        return "ed25519"
    kcls = [key_class(m[4]) for m in meta]
    present = set(kcls)
    wof = {c: next(w for w, k in zip(c5w, kcls) if k == c) for c in ("p256", "p384", "p521", "ed25519") if c in kcls}
    work = {"rsa2048_modexp": rsa_modexp_mads_per_token(74, 2), "rsa3072_modexp": rsa_modexp_mads_per_token(112, 2),
            "rsa4096_modexp": rsa_modexp_mads_per_token(148, 4), "p256_point": p256_point_mads_per_token(wof.get("p256")),
            "p384_point": p384_point_mads_per_token(wof.get("p384")),
            "p521_point": p521_point_mads_per_token(wof.get("p521")),
            "ed25519_point": ed25519_point_mads_per_token(wof.get("ed25519", 20))}
    chunk = args.c5_chunk
    line = config_line(
        ctx, "mixed_10alg_32kid", f"all 10 algs, 32 kids, 5% tampered, 10M stream on 8 GPUs in {chunk}-token chunks "
        "(configs[4]); one chunk per step per GPU, steps alternating between the share's first two chunks",
        pool[:chunk], algs[:chunk], keyidx[:chunk], good[:chunk], chunk,
        max(1, args.steps // 2), 1, dist, world, kernels={k: v for k, v in work.items() if k.split("_")[0] in present},
        class_of_key=kcls,
        second=(pool[chunk:2 * chunk], algs[chunk:2 * chunk], keyidx[chunk:2 * chunk], good[chunk:2 * chunk]))
    line["pool"] = c5_pool_note(args.c5_unique)
    line["table_budget_GiB"] = args.c5_table_budget_gb
    line["key_comb_w"] = {m[0]: w for m, w in zip(meta, c5w) if w}
    # the same workload as a real stream: this GPU's 1/8 share of the 10M
    # tokens (1,250,000) through jg_verify_batch from pinned host memory (H2D,
    # plan, kernels, verdicts back), chunks overlapping
    share = 10_000_000 // 8
    arena, toks = pack(pool, algs, keyidx, share)
    chunks = tuple(c if c == "zc" else int(c) for c in args.stream_chunks.split(","))
    st = measure_pcie(ctx, arena, toks, iters=4, chunks=chunks, warm=3)
    st["workload"] = f"{share} tokens per GPU (10M / 8) streamed with H2D"
    line["stream"] = st
    del arena, toks
    if not args.no_refresh:
        line["refresh"] = measure_refresh(ctx, meta, args.c5_table_budget_gb + 40)
    out["mixed_10alg_32kid"] = line
    C5_E2E.update(pool=pool, good=good, meta=meta)
    return out


C5_E2E = {}           # configs[4]'s token list, for the JWKS end-to-end line after the raw-ABI context closes


def measure_refresh(ctx, meta, budget_gb):
    """JWKS refresh through the C ABI (go-oidc refresh-on-miss behind
    /root/reference/jwt/keyset.go:127; R34): (a) the document unchanged -- the
    common answer to a tampered token's miss -- and (b) a rotated-in P-256 key:
    time until jg_keys_load returns and the new key verifies (narrow W = 20
    table), then until its wide table is swapped in, while the other 32 kids
    keep their tables (shared by content, nothing rebuilt or copied)."""
    from tests import gpu_helpers as H
    keys = [m[3] for m in meta]
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.load_keys(keys, wait_tables=False)
    same_ms = (time.perf_counter() - t0) / reps * 1e3
    gk, gt = H.golden()
    newk = next(k for k in gk if k["kid"] == "p256-a")
    sel = [t for t in gt if t["key"] == "p256-a" and t["alg"] == "ES256"]
    ctx.set_table_budget(int(budget_gb * (1 << 30)))           # room for the new key's W = 26 table too
    t0 = time.perf_counter()
    ctx.load_keys(keys + [H.abi_key(newk)], wait_tables=False)
    load_ms = (time.perf_counter() - t0) * 1e3
    w_at_return = ctx.table_widths()[-1]
    arena, slots = H.jobs_from_tokens(sel, {"p256-a": len(keys)})
    out = ctx.verify(arena)
    first_ms = (time.perf_counter() - t0) * 1e3
    ok_first = [0 if s is None else out[s] for s in slots] == [t["verdict"] for t in sel]
    ctx.wait_tables()
    wide_ms = (time.perf_counter() - t0) * 1e3
    out = ctx.verify(arena)
    ok_wide = [0 if s is None else out[s] for s in slots] == [t["verdict"] for t in sel]
    return {"unchanged_reload_ms": same_ms, "unchanged_reload_note": "jg_keys_load of the identical 32-kid table: "
            "content compared on the host, no device work (no kernel, no copy, no drain)",
            "new_key_load_ms": load_ms, "new_key_width_at_return": w_at_return,
            "new_key_first_verify_ms": first_ms, "new_key_wide_ms": wide_ms,
            "new_key_width_final": ctx.table_widths()[-1], "verdicts_ok": bool(ok_first and ok_wide),
            "tokens": len(sel), "table_budget_GiB": budget_gb}


def measure_jwks_e2e(pool, good, meta, threads):
    """configs[4] as BASELINE states it: a JWKS KeySet over the 32 kids with no
    cache lifetime (max_age 0: every miss refreshes, R34) and Validator
    .ValidateBatch over this GPU's 5 %-tampered share, refreshes included --
    each call's misses trigger one fetch of the (unchanged) JWKS and a retry."""
    from cap_amd import jwt
    jwks = json.dumps({"keys": [m[4] for m in meta]}).encode()
    fetches = [0]

    def fetch(url, ca):
        fetches[0] += 1
        return {"status": 200, "body": jwks, "max_age": 0}
    ks, err = jwt.NewJSONWebKeySet(None, "https://bench.example/jwks", "", fetch)
    assert err is None, err
    v, _ = jwt.NewValidator(ks)
    e = jwt.Expected(Issuer="https://example.com/", Audiences=["www.example.com"], SigningAlgorithms=list(ALG_IDS),
                     Now=lambda: 1611699344 + 60)
    v.ValidateBlob(b"\n".join(pool[:4096]), e)          # warm: first fetch + key staging
    ks.WaitTables()
    blob = b"\n".join(pool)
    best, acc = float("inf"), 0
    f0 = fetches[0]
    for _ in range(2):
        t0 = time.perf_counter()
        ok = v.ValidateBlob(blob, e)
        best = min(best, time.perf_counter() - t0)
        acc = sum(ok)
    want = int(np.asarray(good).sum())
    from cap_amd import _capjwt_host
    res = {"value": len(pool) / best, "unit": "validated JWTs/s", "ms_per_batch": best * 1e3, "tokens": len(pool),
           "accepted": acc, "expected_accepted": want, "fetches_per_call": (fetches[0] - f0) / 2,
           "host_threads": _capjwt_host.host_threads(),
           "note": "NewJSONWebKeySet(max_age 0).ValidateBatch over the 10M / 8 share, all 10 algs allowed: host parse, "
                   "kid routing, one GPU batch, one refresh per call (unchanged JWKS: no device work) and a retry of "
                   "the misses, payload JSON and claims; H2D included; not the headline"}
    if acc != want:
        res["error"] = f"accepted {acc} != expected {want}"
    return res


LINE_MAX_BYTES = 8192       # the driver parses the tail of stdout: keep the one JSON line well under this
DETAIL_DEFAULT = os.path.join("gpurun_out", "bench_detail.json")


def _r(x, nd=4):
    """Round a float to `nd` significant digits for the compact line."""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


def _fracs(roof):
    return {k: _r(v["frac"], 3) for k, v in (roof or {}).items() if isinstance(v, dict) and "frac" in v}


def compact_line(result, detail_path=None):
    """The one stdout JSON line: the contract keys, `roofline`, `cpu_baseline`
    and a compact summary of every other leg (value, accept counts, one `frac`
    per class kernel).  Everything else in `result` (per-kernel times, host
    diagnostics, per-caller tables, phase maps, A/B lines) goes to the detail
    file, referenced by path.  tests/test_bench_contract.py checks the size and
    keys against a full result."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "accepted", "error")
    line = {k: _r(result[k], 6) if k == "value" else result[k] for k in keys if k in result}
    rl = result.get("roofline")
    if rl:
        line["roofline"] = {k: _r(rl[k]) for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic")
                            if k in rl}
        line["roofline"]["traffic_from"] = rl.get("traffic_from")
        line["roofline"]["mads_per_token"] = _r(rl.get("mads_per_token"), 6)
    cb = result.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: _r(cb[k], 6) for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
    oss = result.get("cpu_baseline_openssl") or {}
    if oss:
        line["cpu_openssl"] = {a: _r(v["value"], 6) for a, v in oss.items() if isinstance(v, dict) and "value" in v}
        line["cpu_openssl"]["note"] = "OpenSSL 3 libcrypto EVP_DigestVerify on the same tokens, all cores; not Go"
    if "speedup_vs_cpu" in result:
        line["speedup_vs_cpu"] = {k: _r(v, 4) for k, v in result["speedup_vs_cpu"].items() if k != "note"}
    rs = result.get("rs256")
    if rs:
        line["rs256"] = {"value": _r(rs["value"], 6), "accepted": rs.get("accepted"),
                         "tokens": rs.get("tokens_per_gpu"), "ms_per_step": _r(rs.get("ms_per_step")),
                         "frac": _r(rs.get("roofline", {}).get("frac"), 3)}
        if "error" in rs:
            line["rs256"]["error"] = rs["error"]
    cfgs = {}
    for name, c in (result.get("configs") or {}).items():
        s = {"value": _r(c.get("value"), 6), "accepted": c.get("accepted"), "expected": c.get("expected_accepted"),
             "frac": _fracs(c.get("roofline"))}
        if "error" in c:
            s["error"] = c["error"]
        if "stream" in c:
            s["stream"] = _r(c["stream"].get("value"), 6)
            s["stream_h2d_bound"] = _r(c["stream"].get("h2d_bound"), 4)
        if "jwks_e2e" in c:
            j = c["jwks_e2e"]
            s["jwks_e2e"] = _r(j.get("value"), 6)
            s["jwks_e2e_ok"] = j.get("accepted") == j.get("expected_accepted")
        cfgs[name] = s
    if cfgs:
        line["configs"] = cfgs
    for leg in ("e2e", "single", "multi_device"):
        v = result.get(leg)
        if not v:
            continue
        s = {"value": _r(v.get("value"), 6)}
        for k in ("callers", "p50_us", "p99_us", "host_threads", "devices", "accepted", "expected_accepted",
                  "lone_batch_us", "error"):
            if k in v:
                s[k] = _r(v[k])
        if leg == "e2e" and "fresh_child" in v:
            s["fresh_child"] = _r(v["fresh_child"].get("value"), 6)
        if leg == "multi_device":
            for k in ("verify_batch", "validate_batch"):
                if k in v:
                    s[k] = _r(v[k].get("value"), 6)
        line[leg] = s
    if detail_path:
        line["detail"] = detail_path
    return line


def emit_line(result, detail_path):
    """Write the full `result` to `detail_path` (best effort) and print the
    compact line; the line must fit LINE_MAX_BYTES."""
    where = None
    if detail_path:
        try:
            full = detail_path if os.path.isabs(detail_path) else os.path.join(ROOT, detail_path)
            os.makedirs(os.path.dirname(full), exist_ok=True)
            with open(full, "w") as f:
                json.dump(result, f)
            where = detail_path
        except OSError:
            where = None
    line = json.dumps(compact_line(result, where))
    if len(line) > LINE_MAX_BYTES:
        raise RuntimeError(f"bench line is {len(line)} bytes (> {LINE_MAX_BYTES})")
    print(line, flush=True)


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc pass
    (FETCH_SIZE x2 per the gfx950 correction, calibrated for the streaming and
    80-byte gather patterns in that file, + WRITE_SIZE), or None."""
    try:
        d = json.load(open(TRAFFIC))
        return d["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=1 << 20, help="tokens per GPU per step")
    ap.add_argument("--c5-chunk", type=int, default=625000,
                    help="configs[4] resident chunk (tokens per step; default: half of the GPU's 1.25M share, so the "
                         "two alternating staged chunks cover the whole share)")
    ap.add_argument("--pool", type=int, default=0, help="unique signed ES256 tokens (default: all unique)")
    ap.add_argument("--rs-pool", type=int, default=100000, help="unique RS256 tokens (BASELINE configs[0]: 100k)")
    ap.add_argument("--no-ab", action="store_true", help="skip the replicated-pool A/B line")
    ap.add_argument("--no-rs256", action="store_true")
    ap.add_argument("--no-configs", action="store_true")
    ap.add_argument("--configs-only", action="store_true",
                    help="only the `configs` lines (profiling runs of configs[2..4]); not a bench line")
    ap.add_argument("--c4-pool", type=int, default=1 << 20,
                    help="unique tokens of configs[3] (EdDSA + ES384; default: the whole 1M batch)")
    ap.add_argument("--c5-table-budget-gb", type=float, default=160.0,
                    help="configs[4] table budget over all curves (160 GiB: every kid at its widest tier)")
    ap.add_argument("--stream-chunks", default="zc,196608,262144,524288",
                    help="configs[4] stream: the chunk sizes tried (\"zc\": zero-copy plans); the best is reported")
    ap.add_argument("--c5-legacy-pool", dest="c5_unique", action="store_false",
                    help="configs[4] from 1024 unique tokens per kid (round-2 layout)")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--md-devices", default="auto",
                    help="the one-process multi-device leg's device list (\"auto\": every visible GPU, or the "
                         "one-GPU rehearsal 0,0); \"none\" skips it")
    ap.add_argument("--e2e-child", metavar="TOKFILE", help=argparse.SUPPRESS)   # measure_e2e_fresh's child
    ap.add_argument("--no-refresh", action="store_true", help="skip configs[4]'s JWKS refresh timings "
                    "(profiling passes: they build key tables)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--detail", default=DETAIL_DEFAULT,
                    help="file for the full result (per-kernel times, host diagnostics, A/B lines); the stdout line "
                         "carries the contract keys and a compact summary")
    ap.add_argument("--table-budget-gb", type=float, default=110.0,
                    help="HBM for P-256 key comb tables (jg_set_table_budget): 110 GiB holds the 4 kids at W = 26")
    args = ap.parse_args()
    if args.e2e_child:
        return e2e_child_main(args.e2e_child, args.tokens)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    dev = local
    if dist:
        import torch
        import torch.distributed as td
        ndev = torch.cuda.device_count()          # does not initialise the GPU
        dev = local % max(1, ndev)
        # one rank per GPU over RCCL; more ranks than GPUs (a rehearsal of the
        # N>1 path on a 1-GPU box) share devices and time through gloo
        global COLL_DEVICE
        COLL_DEVICE = "cuda" if world <= ndev else "cpu"
        torch.cuda.set_device(dev)
        td.init_process_group("nccl" if COLL_DEVICE == "cuda" else "gloo")
    from cap_amd import _lib

    cpu = cpu_info()
    # every core this process may use (cgroup quota, affinity), divided among
    # the ranks of one node: N ranks must not each take every core
    host_threads = max(1, cpu["cores_used"] // world)
    if dist:
        cpu["cores_used_per_rank"] = host_threads
        os.environ["CAPJWT_HOST_THREADS"] = str(host_threads)     # the host library's pool (read once, at first use)
    ctx = _lib.Context([dev])
    budget = int(args.table_budget_gb * (1 << 30))
    if dist and COLL_DEVICE == "cpu":
        # ranks sharing one GPU (a rehearsal of N > 1 on a smaller box): each
        # process holds its own tables, so keep them at the 32 GiB default
        budget = min(budget, 32 << 30)
        args.c5_table_budget_gb = min(args.c5_table_budget_gb, 32.0)
    ctx.set_table_budget(budget)
    global P384_BUDGET
    P384_BUDGET = budget
    if args.configs_only:
        res = {"configs_only": True, "configs": run_configs(ctx, args, host_threads, rank, world, dist)}
        ctx.close()
        C5_E2E.clear()
        if rank == 0:
            print(json.dumps(res))
        if dist:
            import torch.distributed as td
            td.destroy_process_group()
        return

    # ---- ES256, P-256 JWKS with 4 kids (configs[1]): 1M unique OpenSSL-signed tokens
    kids = ["p256-a", "p256-b", "p256-c", "p256-d"]
    ctx.load_keys(abi_keys(kids))
    global P256_WQ
    P256_WQ = min(ctx.table_widths())         # the key comb width the library gave the 4 kids
    npool = min(args.pool or args.tokens, args.tokens)
    pool = gen_tokens("ES256", npool, golden_keypaths(kids), host_threads, f"r{rank}")
    arena, toks = pack(pool, [ALG_IDS["ES256"]] * npool, np.arange(npool) % len(kids), args.tokens)
    # the second staged batch of measure(): another npool unique tokens
    pool2 = gen_tokens("ES256", npool, golden_keypaths(kids), host_threads, f"r{rank}b")
    second = pack(pool2, [ALG_IDS["ES256"]] * npool, np.arange(npool) % len(kids), args.tokens)
    del pool2
    el, acc, kms, _ = measure(ctx, arena, toks, args.steps, args.warmup, dist, second=second)
    acc2 = LAST_ACCEPTED2
    es_window = LAST_WINDOW
    del second
    ntok = len(toks)
    value = world * ntok * args.steps / el
    ms_step = el * 1000.0 / args.steps
    point_ms = kms.get("p256_point", float("nan"))
    mads = p256_point_mads_per_token() * ntok
    achieved = mads / (point_ms * 1e-3) / 1e12
    result = {
        "metric": "verified JWTs/sec (RS256-2048, ES256) at 1/2/4/8 MI355X vs all-core Go CPU",
        "value": value,
        "unit": "verified JWTs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (28-bit limbs, 64-bit v_mad_u64_u32 accumulators)",
        "data": f"synthetic: OpenSSL-signed ES256 JWTs (testJWTClaims shape), {npool} unique tokens"
                + (f" replicated to {ntok}" if npool < ntok else "") + " per GPU, no verdict caching; "
                "steps alternate between two staged batches of different tokens (bench.measure)",
        "config": {"workload": "ES256 P-256 JWKS with 4 kids, 1M tokens batch-verified per MI355X (BASELINE configs[1])",
                   "tokens_per_gpu": ntok, "unique_tokens": npool, "kids": 4,
                   "table_budget_GiB": budget / (1 << 30), "p256_key_comb_w": P256_WQ,
                   "parallelism": f"independent shards x{world}"},
        "accepted": acc,
        "roofline": {"bound": "valu", "kernel": "k_ec_point<P256>",
                     "achieved": achieved, "peak": MAD_PEAK_T, "unit": "TMAD/s",
                     "frac": achieved / MAD_PEAK_T, "traffic": load_traffic("p256_point"),
                     "traffic_from": os.path.relpath(TRAFFIC, ROOT),
                     "mads_per_token": p256_point_mads_per_token(),
                     "trace_window": es_window,
                     "note": "integer multiply-add roofline (SURVEY §8d): algorithmic MADs (v_mad_u64_u32 partial "
                             f"products of 28-bit limbs) per token {p256_point_mads_per_token():.0f} for the comb "
                             "algorithm at the run's table widths (not §8(d)'s double-and-add count: the comb tables, "
                             "built outside the timed region, replace the doublings) x tokens / HIP-event kernel time of the "
                             "synchronous runs (trace_window: their CLOCK_BOOTTIME span; the timed steps overlap two "
                             "batches, so their launches share the CUs); peak = measured v_mad_u64_u32 rate; "
                             "traffic = HBM bytes per launch, 2 x FETCH_SIZE + WRITE_SIZE of the rocprofv3 --pmc "
                             f"passes in {os.path.relpath(TRAFFIC, ROOT)} (x2 calibrated for the packed 64-byte "
                             "comb entries by tools/ubench/gather_cal: FETCH counts 64 B per 64-B-aligned entry, "
                             "x2 = the 128-B line holding it; 20 entries per token)"},
        "roofline_other": roofline_line(kms, ntok, {"p256_prep": ("hbm", prep_bytes_per_token(342, 49))}),
        "kernel_ms": kms,
        "cpu": cpu,
    }
    if acc != ntok or acc2 not in (None, ntok):
        result["error"] = f"only {acc}/{ntok} (second batch {acc2}) valid tokens accepted"
    if rank == 0 and world == 1:
        result["pcie"] = measure_pcie(ctx, arena, toks)
    # the same batch at the library's default table budget (what a caller gets
    # without jg_set_table_budget): the 4 kids' key tables at W = 24
    if not args.no_ab and budget != (32 << 30):
        ctx.set_table_budget(32 << 30)
        ctx.load_keys(abi_keys(kids))
        wdef = min(ctx.table_widths())
        eld, accd, kmsd, _ = measure(ctx, arena, toks, max(1, args.steps // 2), 1, dist)
        result["default_budget"] = {"table_budget_GiB": 32, "p256_key_comb_w": wdef,
                                    "value": world * ntok * max(1, args.steps // 2) / eld, "kernel_ms": kmsd,
                                    "accepted": accd,
                                    "note": "same 1M-token batch with the library's default 32 GiB key-table budget "
                                            "(no jg_set_table_budget call); `value` above uses the bench's budget"}
        ctx.set_table_budget(budget)
        ctx.load_keys(abi_keys(kids))
    del arena, toks
    # A/B: the same batch built from a 131072-token pool replicated 8x (round-1 default)
    if not args.no_ab and npool > (1 << 17):
        sub = pool[:1 << 17]
        a2, t2 = pack(sub, [ALG_IDS["ES256"]] * len(sub), np.arange(len(sub)) % len(kids), args.tokens)
        el2, acc2, kms2, _ = measure(ctx, a2, t2, max(1, args.steps // 2), 1, dist)
        result["pool_ab"] = {"replicated_pool": len(sub), "value": world * len(t2) * max(1, args.steps // 2) / el2,
                             "kernel_ms": kms2, "accepted": acc2,
                             "note": "same 1M-token batch from a 131072-token pool replicated 8x; `value` above "
                                     "uses unique tokens"}
        del a2, t2

    # ---- RS256 RSA-2048 (second half of the metric; BASELINE configs[0]'s 100k-token pool)
    if not args.no_rs256:
        ctx.load_keys(abi_keys(["rsa2048-a"]))
        rpool = gen_tokens("RS256", min(args.rs_pool, args.tokens), golden_keypaths(["rsa2048-a"]), host_threads,
                           f"r{rank}")
        rarena, rtoks = pack(rpool, [ALG_IDS["RS256"]] * len(rpool), [0] * len(rpool), args.tokens)
        rsteps = max(1, args.steps // 2)
        rel, racc, rkms, _ = measure(ctx, rarena, rtoks, rsteps, 1, dist)
        mexp = rkms.get("rsa2048_modexp", float("nan"))
        rach = rsa_modexp_mads_per_token(74, 2) * len(rtoks) / (mexp * 1e-3) / 1e12
        result["rs256"] = {"value": world * len(rtoks) * rsteps / rel, "unit": "verified JWTs/s",
                           "ms_per_step": rel * 1000.0 / rsteps, "tokens_per_gpu": len(rtoks),
                           "unique_tokens": len(rpool), "accepted": racc, "kernel_ms": rkms,
                           "roofline": {"bound": "valu", "kernel": "k_rsa_modexp<37,2,8>", "achieved": rach,
                                        "peak": MAD_PEAK_T, "unit": "TMAD/s", "frac": rach / MAD_PEAK_T,
                                        "mads_per_token": rsa_modexp_mads_per_token(74, 2),
                                        "traffic": load_traffic("rsa2048_modexp"), "trace_window": LAST_WINDOW},
                           "roofline_other": roofline_line(rkms, len(rtoks),
                                                           {"rsa2048_prep": ("hbm", prep_bytes_per_token(598, 66))})}
        if racc != len(rtoks):
            result["rs256"]["error"] = f"only {racc}/{len(rtoks)} valid tokens accepted"
        del rarena, rtoks

    # ---- the other BASELINE configs (per-GPU share, same timing rules)
    if not args.no_configs:
        result["configs"] = run_configs(ctx, args, host_threads, rank, world, dist)
    ctx.close()
    if C5_E2E and rank == 0 and not args.no_e2e:
        result["configs"]["mixed_10alg_32kid"]["jwks_e2e"] = measure_jwks_e2e(C5_E2E["pool"], C5_E2E["good"],
                                                                             C5_E2E["meta"], host_threads)
    C5_E2E.clear()

    # ---- end-to-end Validator.ValidateBatch (host + GPU), rank 0 only: in a
    # fresh child process (the line), and inside this long-running bench
    # process beside it
    if rank == 0 and not args.no_e2e:
        jwk = [{"kty": "EC", "kid": f"kid-{i:02d}", "crv": "P-256", **xy} for i, xy in enumerate(p256_jwk_xy(kids))]
        # the line is the rate inside this long-running process (after every
        # other leg: tens of GB of token pools and many contexts behind it);
        # the same measurement in a fresh child process rides beside it
        inproc, phases = with_trace_phases(lambda: measure_e2e(pool, jwk, args.tokens, host_threads))
        inproc["phases_ms_last_pass"] = phases
        inproc["process"] = "the bench process itself, after every other leg"
        fresh = measure_e2e_fresh(pool, args.tokens)
        inproc["fresh_child"] = {k: fresh[k] for k in ("value", "ms_per_batch", "phases_ms_last_pass", "host_diag",
                                                       "process") if k in fresh}
        inproc["in_process_over_fresh"] = inproc["value"] / fresh["value"]
        result["e2e"] = inproc
        result["single"] = measure_single(pool, jwk, host_threads)
    if rank == 0 and world == 1 and args.md_devices != "none":
        jwk = [{"kty": "EC", "kid": f"kid-{i:02d}", "crv": "P-256", **xy} for i, xy in enumerate(p256_jwk_xy(kids))]
        result["multi_device"] = measure_multi_device(pool, kids, jwk, md_devices(args.md_devices), args.tokens,
                                                      host_threads)

    # ---- CPU baselines (rank 0, N = 1 only), both on every core the process
    # may use.  `cpu_baseline` is OpenSSL libcrypto (tools/cpuverify): the
    # closest stand-in for Go's assembly-backed crypto/ecdsa and crypto/rsa
    # available on the box (Go itself is absent).  The repo's clarity-first C
    # oracle (oracle/jws_oracle.c, the "port") is reported beside it.
    if rank == 0 and world == 1 and not args.no_cpu:
        port = cpu_baseline(pool, "ES256", golden_oracle_keys(kids), host_threads, args.cpu_seconds, cpu=cpu)
        result["cpu_baseline_port"] = port
        ossl = {}
        try:
            ossl["es256"] = openssl_baseline(pool[:1 << 16], "ES256", golden_keypaths(kids), host_threads, 5.0)
        except (OSError, subprocess.CalledProcessError, ValueError) as e:
            result["cpu_baseline_openssl_error"] = str(e)
        # the contract's cpu_baseline is the oracle ("port"); OpenSSL rides
        # beside it as cpu_openssl (the closer stand-in for Go's crypto)
        result["cpu_baseline"] = port
        speed = {}
        if "es256" in ossl:
            speed["es256_vs_openssl"] = value / ossl["es256"]["value"]
        speed["es256_vs_port"] = value / port["value"]
        if not args.no_rs256:
            # BASELINE configs[0]: RS256 RSA-2048 StaticKeySet, 100k tokens, all cores
            try:
                ossl["rs256"] = openssl_baseline(rpool, "RS256", golden_keypaths(["rsa2048-a"]), host_threads, 3.0)
                speed["rs256_vs_openssl"] = result["rs256"]["value"] / ossl["rs256"]["value"]
            except (OSError, subprocess.CalledProcessError, ValueError) as e:
                result["cpu_baseline_openssl_error"] = str(e)
            result["cpu_baseline_rs256_port"] = cpu_baseline(rpool, "RS256", golden_oracle_keys(["rsa2048-a"]),
                                                             host_threads, 0, max_tokens=len(rpool), cpu=cpu)
            speed["rs256_vs_port"] = result["rs256"]["value"] / result["cpu_baseline_rs256_port"]["value"]
        result["cpu_baseline_openssl"] = ossl
        speed["note"] = ("GPU value / all-core CPU rate on the same tokens. Neither CPU leg is Go (absent on the GPU "
                         "box): 'openssl' = OpenSSL libcrypto (cpu_baseline), 'port' = the repo's clarity-first C oracle")
        if "single" in result and "es256" in ossl:
            result["single"]["cpu_baseline_openssl"] = ossl["es256"]["value"]
        result["speedup_vs_cpu"] = speed
    if rank == 0:
        emit_line(result, args.detail)
    if dist:
        import torch.distributed as td
        td.destroy_process_group()


def p256_jwk_xy(kids):
    import base64
    from tests import gpu_helpers as H
    kd = {k["kid"]: k for k in H.golden()[0]}
    out = []
    for k in kids:
        d = kd[k]
        out.append({"x": base64.urlsafe_b64encode(int(d["x"], 16).to_bytes(32, "big")).rstrip(b"=").decode(),
                    "y": base64.urlsafe_b64encode(int(d["y"], 16).to_bytes(32, "big")).rstrip(b"=").decode()})
    return out


if __name__ == "__main__":
    main()
