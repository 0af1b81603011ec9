"""Pinned H2D copy bandwidth vs copy size on one stream (back-to-back async
copies, timed by wall clock around a stream sync).  Measurement only."""
import ctypes
import time

hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
hip.hipStreamSynchronize.argtypes = [vp]
TOTAL = 384 << 20
h, d, s = vp(), vp(), vp()
assert hip.hipHostMalloc(ctypes.byref(h), TOTAL, 1) == 0
assert hip.hipMalloc(ctypes.byref(d), TOTAL) == 0
assert hip.hipStreamCreate(ctypes.byref(s)) == 0
ctypes.memset(h, 1, TOTAL)
for mb in (1, 2, 4, 8, 12, 16, 20, 24, 32, 48, 64, 128, 384):
    n = mb << 20
    best = 1e9
    for _ in range(4):
        t0 = time.perf_counter()
        for off in range(0, TOTAL, n):
            hip.hipMemcpyAsync(vp(d.value + off), vp(h.value + off), min(n, TOTAL - off), 1, s)
        hip.hipStreamSynchronize(s)
        best = min(best, time.perf_counter() - t0)
    print(f"copy {mb:4d} MB: {TOTAL / best / 1e9:6.1f} GB/s ({TOTAL // n} copies, {best*1e3:.2f} ms)", flush=True)
