"""Per-call host time of back-to-back pinned H2D copies on one stream, in the
pipeline's pattern (big span from one pinned arena + a small metadata copy
from another pinned buffer + an event), to find host-blocking copies.
Measurement only."""
import ctypes
import sys
import time

hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]
hip.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
hip.hipEventRecord.argtypes = [vp, vp]
TOTAL = 360 << 20
CH, META = 11 << 20, 800 << 10
mode = sys.argv[1] if len(sys.argv) > 1 else "pattern"
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 1
h, d, hm, dm, s = vp(), vp(), vp(), vp(), vp()
assert hip.hipHostMalloc(ctypes.byref(h), TOTAL, flags) == 0
assert hip.hipHostMalloc(ctypes.byref(hm), 8 * META, flags) == 0
assert hip.hipMalloc(ctypes.byref(d), 16 * CH) == 0
assert hip.hipMalloc(ctypes.byref(dm), 8 * META) == 0
assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
ev = [vp() for _ in range(8)]
for e in ev:
    hip.hipEventCreate(ctypes.byref(e))
ctypes.memset(h, 1, TOTAL)
for it in range(3):
    calls = []
    t0 = time.perf_counter()
    for k, off in enumerate(range(0, TOTAL - CH, CH)):
        c0 = time.perf_counter()
        hip.hipMemcpyAsync(vp(d.value + (k % 16) * CH), vp(h.value + off), CH, 1, s)
        if mode == "pattern":
            hip.hipMemcpyAsync(vp(dm.value + (k % 8) * META), vp(hm.value + (k % 8) * META), META, 1, s)
            hip.hipEventRecord(ev[k % 8], s)
        calls.append(time.perf_counter() - c0)
    hip.hipStreamSynchronize(s)
    el = time.perf_counter() - t0
    slow = [(i, round(c * 1e3, 3)) for i, c in enumerate(calls) if c > 2e-4]
    print(f"{mode} flags={flags} iter {it}: {el*1e3:.2f} ms, {len(calls)} chunks, "
          f"{(TOTAL - CH) * (1 + META / CH) / el / 1e9:.1f} GB/s; slow calls {slow}", flush=True)
