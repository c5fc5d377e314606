"""Cost of the per-call scratch allocations the per-rank backends make
(hipHostMalloc / hipMalloc / stream and event creation, and their frees),
by size, on the GPU box. Prints one JSON line per size."""
import ctypes
import json
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipFree(None)
for mib in (1, 4, 16, 32, 64):
    n = mib << 20
    p = ctypes.c_void_p()
    t = {}
    for name, alloc, free in (("hipHostMalloc", lambda: hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0),
                               lambda: hip.hipHostFree(p)),
                              ("hipMalloc", lambda: hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)),
                               lambda: hip.hipFree(p))):
        reps = 10
        ta = tf = 0.0
        for _ in range(reps):
            t0 = time.perf_counter()
            assert alloc() == 0
            t1 = time.perf_counter()
            assert free() == 0
            ta += t1 - t0
            tf += time.perf_counter() - t1
        t[name] = {"alloc_ms": round(ta / reps * 1e3, 3), "free_ms": round(tf / reps * 1e3, 3)}
    print(json.dumps({"MiB": mib, **t}), flush=True)
s = ctypes.c_void_p()
ev = ctypes.c_void_p()
rows = []
for _ in range(6):
    t0 = time.perf_counter()
    hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    t1 = time.perf_counter()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
    t2 = time.perf_counter()
    hip.hipEventDestroy(ev)
    hip.hipStreamDestroy(s)
    t3 = time.perf_counter()
    rows.append([round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 3), round((t3 - t2) * 1e3, 3)])
print(json.dumps({"stream_create_ms, event_create_ms, both_destroy_ms (per iteration)": rows}))
