#!/usr/bin/env python3
"""GPU box probe: how long hipMalloc of large buffers takes as the device
fills (the C5 align-side view allocates ~66 GB with ~115 GB already in use).
Prints one line per step."""
import ctypes
import time

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
GB = 1 << 30


def timed(fn):
    t = time.perf_counter()
    r = fn()
    hip.hipDeviceSynchronize()
    return 1e3 * (time.perf_counter() - t), r


def alloc(n, touch=True):
    p = ctypes.c_void_p()
    ms, r = timed(lambda: hip.hipMalloc(ctypes.byref(p), n))
    ms2 = timed(lambda: hip.hipMemsetAsync(p, 0, n, None))[0] if touch and r == 0 else 0.0
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t))
    print(f"hipMalloc {n / GB:.0f} GB: {ms:.1f} ms (rc {r}), memset {ms2:.1f} ms; free {f.value / GB:.1f} of "
          f"{t.value / GB:.1f} GB", flush=True)
    return p


def free_all(ps):
    ms = sum(timed(lambda: hip.hipFree(p))[0] for p in ps)
    print(f"hipFree x{len(ps)}: {ms:.1f} ms", flush=True)


hip.hipFree(None)
print("-- one 20 GB step at a time", flush=True)
ps = [alloc(20 * GB) for _ in range(12)]
free_all(ps)
print("-- 156 GB at once, then 8", flush=True)
ps = [alloc(156 * GB), alloc(8 * GB)]
free_all(ps)
print("-- 8 GB pieces", flush=True)
ps = [alloc(8 * GB) for _ in range(26)]
free_all(ps)
