#!/usr/bin/env python3
"""What a short CLI process pays around its work on the GPU box: interpreter
start and exit, HIP runtime start, and process teardown with N GiB of device
memory allocated and touched (os._exit, as main.py ends).  Prints one JSON line.

    python scripts/exit_probe.py
"""
import json
import subprocess
import sys
import time

CHILD = r'''
import ctypes, os, sys, time
t0 = time.perf_counter()
gib = int(sys.argv[1])
if gib >= 0:
    h = ctypes.CDLL("libamdhip64.so.7")
    assert h.hipSetDevice(0) == 0
    p = ctypes.c_void_p()
    if gib > 0:
        assert h.hipMalloc(ctypes.byref(p), ctypes.c_size_t(gib << 30)) == 0
        assert h.hipMemset(p, 0, ctypes.c_size_t(gib << 30)) == 0
    assert h.hipDeviceSynchronize() == 0
sys.stderr.write("%.4f\n" % (time.perf_counter() - t0))
sys.stderr.flush()
os._exit(0)
'''


def run(gib):
    t = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", CHILD, str(gib)], stderr=subprocess.PIPE, text=True)
    wall = time.perf_counter() - t
    inner = float(r.stderr.strip().splitlines()[-1])
    return {"gib": gib, "wall_s": round(wall, 4), "inside_s": round(inner, 4), "outside_s": round(wall - inner, 4)}


def main():
    out = {"python_only": run(-1)}
    for g in (0, 4, 16, 64):
        time.sleep(2)
        out[f"hip_{g}gib"] = run(g)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
