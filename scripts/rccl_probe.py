#!/usr/bin/env python3
"""Diagnose pa_comm_init on the GPU box: which librccl / libamdhip64 /
libhsa-runtime64 the process maps, with and without torch imported first.
    python scripts/rccl_probe.py [--torch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd"))
if "--torch" in sys.argv:
    import torch  # noqa: F401
import pa_native as N

print("devices", N.device_count(), flush=True)
try:
    c = N.Comm(0, 1, 0, N.Comm.unique_id())
    print("comm ok, ranks", c.n_ranks, flush=True)
    c.close()
except Exception as e:
    print("comm failed:", e, flush=True)
libs = set()
with open("/proc/self/maps") as f:
    for line in f:
        p = line.split()[-1]
        if any(x in p for x in ("rccl", "amdhip", "hsa-runtime")):
            libs.add(p)
print("\n".join(sorted(libs)))
