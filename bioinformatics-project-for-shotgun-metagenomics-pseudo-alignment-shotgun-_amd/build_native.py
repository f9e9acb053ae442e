"""Build libpa.so (HIP, gfx950) in-tree with hipcc.

    python build_native.py [--force] [--stats]

Objects go to ./build/, the shared library to ./libpa.so next to this file
(both git-ignored; the .so travels to the GPU box with the repo snapshot).
--stats builds the diagnostic variant libpa_stats.so (-DPA_STATS: the fast
kernel counts windows / probes / walk-resolved windows / anchors and pa_align
prints them to stderr); load it with PA_LIBRARY=<path>.
"""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libpa.so")
ARCH = os.environ.get("PA_OFFLOAD_ARCH", "gfx950")

SOURCES = ["pa_index.hip", "pa_align.hip", "pa_fastq.hip", "pa_dump.hip", "pa_kpos.hip", "pa_api.cpp", "pa_ingest.cpp", "pa_comm.cpp", "pa_gz.cpp", "pa_pgz.cpp", "pa_mem.cpp"]
HEADERS = ["pa_device.h", "pa_internal.h", "pa_fast.h", "pa_lane.h", "pa_home.h", "pa_gz.h", "pa_pgz.h"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-value", "-Wno-unused-result", f"-I{INCLUDE}"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, stats: bool = False, variant: str = "",
          defines=()) -> str:
    """Build libpa.so; `stats` or a named `variant` (with extra -D defines) go to
    their own build directory and libpa_<name>.so (experiments, PA_LIBRARY)."""
    name = "stats" if stats else variant
    build_dir = BUILD + (f"_{name}" if name else "")
    lib = os.path.join(HERE, f"libpa_{name}.so") if name else LIB
    flags = FLAGS + (["-DPA_STATS"] if stats else []) + [f"-D{d}" for d in defines]
    os.makedirs(build_dir, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "pa.h")]
    jobs = []
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        if force or _stale(obj, [path, __file__] + headers):
            if src.endswith(".hip"):
                cmd = [hipcc, f"--offload-arch={ARCH}", *flags, "-x", "hip", "-c", path, "-o", obj]
            else:
                cmd = [hipcc, *flags, "-c", path, "-o", obj]
            jobs.append(cmd)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}")
        return r.stdout

    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), 4))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _stale(lib, objs):
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, "-lz", "-lpthread", "-ldl"])
    return lib


def build_tools(force: bool = False) -> str:
    """Measurement tools (not part of libpa.so): profiles/fetch_calib, the
    FETCH_SIZE calibration of the align kernels' access shapes."""
    src = os.path.join(os.path.dirname(HERE), "profiles", "fetch_calib.hip")
    exe = os.path.splitext(src)[0]
    if force or _stale(exe, [src]):
        r = subprocess.run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-o", exe, src],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}")
    return exe


if __name__ == "__main__":
    var = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--variant=")]
    defs = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--define=")]
    print(build(force="--force" in sys.argv, verbose=True, stats="--stats" in sys.argv,
                variant=var[0] if var else "", defines=defs))
