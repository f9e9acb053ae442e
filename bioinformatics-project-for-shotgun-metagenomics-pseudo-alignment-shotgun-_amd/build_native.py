"""Build libpa.so (HIP, gfx950) in-tree with hipcc.

    python build_native.py [--force] [--stats]

Objects go to ./build/, the shared library to ./libpa.so next to this file
(both git-ignored; the .so travels to the GPU box with the repo snapshot).
--stats builds the diagnostic variant libpa_stats.so (-DPA_STATS: the fast
kernel counts windows / probes / walk-resolved windows / anchors and pa_align
prints them to stderr); load it with PA_LIBRARY=<path>.
"""

from __future__ import annotations

import hashlib
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


def _digest(paths, extra=()) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    for e in extra:
        h.update(str(e).encode() + b"\0")
    return h.hexdigest()


def source_hash(stats: bool = False, defines=()) -> str:
    """SHA-256 of every csrc source and header, include/pa.h, the target arch
    and the compile flags: what pa_version() of a library built from this
    checkout reports after "src=" (the library is rebuilt when it changes)."""
    flags = FLAGS + (["-DPA_STATS"] if stats else []) + [f"-D{d}" for d in defines]
    flags = [f.replace(INCLUDE, "<repo>/include") for f in flags]  # (the checkout's path is not part of it)
    paths = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(INCLUDE, "pa.h")]
    return _digest(paths, [ARCH] + flags)


def library_hash(version: str) -> str:
    """The source hash a loaded library reports (pa_version() text)."""
    return version.split("src=", 1)[1].strip() if "src=" in version else ""


def _stamp_ok(target: str, digest: str) -> bool:
    try:
        with open(target + ".sha") as f:
            return os.path.exists(target) and f.read().strip() == digest
    except OSError:
        return False


def _stamp(target: str, digest: str) -> None:
    with open(target + ".sha", "w") as f:
        f.write(digest + "\n")


def build(force: bool = False, verbose: bool = False, stats: bool = False, variant: str = "",
          defines=()) -> str:
    """Build libpa.so; `stats` or a named `variant` (with extra -D defines) go to
    their own build directory and libpa_<name>.so (experiments, PA_LIBRARY)."""
    name = "stats" if stats else variant
    build_dir = BUILD + (f"_{name}" if name else "")
    lib = os.path.join(HERE, f"libpa_{name}.so") if name else LIB
    flags = FLAGS + (["-DPA_STATS"] if stats else []) + [f"-D{d}" for d in defines]
    full = source_hash(stats, defines)
    os.makedirs(build_dir, exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "pa.h")]
    jobs = []
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        # staleness by content: the source, every header and the flags (pa_api
        # embeds the whole checkout's hash, so it follows every file)
        extra = [f"-DPA_SOURCE_HASH=\"{full}\""] if src == "pa_api.cpp" else []
        if src.endswith(".hip"):
            cmd = [hipcc, f"--offload-arch={ARCH}", *flags, *extra, "-x", "hip", "-c", path, "-o", obj]
        else:
            cmd = [hipcc, *flags, *extra, "-c", path, "-o", obj]
        digest = _digest([path] + headers, cmd[1:])
        if force or not _stamp_ok(obj, digest):
            jobs.append((cmd, obj, digest))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}")
        return r.stdout

    def job(j):
        cmd, obj, digest = j
        if os.path.exists(obj + ".sha"):
            os.remove(obj + ".sha")
        run(cmd)
        _stamp(obj, digest)

    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), 4))) as ex:
        list(ex.map(job, jobs))
    if force or jobs or not _stamp_ok(lib, full):
        if os.path.exists(lib + ".sha"):
            os.remove(lib + ".sha")
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, "-lz", "-lpthread", "-ldl"])
        _stamp(lib, full)
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
