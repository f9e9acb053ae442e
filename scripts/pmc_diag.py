#!/usr/bin/env python3
"""Diagnostic counter pass (GPU box): one rocprofv3 --kernel-trace --pmc run of
a bench config's align pass with the counters named, averaged per align kernel.

    python scripts/pmc_diag.py <config> <COUNTER> [<COUNTER> ...] [--reads N]

Keep within one pass's limits (8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_ counters).
Prints one JSON object {kernel: {counter: avg per dispatch, "ms": avg}}."""
import argparse
import glob
import json
import os
import shutil
import sqlite3
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def kernel_short_name(mangled: str):
    """Any kernel's identifier (k_...) from its mangled name: the length prefix
    may run into a preceding digit ("_GLOBAL__N_1" + "10k_nb_build")."""
    import re
    for m in re.finditer(r"(\d+)(k_[A-Za-z0-9_]+)", mangled):
        digits, rest = m.group(1), m.group(2)
        for i in range(len(digits)):
            n = int(digits[i:])
            if n <= len(rest) and (n == len(rest) or rest[n] in "EIv."):
                return rest[:n]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("counters", nargs="+")
    ap.add_argument("--reads", type=int, default=0)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="pa_pmc_", dir="/tmp")
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", *a.counters, "-d", tmp, "-o", "run", "--", sys.executable,
           os.path.join(REPO, "bench.py"), "--traffic-child", "--config", a.config, "--steps", "2", "--warmup", "1"]
    if a.reads:
        cmd += ["--reads-per-gpu", str(a.reads)]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=600)
    if r.returncode != 0:
        print(r.stderr[-2000:], file=sys.stderr)
        sys.exit(r.returncode)
    db = glob.glob(os.path.join(tmp, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    out = {}
    for name, cname, v in c.execute(
            "select s.kernel_name, i.name, avg(e.value) from rocpd_pmc_event e "
            "join rocpd_info_pmc i on e.pmc_id = i.id join rocpd_event ev on e.event_id = ev.id "
            "join rocpd_kernel_dispatch d on d.event_id = ev.id "
            "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name, i.name"):
        short = kernel_short_name(name)
        if short:
            out.setdefault(short, {})[cname] = float(v)
    for name, ns in c.execute("select s.kernel_name, avg(d.end - d.start) from rocpd_kernel_dispatch d "
                              "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name"):
        short = kernel_short_name(name)
        if short in out:
            out[short]["ms"] = float(ns) / 1e6
    shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
