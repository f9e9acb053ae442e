#!/usr/bin/env python3
"""One rocprofv3 counter pass over a bench workload (diagnostics): the align
kernels' per-dispatch averages of the given counters.

    python scripts/pmc_pass.py --config c5 --out gpurun_out/x/c5_tlb.json \
        TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum ...

Runs `rocprofv3 --kernel-trace --pmc <counters> -- python bench.py
--traffic-child --config C` (warmup 1, 2 timed passes) and reads the
database as bench.py's own counter pass does.  Keep to one pass's limits
(8 SQ, 4 TCP, 4 TCC, 2 TA / TD / GRBM counters).
"""
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
from bench import kernel_short_name  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--reads-per-gpu", type=int, default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--kernels", default=None, help="regex on kernel names (default: the align kernels)")
    ap.add_argument("--bench-args", default="", help="extra bench.py arguments")
    ap.add_argument("counters", nargs="+")
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="pa_pmc_", dir="/tmp")
    cmd = [shutil.which("rocprofv3"), "--kernel-trace", "--pmc", *args.counters, "-d", tmp, "-o", "run", "--",
           sys.executable, os.path.join(REPO, "bench.py"), "--traffic-child", "--config", args.config,
           "--steps", "2", "--warmup", "1"]
    if args.reads_per_gpu:
        cmd += ["--reads-per-gpu", str(args.reads_per_gpu)]
    cmd += args.bench_args.split()
    import re
    pat = re.compile(args.kernels) if args.kernels else None

    def short(name):
        if pat is None:
            return kernel_short_name(name)
        m = re.search(r"\d+(k_[A-Za-z0-9_]+)", name)
        base = m.group(1) if m else name
        return base if pat.search(base) else None
    r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=args.timeout)
    if r.returncode:
        sys.exit(f"rocprofv3 rc {r.returncode}: {r.stderr[-1500:]}")
    db = glob.glob(os.path.join(tmp, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    per = {}
    for name, cname, v, n in c.execute(
            "select s.kernel_name, i.name, avg(e.value), count(e.value) from rocpd_pmc_event e "
            "join rocpd_info_pmc i on e.pmc_id = i.id join rocpd_event ev on e.event_id = ev.id "
            "join rocpd_kernel_dispatch d on d.event_id = ev.id "
            "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name, i.name"):
        sh = short(name)
        if sh:
            per.setdefault(sh, {})[cname] = [float(v), int(n)]
    for name, avg_ns, n in c.execute(
            "select s.kernel_name, avg(d.end - d.start), count(*) from rocpd_kernel_dispatch d "
            "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name"):
        sh = short(name)
        if sh and sh in per:
            per[sh]["trace_avg_ms"] = float(avg_ns) / 1e6
            per[sh]["launches"] = int(n)
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"config": args.config, "counters": args.counters, "per_kernel_avg_per_dispatch": per}, f, indent=1)
    for k, d in per.items():
        print(args.config, k, {a: (round(b[0], 1) if isinstance(b, list) else round(b, 3)) for a, b in d.items()})


if __name__ == "__main__":
    main()
