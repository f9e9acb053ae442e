#!/usr/bin/env python3
"""Copy one scripts/measure.sh result into profiles/<round>/ (ROUND, default r04): the bench line, its
counter pass (per-kernel fabric bytes and SQ shares, JSON) and the rocprofv3
kernel summary of the same workload, stamped with the git commit measured.

    python scripts/save_measure.py <tag> [name]      (name defaults to the tag)
"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag: str, name: str) -> None:
    src = os.path.join(REPO, "gpurun_out", f"ms_{tag}")
    dst = os.path.join(REPO, "profiles", os.environ.get("ROUND", "r04"))
    os.makedirs(dst, exist_ok=True)
    head = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=REPO, capture_output=True, text=True).stdout.strip()
    with open(os.path.join(src, "args")) as f:
        args = f.read().strip()
    with open(os.path.join(src, "bench.json")) as f:
        line = f.read()
    with open(os.path.join(dst, f"bench_{name}.json"), "w") as f:
        f.write(line)
    for cj in glob.glob(os.path.join(src, "counters_*.json")):
        with open(cj) as f:
            body = f.read()
        with open(os.path.join(dst, f"{name}_counters.json"), "w") as f:
            f.write(body)
    summ = os.path.join(REPO, "profiles", "rocpd_summary.py")
    for kind, label in (("trace", "kernel_stats"), ("sq", "sq")):
        done = os.path.join(src, f"{label}.txt" if kind == "trace" else "sq.txt")
        dbs = glob.glob(os.path.join(src, kind, "**", "*.db"), recursive=True)
        if os.path.exists(done):  # summarised on the GPU box (measure.sh)
            with open(done) as f:
                out = f.read()
        elif dbs:
            out = subprocess.run([sys.executable, summ, dbs[0]], capture_output=True, text=True, check=True).stdout
        else:
            continue
        with open(os.path.join(dst, f"{name}_{label}.txt"), "w") as f:
            f.write(f"# bench.py --config {args}; measured at commit {head} (+ working tree)\n" + out)
    print("saved", name)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
