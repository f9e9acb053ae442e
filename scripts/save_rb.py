#!/usr/bin/env python3
"""Copy one scripts/round_bench.sh result into profiles/: the bench line, the
rocprofv3 kernel summary, the FETCH_SIZE pass, and traffic_<config>.json (HBM
bytes per align pass = FETCH_SIZE of k_align_lane + k_align_fast, per dispatch).

    python scripts/save_rb.py c2_v11 c2
"""
import glob
import json
import os
import sqlite3
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag: str, config: str) -> None:
    src = os.path.join(REPO, "gpurun_out", f"rb_{tag}")
    cfg, ver = tag.split("_", 1) if "_" in tag else (tag, "v1")
    prof = os.path.join(REPO, "profiles")
    with open(os.path.join(src, "bench.json")) as f:
        line = f.read()
    with open(os.path.join(prof, f"r01_bench_{tag}.json"), "w") as f:
        f.write(line)
    summ = os.path.join(REPO, "profiles", "rocpd_summary.py")
    for kind, name in (("trace", "kernel_stats"), ("pmc", "pmc")):
        db = glob.glob(os.path.join(src, kind, "**", "*.db"), recursive=True)[0]
        out = subprocess.run([sys.executable, summ, db], capture_output=True, text=True, check=True).stdout
        with open(os.path.join(prof, f"r01_{cfg}_{name}_{ver}.txt"), "w") as f:
            f.write(out)
    db = glob.glob(os.path.join(src, "pmc", "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.kernel_name, avg(e.value) from rocpd_pmc_event e join rocpd_info_pmc i on e.pmc_id = i.id "
        "join rocpd_event ev on e.event_id = ev.id join rocpd_kernel_dispatch d on d.event_id = ev.id "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id where i.name = 'FETCH_SIZE' group by s.kernel_name")
    fetch = {}
    for name, v in rows:
        for k in ("k_align_lane", "k_align_fast"):
            if k in name:
                fetch[k] = fetch.get(k, 0.0) + v
    tp = os.path.join(prof, f"traffic_{config}.json")
    old = json.load(open(tp)) if os.path.exists(tp) else {}
    d = {"kernel": "align pass: k_align_lane + k_align_fast",
         "source": f"profiles/r01_{cfg}_pmc_{ver}.txt: rocprofv3 --kernel-trace --pmc FETCH_SIZE, "
                   f"bench.py --config {config} --steps 2 --warmup 1, average per dispatch",
         "fetch_size_kb": fetch,
         "note": old.get("note", "FETCH_SIZE (kB) = TCC_EA0_RDREQ x 64 B as rocprofv3 derives it."),
         "hbm_bytes_per_launch": int(sum(fetch.values()) * 1000)}
    with open(tp, "w") as f:
        json.dump(d, f, indent=2)
    print(tag, json.loads(line)["value"], d["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
