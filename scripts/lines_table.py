#!/usr/bin/env python3
"""profiles/lines_per_read.json: fabric bytes per read of each align kernel, per
bench config, from the counter passes saved under profiles/<round>/
(<config>_counters.json: TCC_EA0_RDREQ_{32B,64B,128B} per dispatch of a
`bench.py --traffic-child` run; <config>.json / bench_<config>.json: its
reads per launch).  bench.py prices an N > 1 rank's dominant-kernel launch with
these bytes (no counter pass runs at N > 1).

    python scripts/lines_table.py profiles/r06 [profiles/r05 ...]   (first found wins per config)
"""
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def main(dirs):
    out = {}
    for d in dirs:
        for path in sorted(glob.glob(os.path.join(REPO, d, "*_counters.json"))):
            cfg = os.path.basename(path)[:-len("_counters.json")]
            if cfg in out:
                continue
            c = json.load(open(path))
            m = re.search(r"--reads-per-gpu (\d+)", c.get("command", ""))
            if not m:
                continue
            reads = int(m.group(1))
            per = {}
            for k, cs in c["per_kernel_avg_per_dispatch"].items():
                b = sum(cs[n][0] * w for n, w in W.items() if n in cs)
                per[k] = {"bytes_per_read": b / reads, "lines_per_read": b / 128.0 / reads}
            out[cfg] = {"reads_per_launch": reads, "kernels": per,
                        "source": os.path.relpath(path, REPO)}
    dst = os.path.join(REPO, "profiles", "lines_per_read.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(dst, sorted(out))


if __name__ == "__main__":
    main(sys.argv[1:] or ["profiles/r05"])
