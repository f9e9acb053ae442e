#!/usr/bin/env python3
"""Summarise a rocprofv3 database (--kernel-trace [--pmc ...]) into a text table.

    python profiles/rocpd_summary.py gpurun_out/prof_c2/run_results.db > profiles/r02/c2_kernel_stats.txt

Per kernel: dispatch count, average / total duration; and, when the database
holds PMC samples, the per-dispatch average of every counter.
"""

import sqlite3
import sys
from collections import defaultdict


def main(path: str) -> None:
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start), "
         "max(s.arch_vgpr_count), max(s.sgpr_count), max(d.group_segment_size) "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by 4 desc")
    print(f"{'kernel':70s} {'calls':>6s} {'avg_ms':>10s} {'total_ms':>10s} {'vgpr':>5s} {'sgpr':>5s} {'lds_B':>7s}")
    for name, n, avg, tot, vg, sg, lds in c.execute(q):
        print(f"{name[:70]:70s} {n:6d} {avg / 1e6:10.4f} {tot / 1e6:10.3f} {vg or 0:5d} {sg or 0:5d} {lds or 0:7d}")
    try:
        rows = list(c.execute(
            "select s.kernel_name, i.name, avg(e.value), count(*) from rocpd_pmc_event e "
            "join rocpd_info_pmc i on e.pmc_id = i.id join rocpd_event ev on e.event_id = ev.id "
            "join rocpd_kernel_dispatch d on d.event_id = ev.id join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
            "group by s.kernel_name, i.name"))
    except sqlite3.Error:
        rows = []
    if rows:
        print("\nPMC (average per dispatch):")
        per = defaultdict(dict)
        for k, cname, v, n in rows:
            per[k][cname] = v
        for k, d in per.items():
            print(f"  {k[:70]}")
            for cname, v in sorted(d.items()):
                print(f"      {cname:32s} {v:18.1f}")
            wc = d.get("SQ_WAVE_CYCLES")
            if wc:  # per-wave shares of the resident cycles
                for cname in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                              "SQ_ACTIVE_INST_VMEM"):
                    if cname in d:
                        print(f"      {cname + ' / SQ_WAVE_CYCLES':48s} {d[cname] / wc:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
