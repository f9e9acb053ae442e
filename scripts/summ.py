#!/usr/bin/env python3
"""Print the headline figures of bench lines: python scripts/summ.py gpurun_out/na3/*.json"""
import json
import sys

for p in sys.argv[1:]:
    if not p.endswith(".json") or "counters_" in p:
        continue
    try:
        d = json.load(open(p))
    except Exception as e:  # (a failed run)
        print(p, "unreadable:", e)
        continue
    r = d["roofline"]
    ps = d.get("parity_sample") or {}
    print(f"{p}: {d['value'] / 1e9:.3f} G reads/s  bound {r['bound']}  frac {r['frac'] and round(r['frac'], 3)}  "
          f"dominant {r['kernel']} {r['kernel_ms']:.3f} ms  pass lines/read {r.get('pass_lines_per_read', 0):.2f}  "
          f"parity {ps.get('bit_exact')} ({ps.get('reads')})")
    for k, v in r["kernels"].items():
        sq = v.get("sq_share_of_wave_cycles") or {}
        print(f"    {k:16s} {v.get('ms_avg', 0):7.3f} ms  lines/read {v.get('lines_per_read', 0):6.2f}  "
              f"frac {v.get('frac', 0) or 0:.3f}  wait {sq.get('wait_any', 0):.2f} valu {sq.get('active_inst_valu', 0):.3f}")
