#!/usr/bin/env python3
"""Parity at a benchmark configuration's FULL reference size.

    python scripts/verify_full.py [--config c4] [--reads 300000]

bench.py checks C2/C3 against the CPU oracle on a prefix of the benchmark's
own reads; C4's 1 Gbp reference makes that too slow for every bench run (the
oracle's index is ~90 GB of host memory and minutes to build), so this script
does it once: the same genomes and device-synthesized reads as
`bench.py --config c4`, the oracle index of all 500 genomes, and a prefix of
the reads aligned by libpa.so and by the oracle on all host threads; counters,
per-genome counts and first keys compared bit for bit.  Prints one JSON line.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import bench  # noqa: E402  (configs, host_threads; also puts the package on sys.path)
import pa_native as N  # noqa: E402
import pa_oracle as O  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=sorted(bench.CONFIGS))
    ap.add_argument("--reads", type=int, default=300_000)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    t0 = time.perf_counter()
    genomes = synth.family_genomes(cfg["n_genomes"], cfg["genome_len"], seed=1, family_size=cfg["family"],
                                   sub_rate=cfg["sub"], conserved_len=cfg["conserved"], n_rate=cfg["n_rate"],
                                   n_run=cfg["n_run"])
    index = N.Index(genomes, cfg["k"], device=0)
    reads = N.Reads.synthesize(index, args.reads, cfg["read_len"], first_read=0, seed=2, sub_rate=cfg["read_err"])
    s, q, off = reads.download()
    pk = cfg["params"]
    kw = dict(m=pk.get("m", 1), p=pk.get("p", 1), mrq=pk.get("mrq"), mkq=pk.get("mkq"), mg=pk.get("mg"))
    res = N.Result(index)
    N.align(index, reads, N.Params.make(kw["m"], kw["p"], kw["mrq"], kw["mkq"], kw["mg"]), 0, res)
    stats, uq, am, fk = res.fetch()
    gpu_s = time.perf_counter() - t0
    print(f"gpu side done in {gpu_s:.1f}s; building the oracle index", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    import threading
    box = {}
    th = threading.Thread(target=lambda: box.setdefault("ix", O.OracleIndex(genomes, cfg["k"])))
    th.start()
    while th.is_alive():  # heartbeat (ctypes releases the GIL inside the C build)
        th.join(timeout=30)
        print(f"  oracle build {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    oix = box["ix"]
    build_s = time.perf_counter() - t0
    print(f"oracle index: {oix.n_kmers} k-mers in {build_s:.0f}s", file=sys.stderr, flush=True)
    threads = bench.host_threads()
    t0 = time.perf_counter()
    o = O.align_counts_parallel(oix, s, q, off, threads, **kw)
    cpu_s = time.perf_counter() - t0
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    out = {"config": cfg["name"], "reads": args.reads, "n_kmers_gpu": int(index.n_kmers),
           "n_kmers_oracle": int(oix.n_kmers),
           "stats_equal": stats.tolist() == o.stats.tolist(), "unique_equal": uq.tolist() == o.unique.tolist(),
           "ambiguous_equal": am.tolist() == o.ambiguous.tolist(), "first_keys_equal": fk.tolist() == ofk.tolist(),
           "stats": [int(x) for x in stats], "oracle_build_s": build_s, "oracle_align_s": cpu_s,
           "oracle_threads": threads}
    out["bit_exact"] = all(out[k] for k in ("stats_equal", "unique_equal", "ambiguous_equal", "first_keys_equal")) \
        and out["n_kmers_gpu"] == out["n_kmers_oracle"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
