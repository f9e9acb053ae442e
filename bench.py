#!/usr/bin/env python3
"""Throughput benchmark of the MI355X pseudo-alignment engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c2|c3|c3raw|c2mix|c2rc|c5|c1]
    torchrun --nproc-per-node N bench.py --gpus N ...            (one rank per GPU)

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset), this
process starts the N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE and
a 127.0.0.1 rendezvous in their environment) before anything touches the GPU,
relays rank 0's line and exits non-zero if any rank fails.  A rank whose
WORLD_SIZE differs from an explicit --gpus exits non-zero.

Metric (BASELINE.json): reads/s pseudo-aligned, k=31, 150 bp reads, at
1/2/4/8 GPUs, plus the achieved fraction of the HBM roofline.  The DEFAULT
workload is the metric's own configuration, C4 (BASELINE.json configs[3], the
north star's "500-genome reference on 8 x MI355X"): 500 synthetic 2 Mbp genomes
in families of 5 (1% substitutions within a family, a 5 kb segment shared by
all, N runs), k=31, and per GPU 62.5M x 150 bp forward-strand reads with 0.5%
substitution errors and raw-ASCII qualities -- 500M reads over 8 GPUs --
synthesized ON the device (resident in HBM before the timed region; nothing
crosses PCIe while timing).  The other configs (--config) are the parity-test
and robustness cases of SURVEY.md section 8d.

A step = one pass of the align kernels over the rank's reads (counters reset,
pa_align, and for N > 1 the RCCL SUM/MIN all-reduce of the counter blocks).
Scaling is weak: rank r aligns global reads [r*R, (r+1)*R) with R = the
config's reads per GPU (rank_reads(); C4 at N = 8 tiles the 500M reads
exactly), and value = all ranks' reads / max-over-ranks time.  With the nccl
backend every rank checks that an RCCL communicator of the job spans all
ranks (ncclCommCount) and exits non-zero otherwise.

At N = 1 the line also carries the end-to-end `dumpalign` CLI figure on the C2
files (scripts/e2e_cli.py, sub-record end_to_end) unless --no-e2e.

roofline (the align pass: k_align_lane + k_align_fast over the reads the lane
kernel leaves; duration from HIP events libpa records on
the stream it launches them on):
  achieved / frac -- ALGORITHMIC bytes: B = L + q*L +
      (L-k+1)*16 per read (ASCII bases, qualities when a quality filter is on,
      one 8-B key + 8-B value slot per window) x reads per pass / duration.
      The lane walk skips most of those table reads, so this can exceed the
      bytes really moved (and even 1.0): it prices the work, not the traffic.
  traffic / measured_frac -- the bytes really moved from HBM / Infinity Cache:
      both kernels' fabric read requests by size (TCC_EA0_RDREQ_32B/64B/128B
      x 32/64/128 B), collected IN THIS RUN by a child process (rank 0, N = 1:
      rocprofv3 --kernel-trace --pmc ... -- python bench.py --traffic-child)
      on the same workload, / duration / peak.  On gfx950 every L2 miss is a
      128-B request, also for the random 8-16 B loads of this kernel, and
      FETCH_SIZE counts it at 64 B (profiles/fetch_calib.hip/.json), so the
      request counters, not FETCH_SIZE, give the bytes.  lines_per_read =
      128-B requests per read; random_line_frac = traffic / duration / the
      measured random-128-B-line ceiling (6.8 TB/s, profiles/fetch_calib.json).

cpu_baseline (rank 0, N=1): the C restatement oracle/pa_oracle.c timed on a
bounded prefix of the same device-generated reads, on one thread and on all the
host threads this job may use (read shards); "value" and
"cores" are the multi-thread figure.  The same prefix is aligned on the GPU and
compared bit-for-bit.
"""

from __future__ import annotations

import argparse
import json
import subprocess
import os
import re
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")
sys.path.insert(0, PKG)

import pa_dist  # noqa: E402
import pa_native as N  # noqa: E402
import synth  # noqa: E402

METRIC = "reads/sec pseudo-aligned (k=31, 150bp) at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

BASE = dict(n_genomes=50, genome_len=2_000_000, family=5, sub=0.01, conserved=5000, n_rate=1e-4, n_run=10, k=31,
            reads_per_gpu=10_000_000, read_len=150, read_err=0.005, params={})
CONFIGS = {
    "c2": dict(BASE, name="C2: 50 x 2 Mbp synthetic genomes, 10M x 150 bp reads per GPU, k=31"),
    "c3": dict(BASE, name="C3: C2 + --min-read-quality 20 --min-kmer-quality 25 --max-genomes 10",
               params=dict(mrq=20, mkq=25, mg=10)),
    "c3raw": dict(BASE, name="C3 raw-ASCII variant: C2 + --min-read-quality 53 --min-kmer-quality 58 "
                             "--max-genomes 10", params=dict(mrq=53, mkq=58, mg=10)),
    # C4 (BASELINE configs[3]): 500 genomes, 500M reads over 8 GPUs = 62.5M reads per GPU (weak scaling)
    "c4": dict(BASE, n_genomes=500, reads_per_gpu=62_500_000,
               name="C4: 500 x 2 Mbp synthetic genomes, 62.5M x 150 bp reads per GPU (500M on 8), k=31"),
    # C5 (BASELINE configs[4]): EXTSIM over 2000 x 4 Mbp genomes in families, then 100M reads
    # every second family is one of near-duplicates (0.03 % apart: ~0.98 of
    # their k-mers shared), so EXTSIM drops 4 of their 5 members
    "c5": dict(BASE, n_genomes=2000, genome_len=4_000_000, reads_per_gpu=100_000_000, generator="fast",
               near_dup_every=2, extsim=0.95,
               name="C5: EXTSIM (threshold 0.95) over 2000 x 4 Mbp synthetic genomes (families of 5, every second "
                    "one near-duplicates), then 100M x 150 bp reads against the kept genomes, k=31"),
    # robustness: 20 % reverse-complemented reads (forward-only
    # lookups: mostly unmapped), 20 % reads of an organism absent from the index,
    # 1.5 % substitutions -- the reads the lane walk cannot settle cheaply
    "c2mix": dict(BASE, read_err=0.015, rc_rate=0.2, foreign_rate=0.2,
                  name="C2 robustness: C2 genomes, 10M reads per GPU: 20% reverse-complement, 20% unindexed "
                       "organism, 1.5% substitutions"),
    # real FASTQ holds about half its reads on the reverse strand, which the
    # forward-only reference (src/kmer.py:423) leaves mostly unmapped: every
    # window of such a read must be shown absent
    "c2rc": dict(BASE, rc_rate=0.5,
                 name="C2 strand mix: C2 genomes, 10M reads per GPU: 50% reverse-complement, 0.5% substitutions"),
    # the other half of c2mix's no-seed reads: half the reads of an organism
    # absent from the index (every window Bloom-tested, k_align_lane_na)
    "c2fg": dict(BASE, foreign_rate=0.5,
                 name="C2 foreign mix: C2 genomes, 10M reads per GPU: 50% unindexed organism, 0.5% substitutions"),
    # the lane path's limits: the reference's demo runs use k = 75
    # and 150 (src/RUN_LOG:30, 67); longer keys and reads than the lane kernels
    # take (k <= 31, <= 176 bp) go to the wave kernel
    "c2k63": dict(BASE, k=63, name="C2 genomes, 10M x 150 bp reads per GPU, k=63 (2-word keys)"),
    "c2k75": dict(BASE, k=75, name="C2 genomes, 10M x 150 bp reads per GPU, k=75 (3-word keys; src/RUN_LOG:30)"),
    "c2l250": dict(BASE, read_len=250, name="C2 genomes, 10M x 250 bp reads per GPU, k=31"),
    "c1": dict(BASE, n_genomes=3, genome_len=5000, family=3, sub=0.02, conserved=300, k=21, reads_per_gpu=1000,
               read_len=100, read_err=0.01, name="C1: 3 x 5 kb genomes, 1k x 100 bp reads, k=21"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def e2e_pass():
    """scripts/e2e_cli.py in a child process: the dumpalign CLI on the C2 files."""
    cmd = [sys.executable, os.path.join(REPO, "scripts", "e2e_cli.py"), "--dir", "/tmp/pa_e2e_bench"]
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
        d = json.loads(line)
    except Exception as e:  # (reported, never fatal to the bench line)
        return {"error": f"{type(e).__name__}: {e}"}
    keep = ("workload", "cli_wall_s", "cli_wall_runs_s", "cli_reads_per_s", "cli_stdout_equals_api",
            "device_parse_path_taken", "host_path_summary_equal", "phases", "dumpref_c2_to_devnull", "fq_gz",
            "fq_plain_gz", "cli_stages", "sharded")
    out = {k: d.get(k) for k in keep}
    out["basis"] = ("median wall time of 3 runs of the whole `main.py -t dumpalign -g c2.fa -k 31 --reads c2.fq` "
                    "command (an idle device between runs), files in the page cache; reads/s = 10 M / that")
    return out


def bytes_per_read(cfg) -> int:
    """SURVEY.md 8(d)'s figure: L + q*L + 16 per window (one 8-B key + 8-B value
    slot read per window).  The lane walk settles most windows without a slot
    read, so this is not a floor of the design (it can pass the peak): kept as
    `survey_8d` for reference only."""
    L, k = cfg["read_len"], cfg["k"]
    q = 1 if (cfg["params"].get("mrq") is not None or cfg["params"].get("mkq") is not None) else 0
    return L + q * L + (L - k + 1) * 16


def design_bytes_per_read(cfg, quality_applied: bool) -> dict:
    """The design's algorithmic bytes per read: what the
    lane kernel must read for a read that is one stretch of one genome, each
    item priced at its own size (no line granularity) --
      read:   L ASCII bases (+ L quality bytes when a quality filter is applied
              after the elision of thresholds no read can fail);
      walk:   the walk blocks over the read's span, 32 B per 64 genome
              positions (2-bit bases + flag planes), (L - 1) / 64 + 1 blocks on
              average over the read's offset in its first block;
      seeds:  the first and last seed windows' slots (16 B each);
      mismatches: one 8-B neighbour word per mismatching base (substitution
              rate x L).
    A floor of the bytes moved, not a count of lines: the measured traffic (128-B
    lines) is several times this, the ratio being the random-access overhead."""
    L = int(cfg["read_len"])
    parts = {"read": L + (L if quality_applied else 0),
             "walk": 32.0 * ((L - 1) / 64.0 + 1.0),
             "seeds": 2 * 16,
             "mismatches": 8.0 * float(cfg["read_err"]) * L}
    return {"bytes_per_read": sum(parts.values()), "parts": parts}


def measured_bytes_per_read(config: str, kernel: str):
    """(fabric bytes per read of `kernel` measured by an N = 1 counter pass of
    `config`, source) from profiles/lines_per_read.json, or (None, reason)."""
    path = os.path.join(REPO, "profiles", "lines_per_read.json")
    try:
        with open(path) as f:
            d = json.load(f)[config]
        return float(d["kernels"][kernel]["bytes_per_read"]), f"N = 1 counter pass, {d['source']}"
    except (OSError, KeyError, ValueError):
        return None, f"no N = 1 measurement of {config}/{kernel} in profiles/lines_per_read.json"


def multi_rank_roofline(config: str, kernel: str, npg: int, slowest_ms: float, design_bpr: float) -> dict:
    """The roofline of an N > 1 line, where no counter pass runs: each rank's
    launch of the dominant kernel priced with the fabric bytes per read an
    N = 1 counter pass of the same config measured (profiles/lines_per_read.json),
    else with the design's algorithmic bytes per read, over the slowest rank's
    average launch."""
    bpr, src = measured_bytes_per_read(config, kernel)
    if bpr is None:
        bpr, src = design_bpr, "the design's algorithmic bytes per read (DESIGN.md section 4)"
    achieved = bpr * npg / (slowest_ms / 1e3) / 1e9
    return {"traffic": bpr * npg, "achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
            "achieved_basis": (f"N > 1 LINES MODEL: {bpr:.1f} fabric bytes per read ({src}) x {npg} reads per rank "
                               f"and launch / the slowest rank's average {kernel} launch (HIP events on each rank's "
                               "stream) / 8 TB/s; no counter pass runs at N > 1")}


def random_line_roofline():
    """(GB/s, source): the measured ceiling of isolated random 128-B line reads."""
    path = os.path.join(REPO, "profiles", "fetch_calib.json")
    if os.path.exists(path):
        with open(path) as f:
            c = json.load(f)
        return float(c["random_line_roofline_GBs"]), "profiles/fetch_calib.json: " + c["random_line_roofline_basis"]
    return None, "profiles/fetch_calib.json absent"


REQ_COUNTERS = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}
# the SQ counters of the same pass (8 SQ counters and 4 TCC fit one rocprofv3
# pass; these count quad-cycles, so only their ratios are used)
SQ_COUNTERS = ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")
ALIGN_KERNELS = ("k_quality_masks", "k_align_lane", "k_align_lane_na", "k_align_lane_rc", "k_rc_seeds",
                 "k_align_fast", "k_align_exact")


def kernel_short_name(mangled: str):
    """The kernel's own identifier from its mangled name (the length prefix
    keeps k_align_lane apart from k_align_lane_na), or None."""
    import re
    # (the digits may run into a preceding name: "_GLOBAL__N_1" + "12k_align_lane")
    for m in re.finditer(r"(\d+)(k_[A-Za-z0-9_]+)", mangled):
        digits, rest = m.group(1), m.group(2)
        for i in range(len(digits)):
            n = int(digits[i:])
            if n <= len(rest) and rest[:n] in ALIGN_KERNELS:
                return rest[:n]
    return None


_PROFILER_LINE = re.compile(r"^([IWEF]\d{8} |\[rocprofv3\]|rocprofv3|\s*$|.*rocprofiler)")


def child_error_lines(stderr: str, n: int = 12) -> str:
    """The counter child's own last stderr lines: the profiler's log lines
    (glog 'I20260101 ...', '[rocprofv3] ...', timers) dropped, so that the
    child's traceback or error message is what is left, whatever the profiler
    printed after it."""
    own = [ln for ln in stderr.splitlines() if not _PROFILER_LINE.match(ln)]
    return " | ".join(own[-n:]) if own else "(no output of its own)"


def counter_pass(args, cfg, kept_path, save_dir=None):
    """Fabric read bytes and SQ cycle shares of the align kernels, measured now:
    a child process repeats this workload under rocprofv3 --kernel-trace --pmc
    (TCC_EA0_RDREQ_{32B,64B,128B} + 5 SQ counters, one pass; 2 passes of the
    align after a warmup).  Returns ({kernel: {...}}, basis) or (None, reason).
    With save_dir, the per-kernel summary is also written there."""
    import glob
    import shutil
    import sqlite3
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="pa_traffic_", dir="/tmp")
    cmd = [prof, "--kernel-trace", "--pmc", *REQ_COUNTERS, *SQ_COUNTERS, "-d", tmp, "-o", "run", "--",
           sys.executable, os.path.abspath(__file__), "--traffic-child", "--config", args.config,
           "--reads-per-gpu", str(cfg["reads_per_gpu"]), "--steps", "2", "--warmup", "1"]
    if args.genome_len:
        cmd += ["--genome-len", str(args.genome_len)]
    if args.read_len:
        cmd += ["--read-len", str(args.read_len)]
    if args.params is not None:
        cmd += ["--params", args.params]
    if kept_path:
        cmd += ["--kept-file", kept_path]
    env = dict(os.environ, TMPDIR="/tmp")
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(v, None)
    # the child's whole stderr is kept in a file (under save_dir when given), so
    # a failure can be read afterwards whatever the profiler printed after it
    err_path = os.path.join(save_dir or tmp, f"counter_child_{args.config}.err")
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
    try:
        with open(err_path, "w") as ef:
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=ef, text=True, timeout=900)
        with open(err_path, errors="replace") as ef:
            stderr = ef.read()
    except subprocess.TimeoutExpired:
        return None, f"rocprofv3 child timed out (stderr: {err_path})"
    if r.returncode != 0:
        return None, (f"rocprofv3 child failed (rc {r.returncode}); its own last lines: "
                      f"{child_error_lines(stderr)} (whole stderr: {err_path})")
    dbs = glob.glob(os.path.join(tmp, "**", "*.db"), recursive=True)
    if not dbs:
        return None, "no rocprofv3 database written"
    raw = {}
    try:
        c = sqlite3.connect(dbs[0])
        for name, cname, v, n in c.execute(
                "select s.kernel_name, i.name, avg(e.value), count(e.value) from rocpd_pmc_event e "
                "join rocpd_info_pmc i on e.pmc_id = i.id join rocpd_event ev on e.event_id = ev.id "
                "join rocpd_kernel_dispatch d on d.event_id = ev.id "
                "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name, i.name"):
            short = kernel_short_name(name)
            if short is not None:
                raw.setdefault(short, {})[cname] = (float(v), int(n))
        durs = {}
        for name, avg_ns, n in c.execute(
                "select s.kernel_name, avg(d.end - d.start), count(*) from rocpd_kernel_dispatch d "
                "join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name"):
            short = kernel_short_name(name)
            if short is not None:
                durs[short] = (float(avg_ns) / 1e6, int(n))
    except sqlite3.Error as e:
        return None, f"rocprofv3 database unreadable: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    per = {}
    for k, cs in raw.items():
        b = sum(cs[c][0] * w for c, w in REQ_COUNTERS.items() if c in cs)
        wave = cs.get("SQ_WAVE_CYCLES", (0.0, 0))[0]
        d = {"bytes_per_launch": b, "launches": max(x[1] for x in cs.values()),
             "trace_avg_ms": durs.get(k, (None, 0))[0]}
        if wave > 0:
            d["sq_share_of_wave_cycles"] = {c[3:].lower(): cs[c][0] / wave for c in SQ_COUNTERS[1:] if c in cs}
        per[k] = d
    if not per:
        return None, "no align-kernel counter samples"
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        with open(os.path.join(save_dir, f"counters_{args.config}.json"), "w") as f:
            json.dump({"command": " ".join(cmd[cmd.index("--") + 1:]), "counters": list(REQ_COUNTERS) +
                       list(SQ_COUNTERS), "per_kernel_avg_per_dispatch": raw, "trace_avg_ms": durs}, f, indent=1)
    return per, ("rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum + SQ_{WAVE,BUSY}_CYCLES, "
                 "SQ_WAIT_ANY, SQ_ACTIVE_INST_{ANY,VALU} of this workload in one pass (child process, 2 passes "
                 "after a warmup, average per dispatch): bytes = 32/64/128 x requests (on gfx950 every L2 miss "
                 "is a request of its size; FETCH_SIZE would count 128-B requests at 64 B, profiles/fetch_calib)")


def bound_of(frac_hbm, sq) -> str:
    """What limits the kernel, from its measured HBM fraction and SQ shares."""
    if frac_hbm is not None and frac_hbm >= 0.7:
        return "hbm"
    if not sq:
        return "unknown (no SQ counters)"
    wait, valu = sq.get("wait_any", 0.0), sq.get("active_inst_valu", 0.0)
    if wait >= 0.4:
        return "latency+valu" if valu >= 0.15 else "latency"
    return "valu" if valu >= 0.3 else "issue"


def host_threads() -> int:
    """Host cores this job may use: the box's CPU share (OMP_NUM_THREADS is set
    to it there), else the affinity mask; at most 16."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(n, 16))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, genomes, index, reads, prm_kw, target_s: float, restricted: bool = False):
    """Time the oracle on a prefix of the reads (1 thread, then all host
    threads over read shards); check GPU == oracle on the multi-thread sample.
    restricted (C5, whose full CPU index would need ~0.7 TB): the oracle index
    holds the sample's k-mers only, each with its full genome list
    (ora_index_build_restricted), built after the sample is chosen."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pa_oracle as O
    kw = dict(m=prm_kw.get("m", 1), p=prm_kw.get("p", 1), mrq=prm_kw.get("mrq"), mkq=prm_kw.get("mkq"),
              mg=prm_kw.get("mg"))
    threads = host_threads()
    bases = sum(len(g) for g in genomes)
    if restricted:
        n = int(min(reads.n, 2_000_000))
        s, q, off = reads.download(0, n)
        t0 = time.perf_counter()
        oix = O.OracleIndex.restricted(genomes, cfg["k"], (s, off), threads=threads)
        build_s, build_threads = time.perf_counter() - t0, threads
        n1 = min(n, 100000)
        s1, q1, off1 = s[:int(off[n1])], q[:int(off[n1])], off[:n1 + 1]
    else:
        t0 = time.perf_counter()
        # one build thread: its pages sit on one NUMA node, as in round 1 (a build
        # spread over the host's threads spreads them and slows the timed align)
        build_threads = 1 if bases < 3e8 else threads
        oix = O.OracleIndex(genomes, cfg["k"], threads=build_threads)
        build_s = time.perf_counter() - t0
        n1 = min(reads.n, 100000)
        s1, q1, off1 = reads.download(0, n1)
    t0 = time.perf_counter()
    oix.align(s1.tobytes(), q1.tobytes(), off1, detail=False, **kw)
    dt1 = time.perf_counter() - t0
    rate1 = n1 / max(dt1, 1e-9)
    if not restricted:
        n = int(min(reads.n, max(n1, rate1 * threads * target_s), 16_000_000))
        s, q, off = reads.download(0, n)
    t0 = time.perf_counter()
    o = O.align_counts_parallel(oix, s, q, off, threads, **kw)
    dt = time.perf_counter() - t0
    # GPU on the same sample
    sample = N.Reads.upload(s, q, off, device=index.device)
    res = N.Result(index)
    N.align(index, sample, N.Params.make(kw["m"], kw["p"], kw["mrq"], kw["mkq"], kw["mg"]), 0, res)
    stats, uq, am, fk = res.fetch()
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    exact = (stats.tolist() == o.stats.tolist() and uq.tolist() == o.unique.tolist()
             and am.tolist() == o.ambiguous.tolist() and fk.tolist() == ofk.tolist())
    what = ("a RESTRICTED oracle index (the sample's k-mers with their full genome lists, streamed from the whole "
            "reference: smaller than the full index, so this CPU rate is flattering)" if restricted else
            "the full oracle index")
    return ({"value": n / dt, "unit": "reads/s", "cores": threads, "kind": "port",
             "single_thread": rate1, "cpu_model": cpu_model(),
             "index_build": {"Mbp_per_s": bases / build_s / 1e6, "s": build_s, "threads": build_threads,
                             "bases": bases, "restricted": restricted},
             "sample": f"first {n} of the benchmark's device-generated reads, oracle/pa_oracle.c on {threads} host "
                       f"threads over read shards ({dt:.1f} s) against {what}; 1 thread: {rate1:.0f} reads/s on "
                       f"the first {n1} reads; oracle index build {build_s:.1f} s ({bases / build_s / 1e6:.1f} "
                       f"Mbp/s on {build_threads} threads) not included"},
            {"reads": n, "bit_exact": bool(exact), "stats": [int(x) for x in stats],
             "oracle": "restricted" if restricted else "full"})


def rank_reads(cfg, rank: int, world: int):
    """(first global read index, reads) of `rank` in a `world`-rank job: weak
    scaling, R = cfg["reads_per_gpu"] reads per rank, contiguous, so the ranks
    of a job tile [0, world * R) exactly (C4 at N = 8: 500M reads)."""
    npg = int(cfg["reads_per_gpu"])
    return rank * npg, npg


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, share_device: bool) -> int:
    """--gpus N > 1 without torchrun: one child process per rank (this parent
    never initialises the GPU), rank i on device i (share_device: all on device
    0, the 1-GPU rehearsal).  Relays rank 0's stdout; a failed rank stops the
    others.  Returns the exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0" if share_device else str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PA_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode().splitlines()), daemon=True)
    reader.start()
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            log(f"[launcher] a rank exited with {rc}: stopping the others")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    reader.join(timeout=30)
    rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    for line in out0:
        print(line, flush=True)
    if rc == 0 and not any(x.startswith("{") for x in out0):
        log("[launcher] rank 0 printed no result line")
        rc = 1
    return rc


def job_plan(config: str, world: int, reduce: str, cuda_available: bool) -> dict:
    """What a `world`-rank run of `config` does, before any device call: the
    reads of every rank (global index ranges, rank_reads), the reduction path
    and the torch.distributed backend pa_dist picks (RCCL on a GPU node).
    `python bench.py --gpus N --plan` prints it without touching the GPU."""
    import pa_dist
    cfg = CONFIGS[config]
    spans = [rank_reads(cfg, r, world) for r in range(world)]
    return {"config": config, "workload": cfg["name"], "world": world,
            "rank_reads": [{"rank": r, "first": f, "n": n} for r, (f, n) in enumerate(spans)],
            "job_reads_per_step": sum(n for _, n in spans),
            "reduce": reduce if world > 1 else None,
            "backend": pa_dist.default_backend(cuda_available) if world > 1 else None}


def counters_digest(result) -> dict:
    """The job's counters after the last step (every rank holds them once
    reduced): statistics plus a SHA-256 of the sum and min blocks, so a test can
    compare an N-rank run with one process aligning the same global reads."""
    import hashlib
    stats, uq, am, fk = result.fetch()
    h = hashlib.sha256()
    for a in (stats, uq, am, fk):
        h.update(np.ascontiguousarray(a, dtype=np.uint64).tobytes())
    return {"stats": [int(x) for x in stats], "sha256": h.hexdigest()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (GPUs); default WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS),
                    help="workload (default c4: the metric's configuration, BASELINE.json configs[3])")
    ap.add_argument("--reads-per-gpu", type=int, default=None)
    ap.add_argument("--genome-len", type=int, default=None, help="override the genome length (experiments)")
    ap.add_argument("--read-len", type=int, default=None, help="override the read length (experiments)")
    ap.add_argument("--job-table", choices=("auto", "full"), default="auto",
                    help="the job index's k-mer table: compact below the break-even (auto, as the CLI) or the "
                         "serving index's (full: the line's neighbour-bit break-even is then measurable)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-traffic", action="store_true", help="skip the in-run counter pass (traffic, SQ shares)")
    ap.add_argument("--profile-dir", default=None, help="also write the counter pass's per-kernel summary here")
    ap.add_argument("--traffic-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--kept-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--reduce", choices=("torch", "capi"), default="torch",
                    help="N > 1: all-reduce through torch.distributed (RCCL) or libpa's pa_counters_reduce")
    ap.add_argument("--no-e2e", action="store_true",
                    help="N=1: skip the end-to-end dumpalign CLI figure on the C2 files (scripts/e2e_cli.py)")
    ap.add_argument("--ranks-share-device", action="store_true", help=argparse.SUPPRESS)  # 1-GPU rehearsal
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default=None, help=argparse.SUPPRESS)
    ap.add_argument("--fail-rank", type=int, default=None, help=argparse.SUPPRESS)  # launcher test: this rank dies
    ap.add_argument("--params", default=None,
                    help='override the filter arguments, JSON, e.g. \'{"mg": 10}\' (experiments; named in config)')
    ap.add_argument("--plan", action="store_true",
                    help="print the job plan (every rank's reads, reduction, backend) and exit; no device call")
    args = ap.parse_args()
    if args.plan:
        import torch
        # (device_count does not initialise the GPU on this image)
        print(json.dumps(job_plan(args.config, args.gpus or int(os.environ.get("WORLD_SIZE", "1")), args.reduce,
                                  torch.cuda.device_count() > 0)), flush=True)
        return
    if (args.gpus or 1) > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, args.ranks_share_device))
    cfg = dict(CONFIGS[args.config])
    if args.params is not None:
        cfg["params"] = json.loads(args.params)
        cfg["name"] += f" [filters overridden: {args.params}]"
    if args.reads_per_gpu:
        cfg["reads_per_gpu"] = args.reads_per_gpu
    if args.genome_len:
        cfg["genome_len"] = args.genome_len
        cfg["name"] += f" [genome_len overridden: {args.genome_len}]"
    if args.read_len:
        cfg["read_len"] = args.read_len
        cfg["name"] += f" [read_len overridden: {args.read_len}]"

    import torch
    rank, world, local = pa_dist.init_process_group(args.dist_backend)
    if args.fail_rank == rank:
        log(f"[rank {rank}] --fail-rank: exiting")
        sys.exit(3)
    if args.gpus is not None and world != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = torch.distributed.get_backend() if world > 1 else None

    t0 = time.perf_counter()
    gkw = dict(seed=1, family_size=cfg["family"], sub_rate=cfg["sub"], conserved_len=cfg["conserved"],
               n_rate=cfg["n_rate"], n_run=cfg["n_run"])
    if cfg.get("generator") == "fast":
        genomes = synth.family_genomes_fast(cfg["n_genomes"], cfg["genome_len"],
                                            near_dup_every=cfg.get("near_dup_every", 0), **gkw)
    else:
        genomes = synth.family_genomes(cfg["n_genomes"], cfg["genome_len"], **gkw)
    gen_s = time.perf_counter() - t0
    log(f"[rank {rank}] genomes: {len(genomes)} x {cfg['genome_len']} in {gen_s:.1f}s")
    stream = torch.cuda.current_stream(dev)
    # EXTSIM configs: the first index (all genomes) feeds the statistics only,
    # so its align-side view is deferred (PA_BUILD_DEFER_TILES) and never made
    # unless no genome is dropped
    filtering = cfg.get("extsim") is not None or args.kept_file
    # the library's own HIP runtime (context, code objects) is started before the
    # timed build, as the CLI starts it at entry beside the imports: a one-genome
    # index, closed at once (its device memory stays in the library's pool)
    N.Index([np.frombuffer(b"ACGT" * 64, dtype=np.uint8)], cfg["k"], device=local, stream=stream).close()
    torch.cuda.synchronize(dev)
    first_read, npg = rank_reads(cfg, rank, world)
    all_genomes = genomes
    kept_path = None
    kept_from_file = None
    if args.kept_file:  # traffic child: the parent's EXTSIM outcome
        with open(args.kept_file) as f:
            kept_from_file = json.load(f)

    def build_index(expected_reads):
        """genomes in host memory -> an align-ready index: build (the view
        deferred), EXTSIM + the rebuild of the kept genomes (C5), then the
        align-side view -- for a job of `expected_reads` reads
        (pa_index_prepare_ex: the neighbour bits only past their break-even),
        or, with None, the full view (the serving index, pa_index_prepare).
        Returns (index, kept genomes, timings)."""
        nonlocal kept_path
        t_all = t0 = time.perf_counter()
        # the job's table compact (PA_BUILD_COMPACT: 2 slots per genome window)
        # below the break-even PA_COMPACT_READS_PER_BASE, as the CLI's jobs
        bases = sum(len(g) for g in all_genomes)
        compact = (expected_reads is not None and args.job_table == "auto" and
                   expected_reads < N.PA_COMPACT_READS_PER_BASE * bases)
        ix = N.Index(all_genomes, cfg["k"], device=local, stream=stream, defer_tiles=True, compact=compact)
        torch.cuda.synchronize(dev)
        ii = ix.info()  # (the library takes the flag for one-word keys on window-sized tables only)
        tm = {"first_build_s": time.perf_counter() - t0, "bases_built": bases, "extsim": None,
              "compact_table": bool(compact and int(ii.table_slots) == (2 * int(ii.total_windows) + 64 + 3) // 4 * 4)}
        kept = all_genomes
        if kept_from_file is not None:
            kept = [all_genomes[i] for i in kept_from_file]
            ix.reduce(kept_from_file, stream)
            torch.cuda.synchronize(dev)
        elif cfg.get("extsim") is not None:
            # EXTSIM (src/kmer.py:152-263): GPU statistics + the greedy pass; a
            # genome dropped -> the index of the kept genomes
            import kmer
            t0 = time.perf_counter()
            idents = [f"genome_{i}" for i in range(len(all_genomes))]
            keep, sim_info = kmer.extsim_filter(ix, idents, [len(g) for g in all_genomes], cfg["extsim"])
            stats_s = time.perf_counter() - t0
            kept_idx = [j for j, i in enumerate(idents) if i in keep]
            t1 = time.perf_counter()
            if len(keep) != len(idents):  # the kept genomes' index, from their codes on the device
                kept = [all_genomes[j] for j in kept_idx]
                ix.reduce(kept_idx, stream)
                torch.cuda.synchronize(dev)
                tm["bases_built"] += sum(len(g) for g in kept)
            rebuild_s = time.perf_counter() - t1
            if kept_path is None:
                import tempfile
                fd, kept_path = tempfile.mkstemp(prefix="pa_kept_", suffix=".json", dir="/tmp")
                with os.fdopen(fd, "w") as f:
                    json.dump(kept_idx, f)
            scores = [v["similarity_score"] for v in sim_info.values() if v["kept"] == "no"]
            tm["extsim"] = {"threshold": cfg["extsim"], "genomes_in": len(idents), "genomes_kept": len(keep),
                            "stats_and_greedy_s": stats_s, "rebuild_kept_s": rebuild_s,
                            "total_s": time.perf_counter() - t0, "min_dropped_score": min(scores) if scores else None,
                            "max_kept_pair_score_below": cfg["extsim"]}
            log(f"[rank {rank}] EXTSIM: kept {len(keep)} of {len(idents)} in {tm['extsim']['total_s']:.1f}s")
        t0 = time.perf_counter()
        ix.prepare(stream, expected_reads=expected_reads)
        torch.cuda.synchronize(dev)
        tm["prepare_s"] = time.perf_counter() - t0
        tm["build_s"] = time.perf_counter() - t_all
        return ix, kept, tm

    def make_reads(ix):
        t0 = time.perf_counter()
        r = N.Reads.synthesize(ix, npg, cfg["read_len"], first_read=first_read, seed=2, sub_rate=cfg["read_err"],
                               stream=stream, rc_rate=cfg.get("rc_rate", 0.0),
                               foreign_rate=cfg.get("foreign_rate", 0.0))
        torch.cuda.synchronize(dev)
        return r, time.perf_counter() - t0

    pk = cfg["params"]
    prm = N.Params.make(pk.get("m", 1), pk.get("p", 1), pk.get("mrq"), pk.get("mkq"), pk.get("mg"))
    comm = pa_dist.make_comm(local) if (world > 1 and args.reduce == "capi") else None
    # the ranks an RCCL communicator of this job really spans (ncclCommCount);
    # the torch path's communicator is torch's own, so one is made to ask
    rccl_ranks = None
    if world > 1 and backend == "nccl":
        probe = comm if comm is not None else pa_dist.make_comm(local)
        rccl_ranks = probe.n_ranks
        if probe is not comm:
            probe.close()
        if rccl_ranks != world:
            log(f"[rank {rank}] error: the RCCL communicator spans {rccl_ranks} ranks, WORLD_SIZE is {world}")
            sys.exit(4)
    cur = {}

    def step():
        index, reads, result = cur["index"], cur["reads"], cur["result"]
        result.reset(stream)
        N.align(index, reads, prm, first_read, result, stream)
        if world > 1:
            if comm is not None:
                pa_dist.reduce_result_capi(result, comm, stream)
            else:
                pa_dist.reduce_result(result, dev, stream)

    def timed_passes(n):
        """n passes between barriers + device syncs; (max-over-ranks seconds,
        {kernel: (ms, launches)} of HIP events around each launch)."""
        index = cur["index"]
        index.profile_read()  # (drop earlier events)
        index.profile_enable(True)
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        kern = index.profile_read_kernels()
        index.profile_enable(False)
        return max_over_ranks(el), kern

    def max_over_ranks(*vals):
        t = torch.tensor(list(vals), dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        if world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        out = [float(x) for x in t.tolist()]
        return out[0] if len(out) == 1 else out

    # 1) the job as the product runs it: the index built for this rank's npg
    #    reads (the neighbour bits only past their break-even), then one pass of
    #    them (timed over a few passes: fewer than would bring the reads aligned
    #    past the break-even, where the align would make the bits itself)
    product = None
    job_tm = None
    if not args.traffic_child:
        jix, _, job_tm = build_index(npg)
        job_bytes = int(jix.info().device_bytes)
        jreads, _ = make_reads(jix)
        cur.update(index=jix, reads=jreads, result=N.Result(jix))
        step()  # (warmup)
        torch.cuda.synchronize(dev)
        np_ = max(1, min(args.steps, 5))
        p_el, p_kern = timed_passes(np_)
        product = {"passes": np_, "pass_s": p_el / np_, "reads_per_s": world * npg * np_ / p_el,
                   "kernels_ms": {k: v[0] / v[1] for k, v in p_kern.items() if v[1]},
                   "device_bytes": job_bytes, "valid": int(jix.info().device_bytes) == job_bytes,
                   "compact_table": job_tm["compact_table"], "table_slots": int(jix.info().table_slots)}
        for h in ("result", "reads", "index"):
            cur.pop(h).close()
        torch.cuda.synchronize(dev)
    # 2) the serving index -- the full align-side view (neighbour bits), what a
    #    long-lived aligner keeps and what pa_index_build makes -- built anew
    #    from the same genomes: the measured passes below run on it
    index, genomes, srv_tm = build_index(None)
    build_s, prepare_s, index_total_s = srv_tm["first_build_s"], srv_tm["prepare_s"], srv_tm["build_s"]
    build_bases = srv_tm["bases_built"]
    extsim = srv_tm["extsim"] or (job_tm or {}).get("extsim")
    reads, reads_make_s = make_reads(index)
    result = N.Result(index)
    cur.update(index=index, reads=reads, result=result)
    info = index.info()
    nb_built = product is not None and int(info.device_bytes) > product["device_bytes"]
    nb_s = index_total_s - job_tm["build_s"] if job_tm else 0.0
    # the filters a pass really applies: thresholds at or below the batch's
    # smallest quality byte filter nothing (quirk 5) and are dropped
    eff, q_min = reads.effective(prm, stream)
    applied = {}
    if eff.flags & N.HAS_MRQ:
        applied["mrq"] = pk.get("mrq")
    if eff.flags & N.HAS_MKQ:
        applied["mkq"] = pk.get("mkq")
    if eff.flags & N.HAS_MG:
        applied["mg"] = pk.get("mg")
    elided = [n for n, f in (("mrq", N.HAS_MRQ), ("mkq", N.HAS_MKQ)) if (prm.flags & f) and not (eff.flags & f)]
    quality_applied = bool(eff.flags & (N.HAS_MRQ | N.HAS_MKQ))
    log(f"[rank {rank}] genomes {gen_s:.1f}s, serving index {index_total_s:.2f}s (first build {build_s:.2f}s, "
        f"align-side view {prepare_s:.2f}s), job index {job_tm['build_s'] if job_tm else float('nan'):.2f}s: "
        f"{info.n_kmers} k-mers, {info.n_multi_classes} multi-genome sets, table {info.table_bytes / 2**30:.2f} GiB; "
        f"{npg} reads")

    if args.traffic_child:  # under rocprofv3: warmup + the measured passes, nothing else
        for _ in range(args.warmup + args.steps):
            step()
        torch.cuda.synchronize(dev)
        return

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    index.profile_read()  # drop warmup events
    index.profile_enable(True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms, launches, deferred = index.profile_read()
    kern = index.profile_read_kernels()
    index.profile_enable(False)
    elapsed = max_over_ranks(elapsed)
    job_build_s = job_tm["build_s"] if job_tm else index_total_s
    build_max, srv_build_max, nb_max = max_over_ranks(job_build_s, index_total_s, nb_s)
    # every rank's align-kernel times (HIP events on its own stream), for the
    # rank-0 line: at N > 1 no counter pass runs, so the roofline of a scaling
    # run comes from these and the section 8(d) algorithmic bytes
    mine = {"rank": rank, "kernels_ms": {k: v[0] / v[1] for k, v in kern.items() if v[1]}}
    if world > 1:
        ranks_kern = [None] * world
        torch.distributed.all_gather_object(ranks_kern, mine)
    else:
        ranks_kern = [mine]
    job_counters = counters_digest(result)

    total_reads = world * npg * args.steps
    value = total_reads / elapsed
    pass_s = kern_ms / max(launches, 1) / 1e3
    b_read = bytes_per_read(cfg)
    design = design_bytes_per_read(cfg, quality_applied)
    # the dominant kernel: the largest share of the timed align passes
    dominant = max((k for k in kern if kern[k][1] > 0), key=lambda k: kern[k][0], default="k_align_lane")
    dom_s = kern[dominant][0] / max(kern[dominant][1], 1) / 1e3
    alg_achieved = design["bytes_per_read"] * npg / dom_s / 1e9 if dom_s > 0 else 0.0
    # the job as the product runs it (section 1 above): build + one pass, per GPU
    job = None
    if product is not None:
        job_s = build_max + product["pass_s"]
        job = {"reads_per_gpu": npg, "index_build_s": build_max, "align_pass_s": product["pass_s"],
               "job_s": job_s, "job_reads_per_s_per_gpu": npg / job_s, "job_reads_per_s": world * npg / job_s,
               "plan_8_gpus": {"reads": 8 * npg, "job_reads_per_s": 8 * npg / job_s,
                               "basis": "8 ranks each building the same replica and aligning its npg reads in the "
                                        "same time as this rank (weak scaling, one latency-bound all-reduce)"},
               "compact_table": product["compact_table"],
               "basis": ("the index built for this rank's reads (pa_index_prepare_ex with expected_reads = npg: "
                         "neighbour bits only past their break-even; the compact k-mer table, PA_BUILD_COMPACT, "
                         "below PA_COMPACT_READS_PER_BASE -- as the CLI builds them) from genomes in host memory, "
                         "plus one align pass of the npg device-resident reads on it; max over ranks")}
    serving_pass_s = elapsed / args.steps
    breakeven = None
    if product is not None and product["compact_table"]:
        breakeven = {"basis": "not measured in this line: the job index has the compact k-mer table "
                              "(PA_BUILD_COMPACT), so job vs serving index differ in more than the neighbour "
                              "bits; bench.py --job-table full measures it (round-6 figures: include/pa.h)"}
    elif product is not None and product["valid"] and nb_built:
        saved = (product["pass_s"] - serving_pass_s) / npg
        per_base = nb_max / max(int(info.total_windows), 1)
        breakeven = {"neighbour_bits_s": nb_max, "saved_ns_per_read": saved * 1e9,
                     "cost_ns_per_base": per_base * 1e9,
                     "reads_per_base": per_base / saved if saved > 0 else None,
                     "policy_reads_per_base": (N.PA_NB_READS_PER_KBASE if cfg["k"] <= 31 else
                                               N.PA_NB_READS_PER_KBASE_2W if cfg["k"] <= 63 else
                                               N.PA_NB_READS_PER_KBASE_3W) / 1000,
                     "basis": "neighbour bits' build time per genome window / align time they save per read "
                              "(job-index pass - serving-index pass, per read)"}
    out = {
        "metric": METRIC, "value": value, "unit": "reads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: seeded numpy genomes, reads sampled on the device (resident in HBM before timing)",
        "config": {"workload": cfg["name"], "genomes": cfg["n_genomes"], "genome_len": cfg["genome_len"],
                   "k": cfg["k"], "reads_per_gpu": npg, "job_reads_per_step": world * npg,
                   "read_len": cfg["read_len"],
                   "filters": cfg["params"] or None,
                   "filters_applied": applied or None,
                   "filters_note": (f"{'/'.join(elided)} elided (q_min = {q_min}: a threshold at or below the batch's "
                                    "smallest quality byte filters nothing, strict <, quirk 5; measured when the reads "
                                    "are made, outside the timed step)") if elided else None,
                   "index": ("serving: the full align-side view, neighbour bits included (built anew after the "
                             "job-index passes, pa_index_prepare)"),
                   "parallelism": f"read-sharded x{world}, index replicated",
                   "reduce": args.reduce if world > 1 else None, "backend": backend, "rccl_ranks": rccl_ranks,
                   "read_mix": {"reverse_complement": cfg.get("rc_rate", 0.0), "foreign": cfg.get("foreign_rate", 0.0),
                                "substitution_rate": cfg["read_err"]}},
        "roofline": {"bound": None, "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                     "traffic": None, "kernel": dominant, "kernel_ms": dom_s * 1e3,
                     "achieved_basis": ("MEASURED fabric read bytes of the dominant kernel per launch (traffic, "
                                        "counter pass) / its average duration (HIP events around each launch on "
                                        "its stream over the timed steps) / 8 TB/s"),
                     "algorithmic": {"model": "design bytes per read (DESIGN.md section 4)",
                                     "bytes_per_read": design["bytes_per_read"], "parts": design["parts"],
                                     "bytes_per_launch": design["bytes_per_read"] * npg,
                                     "kernel_ms": dom_s * 1e3, "achieved": alg_achieved,
                                     "frac": alg_achieved / HBM_PEAK_GBS,
                                     "basis": ("the lane design's bytes per read, each item at its own size: the read "
                                               "(+ qualities when a quality filter is applied), the walk blocks over "
                                               "its span (32 B per 64 positions), two seed slots (16 B), one 8-B "
                                               "neighbour word per mismatching base -- x reads per launch / the "
                                               "dominant kernel's average launch: a floor of the bytes moved"),
                                     "survey_8d": {"bytes_per_read": b_read, "pass_ms": pass_s * 1e3,
                                                   "achieved": b_read * npg / pass_s / 1e9 if pass_s > 0 else None,
                                                   "note": ("SURVEY.md 8d prices one 16-B slot read per window, "
                                                            "which the walk skips: not a bound of this design "
                                                            "(it can pass the peak); reference only")}},
                     "kernels": {k: {"ms_avg": v[0] / v[1], "launches": v[1]} for k, v in kern.items() if v[1]}},
        "job": job,
        "job_index": (dict(product, neighbour_bits=not nb_built) if product is not None else None),
        "neighbour_bits_breakeven": breakeven,
        "deferred_read_fraction": deferred / max(npg * args.steps, 1),
        "job_counters": job_counters,
        "index": {"build_s": job_build_s, "serving_build_s": index_total_s,
                  "serving_first_build_s": build_s, "serving_prepare_s": prepare_s,
                  "job_first_build_s": job_tm["first_build_s"] if job_tm else None,
                  "job_prepare_s": job_tm["prepare_s"] if job_tm else None,
                  "neighbour_bits_s": nb_s, "reads_make_s": reads_make_s,
                  "build_basis": ("FASTA genomes in host memory -> an align-ready index: table + genome sets"
                                  + (", EXTSIM statistics and greedy pass, rebuild of the kept genomes" if extsim else "")
                                  + ", tiles / Bloom filter; build_s: the job's index (neighbour bits only when the "
                                    "job repays them), serving_build_s: the serving index the timed passes run on "
                                    "(every bit; built anew), neighbour_bits_s: their difference"),
                  "n_kmers": int(info.n_kmers), "multi_genome_sets": int(info.n_multi_classes),
                  "table_bytes": int(info.table_bytes), "table_slots": int(info.table_slots)},
        "extsim": extsim,
        "cpu_baseline": None,
    }
    # index-build roofline (B_bp = 17 B per genome base -- one
    # base read + one 16-B slot touched -- over every build of the job)
    bases_built = int(build_bases)
    ib = out["index"]
    ib["bases_built"] = bases_built
    ib["Mbp_per_s"] = bases_built / job_build_s / 1e6 if job_build_s > 0 else None
    ib["roofline"] = {"bytes_per_base": 17, "achieved": 17 * bases_built / job_build_s / 1e9,
                      "frac": 17 * bases_built / job_build_s / 1e9 / HBM_PEAK_GBS, "unit": "GB/s",
                      "basis": "17 B per genome base of every build (first build + EXTSIM rebuild) / build_s "
                               "(the job's index)"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        torch.cuda.synchronize(dev)
        # C5: the oracle's full index of the kept ~5 Gbp would need ~0.7 TB of host memory
        base, parity = cpu_baseline(cfg, genomes, index, reads, pk, args.cpu_seconds,
                                    restricted=args.config == "c5")
        out["cpu_baseline"] = base
        out["parity_sample"] = parity
    # the counter pass last, after this process's device memory is released:
    # its child rebuilds the same index and reads (C5's would not fit twice)
    per = None
    line_peak, line_src = random_line_roofline()
    if rank == 0 and world == 1 and not args.no_traffic:
        result.close()
        reads.close()
        index.close()
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        # the library's slab pool keeps freed index buffers for the next build
        # (pa_mem.cpp): handed back here, or C5's child finds no room for its own
        N.mem_trim(local)
        per, tnote = counter_pass(args, cfg, kept_path, args.profile_dir)
    else:
        tnote = "not measured (--no-traffic, or a rank of a multi-GPU run)"
    rl = out["roofline"]
    rl["traffic_basis"] = tnote
    dom_rank_ms = [r["kernels_ms"].get(dominant) for r in ranks_kern]
    rl["per_rank"] = [{"rank": r["rank"], "dominant_kernel_ms": r["kernels_ms"].get(dominant),
                       "kernels_ms": r["kernels_ms"]} for r in ranks_kern]
    if world > 1 and all(dom_rank_ms):
        # no counter pass at N > 1: each rank's dominant-kernel launch priced
        # with the fabric bytes per read a counter pass of the same config
        # measured at N = 1 (profiles/lines_per_read.json), else with the
        # design's algorithmic bytes
        rl.update(multi_rank_roofline(args.config, dominant, npg, max(dom_rank_ms), design["bytes_per_read"]))
    rl["random_line_peak"], rl["random_line_peak_source"] = line_peak, line_src
    if per is not None:
        for k, d in per.items():
            kd = rl["kernels"].setdefault(k, {})
            kd.update(d)
            ms = kd.get("ms_avg")
            if ms:
                kd["measured_GBs"] = d["bytes_per_launch"] / (ms / 1e3) / 1e9
                kd["frac"] = kd["measured_GBs"] / HBM_PEAK_GBS
            kd["lines_per_read"] = d["bytes_per_launch"] / 128.0 / npg
        if dominant in per and dom_s > 0:
            d = per[dominant]
            rl["traffic"] = d["bytes_per_launch"]
            rl["achieved"] = d["bytes_per_launch"] / dom_s / 1e9
            rl["frac"] = rl["achieved"] / HBM_PEAK_GBS
            rl["sq"] = d.get("sq_share_of_wave_cycles")
            rl["random_line_frac"] = rl["achieved"] / line_peak if line_peak else None
            rl["pass_lines_per_read"] = sum(x["bytes_per_launch"] for x in per.values()) / 128.0 / npg
            log(f"[rank 0] {dominant}: {rl['traffic'] / 1e9:.2f} GB per launch in {dom_s * 1e3:.3f} ms "
                f"= {rl['achieved']:.0f} GB/s ({rl['frac']:.3f} of HBM peak)")
    # (at N > 1 frac is the algorithmic one, which prices skipped slot reads: no bound from it)
    rl["bound"] = bound_of(rl["frac"] if world == 1 else None, rl.get("sq"))
    out["libpa"] = N.lib().pa_version().decode()
    if kept_path:
        os.unlink(kept_path)
    if rank == 0 and world == 1 and not args.no_e2e and not args.traffic_child:
        # the user-visible figure beside the device-resident one: `main.py -t
        # dumpalign` on the C2 files (FASTA + 3.2 GB FASTQ, page cache warm)
        for h in (result, reads, index):
            h.close()
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        N.mem_trim(local)
        out["end_to_end"] = e2e_pass()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
