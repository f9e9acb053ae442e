#!/usr/bin/env python3
"""End-to-end dumpalign figure (host parse, index build
and the CLI measured separately from the device-resident bench).

    python scripts/e2e_cli.py [--reads N] [--dir DIR]

Writes the C2 genomes (FASTA, 80-column lines) and N x 150 bp reads (FASTQ)
to DIR, then
  1. times each phase of the drop-in API in one process: FASTAFile (native
     ingest), KmerReference (device index build + align-side view), the CLI's
     PseudoAlignment.align_reads_from_file (FASTQ parsed on the device and
     aligned in windows), and for comparison the host path (FASTAQFile native
     host parse + align_reads_from_container);
  2. runs `main.py -t dumpalign` as a subprocess and times the whole command,
     checking that its stdout equals the in-process summary.
Prints one JSON line.
"""

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")
sys.path.insert(0, PKG)

import synth  # noqa: E402


def write_fastq(path, genomes, n, chunk=1_000_000):
    """Fixed-width records '@r%09d' / 150 bases / '+' / 150 qualities."""
    L = 150
    rec = 12 + L + 1 + 2 + L + 1
    with open(path, "wb") as f:
        for b in range(0, n, chunk):
            m = min(chunk, n - b)
            seq, qual, _ = synth.sample_reads(genomes, m, L, seed=2 + b // chunk, err_rate=0.005)
            buf = np.empty((m, rec), dtype=np.uint8)
            ids = np.char.zfill(np.arange(b, b + m).astype(str), 9).astype("S9")
            buf[:, 0] = ord("@")
            buf[:, 1] = ord("r")
            buf[:, 2:11] = np.frombuffer(ids.tobytes(), dtype=np.uint8).reshape(m, 9)
            buf[:, 11] = 10
            buf[:, 12:12 + L] = seq
            buf[:, 12 + L] = 10
            buf[:, 13 + L] = ord("+")
            buf[:, 14 + L] = 10
            buf[:, 15 + L:15 + 2 * L] = qual
            buf[:, 15 + 2 * L] = 10
            buf.tofile(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--dir", default="/tmp/pa_e2e")
    ap.add_argument("--keep", action="store_true", help="leave the generated files in --dir (profiling runs)")
    ap.add_argument("--no-gz", action="store_true", help="skip the .fq.gz runs (BGZF and one plain member)")
    args = ap.parse_args()
    os.makedirs(args.dir, exist_ok=True)
    fa, fq = os.path.join(args.dir, "c2.fa"), os.path.join(args.dir, "c2.fq")
    t0 = time.perf_counter()
    genomes = synth.family_genomes(50, 2_000_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=5000,
                                   n_rate=1e-4, n_run=10)
    with open(fa, "w") as f:
        f.write(synth.fasta_text([f"genome_{i} synthetic C2" for i in range(50)], genomes, width=80))
    write_fastq(fq, genomes, args.reads)
    gen_s = time.perf_counter() - t0
    print(f"files written in {gen_s:.1f}s: {os.path.getsize(fq) / 1e9:.2f} GB FASTQ", file=sys.stderr, flush=True)

    from data_file import FASTAFile, FASTAQFile
    from kmer import KmerReference, PseudoAlignment
    ph = {}
    t = time.perf_counter()
    gc = FASTAFile(fa).container
    ph["parse_fasta_s"] = time.perf_counter() - t
    t = time.perf_counter()
    ref = KmerReference(31, gc)
    ref.index.prepare()  # the align-side view (otherwise made by the first align)
    import pa_native as N
    N.lib()
    ph["index_build_s"] = time.perf_counter() - t
    # the CLI's path: the FASTQ file parsed on the device, aligned in windows
    t = time.perf_counter()
    pa = PseudoAlignment(ref)
    pa.align_reads_from_file(fq)
    ph["fastq_device_parse_align_s"] = time.perf_counter() - t
    streamed = getattr(pa, "_streamed_records", None) == args.reads
    summary = json.dumps(pa.get_summary(), indent=4)
    del pa
    # the host path (round 1): native host parse into a container, then upload + align
    t = time.perf_counter()
    rc = FASTAQFile(fq).container
    ph["host_parse_fastq_s"] = time.perf_counter() - t
    t = time.perf_counter()
    pb = PseudoAlignment(ref)
    pb.align_reads_from_container(rc)
    ph["host_upload_align_s"] = time.perf_counter() - t
    host_equal = json.dumps(pb.get_summary(), indent=4) == summary
    del rc, pb

    cmd = [sys.executable, os.path.join(PKG, "main.py"), "-t", "dumpalign", "-g", fa, "-k", "31", "--reads", fq]
    walls = []
    for _ in range(3):  # the median of three runs of the whole command
        # (each on an idle device: a process's GPU memory is reclaimed by the
        # driver after it exits, which delays the next process's runtime start)
        time.sleep(3)
        t = time.perf_counter()
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        walls.append(time.perf_counter() - t)
    cli_s = sorted(walls)[1]
    # the same command again with stage times on stderr (not the timed run)
    time.sleep(3)
    t = time.perf_counter()
    rt = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                        env=dict(os.environ, PA_CLI_TIMING="1", PA_STREAM_TIMING="1"))
    stages = {"wall_s": time.perf_counter() - t, "stderr": rt.stderr.strip().splitlines()[-12:]}
    time.sleep(3)
    t = time.perf_counter()
    rs = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                        env=dict(os.environ, PA_CLI_TIMING="1", PA_FAST_EXIT="0"))
    stages["normal_exit"] = {"wall_s": time.perf_counter() - t, "stderr": rs.stderr.strip().splitlines()[-3:]}
    # the same command read-sharded over two devices (PA_GPUS=2, pa_shard.py;
    # on a one-GPU box both replicas on device 0: PA_GPUS_SHARE=1)
    shard_env = dict(os.environ, PA_GPUS="2", PA_CLI_TIMING="1")
    if N.device_count() < 2:
        shard_env["PA_GPUS_SHARE"] = "1"
    time.sleep(3)
    t = time.perf_counter()
    rsh = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=shard_env)
    sharded = {"gpus": 2, "shared_device": shard_env.get("PA_GPUS_SHARE") == "1",
               "wall_s": time.perf_counter() - t, "rc": rsh.returncode,
               "stdout_equals_api": rsh.stdout == summary + "\n",
               "sharded_path_taken": "reads aligned (sharded)" in rsh.stderr,
               "stages": [x for x in rsh.stderr.strip().splitlines() if x.startswith("[pa_cli]")][-8:]}
    t = time.perf_counter()
    subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import main" % PKG])
    stages["python_and_imports_s"] = time.perf_counter() - t
    # dumpref of the C2 reference (46 M k-mers: ~6 GB of JSON) to /dev/null
    t = time.perf_counter()
    with open(os.devnull, "w") as dn:
        rd = subprocess.run([sys.executable, os.path.join(PKG, "main.py"), "-t", "dumpref", "-g", fa, "-k", "31"],
                            stdout=dn, stderr=subprocess.PIPE, text=True)
    dumpref = {"wall_s": time.perf_counter() - t, "rc": rd.returncode}
    # the same reads as a BGZF .fq.gz (bgzip's format, level 6): members inflated
    # on host threads (pa_gz.cpp) while the device parses and aligns
    gz = {}
    if not args.no_gz:
        fqz = fq + ".gz"
        t = time.perf_counter()
        with open(fq, "rb") as f:
            synth.write_bgzf(fqz, f.read(), level=6, workers=min(16, os.cpu_count() or 1))
        gz["write_s"] = time.perf_counter() - t
        cmdz = cmd[:-1] + [fqz]
        wz = []
        for _ in range(3):
            time.sleep(3)
            t = time.perf_counter()
            rz = subprocess.run(cmdz, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
            wz.append(time.perf_counter() - t)
        gz.update({"fastq_gz_bytes": os.path.getsize(fqz), "format": "BGZF (bgzip layout), zlib level 6",
                   "cli_wall_s": sorted(wz)[1], "cli_wall_runs_s": wz, "cli_reads_per_s": args.reads / sorted(wz)[1],
                   "cli_rc": rz.returncode, "cli_stdout_equals_api": rz.stdout == summary + "\n"})
        if rz.returncode:
            gz["cli_stderr"] = rz.stderr[-2000:]
        if not args.keep:
            os.remove(fqz)
    # the same reads as ONE ordinary gzip member (what `gzip` / pigz write, the
    # reference's gzip.open path, src/data_file.py:123-125): inflated by chunks
    # on host threads (pa_pgz.cpp), their block boundaries found by search
    pgz = {}
    if not args.no_gz:
        fqz = fq[:-3] + "_plain.fq.gz"  # (the CLI takes .fq / .fq.gz names only)
        t = time.perf_counter()
        with open(fq, "rb") as f:
            synth.write_gzip(fqz, f.read(), level=6, workers=min(16, os.cpu_count() or 1))
        pgz["write_s"] = time.perf_counter() - t
        cmdz = cmd[:-1] + [fqz]
        wz = []
        for _ in range(3):
            time.sleep(3)
            t = time.perf_counter()
            rz = subprocess.run(cmdz, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
            wz.append(time.perf_counter() - t)
        pgz.update({"fastq_gz_bytes": os.path.getsize(fqz),
                    "format": "one gzip member (pigz layout: 1 MiB slices, sync flushes), zlib level 6",
                    "cli_wall_s": sorted(wz)[1], "cli_wall_runs_s": wz, "cli_reads_per_s": args.reads / sorted(wz)[1],
                    "cli_rc": rz.returncode, "cli_stdout_equals_api": rz.stdout == summary + "\n"})
        if rz.returncode:
            pgz["cli_stderr"] = rz.stderr[-2000:]
        if not args.keep:
            os.remove(fqz)
    out = {"workload": f"dumpalign C2: 50 x 2 Mbp FASTA, {args.reads} x 150 bp FASTQ, k=31",
           "fq_gz": gz, "fq_plain_gz": pgz, "sharded": sharded,
           "fastq_bytes": os.path.getsize(fq), "cli_wall_s": cli_s, "cli_wall_runs_s": walls, "cli_reads_per_s": args.reads / cli_s,
           "cli_rc": r.returncode, "cli_stdout_equals_api": r.stdout == summary + "\n",
           "device_parse_path_taken": streamed, "host_path_summary_equal": host_equal,
           "phases": ph, "cli_stages": stages, "dumpref_c2_to_devnull": dumpref, "ingest_threads": N.ingest_threads(),
           "fastq_device_parse_align_GBps": os.path.getsize(fq) / ph["fastq_device_parse_align_s"] / 1e9,
           "fastq_host_parse_GBps": os.path.getsize(fq) / ph["host_parse_fastq_s"] / 1e9}
    if r.returncode:
        out["cli_stderr"] = r.stderr[-2000:]
    print(json.dumps(out), flush=True)
    if not args.keep:
        for p in (fa, fq):
            os.remove(p)


if __name__ == "__main__":
    main()
