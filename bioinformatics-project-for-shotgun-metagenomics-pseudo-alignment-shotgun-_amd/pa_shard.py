"""The dumpalign job read-sharded over the GPUs of one node (PA_GPUS=N).

The reference aligns one FASTQ file in one process (src/main.py:289-310 ->
src/kmer.py:600-620).  Here, with PA_GPUS=N (N > 1), `main.py -t dumpalign
-g G.fa -k K --reads R.fq` builds one index replica per device and aligns one
byte range of the FASTQ file on each:

* the file is cut into N byte ranges on record boundaries (fastq_shards);
* the replicas are built on host threads, one per device, concurrently (the
  library's calls release the GIL); EXTSIM runs on each replica alike;
* each range is parsed and aligned on its device (pa_align_fastq_range) with
  the range's byte offset as its read-index base, which keeps the Summary key
  order of one pass over the file (every record takes more than one byte);
* the ranges' read ids are checked for duplicates across ranges
  (pa_idsets_disjoint; DuplicateRecordError, src/records.py:290-302);
* the counters are reduced on the host (SUM of the sum blocks, MIN of the
  first-appearance keys) and loaded into replica 0's result, so the
  PseudoAlignment answers get_summary() -- and everything else -- as the
  one-GPU pass does.

Whatever the sharded path cannot take (a .gz file, a range outside the
device-parsed grammar subset, a duplicate id across ranges, fewer records
than ranges) returns None and the caller takes the one-GPU path, which also
raises the reference's errors.  PA_GPUS_SHARE=1 puts every replica on device
0 (the two-rank rehearsal of the one-GPU test box).
"""

from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

import pa_native as N


def gpus_from_env() -> Tuple[int, bool]:
    """(N, share): PA_GPUS (default 1) and PA_GPUS_SHARE=1 (all on device 0)."""
    env = os.environ.get("PA_GPUS", "1")
    n = int(env) if env.isdigit() and int(env) > 0 else 1
    return n, os.environ.get("PA_GPUS_SHARE") == "1"


def devices_for(n: int, share: bool) -> List[int]:
    """The devices of an n-way job: 0..n-1 (at most the visible ones), or n
    times device 0 with `share`."""
    if share:
        return [0] * n
    return list(range(min(n, max(N.device_count(), 1))))


def _record_start(buf: bytes, p: int) -> bool:
    """Line p of the text starts a canonical 4-line record: '@' here and '+'
    two lines on.  (A quality line may start with '@', but two lines after it
    comes a sequence line -- ACGT, never '+' -- so the test is exact for the
    4-line records the device parser takes; anything else fails that parser,
    and the whole file takes the exact path.)"""
    if p >= len(buf) or buf[p] != 0x40:
        return False
    e0 = buf.find(b"\n", p)
    if e0 < 0:
        return False
    e1 = buf.find(b"\n", e0 + 1)
    return e1 >= 0 and e1 + 1 < len(buf) and buf[e1 + 1] == 0x2B


def fastq_shards(path: str, n: int, probe: int = 1 << 20) -> Optional[List[Tuple[int, int]]]:
    """Up to n byte ranges [(offset, length)] of a plain FASTQ file, cut at
    record starts near i * size / n; None if the file is empty or no cut is
    found (the caller then aligns the whole file on one device)."""
    try:
        size = os.path.getsize(path)
    except OSError:
        return None
    if size == 0 or n < 1:
        return None
    cuts = [0]
    with open(path, "rb") as f:
        for i in range(1, n):
            target = max(i * size // n, cuts[-1] + 1)
            if target >= size:
                break
            f.seek(target - 1)
            buf = f.read(probe)
            at = None
            q = buf.find(b"\n")
            while 0 <= q < len(buf) - 1:
                if _record_start(buf, q + 1):
                    at = target - 1 + q + 1
                    break
                q = buf.find(b"\n", q + 1)
            if at is None or at >= size:
                continue
            cuts.append(at)
    if len(cuts) < 2:
        return None
    cuts.append(size)
    return [(a, b - a) for a, b in zip(cuts[:-1], cuts[1:])]


def _records_estimate(path: str, offset: int, length: int, probe: int = 1 << 20) -> int:
    """Records in a range from the line feeds of its first megabyte (the
    align-side view's hint: pa_index_prepare_ex)."""
    with open(path, "rb") as f:
        f.seek(offset)
        head = f.read(min(probe, length))
    if not head:
        return 0
    return int(length * (head.count(b"\n") / 4.0) / len(head)) + 1


def _run_threads(fns) -> list:
    """Run callables on threads; their results in order, the first error re-raised."""
    out = [None] * len(fns)
    err = []

    def run(i):
        try:
            out[i] = fns[i]()
        except BaseException as e:  # (re-raised on the calling thread)
            err.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return out


def build_replicas(k: int, container, devices: Sequence[int], filter_similar: bool = False,
                   similarity_threshold: float = 0.95, compact_table: bool = False):
    """One KmerReference per device, built concurrently on host threads
    (KmerReference(k, container, ..., device=d) each: the same genomes, the same
    EXTSIM outcome; compact_table: PA_BUILD_COMPACT, main.compact_for_job)."""
    from kmer import KmerReference
    N.lib()  # (bound once, before the threads)
    return _run_threads([lambda d=d: KmerReference(k, container, filter_similar=filter_similar,
                                                   similarity_threshold=similarity_threshold, device=d,
                                                   compact_table=compact_table)
                         for d in devices])


def align_sharded(refs: Sequence, reads_file: str, m: int = 1, p: int = 1, min_read_quality=None,
                  min_kmer_quality=None, max_genomes=None):
    """The PseudoAlignment of `reads_file` against refs[0] computed as one byte
    range per replica (module docstring), or None where the sharded path does
    not apply."""
    from data_file import FASTAQFile
    from kmer import PseudoAlignment, _FileBatch, _check_align_args
    if len(refs) < 2 or reads_file.endswith(".gz"):
        return None
    if _check_align_args(refs[0], m, p, min_read_quality, min_kmer_quality, max_genomes) is not None:
        return None  # (the one-GPU path raises the reference's error)
    FASTAQFile.check_extension(reads_file)
    shards = fastq_shards(reads_file, len(refs))
    if shards is None:
        return None
    refs = list(refs)[:len(shards)]
    prm = N.Params.make(m, p, min_read_quality, min_kmer_quality, max_genomes)
    results = [N.Result(r.index) for r in refs]
    threads = max(2, N.ingest_threads() // len(refs))

    def shard(i):
        off, ln = shards[i]
        refs[i].index.prepare(expected_reads=_records_estimate(reads_file, off, ln))
        return N.align_fastq_range(refs[i].index, reads_file, off, ln, prm, off, results[i], threads=threads)

    outs = _run_threads([lambda i=i: shard(i) for i in range(len(refs))])
    try:
        if any(o is None for o in outs):
            return None
        if not N.idsets_disjoint([o[1] for o in outs], device=refs[0].index.device):
            return None
    finally:
        for o in outs:
            if o is not None and o[1] is not None:
                o[1].close()
    # host SUM / MIN of the shards' counters into replica 0's result
    parts = [r.fetch() for r in results]
    stats = sum(x[0] for x in parts)
    uq = sum(x[1] for x in parts)
    am = sum(x[2] for x in parts)
    fk = parts[0][3].copy()
    for x in parts[1:]:
        fk = np.minimum(fk, x[3])
    results[0].load(stats, uq, am, fk)
    for r in results[1:]:
        r.close()
    n_total = sum(o[0] for o in outs)
    pa = PseudoAlignment(refs[0])
    if min_read_quality is not None:
        pa.filter_read_quality_flag = True
    if min_kmer_quality is not None:
        pa.filter_kmer_quality_flag = True
    if max_genomes is not None:
        pa.filter_max_genomes_flag = True
    pa._result = results[0]
    pa._gpu_stats = stats
    pa.filtered_quality_reads = int(stats[3])
    pa.filtered_quality_kmers = int(stats[4])
    pa.filtered_hr_kmers = int(stats[5])
    # per-read results, if asked for, come from one host parse of the whole
    # file aligned on replica 0 (read indices from 0: the order is the file's)
    pa._batches.append(_FileBatch(0, reads_file, prm, min_read_quality, n_total))
    pa._next_index = n_total
    pa._shards = [(off, ln, o[0]) for (off, ln), o in zip(shards, outs)]
    return pa
