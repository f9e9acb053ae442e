#!/usr/bin/env python3
"""Command-line interface, drop-in for the reference's src/main.py.

    python3 main.py -t dumpalign -g GENOMES.fa -k 31 --reads READS.fq [-m M] [-p P]
                    [--min-read-quality Q] [--min-kmer-quality QK] [--max-genomes MG]
                    [--filter-similar [--similarity-threshold T]]

Same tasks (reference | dumpref | align | dumpalign), flags, flag-combination
checks, default coercions and error exits as src/main.py:61-402:

* ``-m 0`` / ``-p 0`` / ``--similarity-threshold 0`` are falsy and coerced to
  their defaults (1, 1, 0.95), exactly like src/main.py:337-342;
* errors end the process with ``sys.exit(message)`` (non-zero, message on
  stderr).

The ``.kdb`` / ``.aln`` files are gzip pickles, loaded by a restricted
unpickler (kmer._KdbUnpickler) that admits only the classes such files hold;
the classes keep the reference's module and class names, so files written by
the reference load too (a loaded reference rebuilds its device index).
``dumpref`` streams its JSON from the device index (pa_index_dumpref).
"""

from __future__ import annotations

import argparse
import atexit
import gzip
import json
import os
import sys
import time
from typing import List, Optional

_T0 = time.perf_counter()

_EARLY_PREFETCH = None  # (path, native handle) of a FASTQ prefetch started at entry


_FQ_PLAIN_EXT = ".fq"  # (FASTAQFile.EXTENSIONS without ".fq.gz": the file types the prefetch takes)


def _early_reads_path(argv: List[str]) -> Optional[str]:
    """The --reads file of a `-t dumpalign` command line, read off argv before
    argparse and the heavy imports (every spelling argparse accepts: `-t X`,
    `-tX`, `--task X`, `--task=X`, `--reads X`, `--reads=X`), when it is a file
    the later prefetch would take too (_prefetch_reads: a plain `.fq`, streaming
    and prefetch on).  A guess: main() still validates everything and ignores
    the early prefetch unless it names the same file."""
    task = reads = None
    i = 0
    while i < len(argv):
        a = argv[i]
        nxt = argv[i + 1] if i + 1 < len(argv) else None
        if a in ("-t", "--task"):
            task, i = nxt, i + 2
            continue
        if a == "--reads":
            reads, i = nxt, i + 2
            continue
        if a.startswith("--task="):
            task = a.split("=", 1)[1]
        elif a.startswith("-t") and not a.startswith("--") and len(a) > 2:
            task = a[2:]
        elif a.startswith("--reads="):
            reads = a.split("=", 1)[1]
        i += 1
    if task != "dumpalign" or not reads or not reads.endswith(_FQ_PLAIN_EXT):
        return None
    if os.environ.get("PA_GPUS", "1") not in ("", "0", "1"):  # (read-sharded over GPUs: no whole-file prefetch)
        return None
    if os.environ.get("PA_STREAM", "1") == "0" or os.environ.get("PA_PREFETCH", "1") == "0":
        return None
    return reads


def _stream_window() -> int:
    """PA_STREAM_WINDOW (bytes; 0: the library's default), as pa_native reads it."""
    env = os.environ.get("PA_STREAM_WINDOW")
    return int(env) if env and env.isdigit() else 0


if __name__ == "__main__":  # the HIP runtime starts on a native thread while the modules below import
    try:
        import ctypes
        _here = os.path.dirname(os.path.abspath(__file__))
        _lib = ctypes.CDLL(os.environ.get("PA_LIBRARY", os.path.join(_here, "libpa.so")))
        _dev = int(os.environ.get("PA_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        _lib.pa_runtime_start(_dev)
        # a plain FASTQ's copy into device memory starts now too (pa_fastq_prefetch_start
        # makes no HIP call on this thread): it overlaps the imports, not only the build
        _r = _early_reads_path(sys.argv[1:])
        if _r and os.path.isfile(_r) and os.environ.get("PA_EARLY_PREFETCH", "1") != "0":
            _n = len(os.sched_getaffinity(0))
            _omp = os.environ.get("OMP_NUM_THREADS", "")
            _thr = os.environ.get("PA_INGEST_THREADS", "")
            _threads = int(_thr) if _thr.isdigit() and int(_thr) > 0 else \
                max(1, min(min(_n, int(_omp)) if _omp.isdigit() and int(_omp) > 0 else _n, 16))
            _h = ctypes.c_void_p()
            _lib.pa_fastq_prefetch_start.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
            if (_lib.pa_fastq_prefetch_start(os.fsencode(_r), _dev, _threads, _stream_window(), ctypes.byref(_h)) == 0
                    and _h.value):
                _EARLY_PREFETCH = (os.path.abspath(_r), _h)

                def _free_early_prefetch():  # (an early exit: argument errors, another task)
                    if _EARLY_PREFETCH is not None:
                        _lib.pa_fastq_prefetch_free.argtypes = [ctypes.c_void_p]
                        _lib.pa_fastq_prefetch_free(_EARLY_PREFETCH[1])
                atexit.register(_free_early_prefetch)
    except (OSError, AttributeError, ValueError):
        pass  # (no library: pa_native raises at the first device call)

from constants import DEFAULT_AMBIGUOUS_THRESHOLD, DEFAULT_SIMILARITY_THRESHOLD, DEFAULT_UNIQUE_THRESHOLD
from data_file import FASTAFile, FASTAQFile, InvalidExtensionError, NoRecordsInDataFile
from kmer import AddingExistingRead, KmerReference, NotValidatingUniqueMapping, PseudoAlignment

_TIMING = os.environ.get("PA_CLI_TIMING") == "1"  # stage times on stderr (diagnostic)


def _stage(name: str) -> None:
    if _TIMING:
        print(f"[pa_cli] {name}: {time.perf_counter() - _T0:.3f} s", file=sys.stderr, flush=True)


def validate_file_readable(filepath: str, description: str) -> None:
    if not os.path.isfile(filepath):
        sys.exit(f"Error: {description} file '{filepath}' does not exist or is not a file.")
    if not os.access(filepath, os.R_OK):
        sys.exit(f"Error: {description} file '{filepath}' is not readable.")


def validate_file_writable(filepath: str, description: str) -> None:
    dir_path = os.path.dirname(filepath) or "."
    if os.path.exists(filepath) and not os.access(filepath, os.W_OK):
        sys.exit(f"Error: {description} file '{filepath}' is not writable.")
    if not os.path.exists(filepath) and not os.access(dir_path, os.W_OK):
        sys.exit(f"Error: Directory '{dir_path}' is not writable to create {description} file '{filepath}'.")


def parse_arguments(args: Optional[List[str]] = None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(prog="Biosequence project")
    parser.add_argument("-t", "--task", required=True, help="Task to execute")
    parser.add_argument("-g", "--genomefile", help="Genome FASTA file (multiple records)")
    parser.add_argument("-k", "--kmer-size", type=int, help="Length of k-mers")
    parser.add_argument("-r", "--referencefile", help="KDB file (input/output)")
    parser.add_argument("-a", "--alignfile", help="aln file. Can be either input or name for output file")
    parser.add_argument("--reads", help="FASTQ reads file")
    parser.add_argument("-m", "--unique-threshold", help="unique k-mer threshold", type=int)
    parser.add_argument("-p", "--ambiguous-threhold", help="ambiguous k-mer threshold", type=int)
    parser.add_argument("--reverse-complement", action="store_true")  # parsed, unused (as in the reference)
    parser.add_argument("--min-read-quality", type=int, default=None)
    parser.add_argument("--min-kmer-quality", type=int, default=None)
    parser.add_argument("--max-genomes", type=int, default=None)
    parser.add_argument("--filter-similar", action="store_true")
    parser.add_argument("--similarity-threshold", type=float)
    return parser.parse_args(args)


def _load_reference(reference_file: str) -> KmerReference:
    try:
        return KmerReference.load(reference_file)
    except gzip.BadGzipFile:
        sys.exit("Error: Incorrect format of input file.")


def compact_for_job(reads_file: Optional[str], container, shards: int = 1) -> bool:
    """The reference of a one-FASTQ job gets the compact k-mer table
    (PA_BUILD_COMPACT) when the job has fewer than PA_COMPACT_READS_PER_BASE
    reads per genome base -- the reads counted high, one per 64 bytes of the
    file (4x that for gzip), over `shards` replicas."""
    env = os.environ.get("PA_COMPACT_TABLE")  # (A/B: 0 / 1 overrides the policy)
    if env in ("0", "1"):
        return env == "1"
    if not reads_file:
        return False
    import pa_native as N
    try:
        size = os.path.getsize(reads_file)
    except OSError:
        return False
    reads = (size * (4 if reads_file.endswith(".gz") else 1)) // 64 // max(shards, 1)
    bases = sum(len(g["genome"]) for g in container)
    return reads < N.PA_COMPACT_READS_PER_BASE * bases


def create_reference(fasta_file: str, kmer_size: int, filter_similar: bool = False,
                     similarity_threshold: float = 0.95, reads_file: Optional[str] = None) -> KmerReference:
    container = FASTAFile(fasta_file).container
    _stage("fasta parsed")
    return KmerReference(kmer_size, container, filter_similar=filter_similar,
                         similarity_threshold=similarity_threshold,
                         compact_table=compact_for_job(reads_file, container))


def _prefetch_reads(reads_file: str):
    """Start moving a plain FASTQ file into device memory (pa_fastq_prefetch_start)
    so that the copy overlaps the reference build; None where the file takes
    another path (a .gz or wrong extension, PA_STREAM=0 / PA_PREFETCH=0)."""
    if os.environ.get("PA_STREAM", "1") == "0" or os.environ.get("PA_PREFETCH", "1") == "0":
        return None
    if reads_file.endswith(".gz") or not any(reads_file.endswith(e) for e in FASTAQFile.EXTENSIONS):
        return None
    try:
        import pa_native as N
        global _EARLY_PREFETCH
        early = _EARLY_PREFETCH
        if early is not None and early[0] == os.path.abspath(reads_file):  # started at entry
            _EARLY_PREFETCH = None  # (owned by pf from here on)
            pf = N.FastqPrefetch.adopt(early[1], reads_file)
        else:
            pf = N.FastqPrefetch(reads_file)
    except Exception:  # (no device, unreadable file: the exact path reports it in the reference's order)
        return None
    atexit.register(pf.close)
    return pf


def create_alignment_from_reference(kmer_reference: KmerReference, reads_file: str, m: int, p: int,
                                    min_read_quality, min_kmer_quality, max_genomes,
                                    prefetch=None, per_read: bool = False) -> PseudoAlignment:
    # the FASTQ file goes straight to the device (parsed there, aligned in
    # windows); a file outside that subset of the grammar is parsed the exact
    # way (FASTAQFile), which also raises the reference's errors.  per_read
    # (task 'align': the .aln file holds every read's result): the host parse,
    # whose records the per-read results are made from -- the device parse
    # would only have to be repeated on the host for them
    FASTAQFile.check_extension(reads_file)
    _stage("reference built")
    alignment = PseudoAlignment(kmer_reference)
    if per_read:
        alignment.align_reads_from_container(FASTAQFile(reads_file).container, m, p, min_read_quality,
                                             min_kmer_quality, max_genomes)
    else:
        alignment.align_reads_from_file(reads_file, m, p, min_read_quality, min_kmer_quality, max_genomes,
                                        prefetch=prefetch)
    _stage("reads aligned")
    return alignment


def _print_json(obj) -> None:
    print(json.dumps(obj, indent=4))


def _dump_reference(ref: KmerReference) -> None:
    """print(json.dumps(ref.get_summary(), indent=4)) (src/main.py:121-127), the
    text streamed to stdout from the device index instead of built as a dict."""
    if not isinstance(ref, KmerReference):  # (another object in the file: its own summary, as the reference)
        _print_json(ref.get_summary())
        return
    sys.stdout.flush()
    fd = sys.stdout.fileno()
    ref.write_summary(fd)
    os.write(fd, b"\n")


def _check_task(args: argparse.Namespace) -> None:
    """Flag combinations (src/main.py:321-334), truthiness-based like the reference."""
    extra = (args.reads or args.alignfile or args.unique_threshold or args.ambiguous_threhold
             or args.min_read_quality or args.min_kmer_quality or args.max_genomes)
    if args.task == "reference":
        if extra:
            sys.exit("Error: For task 'reference', only -g, -k, -r, --filter-similar, and --similarity-threshold "
                     "are allowed.")
    elif args.task == "dumpref":
        if extra:
            sys.exit("Error: For task 'dumpref', only -r or (-g and -k) with --filter-similar and "
                     "--similarity-threshold are allowed.")
    elif args.task == "align":
        if not ((args.referencefile and args.reads and args.alignfile)
                or (args.genomefile and args.kmer_size and args.reads and args.alignfile)):
            sys.exit("Error: For task 'align', provide either -r (reference file) or -g and -k (genome file and "
                     "kmer size) along with --reads and -a.")
    elif args.task == "dumpalign":
        if not ((args.referencefile and args.reads) or (args.genomefile and args.kmer_size and args.reads)
                or args.alignfile):
            sys.exit("Error: For task 'dumpalign', provide either -r and --reads, or -g, -k, and --reads, or -a.")
    else:
        sys.exit("Error: Unsupported task.")


def _dumpalign_sharded(args: argparse.Namespace, filt) -> Optional[PseudoAlignment]:
    """PA_GPUS=N > 1: the dumpalign job read-sharded over N devices (pa_shard:
    one index replica per device, one byte range of the FASTQ file each, the
    counters reduced on the host); None where it does not apply -- one GPU,
    a .gz or non-canonical file, a duplicate id across ranges -- and the
    one-GPU path runs (and raises the reference's errors)."""
    import pa_shard
    n, share = pa_shard.gpus_from_env()
    if n < 2 or args.reads.endswith(".gz"):
        return None
    FASTAQFile.check_extension(args.reads)
    devices = pa_shard.devices_for(n, share)
    if len(devices) < 2:
        return None
    container = FASTAFile(args.genomefile).container
    _stage("fasta parsed")
    refs = pa_shard.build_replicas(args.kmer_size, container, devices, args.filter_similar,
                                   args.similarity_threshold,
                                   compact_table=compact_for_job(args.reads, container, len(devices)))
    _stage(f"{len(refs)} references built")
    pa = pa_shard.align_sharded(refs, args.reads, *filt)
    _stage("reads aligned (sharded)" if pa is not None else "sharded path not taken")
    if pa is None:
        return None
    if _TIMING:
        print(f"[pa_cli] shards (offset, bytes, records): {pa._shards}", file=sys.stderr, flush=True)
    return pa


def _run(args: argparse.Namespace) -> None:
    filt = (args.unique_threshold, args.ambiguous_threhold, args.min_read_quality, args.min_kmer_quality,
            args.max_genomes)
    if args.task == "reference":
        validate_file_readable(args.genomefile, "Genome FASTA")
        validate_file_writable(args.referencefile, "Reference database output")
        create_reference(args.genomefile, args.kmer_size, args.filter_similar,
                         args.similarity_threshold).save(args.referencefile)
    elif args.task == "dumpref":
        if args.referencefile:
            validate_file_readable(args.referencefile, "Reference database")
            _dump_reference(_load_reference(args.referencefile))
        elif args.genomefile and args.kmer_size:
            validate_file_readable(args.genomefile, "Genome FASTA")
            _dump_reference(create_reference(args.genomefile, args.kmer_size, args.filter_similar,
                                             args.similarity_threshold))
    elif args.task == "align":
        validate_file_readable(args.reads, "FASTQ reads")
        validate_file_writable(args.alignfile, "Alignment output")
        if args.referencefile and args.reads and args.alignfile:
            validate_file_readable(args.referencefile, "Reference database")
            ref = _load_reference(args.referencefile)
        else:
            validate_file_readable(args.genomefile, "Genome FASTA")
            ref = create_reference(args.genomefile, args.kmer_size, args.filter_similar, args.similarity_threshold,
                                   reads_file=args.reads)
            # saved unconditionally, as src/main.py:370 does: without -r that is
            # gzip.open(None), a TypeError the reference does not catch
            # (src/main.py:401), so the command ends with a traceback and exit
            # status 1 before any alignment is written -- reproduced, not fixed
            ref.save(args.referencefile)
        create_alignment_from_reference(ref, args.reads, *filt, per_read=True).save(args.alignfile)
    elif args.task == "dumpalign":
        if args.referencefile and args.reads:
            validate_file_readable(args.reads, "FASTQ reads")
            pf = _prefetch_reads(args.reads)
            ref = _load_reference(args.referencefile)
            _print_json(create_alignment_from_reference(ref, args.reads, *filt, prefetch=pf).get_summary())
        elif args.genomefile and args.kmer_size and args.reads:
            validate_file_readable(args.reads, "FASTQ reads")
            validate_file_readable(args.genomefile, "Genome FASTA")
            sharded = _dumpalign_sharded(args, filt)
            if sharded is not None:
                _print_json(sharded.get_summary())
                return
            pf = _prefetch_reads(args.reads)
            ref = create_reference(args.genomefile, args.kmer_size, args.filter_similar, args.similarity_threshold,
                                   reads_file=args.reads)
            _print_json(create_alignment_from_reference(ref, args.reads, *filt, prefetch=pf).get_summary())
        elif args.alignfile:
            validate_file_readable(args.alignfile, "Alignment output")
            try:
                alignment = PseudoAlignment.load(args.alignfile)
            except gzip.BadGzipFile:
                sys.exit("Error: Incorrect format of input file.")
            _print_json(alignment.get_summary())
        else:
            sys.exit("Error: Provide either -g and -k with --reads, or -r with --reads, or -a.")
    else:
        sys.exit("Error: Unsupported task.")


def main(argv: Optional[List[str]] = None) -> None:
    _stage("imports done")
    args = parse_arguments(argv)
    _check_task(args)
    # falsy -> default, as src/main.py:337-342 (so -m 0 and -p 0 become 1)
    if not args.unique_threshold:
        args.unique_threshold = DEFAULT_UNIQUE_THRESHOLD
    if not args.ambiguous_threhold:
        args.ambiguous_threhold = DEFAULT_AMBIGUOUS_THRESHOLD
    if not args.similarity_threshold:
        args.similarity_threshold = DEFAULT_SIMILARITY_THRESHOLD
    try:
        _run(args)
        _stage("printed")
    except gzip.BadGzipFile:
        sys.exit("Error: Incorrect format of input file.")
    except (InvalidExtensionError, NoRecordsInDataFile, NotValidatingUniqueMapping, AddingExistingRead,
            ValueError) as err:
        sys.exit(err)


if __name__ == "__main__":
    main()
    # done: the output is flushed and the process ends without releasing the
    # device index allocation by allocation (the driver reclaims it at exit);
    # PA_FAST_EXIT=0 keeps the normal interpreter exit (profilers write their
    # results from exit handlers)
    if os.environ.get("PA_FAST_EXIT", "1") != "0":
        _stage("exit")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
