"""ctypes wrapper of the CPU restatement (oracle/pa_oracle.c) + host helpers.

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's ``cpu_baseline`` leg, never by the product package.  The product's
drop-in modules live in the package directory and call libpa.so (HIP) only.

Besides the C restatement this module restates, in Python, the two pieces of
the reference that are pure host control flow:

* the EXTSIM greedy pass (``src/kmer.py:179-230``), fed with the per-identifier
  k-mer statistics that ``ora_extsim_stats`` computes (``src/kmer.py:152-177``);
* ``PseudoAlignment.get_summary`` (``src/kmer.py:622-657``), computed the
  reference's way, by walking per-read genome lists in read order;
* ``KmerReference.get_summary`` (dumpref, ``src/kmer.py:300-329``) over the
  reference's own dict (``src/kmer.py:135-150``, pruned by identifier as
  ``src/kmer.py:232-245`` does), pure Python: small references only;
* ``get_kmer_references`` / ``get_kmer_and_reverse_references``
  (``src/kmer.py:292-298, 331-351``) over that dict (``kmer_dict`` +
  ``kmer_references``).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from collections import defaultdict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "pa_oracle.c")
LIB = os.path.join(HERE, "_build", "libpa_oracle.so")

DROPPED, UNMAPPED, UNIQUE, AMBIGUOUS = 0, 1, 2, 3
TYPE_NAMES = {DROPPED: "DROPPED", UNMAPPED: "UNMAPPED", UNIQUE: "UNIQUELY_MAPPED", AMBIGUOUS: "AMBIGUOUSLY_MAPPED"}
HAS_MRQ, HAS_MKQ, HAS_MG = 1, 2, 4
U64 = ctypes.c_uint64
P = ctypes.c_void_p


def build(force: bool = False) -> str:
    """Compile the restatement with gcc into oracle/_build/ (gitignored)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-std=c11", "-shared", "-fPIC", "-pthread", "-o", LIB, SRC])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.ora_index_build.restype = P
        L.ora_index_build.argtypes = [ctypes.c_char_p, P, ctypes.c_uint32, ctypes.c_int64]
        L.ora_index_build_mt.restype = P
        L.ora_index_build_mt.argtypes = [ctypes.c_char_p, P, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int]
        L.ora_index_build_restricted.restype = P
        L.ora_index_build_restricted.argtypes = [P, P, ctypes.c_uint32, ctypes.c_int64, P, P, ctypes.c_uint32,
                                                 ctypes.c_int]
        L.ora_index_free.argtypes = [P]
        L.ora_index_n_kmers.restype = U64
        L.ora_index_n_kmers.argtypes = [P]
        L.ora_index_lookup.restype = ctypes.c_int64
        L.ora_index_lookup.argtypes = [P, ctypes.c_char_p, P, ctypes.c_uint32]
        L.ora_index_export.restype = ctypes.c_int64
        L.ora_index_export.argtypes = [P, P, P, P]
        L.ora_extsim_stats.argtypes = [P, P, ctypes.c_uint32, P, P, P]
        L.ora_align.restype = ctypes.c_int
        L.ora_align.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, P, U64, U64,
                                ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                ctypes.c_uint32, P, P, P, P, P, U64, P, P, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def concat(chunks: Sequence) -> Tuple[bytes, np.ndarray]:
    """Concatenate str/bytes/uint8 chunks; returns (bytes, uint64 CSR offsets)."""
    bs = [c.encode() if isinstance(c, str) else bytes(c) for c in chunks]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    return b"".join(bs), off


def _packed(x) -> Tuple[np.ndarray, np.ndarray]:
    """(uint8 buffer, uint64 CSR offsets) of a sequence list, or the pair as is."""
    if isinstance(x, tuple) and len(x) == 2 and isinstance(x[1], np.ndarray):
        buf, off = x
        buf = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
        return buf, np.ascontiguousarray(off, dtype=np.uint64)
    text, off = concat(x)
    buf = np.frombuffer(text, dtype=np.uint8) if text else np.zeros(1, dtype=np.uint8)
    return buf, off


@dataclass
class AlignResult:
    types: np.ndarray          # uint8 per read (DROPPED/UNMAPPED/UNIQUE/AMBIGUOUS)
    qf: np.ndarray             # windows filtered by k-mer quality, per read
    hr: np.ndarray             # windows filtered as highly redundant, per read
    list_off: np.ndarray       # CSR offsets of genomes_mapped_to
    lists: np.ndarray          # genome indices
    stats: np.ndarray          # unique, ambiguous, unmapped, filt reads, filt q windows, filt hr windows
    unique: np.ndarray         # per genome
    ambiguous: np.ndarray      # per genome
    first_key: np.ndarray      # per genome, (read << 20 | list position), 2^64-1 if never

    def genomes_of(self, r: int) -> List[int]:
        return [int(x) for x in self.lists[self.list_off[r]:self.list_off[r + 1]]]


def host_threads() -> int:
    """Host threads this job may use: OMP_NUM_THREADS (the GPU box's CPU share)
    capped by the affinity mask, at most 16."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, min(n, 16))


def pack_params(m=1, p=1, mrq=None, mkq=None, mg=None):
    flags = (HAS_MRQ if mrq is not None else 0) | (HAS_MKQ if mkq is not None else 0) | (HAS_MG if mg is not None else 0)
    return int(m), int(p), int(mrq or 0), int(mkq or 0), int(mg or 0), flags


class OracleIndex:
    """CPU k-mer index: genomes in FASTA order, k-mers with 'N' skipped."""

    def __init__(self, genomes: Sequence, k: int, threads: Optional[int] = None):
        """``threads`` host threads build it (default: this job's CPU share, at
        most 16); the index -- every k-mer's genome list included -- does not
        depend on the thread count."""
        self.k = int(k)
        text, off = concat(genomes)
        self.n_genomes = len(off) - 1
        self._off = off
        self._h = lib().ora_index_build_mt(text, _ptr(off), self.n_genomes, self.k,
                                           int(threads if threads else host_threads()))
        if not self._h:
            raise MemoryError("oracle index build failed")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().ora_index_free(h)
            self._h = None

    @classmethod
    def restricted(cls, genomes, k: int, seeds, threads: Optional[int] = None) -> "OracleIndex":
        """The k-mers of ``seeds`` only, each with exactly the genome list the full
        index gives it (ora_index_build_restricted): reads drawn from the seeds
        align as against the full index, and for every genome in the seeds
        ``extsim_stats`` rows are exact.  Memory scales with the seeds, so BASELINE
        configs 4-5 (1 and 8 Gbp) get full-size parity.  ``genomes`` / ``seeds``:
        sequences, or already concatenated ``(uint8 array, uint64 offsets)``."""
        self = cls.__new__(cls)
        self.k = int(k)
        gbuf, goff = _packed(genomes)
        sbuf, soff = _packed(seeds)
        self.n_genomes = len(goff) - 1
        self._off = goff
        self._h = lib().ora_index_build_restricted(_ptr(gbuf), _ptr(goff), self.n_genomes, self.k, _ptr(sbuf),
                                                   _ptr(soff), len(soff) - 1,
                                                   int(threads if threads else host_threads()))
        if not self._h:
            raise MemoryError("oracle restricted index build failed")
        return self

    @property
    def n_kmers(self) -> int:
        """Distinct k-mers (a restricted index: those of its seeds that some genome holds)."""
        return int(lib().ora_index_n_kmers(self._h))

    def lookup(self, kmer: str) -> List[int]:
        buf = np.zeros(self.n_genomes + 1, dtype=np.uint32)
        n = lib().ora_index_lookup(self._h, kmer.encode(), _ptr(buf), buf.size)
        return [int(x) for x in buf[:n]]

    def export(self) -> Dict[str, List[int]]:
        n = self.n_kmers
        total = lib().ora_index_export(self._h, None, None, None)
        kbuf = ctypes.create_string_buffer(max(1, n * max(self.k, 0)))
        off = np.zeros(n + 1, dtype=np.uint64)
        lists = np.zeros(max(total, 1), dtype=np.uint32)
        lib().ora_index_export(self._h, ctypes.cast(kbuf, ctypes.c_void_p), _ptr(off), _ptr(lists))
        raw = kbuf.raw
        return {raw[i * self.k:(i + 1) * self.k].decode(): [int(x) for x in lists[off[i]:off[i + 1]]]
                for i in range(n)}

    def extsim_stats(self, group_of: Sequence[int], n_groups: int):
        g = np.asarray(group_of, dtype=np.uint32)
        total = np.zeros(n_groups, dtype=np.uint64)
        uniq = np.zeros(n_groups, dtype=np.uint64)
        inter = np.zeros(n_groups * n_groups, dtype=np.uint64)
        lib().ora_extsim_stats(self._h, _ptr(g), n_groups, _ptr(total), _ptr(uniq), _ptr(inter))
        return total, uniq, inter.reshape(n_groups, n_groups)

    def align(self, seq: bytes, qual: bytes, read_off: np.ndarray, m=1, p=1, mrq=None, mkq=None, mg=None,
              read_base: int = 0, detail: bool = True) -> AlignResult:
        n = len(read_off) - 1
        read_off = np.ascontiguousarray(read_off, dtype=np.uint64)
        G = self.n_genomes
        types = np.zeros(n, dtype=np.uint8)
        qf = np.zeros(n, dtype=np.uint32)
        hr = np.zeros(n, dtype=np.uint32)
        stats = np.zeros(6, dtype=np.uint64)
        uq = np.zeros(G, dtype=np.uint64)
        am = np.zeros(G, dtype=np.uint64)
        fk = np.full(G, np.iinfo(np.uint64).max, dtype=np.uint64)
        mm, pp, a, b, c, flags = pack_params(m, p, mrq, mkq, mg)
        if detail:
            lo = np.zeros(n + 1, dtype=np.uint64)
            cap = n * (G + 2) if G < 64 else 4 * n + 64
            while True:
                lists = np.zeros(max(cap, 1), dtype=np.uint32)
                stats[:] = 0; uq[:] = 0; am[:] = 0; fk[:] = np.iinfo(np.uint64).max
                rc = lib().ora_align(self._h, seq, qual, _ptr(read_off), n, read_base, mm, pp, a, b, c, flags,
                                     _ptr(types), _ptr(qf), _ptr(hr), _ptr(lo), _ptr(lists), cap,
                                     _ptr(stats), _ptr(uq), _ptr(am), _ptr(fk))
                if rc == -1:
                    cap = int(lo[-1]) + 1
                    continue
                break
        else:
            lo = np.zeros(1, dtype=np.uint64)
            lists = np.zeros(0, dtype=np.uint32)
            rc = lib().ora_align(self._h, seq, qual, _ptr(read_off), n, read_base, mm, pp, a, b, c, flags,
                                 _ptr(types), _ptr(qf), _ptr(hr), None, None, 0,
                                 _ptr(stats), _ptr(uq), _ptr(am), _ptr(fk))
        if rc == -2:
            raise MemoryError("oracle align allocation failed")
        if detail:
            lists = lists[:int(lo[-1])]
        return AlignResult(types, qf, hr, lo, lists, stats, uq, am, fk)


def align_counts_parallel(index: "OracleIndex", seq: np.ndarray, qual: np.ndarray, read_off: np.ndarray,
                          threads: int, m=1, p=1, mrq=None, mkq=None, mg=None, read_base: int = 0) -> AlignResult:
    """Counters of ``index.align(..., detail=False)`` computed by ``threads`` host
    threads over contiguous read shards (ctypes releases the GIL inside
    ``ora_align``; the index is read-only).  Sums of the per-shard counters and
    min of the first keys (shards carry their global read base) equal the
    single-thread result exactly.  CPU-baseline helper for bench.py."""
    from concurrent.futures import ThreadPoolExecutor

    n = len(read_off) - 1
    threads = max(1, min(int(threads), max(n, 1)))
    cuts = [n * i // threads for i in range(threads + 1)]

    def shard(i):
        a, b = cuts[i], cuts[i + 1]
        lo, hi = int(read_off[a]), int(read_off[b])
        off = (read_off[a:b + 1] - read_off[a]).astype(np.uint64)
        return index.align(seq[lo:hi].tobytes(), qual[lo:hi].tobytes(), off, m=m, p=p, mrq=mrq, mkq=mkq, mg=mg,
                           read_base=read_base + a, detail=False)

    with ThreadPoolExecutor(max_workers=threads) as ex:
        parts = list(ex.map(shard, range(threads)))
    G = index.n_genomes
    out = AlignResult(np.zeros(0, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint32),
                      np.zeros(1, np.uint64), np.zeros(0, np.uint32), np.zeros(6, np.uint64),
                      np.zeros(G, np.uint64), np.zeros(G, np.uint64),
                      np.full(G, np.iinfo(np.uint64).max, dtype=np.uint64))
    for r in parts:
        out.stats += r.stats
        out.unique += r.unique
        out.ambiguous += r.ambiguous
        np.minimum(out.first_key, r.first_key, out=out.first_key)
    return out


def summary_by_walk(result: AlignResult, identifiers: Sequence[str], mrq=None, mkq=None, mg=None) -> dict:
    """get_summary (src/kmer.py:622-657) computed by walking reads in order."""
    stats = {"unique_mapped_reads": 0, "ambiguous_mapped_reads": 0, "unmapped_reads": 0}
    if mrq is not None:
        stats["filtered_quality_reads"] = int(result.stats[3])
    if mkq is not None:
        stats["filtered_quality_kmers"] = int(result.stats[4])
    if mg is not None:
        stats["filtered_hr_kmers"] = int(result.stats[5])
    genomes: Dict[str, Dict[str, int]] = {}
    for r, t in enumerate(result.types):
        if t == DROPPED:
            continue
        if t == UNMAPPED:
            stats["unmapped_reads"] += 1
            continue
        key = "unique_reads" if t == UNIQUE else "ambiguous_reads"
        stats["unique_mapped_reads" if t == UNIQUE else "ambiguous_mapped_reads"] += 1
        for g in result.genomes_of(r):
            genomes.setdefault(identifiers[g], {"unique_reads": 0, "ambiguous_reads": 0})[key] += 1
    return {"Statistics": stats, "Summary": genomes}


def extsim(identifiers: Sequence[str], genome_lengths: Sequence[int], index: OracleIndex, threshold: float):
    """EXTSIM (src/kmer.py:152-263) on the oracle index.

    Returns (kept record indices in FASTA order, similarity_info dict)."""
    # group records by identifier, as genome_to_kmers is keyed by identifier (:162-163)
    gid: Dict[str, int] = {}
    group_of = []
    for ident in identifiers:
        group_of.append(gid.setdefault(ident, len(gid)))
    ng = len(gid)
    total, uniq, inter = index.extsim_stats(group_of, ng)
    stats: Dict[str, dict] = {}
    for order, ident in enumerate(identifiers):  # later records overwrite (:165-176)
        a = gid[ident]
        stats[ident] = {"unique_kmers": int(uniq[a]), "total_kmers": int(total[a]),
                        "genome_length": int(genome_lengths[order]), "order": order}
    ordered = sorted(stats.items(), key=lambda x: (x[1]["unique_kmers"], x[1]["total_kmers"],
                                                   x[1]["genome_length"], x[1]["order"]))
    kept: List[str] = []
    info: Dict[str, dict] = {}
    for ident, st in ordered:
        a = gid[ident]
        dropped = False
        for kid in kept:
            b = gid[kid]
            mc = min(int(total[a]), int(total[b]))
            score = (int(inter[a, b]) / mc) if mc > 0 else 0
            if score > threshold:
                info[ident] = {"kept": "no", "unique_kmers": st["unique_kmers"], "total_kmers": st["total_kmers"],
                               "genome_length": st["genome_length"], "similar_to": kid, "similarity_score": score}
                dropped = True
                break
        if not dropped:
            info[ident] = {"kept": "yes", "unique_kmers": st["unique_kmers"], "total_kmers": st["total_kmers"],
                           "genome_length": st["genome_length"], "similar_to": "NA", "similarity_score": "NA"}
            kept.append(ident)
    keep_ids = set(kept)
    return [i for i, ident in enumerate(identifiers) if ident in keep_ids], info


def dumpref_summary(genomes: Sequence[Tuple[str, str]], k: int, kept_ids=None, similarity_info=None) -> dict:
    """KmerReference.get_summary() (src/kmer.py:300-329) restated on the
    reference's dict: ``genomes`` = (description, sequence) in FASTA order;
    ``kept_ids``: identifiers EXTSIM kept (None: no filtering)."""
    kmers: Dict[str, Dict[int, set]] = {}
    for gi, (_, seq) in enumerate(genomes):
        if k <= 0 or k > len(seq):  # extract_kmers_from_genome, src/kmer.py:84-94
            continue
        for pos in range(len(seq) - k + 1):
            km = seq[pos:pos + k]
            if "N" in km:  # src/kmer.py:145
                continue
            kmers.setdefault(km, {}).setdefault(gi, set()).add(pos)
    if kept_ids is not None:  # _remove_filtered_genomes_from_kmers, src/kmer.py:232-245
        for km in list(kmers):
            m = kmers[km]
            for gi in list(m):
                if genomes[gi][0] not in kept_ids:
                    del m[gi]
            if not m:
                del kmers[km]
    details = {km: {genomes[gi][0]: sorted(p) for gi, p in m.items()} for km, m in kmers.items()}
    summary: Dict[str, dict] = defaultdict(lambda: {"total_bases": 0, "unique_kmers": 0, "multi_mapping_kmers": 0})
    per: Dict[str, set] = defaultdict(set)
    for km, m in kmers.items():
        for gi in m:
            d = genomes[gi][0]
            summary[d]["total_bases"] = len(genomes[gi][1])
            per[d].add(km)
    for d, kms in per.items():
        u = sum(1 for km in kms if len(kmers[km]) == 1)
        summary[d]["unique_kmers"] = u
        summary[d]["multi_mapping_kmers"] = len(kms) - u
    out = {"Kmers": details, "Summary": dict(summary)}
    if similarity_info is not None:
        out["Similarity"] = similarity_info
    return out


def kmer_dict(seqs: Sequence[str], k: int) -> Dict[str, Dict[int, set]]:
    """The reference's ``kmers`` dict (src/kmer.py:135-150) keyed by genome
    index: {k-mer: {genome: positions}} in insertion order, 'N' k-mers skipped."""
    kmers: Dict[str, Dict[int, set]] = {}
    for gi, seq in enumerate(seqs):
        if k <= 0 or k > len(seq):  # src/kmer.py:84-94
            continue
        for pos in range(len(seq) - k + 1):
            km = seq[pos:pos + k]
            if "N" not in km:  # src/kmer.py:145
                kmers.setdefault(km, {}).setdefault(gi, set()).add(pos)
    return kmers


def reverse_complement(seq: str) -> str:
    """src/kmer.py:96-103: A<->T, C<->G, anything else kept, reversed."""
    return seq.translate(str.maketrans("ACGT", "TGCA"))[::-1]


def kmer_references(kmers: Dict[str, Dict[int, set]], kmer: str, reverse: bool = False) -> List[Tuple[int, List[int]]]:
    """get_kmer_references (src/kmer.py:292-298) or, with reverse,
    get_kmer_and_reverse_references (src/kmer.py:331-351): [(genome, sorted
    positions)] in the result dict's order."""
    out: Dict[int, set] = {g: set(p) for g, p in kmers.get(kmer, {}).items()}
    if reverse:
        rev = reverse_complement(kmer)
        if rev != kmer:
            for g, p in kmers.get(rev, {}).items():
                out.setdefault(g, set()).update(p)
    return [(g, sorted(p)) for g, p in out.items()]
