"""K-mer reference and pseudo-alignment, backed by the MI355X engine (libpa.so).

Drop-in for the reference's src/kmer.py: same names, constructor arguments,
attributes, return values and exceptions.  What changes is where the work runs:

* ``KmerReference`` builds a device-resident open-addressing hash table of
  2-bit-packed k-mers and their genome sets (``pa_index_build``) instead of
  ``Dict[str, Dict[Record, Set[int]]]`` (src/kmer.py:113-150).
* ``PseudoAlignment.align_reads_from_container`` ships the reads column-wise to
  HBM and classifies all of them in one kernel pass (``pa_align``,
  src/kmer.py:482-620); only per-genome counters and filter statistics come
  back.  ``PseudoAlignment.reads`` (per-read mapping types and genome lists)
  is materialised on first access by the per-read kernel (``pa_align_detail``).
* ``KmerReference.kmers`` -- positions included -- is an introspection view
  built on the host on first access; nothing on the align path reads it.
  ``KmerReference.get_summary`` (dumpref) is made on the device instead
  (``pa_index_dumpref``: k-mers in insertion order by a device sort, the JSON
  text streamed by host threads), so it scales to references whose dict the
  reference could not hold.
* ``.kdb`` / ``.aln`` files load through a restricted unpickler that admits
  only the classes such files hold -- this package's, or the reference's
  same-named ones, so files written by the reference load too.

Results (per-genome unique/ambiguous counts, filtered_* counters, the Summary
key order) are bit-exact to the reference; see DESIGN.md for the quirk list
this reproduces.  Known deviations: k above 255 raises PaUnsupported; argument
errors of a batch (TypeError / ValueError / AddingExistingRead) are raised
before any read of the batch is counted rather than at the offending read.
"""

from __future__ import annotations

import gzip
import json
import os
import pickle
import tempfile
from collections import defaultdict, namedtuple
from enum import Enum
from typing import Any, Dict, Iterator, List, Optional, Sequence, Set, Tuple, Union

import numpy as np

import constants
import pa_native as N
from records import FASTAQRecordContainer, FASTARecordContainer, Record

IGNORE_AMBIGUOUS_THRESHOLD = 0
M_THRESHOLD = 0
_NO_KEY = int(N.NO_FIRST_KEY)
_DROPPED = 0  # PA_DROPPED


class NotValidatingUniqueMapping(Exception):
    def __init__(self, message: str) -> None:
        super().__init__(message)


class AddingExistingRead(Exception):
    def __init__(self, message: str) -> None:
        super().__init__(message)


class ReadMappingType(Enum):
    UNMAPPED = 1
    UNIQUELY_MAPPED = 2
    AMBIGUOUSLY_MAPPED = 3


class KmerSpecifity(Enum):
    SPECIFIC = 1
    UNSPECIFIC = 2


ReadKmer = namedtuple("ReadKmer", ["specifity", "references"])
ReadMapping = namedtuple("ReadMapping", ["type", "genomes_mapped_to"])


def extract_k_max_value_keys_from_dict(d: Dict[str, int], k: int) -> List[str]:
    if not isinstance(d, dict):
        raise ValueError("Input must be a dictionary.")
    return sorted(d, key=lambda x: d[x], reverse=True)[:k] if d else []


def extract_kmers_from_genome(k: int, genome: str) -> Iterator[Tuple[int, str]]:
    """All (position, k-mer) windows of ``genome`` (src/kmer.py:84-94).

    Host helper kept for API compatibility; the engine extracts windows on
    the GPU (2-bit rolling keys in the build, funnel shifts in the align)."""
    if k > len(genome) or k <= 0:
        return iter([])
    return ((i, genome[i:i + k]) for i in range(len(genome) - k + 1))


def reverse_complement(seq: str) -> str:
    return seq.translate(str.maketrans("ACGT", "TGCA"))[::-1]


def _kmer_positions(genome: str, kmer: str) -> Set[int]:
    out, i = set(), genome.find(kmer)
    while i >= 0:
        out.add(i)
        i = genome.find(kmer, i + 1)
    return out


def _check_align_args(kmer_reference, m, p, mrq, mkq, mg, debug=False) -> Optional[Exception]:
    """The checks of Read.pseudo_align (src/kmer.py:501-510) as an exception, or None."""
    if not (isinstance(kmer_reference, KmerReference) and isinstance(m, int) and isinstance(p, int)
            and (mrq is None or isinstance(mrq, int)) and (mkq is None or isinstance(mkq, int))
            and (mg is None or isinstance(mg, int)) and isinstance(debug, bool)):
        return TypeError(f"Invalid types given to pseudo align: {type(kmer_reference)}, {type(p)}, {type(m)}, "
                         f"{type(debug)}")
    if m < M_THRESHOLD:
        return ValueError(f"m must be bigger than or equal to {M_THRESHOLD}")
    return None


def extsim_filter(index: N.Index, identifiers: Sequence[str], genome_lengths: Sequence[int],
                  similarity_threshold: float) -> Tuple[Set[str], Dict[str, Dict[str, Union[str, int, float]]]]:
    """EXTSIM greedy similar-genome filter (src/kmer.py:152-230) on a device index.

    Per-identifier statistics and pairwise intersections come from the GPU
    (``pa_index_extsim_stats``: distinct k-mers, specific k-mers, and shared
    k-mers of every pair of identifiers, src/kmer.py:152-177); the greedy pass
    is the reference's: genomes sorted ascending by (unique, total, length,
    order), each compared with the kept ones in keep order by the overlap
    coefficient |A & B| / min(|A|, |B|) (0 if min is 0) and dropped on the first
    score strictly above the threshold.  Returns (kept identifiers,
    similarity_info).  Duplicate identifiers form one group, later records
    overwriting the length/order of earlier ones, as in the reference."""
    gid: Dict[str, int] = {}
    group_of = [gid.setdefault(i, len(gid)) for i in identifiers]
    total, uniq, inter = index.extsim_stats(group_of, len(gid))
    stats: Dict[str, Dict[str, int]] = {}
    for order, (ident, glen) in enumerate(zip(identifiers, genome_lengths)):
        a = gid[ident]
        stats[ident] = {"unique_kmers": int(uniq[a]), "total_kmers": int(total[a]), "genome_length": int(glen),
                        "order": order}
    ordered = sorted(stats.items(), key=lambda x: (x[1]["unique_kmers"], x[1]["total_kmers"],
                                                   x[1]["genome_length"], x[1]["order"]))
    kept: List[str] = []
    info: Dict[str, Dict[str, Union[str, int, float]]] = {}
    for ident, st in ordered:
        a = gid[ident]
        similar_to = None
        for kid in kept:
            b = gid[kid]
            min_count = min(int(total[a]), int(total[b]))
            score = (int(inter[a, b]) / min_count) if min_count > 0 else 0
            if score > similarity_threshold:  # overlap coefficient, strict (src/kmer.py:206-208)
                similar_to = (kid, score)
                break
        base = {"unique_kmers": st["unique_kmers"], "total_kmers": st["total_kmers"],
                "genome_length": st["genome_length"]}
        if similar_to is None:
            info[ident] = {"kept": "yes", **base, "similar_to": "NA", "similarity_score": "NA"}
            kept.append(ident)
        else:
            info[ident] = {"kept": "no", **base, "similar_to": similar_to[0], "similarity_score": similar_to[1]}
    return set(kept), info


class _KdbUnpickler(pickle.Unpickler):
    """Loader of .kdb / .aln files (src/kmer.py:265-282, 671-699): only the
    classes such files hold are resolved -- this package's, whose module and
    class names are the reference's own (kmer.KmerReference, records.Record,
    ...), so a file written by the reference resolves to these classes and
    their __setstate__ converts its state.  Anything else is refused."""

    _OWN = {("kmer", n) for n in ("KmerReference", "PseudoAlignment", "ReadMappingType", "KmerSpecifity",
                                  "ReadMapping", "ReadKmer")} | {("records", "Record")}
    _LIB = {("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
            ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
            ("numpy._core.multiarray", "scalar"), ("builtins", "set"), ("builtins", "frozenset"),
            ("collections", "defaultdict"), ("collections", "OrderedDict")}

    def find_class(self, module: str, name: str):
        if (module, name) in self._OWN:
            if module == "records":
                import records
                return getattr(records, name)
            return globals()[name]
        if (module, name) in self._LIB:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"{module}.{name} is not a class a .kdb / .aln file holds")


def _load_pickle(path: str):
    with gzip.open(path, "rb") as f:
        return _KdbUnpickler(f).load()


def _write_fd(fd: int, data: bytes) -> None:
    view = memoryview(data)
    while view:
        view = view[os.write(fd, view):]


class KmerReference:
    """Device-resident k-mer reference of a FASTA container (src/kmer.py:109-351)."""

    def __init__(self, k: int, fasta_record_container: FASTARecordContainer, filter_similar: bool = False,
                 similarity_threshold: float = 0.95, device: Optional[int] = None, *,
                 compact_table: bool = False) -> None:
        """compact_table (not in the reference): the k-mer table at 2 slots per
        genome window (PA_BUILD_COMPACT) -- for a job of few reads per genome
        base, as the CLI's dumpalign / align jobs are (main.create_reference)."""
        if filter_similar and not (0 <= similarity_threshold <= 1):
            raise ValueError("similarity_threshold must be between 0 and 1")
        if not isinstance(k, int):
            raise TypeError(f"k must be an int, got {type(k)}")
        self.genomes: List[Record] = list(fasta_record_container)
        pg = getattr(fasta_record_container, "packed_genomes", None)
        self._packed = pg(self.genomes) if pg is not None else None  # (the parser's concatenated genomes)
        self._all_genomes: Optional[List[Record]] = None  # before EXTSIM dropped any (k-mer view order)
        self._ref_kmers: Optional[Dict[str, Dict[Record, Set[int]]]] = None  # the dict of a reference-written .kdb
        self.kmer_len: int = k
        self._device = N.default_device() if device is None else int(device)
        self._compact = bool(compact_table)
        self._build()
        if filter_similar:
            self._filter_similar_genomes(similarity_threshold)

    # -- device index -------------------------------------------------------

    def _build(self) -> None:
        # the align-side view (tiles, neighbour bits) is made at the first align:
        # an index that EXTSIM then rebuilds from the kept genomes never needs it
        packed, self._packed = getattr(self, "_packed", None), None  # (only for the first build)
        self._index = N.Index(None if packed is not None else [g["genome"] for g in self.genomes], self.kmer_len,
                              device=self._device, defer_tiles=True, packed=packed,
                              compact=getattr(self, "_compact", False))
        self._view: Optional[Dict[str, Dict[Record, Set[int]]]] = None

    @property
    def index(self) -> N.Index:
        return self._index

    @property
    def n_kmers(self) -> int:
        """Number of distinct k-mers (== len(self.kmers))."""
        return self._index.n_kmers

    # -- EXTSIM (src/kmer.py:152-263) --------------------------------------

    def _filter_similar_genomes(self, similarity_threshold: float) -> None:
        keep, info = extsim_filter(self._index, [g.identifier for g in self.genomes],
                                   [len(g["genome"]) for g in self.genomes], similarity_threshold)
        if len(keep) != len({g.identifier for g in self.genomes}):
            sel = [i for i, g in enumerate(self.genomes) if g.identifier in keep]
            # pruning dropped genomes == building from the kept ones: in place,
            # from their codes already on the device (pa_index_reduce); the
            # genome lists change only once that succeeded
            self._index.reduce(sel)
            self._all_genomes = self.genomes
            self.genomes = [self.genomes[i] for i in sel]
            self._view = None
        self.similarity_info = info

    # -- persistence ----------------------------------------------------------

    def __getstate__(self):
        state = {k: v for k, v in self.__dict__.items() if k not in ("_index", "_view", "_packed")}
        return state

    def __setstate__(self, state):
        if "kmers" in state and "_device" not in state:
            # written by the reference (src/kmer.py:265-282): genomes (the kept
            # ones after EXTSIM), kmer_len, its kmers dict, similarity_info.  The
            # device index is built from the genomes; the dict stays the k-mer
            # view, since after EXTSIM its order comes from genomes the file no
            # longer holds.
            self.genomes = list(state["genomes"])
            self.kmer_len = state["kmer_len"]
            self._all_genomes = None
            self._device = N.default_device()
            if "similarity_info" in state:
                self.similarity_info = state["similarity_info"]
            self._build()
            self._ref_kmers = state["kmers"]
            self._view = self._ref_kmers
            return
        self.__dict__.update(state)
        self.__dict__.setdefault("_ref_kmers", None)
        self._build()
        if self._ref_kmers is not None:
            self._view = self._ref_kmers

    def save(self, ref_file: str) -> None:
        with gzip.open(ref_file, "wb") as f:
            pickle.dump(self, f)

    @classmethod
    def load(cls, ref_file: str) -> "KmerReference":
        return _load_pickle(ref_file)  # (any object, as pickle.load)

    # -- lookups ----------------------------------------------------------------

    @property
    def kmers(self) -> Dict[str, Dict[Record, Set[int]]]:
        """Introspection view ``{kmer: {Record: positions}}`` in the reference's
        insertion order (built on the host on first access; not used to align)."""
        if self._view is None:
            # After EXTSIM the reference deletes the dropped genomes' entries from
            # the full dict (src/kmer.py:232-245): the remaining k-mers keep the
            # order of the full build, so walk every original genome and keep
            # the kept ones' positions only.
            kept = None if self._all_genomes is None else {id(g) for g in self.genomes}
            view: Dict[str, Dict[Record, Set[int]]] = {}
            for rec in (self.genomes if kept is None else self._all_genomes):
                keep = kept is None or id(rec) in kept
                for pos, km in extract_kmers_from_genome(self.kmer_len, rec["genome"]):
                    if constants.NULL_NUCLEOTIDES_CHAR not in km:
                        entry = view.setdefault(km, {})
                        if keep:
                            entry.setdefault(rec, set()).add(pos)
            self._view = view if kept is None else {km: gs for km, gs in view.items() if gs}
        return self._view

    def _genome_set(self, kmer: str) -> List[int]:
        cls, _ = self._index.lookup([kmer])
        return [] if cls[0] < 0 else self._index.class_genomes(int(cls[0]))

    def _references(self, kmer: str, reverse: bool) -> Dict[Record, Set[int]]:
        """{genome record: positions} of the k-mer (and of its reverse complement)
        from the device index (pa_index_positions): genomes in FASTA order, the
        reverse complement's new genomes after the k-mer's own, as the
        reference's dict merge orders them (src/kmer.py:338-351)."""
        out: Dict[Record, Set[int]] = {}
        for q, g, p in self._index.positions([kmer], reverse).tolist():
            out.setdefault(self.genomes[g], set()).add(p)
        return out

    def _references_many(self, kmers: List[str]) -> List[Dict[Record, Set[int]]]:
        """get_kmer_references of every k-mer of the list: one device scan
        (pa_index_positions over the whole batch), hits split by query."""
        if self._view is not None:
            return [self._view.get(km, {}) for km in kmers]
        out: List[Dict[Record, Set[int]]] = [{} for _ in kmers]
        if kmers:
            for q, g, p in self._index.positions(kmers, False).tolist():
                out[q].setdefault(self.genomes[g], set()).add(p)
        return out

    def get_kmer_references(self, kmer: str) -> Dict[Record, Set[int]]:
        if self._view is not None:
            return self._view.get(kmer, {})
        return self._references(kmer, False)

    def __getitem__(self, kmer: str) -> Optional[Dict[Record, Set[int]]]:
        return self.get_kmer_references(kmer) or None

    def get_kmer_and_reverse_references(self, kmer: str) -> Dict[Record, Set[int]]:
        if self._view is None:
            return self._references(kmer, True)
        result: Dict[Record, Set[int]] = {g: set(p) for g, p in self.get_kmer_references(kmer).items()}
        rev = reverse_complement(kmer)
        if rev != kmer:
            for g, p in self.get_kmer_references(rev).items():
                result.setdefault(g, set()).update(p)
        return result

    # -- dumpref (src/kmer.py:300-329) ---------------------------------------------

    def write_summary(self, fd: int) -> None:
        """``json.dumps(self.get_summary(), indent=4)`` written to file descriptor
        ``fd`` (no final line break): the "Kmers" object streamed from the device
        index by pa_index_dumpref, then Summary (and Similarity) from its counts."""
        if self._ref_kmers is not None:  # a reference-written .kdb: its own dict is the k-mer order
            _write_fd(fd, json.dumps(self._summary_from_view(), indent=4).encode())
            return
        if self._all_genomes is None:
            index, genomes, keep, tmp = self._index, self.genomes, None, False
        else:
            # EXTSIM dropped genomes: the reference deletes their entries from the
            # full dict (src/kmer.py:232-245), so the k-mers keep the full
            # build's order -- dump an index of every original genome, masked
            genomes = self._all_genomes
            index = N.Index([g["genome"] for g in genomes], self.kmer_len, device=self._device, defer_tiles=True)
            kept = {id(g) for g in self.genomes}
            keep = np.fromiter((id(g) in kept for g in genomes), dtype=np.uint8, count=len(genomes))
            tmp = True
        descs: Dict[str, int] = {}
        desc_of = np.empty(len(genomes), dtype=np.uint32)
        for i, g in enumerate(genomes):
            desc_of[i] = descs.setdefault(g["description"], len(descs))
        names = list(descs)
        try:
            _write_fd(fd, b'{\n    "Kmers": ')
            uniq, multi, order, last, _ = N.index_dumpref(index, keep, desc_of, [json.dumps(d) for d in names], fd)
        finally:
            if tmp:
                index.close()
        present = sorted((d for d in range(len(names)) if int(order[d]) != N.NO_ORDER), key=lambda d: int(order[d]))
        summary = {names[d]: {"total_bases": len(genomes[int(last[d])]["genome"]), "unique_kmers": int(uniq[d]),
                              "multi_mapping_kmers": int(multi[d])} for d in present}
        tail: Dict[str, Any] = {"Kmers": 0, "Summary": summary}
        if hasattr(self, "similarity_info"):
            tail["Similarity"] = self.similarity_info
        text = json.dumps(tail, indent=4)
        _write_fd(fd, text[text.index('"Kmers": 0') + len('"Kmers": 0'):].encode())

    def get_summary(self) -> Dict[str, Any]:
        """dumpref summary (src/kmer.py:300-329): {"Kmers", "Summary"[, "Similarity"]}."""
        if self._ref_kmers is not None:
            return self._summary_from_view()
        with tempfile.TemporaryFile() as f:
            self.write_summary(f.fileno())
            f.seek(0)
            return json.loads(f.read())

    def _summary_from_view(self) -> Dict[str, Any]:
        """The same summary from the host view (a reference-written .kdb's dict)."""
        kmers = self.kmers
        details = {km: {g["description"]: sorted(p) for g, p in gs.items()} for km, gs in kmers.items()}
        summary: Dict[str, Dict[str, int]] = defaultdict(
            lambda: {"total_bases": 0, "unique_kmers": 0, "multi_mapping_kmers": 0})
        per_genome: Dict[str, Set[str]] = defaultdict(set)
        for km, gs in kmers.items():
            for g in gs:
                summary[g["description"]]["total_bases"] = len(g["genome"])
                per_genome[g["description"]].add(km)
        for desc, kms in per_genome.items():
            uniq = sum(1 for km in kms if len(kmers[km]) == 1)
            summary[desc]["unique_kmers"] = uniq
            summary[desc]["multi_mapping_kmers"] = len(kms) - uniq
        out = {"Kmers": details, "Summary": dict(summary)}
        if hasattr(self, "similarity_info"):
            out["Similarity"] = self.similarity_info
        return out


class Read:
    """One FASTQ read (src/kmer.py:357-526); pseudo_align runs on the GPU."""

    def __init__(self, fastaq_record: Record) -> None:
        self.identifier = fastaq_record.identifier
        self.mapping = ReadMapping(ReadMappingType.UNMAPPED, [])
        self.__raw_read: str = fastaq_record["sequence"]
        self.__quality_scores: str = fastaq_record["quality_sequence"]
        self.num_quality_filtered_kmers: int = 0
        self.num_redundant_kmers: int = 0
        self._kmers: Dict[str, ReadKmer] = {}
        self._kmer_args = None

    def __str__(self) -> str:
        rows = [f"Mapping: {self.mapping}"]
        for kmer, rk in self.kmers.items():
            rows += [f"k-mer: {kmer}", f"specifity: {rk.specifity}", "Genome References:"]
            rows += [f"\t{ref}" for ref in rk.references]
        return "\n".join(rows)

    __repr__ = __str__

    def mean_quality(self) -> float:
        return sum(map(ord, self.__quality_scores)) / len(self.__quality_scores)

    def kmer_quality(self, start: int, k: int) -> float:
        return sum(map(ord, self.__quality_scores[start:start + k])) / k

    @property
    def kmers(self) -> Dict[str, ReadKmer]:
        """The read's distinct indexed k-mers (src/kmer.py:410-429), from GPU lookups."""
        if self._kmer_args is not None:
            ref, mkq, mg = self._kmer_args
            self._kmer_args = None
            k = ref.kmer_len
            windows = list(extract_kmers_from_genome(k, self.__raw_read))
            cls, size = ref.index.lookup([w for _, w in windows]) if windows else ([], [])
            kept: Dict[str, int] = {}  # included k-mer -> its set size, first inclusion order
            for (start, km), c, s in zip(windows, cls, size):
                if mkq is not None and self.kmer_quality(start, k) < mkq:
                    continue
                if c < 0 or (mg is not None and int(s) > mg):
                    continue
                kept.setdefault(km, int(s))
            # every included k-mer's references from one batched device scan
            names = list(kept)
            for km, refs in zip(names, ref._references_many(names)):
                self._kmers[km] = ReadKmer(KmerSpecifity.SPECIFIC if kept[km] == 1 else KmerSpecifity.UNSPECIFIC, refs)
        return self._kmers

    def _packed(self):
        seq = np.frombuffer(self.__raw_read.encode("ascii", errors="replace"), dtype=np.uint8)
        qual = np.frombuffer(self.__quality_scores.encode("latin-1", errors="replace"), dtype=np.uint8)
        return seq, qual, np.array([0, seq.size], dtype=np.uint64)

    def pseudo_align(self, kmer_reference: KmerReference, m: int = 1, p: int = 1,
                     min_read_quality: Optional[int] = None, min_kmer_quality: Optional[int] = None,
                     max_genomes: Optional[int] = None, debug: bool = False) -> ReadMappingType:
        err = _check_align_args(kmer_reference, m, p, min_read_quality, min_kmer_quality, max_genomes, debug)
        if err is not None:
            raise err
        if min_read_quality is not None and self.mean_quality() < min_read_quality:
            return ReadMappingType.UNMAPPED
        seq, qual, off = self._packed()
        reads = N.Reads.upload(seq, qual, off, device=kmer_reference.index.device)
        prm = N.Params.make(m, p, None, min_kmer_quality, max_genomes)
        types, qf, hr, loff, lists = N.align_detail(kmer_reference.index, reads, prm)
        reads.close()
        self.num_quality_filtered_kmers += int(qf[0])
        self.num_redundant_kmers += int(hr[0])
        self._kmer_args = (kmer_reference, min_kmer_quality, max_genomes)
        t = ReadMappingType(int(types[0]))
        if t != ReadMappingType.UNMAPPED:
            self.mapping = ReadMapping(t, [kmer_reference.genomes[int(g)] for g in lists[loff[0]:loff[1]]])
        if debug:
            print(f"[DEBUG pseudo_align]: self.mapping: {self.mapping.type}, mapped to: {self.mapping}")
        return t


class _Batch:
    """A container batch aligned on the GPU, kept for lazy per-read results.
    ``all_dropped``: every read failed --min-read-quality on the host (no GPU
    pass was needed, see _align_columns)."""

    __slots__ = ("base", "ids", "seq", "qual", "off", "params", "mrq", "entries", "all_dropped", "_dropped")

    def __init__(self, base, ids, seq, qual, off, params, mrq, all_dropped=False):
        self.base, self.ids, self.seq, self.qual, self.off, self.params = base, ids, seq, qual, off, params
        self.mrq, self.all_dropped, self.entries, self._dropped = mrq, all_dropped, None, None

    def load(self) -> None:
        pass

    def dropped(self) -> Optional[np.ndarray]:
        """Reads dropped by --min-read-quality (not in PseudoAlignment.reads), or None if none can be."""
        self.load()
        if self.all_dropped:
            return np.ones(len(self.ids), dtype=bool)
        if self.mrq is None:
            return None
        if self._dropped is None:
            self._dropped = _dropped_mask(self.qual, self.off, self.mrq)
        return self._dropped


class _FileBatch(_Batch):
    """A FASTQ file aligned by pa_align_fastq_file: its columns (ids, bases,
    qualities) are parsed from the file only when per-read results or ids are
    asked for."""

    __slots__ = ("path", "n")

    def __init__(self, base, path, params, mrq, n):
        super().__init__(base, None, None, None, None, params, mrq)
        self.path, self.n = path, n

    def load(self) -> None:
        if self.ids is None:
            from data_file import FASTAQFile
            self.ids, self.seq, self.qual, self.off = _columnar(FASTAQFile(self.path).container)


def _dropped_mask(qual: np.ndarray, off: np.ndarray, mrq) -> np.ndarray:
    """Read.mean_quality() < min_read_quality per read (src/kmer.py:394-399, 587),
    raw ASCII: an exact integer test for an int threshold, the reference's own
    float division (IEEE double, as numpy's) otherwise."""
    off = np.asarray(off, dtype=np.int64)
    lens = np.diff(off)
    n = lens.size
    sums = np.zeros(n, dtype=np.int64)
    if qual.size and n:
        nz = lens > 0
        sums[nz] = np.add.reduceat(qual.astype(np.int64), off[:-1][nz])
    if isinstance(mrq, int):
        return sums < int(mrq) * lens
    with np.errstate(divide="ignore", invalid="ignore"):
        return (sums / lens) < float(mrq)


def _columnar(container) -> Tuple[List[str], np.ndarray, np.ndarray, np.ndarray]:
    if isinstance(container, FASTAQRecordContainer):
        return container.id_sequence(), container.seq, container.qual, container.offsets
    ids, seqs, quals = [], [], []
    for rec in container:
        ids.append(rec.identifier)
        seqs.append(rec["sequence"])
        quals.append(rec["quality_sequence"])
    seq, off = N.concat(seqs)
    qual, _ = N.concat(quals)
    return ids, seq, qual, off


class PseudoAlignment:
    """Pseudo-alignment of reads against a KmerReference (src/kmer.py:532-699)."""

    def __init__(self, kmer_reference: KmerReference) -> None:
        self.kmer_reference: KmerReference = kmer_reference
        self.filtered_quality_reads: int = 0
        self.filtered_quality_kmers: int = 0
        self.filtered_hr_kmers: int = 0
        self.filter_read_quality_flag: bool = False
        self.filter_kmer_quality_flag: bool = False
        self.filter_max_genomes_flag: bool = False
        self._next_index = 0
        self._result: Optional[N.Result] = None
        self._gpu_stats = np.zeros(6, dtype=np.uint64)
        self._batches: List[_Batch] = []
        self._host: List[Tuple[int, str, Dict[str, Any]]] = []  # (index, id, entry) of add_read()
        self._ids: Optional[Set[str]] = None

    # -- bookkeeping ------------------------------------------------------------

    def _known_ids(self) -> Set[str]:
        """Identifiers already in ``reads`` (src/kmer.py:557): reads dropped by
        --min-read-quality never entered it."""
        if self._ids is None:
            ids: Set[str] = set()
            for b in self._batches:
                d = b.dropped()  # (loads a file batch's columns)
                ids.update(b.ids if d is None else (i for i, x in zip(b.ids, d) if not x))
            ids.update(i for _, i, _ in self._host)
            self._ids = ids
        return self._ids

    def _add_ids(self, ids: Sequence[str], dropped: Optional[np.ndarray], unique_batch: bool) -> None:
        """AddingExistingRead for an identifier already aligned -- before or
        earlier in this batch (src/kmer.py:557-558).  ``unique_batch``: the ids
        come from one parsed FASTQ container, which the grammar made unique."""
        if not self._batches and not self._host and unique_batch:
            return
        known = self._known_ids()
        seen: Set[str] = set()
        for i, rid in enumerate(ids):
            if dropped is not None and dropped[i]:
                continue
            if rid in known or (not unique_batch and rid in seen):
                raise AddingExistingRead(f"There already exists a read with identifier: {rid}")
            if not unique_batch:
                seen.add(rid)

    def add_read(self, read: Read) -> None:
        self._add_ids([read.identifier], None, False)
        if self._ids is not None:
            self._ids.add(read.identifier)
        entry = {"mapping_type": read.mapping.type,
                 "genomes_mapped_to": [g.identifier for g in read.mapping.genomes_mapped_to]}
        self._host.append((self._next_index, read.identifier, entry))
        self._next_index += 1

    def add_read_from_read_record(self, read_record: Record, m: int = 1, p: int = 1,
                                  min_read_quality: Optional[int] = None, min_kmer_quality: Optional[int] = None,
                                  max_genomes: Optional[int] = None) -> None:
        ids = [read_record.identifier]
        seq, off = N.concat([read_record["sequence"]])
        qual = np.frombuffer(read_record["quality_sequence"].encode("latin-1", errors="replace"), dtype=np.uint8)
        self._align_columns(ids, seq, qual, off, m, p, min_read_quality, min_kmer_quality, max_genomes)

    def align_reads_from_container(self, reads_container: FASTAQRecordContainer, m: int = 1, p: int = 1,
                                   min_read_quality: Optional[int] = None, min_kmer_quality: Optional[int] = None,
                                   max_genomes: Optional[int] = None) -> None:
        ids, seq, qual, off = _columnar(reads_container)
        self._align_columns(ids, seq, qual, off, m, p, min_read_quality, min_kmer_quality, max_genomes,
                            unique_batch=isinstance(reads_container, FASTAQRecordContainer))

    def align_reads_from_file(self, reads_file: str, m: int = 1, p: int = 1, min_read_quality: Optional[int] = None,
                              min_kmer_quality: Optional[int] = None, max_genomes: Optional[int] = None, *,
                              prefetch: Optional["N.FastqPrefetch"] = None) -> None:
        """FASTAQFile(reads_file).container + align_reads_from_container as one
        device pass (pa_align_fastq_file: the file is parsed on the GPU and
        aligned in windows while the host reads the next).  Per-read results
        (``reads``) parse the file again when asked for.  A file outside the
        device-parsed subset of the grammar, a duplicate id, arguments the
        reference rejects, or reads already added take the exact path.
        ``prefetch``: the same file already on its way to the device
        (N.FastqPrefetch, started before the index build); consumed here."""
        from data_file import FASTAQFile
        fresh = not self._batches and not self._host and self._result is None
        err = _check_align_args(self.kmer_reference, m, p, min_read_quality, min_kmer_quality, max_genomes)
        n = None
        if fresh and err is None and os.environ.get("PA_STREAM", "1") != "0":
            FASTAQFile.check_extension(reads_file)
            ref = self.kmer_reference
            result = N.Result(ref.index)
            prm = N.Params.make(m, p, min_read_quality, min_kmer_quality, max_genomes)
            if prefetch is not None and prefetch.device == ref.index.device:
                n = N.align_fastq_prefetched(ref.index, prefetch, prm, self._next_index, result)
            else:
                n = N.align_fastq_file(ref.index, reads_file, prm, self._next_index, result)
            if n is None:
                result.close()
        if prefetch is not None:
            prefetch.close()
        if n is None:
            self.align_reads_from_container(FASTAQFile(reads_file).container, m, p, min_read_quality,
                                            min_kmer_quality, max_genomes)
            return
        if min_read_quality is not None:
            self.filter_read_quality_flag = True
        if min_kmer_quality is not None:
            self.filter_kmer_quality_flag = True
        if max_genomes is not None:
            self.filter_max_genomes_flag = True
        self._result = result
        stats, _, _, _ = result.fetch()
        self._gpu_stats = stats
        self.filtered_quality_reads += int(stats[3])
        self.filtered_quality_kmers += int(stats[4])
        self.filtered_hr_kmers += int(stats[5])
        self._batches.append(_FileBatch(self._next_index, reads_file, prm, min_read_quality, n))
        self._next_index += n
        self._streamed_records = n  # (diagnostics: the device-parsed path was taken)

    def _align_columns(self, ids, seq, qual, off, m, p, mrq, mkq, mg, unique_batch=False) -> None:
        n = len(ids)
        if n == 0:
            return
        if mrq is not None:
            self.filter_read_quality_flag = True
        if mkq is not None:
            self.filter_kmer_quality_flag = True
        if mg is not None:
            self.filter_max_genomes_flag = True
        err = _check_align_args(self.kmer_reference, m, p, mrq, mkq, mg)
        all_dropped = False
        if err is not None:
            # the reference checks the arguments (Read.pseudo_align) only for
            # reads that pass --min-read-quality (src/kmer.py:587-592): a batch
            # whose every read is dropped by it is only counted
            if mrq is None or isinstance(mrq, bool) or not isinstance(mrq, (int, float)):
                raise err
            if not _dropped_mask(qual, off, mrq).all():
                raise err
            all_dropped = True
        dropped = _dropped_mask(qual, off, mrq) if (mrq is not None and (self._batches or self._host
                                                                          or not unique_batch)) else None
        self._add_ids(ids, np.ones(n, dtype=bool) if all_dropped else dropped, unique_batch)
        ref = self.kmer_reference
        prm = None
        if all_dropped:
            self.filtered_quality_reads += n
        else:
            if self._result is None:
                self._result = N.Result(ref.index)
            prm = N.Params.make(m, p, mrq, mkq, mg)
            # the align-side view this batch repays (the neighbour bits only
            # past their break-even in reads per genome base; pa_index_prepare_ex)
            ref.index.prepare(expected_reads=n)
            reads = N.Reads.upload(seq, qual, off, device=ref.index.device)
            N.align(ref.index, reads, prm, self._next_index, self._result)
            stats, _, _, _ = self._result.fetch()
            reads.close()
            delta = stats - self._gpu_stats
            self._gpu_stats = stats
            self.filtered_quality_reads += int(delta[3])
            self.filtered_quality_kmers += int(delta[4])
            self.filtered_hr_kmers += int(delta[5])
        b = _Batch(self._next_index, ids, seq, qual, off, prm, mrq, all_dropped)
        b._dropped = dropped
        self._batches.append(b)
        if self._ids is not None:
            d = b.dropped()
            self._ids.update(ids if d is None else (i for i, x in zip(ids, d) if not x))
        self._next_index += n

    # -- results ----------------------------------------------------------------

    @property
    def reads(self) -> Dict[str, Dict[str, Any]]:
        """``{read id: {"mapping_type", "genomes_mapped_to"}}`` in insertion order;
        reads dropped by --min-read-quality are absent (src/kmer.py:587-589)."""
        ref = self.kmer_reference
        items: List[Tuple[int, str, Dict[str, Any]]] = list(self._host)
        for b in self._batches:
            if b.all_dropped:
                continue
            if b.entries is None:
                b.load()
                reads = N.Reads.upload(b.seq, b.qual, b.off, device=ref.index.device)
                types, _, _, loff, lists = N.align_detail(ref.index, reads, b.params)
                reads.close()
                names = [g.identifier for g in ref.genomes]
                ent = []
                for i, t in enumerate(types):
                    if t == _DROPPED:  # filtered by --min-read-quality: not a read of the alignment
                        continue
                    gl = [names[int(g)] for g in lists[loff[i]:loff[i + 1]]]
                    ent.append((b.base + i, b.ids[i], {"mapping_type": ReadMappingType(int(t)),
                                                       "genomes_mapped_to": gl}))
                b.entries = ent
            items.extend(b.entries)
        items.sort(key=lambda x: x[0])
        return {rid: e for _, rid, e in items}

    def get_summary(self) -> Dict[str, Dict[str, Union[int, Dict[str, int]]]]:
        stats = self._gpu_stats.astype(np.int64)
        summary: Dict[str, Union[int, Dict[str, int]]] = {
            "unique_mapped_reads": int(stats[0]),
            "ambiguous_mapped_reads": int(stats[1]),
            "unmapped_reads": int(stats[2]),
        }
        if self.filter_read_quality_flag:
            summary["filtered_quality_reads"] = self.filtered_quality_reads
        if self.filter_kmer_quality_flag:
            summary["filtered_quality_kmers"] = self.filtered_quality_kmers
        if self.filter_max_genomes_flag:
            summary["filtered_hr_kmers"] = self.filtered_hr_kmers
        counts: Dict[str, List[int]] = {}
        first: Dict[str, int] = {}
        if self._result is not None:
            _, uq, am, fk = self._result.fetch()
            for g in np.flatnonzero(fk != N.NO_FIRST_KEY):
                name = self.kmer_reference.genomes[int(g)].identifier
                c = counts.setdefault(name, [0, 0])
                c[0] += int(uq[g])
                c[1] += int(am[g])
                first[name] = min(first.get(name, _NO_KEY), int(fk[g]))
        for idx, _, e in self._host:
            t = e["mapping_type"]
            if t == ReadMappingType.UNMAPPED:
                summary["unmapped_reads"] += 1
                continue
            col = 0 if t == ReadMappingType.UNIQUELY_MAPPED else 1
            summary["unique_mapped_reads" if col == 0 else "ambiguous_mapped_reads"] += 1
            for pos, name in enumerate(e["genomes_mapped_to"]):
                counts.setdefault(name, [0, 0])[col] += 1
                first[name] = min(first.get(name, _NO_KEY), (idx << 20) | pos)
        genome_mapping = {name: {"unique_reads": counts[name][0], "ambiguous_reads": counts[name][1]}
                          for name in sorted(first, key=first.get)}
        return {"Statistics": summary, "Summary": genome_mapping}

    def get_reads_by_mapping_type(self, mapping_type: ReadMappingType) -> List[str]:
        return [rid for rid, d in self.reads.items() if d["mapping_type"] == mapping_type]

    def export_summary_to_json(self, json_file: str) -> None:
        with open(json_file, "w") as f:
            json.dump(self.get_summary(), f, indent=4)

    def __repr__(self) -> str:
        return json.dumps(self.get_summary(), indent=4)

    # -- persistence: per-read results are materialised, device state dropped ----

    def __getstate__(self):
        reads = self.reads
        state = {k: v for k, v in self.__dict__.items() if k not in ("_result", "_batches", "_host", "_ids")}
        state["_host"] = [(i, rid, e) for i, (rid, e) in enumerate(reads.items())]
        state["_next_index"] = len(reads)
        state["_gpu_stats"] = np.zeros(6, dtype=np.uint64)
        return state

    def __setstate__(self, state):
        if "reads" in state and "_host" not in state:
            # written by the reference (src/kmer.py:536-548, 659-699): its reads
            # dict becomes the host entries, in the same order
            reads = state.pop("reads")
            state["_host"] = [(i, rid, e) for i, (rid, e) in enumerate(reads.items())]
            state["_next_index"] = len(reads)
            state["_gpu_stats"] = np.zeros(6, dtype=np.uint64)
        self.__dict__.update(state)
        self._result = None
        self._batches = []
        self._ids = None

    def save(self, align_file: str) -> None:
        with gzip.open(align_file, "wb") as f:
            pickle.dump(self, f)

    @classmethod
    def load(cls, align_file: str) -> "PseudoAlignment":
        return _load_pickle(align_file)  # (any object, as pickle.load)
