"""ctypes binding of libpa.so (include/pa.h).

This is the only module that talks to the native library.  There is no CPU
fallback: if libpa.so is missing or no HIP device is visible, every call fails
loudly (ImportError / PaDeviceError).
"""

from __future__ import annotations

import ctypes
import os
import sys
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_TIMING = os.environ.get("PA_CLI_TIMING") == "1"  # (diagnostic stage times on stderr)
LIB_PATH = os.environ.get("PA_LIBRARY", os.path.join(HERE, "libpa.so"))

PA_OK, PA_EINVAL, PA_ETYPE, PA_ENOMEM, PA_EDEVICE, PA_EUNSUPPORTED, PA_EINTERNAL, PA_ENOTCANON, PA_EIO = range(9)
PA_FASTA, PA_FASTQ = 0, 1
PA_MAX_K = 255
PA_MAX_GENOMES = (1 << 20) - 1
PA_COMM_ID_BYTES = 128
HAS_MRQ, HAS_MKQ, HAS_MG = 1, 2, 4
NO_FIRST_KEY = np.uint64(2 ** 63 - 1)  # PA_NO_FIRST_KEY
PA_BUILD_DEFER_TILES = 1
PA_BUILD_COMPACT = 2
PA_COMPACT_READS_PER_BASE = 3  # (include/pa.h: the measured break-even of the compact table)
PA_POS_REVERSE, PA_POS_RC_BIT = 1, 0x80000000
PA_READS_UNKNOWN = 2 ** 64 - 1
PA_NB_READS_PER_KBASE = 2500  # (include/pa.h: the neighbour bits' break-even, reads per 1000 genome bases)
PA_NB_READS_PER_KBASE_2W, PA_NB_READS_PER_KBASE_3W = 10000, 18000  # (two- / three-word keys)

# every symbol declared in include/pa.h
EXPORTS = (
    "pa_last_error", "pa_version", "pa_device_count", "pa_runtime_start",
    "pa_index_build", "pa_index_build_ex", "pa_index_reduce", "pa_index_prepare", "pa_index_prepare_ex", "pa_index_free", "pa_index_get_info", "pa_index_lookup", "pa_index_class_genomes",
    "pa_index_positions",
    "pa_index_extsim_stats", "pa_index_dumpref",
    "pa_reads_upload", "pa_reads_synthesize", "pa_reads_synthesize_mix", "pa_reads_info", "pa_params_effective",
    "pa_reads_download", "pa_reads_free",
    "pa_result_create", "pa_result_reset", "pa_result_fetch", "pa_result_device_view", "pa_result_copy_out",
    "pa_result_copy_in", "pa_result_load", "pa_result_free",
    "pa_align", "pa_align_detail", "pa_align_batch", "pa_align_fastq_file", "pa_align_fastq_range",
    "pa_idsets_disjoint", "pa_idset_free",
    "pa_fastq_prefetch_start", "pa_align_fastq_prefetched", "pa_fastq_prefetch_free",
    "pa_comm_unique_id", "pa_comm_init", "pa_comm_free", "pa_comm_count", "pa_counters_reduce",
    "pa_profile_enable", "pa_profile_read", "pa_profile_read_kernels", "pa_mem_trim",
    "pa_parse_text", "pa_parse_file", "pa_seqset_sizes", "pa_seqset_export", "pa_seqset_free", "pa_gz_inflate_file",
)


class PaError(RuntimeError):
    pass


class PaDeviceError(PaError):
    pass


class PaUnsupported(PaError):
    pass


class Params(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("p", ctypes.c_int64), ("min_read_quality", ctypes.c_int64),
                ("min_kmer_quality", ctypes.c_int64), ("max_genomes", ctypes.c_int64),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]

    @classmethod
    def make(cls, m=1, p=1, min_read_quality=None, min_kmer_quality=None, max_genomes=None) -> "Params":
        flags = ((HAS_MRQ if min_read_quality is not None else 0) | (HAS_MKQ if min_kmer_quality is not None else 0)
                 | (HAS_MG if max_genomes is not None else 0))

        def clamp(v):  # Python ints are unbounded; the C side clamps again to semantic ranges
            return max(min(int(v), 2 ** 62), -2 ** 62)
        return cls(clamp(m), clamp(p), clamp(min_read_quality or 0), clamp(min_kmer_quality or 0),
                   clamp(max_genomes or 0), flags, 0)


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("unique_mapped_reads", "ambiguous_mapped_reads", "unmapped_reads",
                                               "filtered_quality_reads", "filtered_quality_kmers",
                                               "filtered_hr_kmers")]


class IndexInfo(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint32), ("n_genomes", ctypes.c_uint32), ("key_words", ctypes.c_uint32),
                ("slot_bytes", ctypes.c_uint32)] + [
        (n, ctypes.c_uint64) for n in ("n_kmers", "n_multi_classes", "class_genome_entries", "table_slots",
                                       "table_bytes", "total_windows", "device_bytes")]


_lib = None
P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
U64 = ctypes.c_uint64
I64 = ctypes.c_int64
U32 = ctypes.c_uint32
I32 = ctypes.c_int32


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpa.so not found at {LIB_PATH}; build it with `python build_native.py` "
                          "(there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "pa_last_error": (ctypes.c_char_p, []),
        "pa_version": (ctypes.c_char_p, []),
        "pa_device_count": (I32, [ctypes.POINTER(I32)]),
        "pa_runtime_start": (I32, [I32]),
        "pa_index_build": (I32, [I32, ctypes.c_char_p, P, U32, I64, P, PP]),
        "pa_index_build_ex": (I32, [I32, ctypes.c_char_p, P, U32, I64, U32, P, PP]),
        "pa_index_reduce": (I32, [P, P, U32, U32, P]),
        "pa_index_prepare": (I32, [P, P]),
        "pa_index_prepare_ex": (I32, [P, U64, P]),
        "pa_index_free": (None, [P]),
        "pa_index_get_info": (I32, [P, ctypes.POINTER(IndexInfo)]),
        "pa_index_lookup": (I32, [P, ctypes.c_char_p, U64, U32, P, P, P]),
        "pa_index_class_genomes": (I32, [P, I64, P, U32, ctypes.POINTER(U32), P]),
        "pa_index_positions": (I32, [P, ctypes.c_char_p, U64, U32, U32, P, U64, ctypes.POINTER(U64), P]),
        "pa_index_extsim_stats": (I32, [P, P, U32, P, P, P, P]),
        "pa_index_dumpref": (I32, [P, P, P, U32, ctypes.POINTER(ctypes.c_char_p), I32, I32, P, P, P, P,
                                   ctypes.POINTER(U64)]),
        "pa_reads_upload": (I32, [I32, P, P, P, U64, P, PP]),
        "pa_reads_synthesize": (I32, [P, U64, U32, U64, U64, ctypes.c_double, P, PP]),
        "pa_reads_synthesize_mix": (I32, [P, U64, U32, U64, U64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                          P, PP]),
        "pa_reads_info": (I32, [P, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U32)]),
        "pa_params_effective": (I32, [P, ctypes.POINTER(Params), ctypes.POINTER(Params), ctypes.POINTER(I32), P]),
        "pa_reads_download": (I32, [P, U64, U64, P, P, P, P]),
        "pa_reads_free": (None, [P]),
        "pa_result_create": (I32, [P, PP]),
        "pa_result_reset": (I32, [P, P]),
        "pa_result_fetch": (I32, [P, ctypes.POINTER(Stats), P, P, P, P]),
        "pa_result_device_view": (I32, [P, PP, ctypes.POINTER(U64), PP, ctypes.POINTER(U64)]),
        "pa_result_copy_out": (I32, [P, P, P, P]),
        "pa_result_copy_in": (I32, [P, P, P, P]),
        "pa_result_load": (I32, [P, P, P]),
        "pa_result_free": (None, [P]),
        "pa_align": (I32, [P, P, ctypes.POINTER(Params), U64, P, P]),
        "pa_align_detail": (I32, [P, P, ctypes.POINTER(Params), P, P, P, P, P, U64, ctypes.POINTER(U64), P]),
        "pa_align_batch": (I32, [P, P, P, P, U64, U64, ctypes.POINTER(Params), ctypes.POINTER(Stats), P, P, P, P]),
        "pa_align_fastq_file": (I32, [P, ctypes.c_char_p, ctypes.POINTER(Params), U64, P, I32, U64, P,
                                      ctypes.POINTER(U64)]),
        "pa_align_fastq_range": (I32, [P, ctypes.c_char_p, U64, U64, ctypes.POINTER(Params), U64, P, I32, U64, P,
                                       ctypes.POINTER(U64), PP]),
        "pa_idsets_disjoint": (I32, [ctypes.POINTER(P), U32, I32, ctypes.POINTER(I32)]),
        "pa_idset_free": (None, [P]),
        "pa_fastq_prefetch_start": (I32, [ctypes.c_char_p, I32, I32, U64, PP]),
        "pa_align_fastq_prefetched": (I32, [P, P, ctypes.POINTER(Params), U64, P, P, ctypes.POINTER(U64)]),
        "pa_fastq_prefetch_free": (None, [P]),
        "pa_comm_unique_id": (I32, [P]),
        "pa_comm_init": (I32, [I32, I32, I32, P, PP]),
        "pa_comm_free": (I32, [P]),
        "pa_comm_count": (I32, [P, ctypes.POINTER(I32)]),
        "pa_counters_reduce": (I32, [P, P, P]),
        "pa_profile_enable": (I32, [P, I32]),
        "pa_profile_read": (I32, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "pa_profile_read_kernels": (I32, [P, P, P]),
        "pa_mem_trim": (I32, [I32, ctypes.POINTER(U64)]),
        "pa_parse_text": (I32, [I32, P, U64, I32, I32, PP]),
        "pa_parse_file": (I32, [I32, ctypes.c_char_p, I32, PP]),
        "pa_gz_inflate_file": (I32, [ctypes.c_char_p, I32, P, U64, ctypes.POINTER(U64)]),
        "pa_seqset_sizes": (I32, [P, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "pa_seqset_export": (I32, [P, P, P, P, P]),
        "pa_seqset_free": (None, [P]),
    }
    # PA_LIBRARY_PARTIAL=1: an older libpa (A/B experiments) may lack newer entry points
    partial = os.environ.get("PA_LIBRARY_PARTIAL") == "1"
    for name, (res, args) in sig.items():
        if partial and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(status: int) -> None:
    if status == PA_OK:
        return
    msg = lib().pa_last_error().decode(errors="replace")
    if status == PA_EINVAL:
        raise ValueError(msg)
    if status == PA_ETYPE:
        raise TypeError(msg)
    if status == PA_ENOMEM:
        raise MemoryError(msg)
    if status == PA_EDEVICE:
        raise PaDeviceError(msg)
    if status == PA_EUNSUPPORTED:
        raise PaUnsupported(msg)
    raise PaError(msg)


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _stream(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(getattr(stream, "cuda_stream", stream))


def device_count() -> int:
    n = I32(0)
    try:
        _check(lib().pa_device_count(ctypes.byref(n)))
    except PaDeviceError:
        return 0
    return int(n.value)


def default_device() -> int:
    return int(os.environ.get("PA_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def mem_trim(device: int = -1) -> int:
    """Give the library's idle device slabs back to the driver (pa_mem_trim);
    returns the bytes released.  Closed indexes and reads leave their large
    buffers in the library's pool for the next build (csrc/pa_mem.cpp)."""
    n = U64(0)
    _check(lib().pa_mem_trim(int(device), ctypes.byref(n)))
    return int(n.value)


def gz_inflate_file(path: str, cap: int, threads: Optional[int] = None) -> bytes:
    """gzip.open(path).read() (src/data_file.py:123-125) on host threads
    (pa_gz_inflate_file: BGZF members or search-split chunks in parallel, CRC-32
    checked).  PaError (PA_ENOTCANON) for data gzip would not read cleanly; cap bounds
    the text (ValueError past it)."""
    buf = np.empty(max(int(cap), 1), dtype=np.uint8)
    n = U64(0)
    _check(lib().pa_gz_inflate_file(path.encode(), ingest_threads() if threads is None else int(threads),
                                    buf.ctypes.data_as(P), int(cap), ctypes.byref(n)))
    return buf[:n.value].tobytes()


def ingest_threads() -> int:
    """Host threads for ingest: PA_INGEST_THREADS if set, else this job's CPU
    share (OMP_NUM_THREADS on the GPU box) capped by the affinity mask, at most 16."""
    env = os.environ.get("PA_INGEST_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 16))


class IdBlob(Sequence):
    """Read ids held as one ASCII blob (each id followed by a line break), a
    read-only str sequence that materialises ids only when they are asked for:
    aligning a container never needs them (only PseudoAlignment.reads does)."""

    __slots__ = ("_blob", "_n", "_ends", "_list")

    def __init__(self, blob: bytes, n: int):
        self._blob, self._n, self._ends, self._list = blob, int(n), None, None

    def __len__(self) -> int:
        return self._n

    def _offsets(self):
        if self._ends is None:
            self._ends = np.flatnonzero(np.frombuffer(self._blob, dtype=np.uint8) == 10)
        return self._ends

    def __getitem__(self, i):
        if self._list is not None:
            return self._list[i]
        if isinstance(i, slice):
            return self.tolist()[i]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        e = self._offsets()
        s = int(e[i - 1]) + 1 if i else 0
        return self._blob[s:int(e[i])].decode("ascii")

    def __iter__(self):
        return iter(self.tolist())

    def tolist(self):
        if self._list is None:
            self._list = self._blob.decode("ascii").split("\n")[:self._n]
        return self._list


class SeqColumns:
    """Parsed FASTA/FASTQ columns: ``names`` (IdBlob, a str sequence), ``seq`` /
    ``qual`` (uint8; ``qual`` is None for FASTA) and ``off`` (uint64 CSR, n + 1)."""

    __slots__ = ("names", "seq", "qual", "off")

    def __init__(self, names, seq, qual, off):
        self.names, self.seq, self.qual, self.off = names, seq, qual, off


def _seqset_columns(h, kind: int) -> SeqColumns:
    n, nb, nn = U64(), U64(), U64()
    try:
        _check(lib().pa_seqset_sizes(h, ctypes.byref(n), ctypes.byref(nb), ctypes.byref(nn)))
        seq = np.empty(nb.value, dtype=np.uint8)
        qual = np.empty(nb.value, dtype=np.uint8) if kind == PA_FASTQ else None
        off = np.empty(n.value + 1, dtype=np.uint64)
        names = ctypes.create_string_buffer(max(1, nn.value))
        _check(lib().pa_seqset_export(h, _ptr(seq), _ptr(qual), _ptr(off), ctypes.cast(names, P)))
    finally:
        lib().pa_seqset_free(h)
    return SeqColumns(IdBlob(names.raw[:nn.value], n.value), seq, qual, off)


def parse_file(kind: int, path: str, threads: Optional[int] = None) -> Optional[SeqColumns]:
    """Native multi-threaded parse of a FASTA/FASTQ file (pa_parse_file); None if
    the file is outside the canonical subset or unreadable -- the caller then
    uses the exact grammar of records.py, which also raises the reference's errors."""
    h = P()
    st = lib().pa_parse_file(int(kind), os.fsencode(path), int(threads or ingest_threads()), ctypes.byref(h))
    if st in (PA_ENOTCANON, PA_EIO):
        return None
    _check(st)
    return _seqset_columns(h, kind)


def parse_text(kind: int, text, threads: Optional[int] = None, universal_newlines: bool = False
               ) -> Optional[SeqColumns]:
    """Like parse_file, on text (str or bytes) in memory (pa_parse_text); by
    default the text is taken as is, like the regexes of records.py see a str."""
    data = text.encode("utf-8") if isinstance(text, str) else bytes(text)
    h = P()
    buf = ctypes.create_string_buffer(data, len(data)) if data else None
    st = lib().pa_parse_text(int(kind), ctypes.cast(buf, P) if buf is not None else None, len(data),
                             int(threads or ingest_threads()), int(bool(universal_newlines)), ctypes.byref(h))
    if st == PA_ENOTCANON:
        return None
    _check(st)
    return _seqset_columns(h, kind)


def _contiguous_views(chunks) -> bool:
    """uint8 arrays that are views of one C-contiguous buffer, back to back."""
    base = chunks[0].base
    if base is None or not isinstance(base, np.ndarray) or not base.flags.c_contiguous or base.dtype != np.uint8:
        return False
    at = chunks[0].ctypes.data
    for c in chunks:
        if c.base is not base or c.ctypes.data != at or not c.flags.c_contiguous:
            return False
        at += c.size
    return True


def concat(chunks: Sequence) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate str/bytes/uint8 chunks into (uint8 array, uint64 CSR offsets)."""
    if chunks and all(isinstance(c, np.ndarray) and c.dtype == np.uint8 and c.ndim == 1 for c in chunks):
        off = np.zeros(len(chunks) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([c.size for c in chunks], dtype=np.uint64)
        if _contiguous_views(chunks):  # consecutive views of one buffer: no copy
            whole = chunks[0].base if chunks[0].base is not None else chunks[0]
            start = chunks[0].ctypes.data - whole.ctypes.data
            return whole.reshape(-1)[start:start + int(off[-1])], off
        return np.concatenate(chunks), off  # (one copy: multi-Gbp references, BASELINE config 5)
    bs = [c.encode() if isinstance(c, str) else (c.tobytes() if isinstance(c, np.ndarray) else bytes(c))
          for c in chunks]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8) if bs else np.zeros(0, dtype=np.uint8)
    return buf, off


class Index:
    """A device-resident k-mer index (pa_index)."""

    def __init__(self, genomes: Sequence, k: int, device: Optional[int] = None, stream=None,
                 defer_tiles: bool = False, packed: Optional[Tuple[np.ndarray, np.ndarray]] = None,
                 compact: bool = False):
        """defer_tiles: build the table and genome sets only (PA_BUILD_DEFER_TILES);
        the align-side view is made by prepare() or the first align.  packed:
        the genomes already concatenated (uint8 bytes, uint64 offsets).
        compact: the table at 2 slots per genome window (PA_BUILD_COMPACT: a
        job of few reads per genome base; kept by reduce())."""
        t0 = time.perf_counter()
        buf, off = packed if packed is not None else concat(genomes)
        t1 = time.perf_counter()
        self.device = default_device() if device is None else int(device)
        self.k = int(k)
        h = P()
        kk = max(min(self.k, 2 ** 62), -2 ** 62)
        _check(lib().pa_index_build_ex(self.device, buf.ctypes.data_as(ctypes.c_char_p) if buf.size else None,
                                       _ptr(off), len(off) - 1, kk,
                                       (PA_BUILD_DEFER_TILES if defer_tiles else 0) |
                                       (PA_BUILD_COMPACT if compact else 0), _stream(stream), ctypes.byref(h)))
        if _TIMING:
            print(f"[pa_index] concat {1e3 * (t1 - t0):.1f} ms, pa_index_build_ex {1e3 * (time.perf_counter() - t1):.1f} "
                  "ms", file=sys.stderr, flush=True)
        self._h = h
        self.n_genomes = len(off) - 1
        self.compact = bool(compact)

    @property
    def handle(self):
        return self._h

    def reduce(self, keep: Sequence[int], stream=None, defer_tiles: bool = True) -> None:
        """Rebuild this index over the genomes numbered ``keep`` (ascending), in
        place, from their 2-bit codes already on the device (pa_index_reduce):
        the EXTSIM rebuild without uploading the kept genomes again.  On an
        error the index is left empty and closed."""
        sel = np.ascontiguousarray(np.asarray(keep, dtype=np.uint32))
        st = lib().pa_index_reduce(self._h, _ptr(sel), len(sel),
                                   (PA_BUILD_DEFER_TILES if defer_tiles else 0) |
                                   (PA_BUILD_COMPACT if self.compact else 0), _stream(stream))
        if st != PA_OK and st != PA_EINVAL:
            self.close()
        _check(st)
        self.n_genomes = len(sel)

    def prepare(self, stream=None, expected_reads: Optional[int] = None) -> None:
        """Make a deferred build's align-side view now (pa_index_prepare), or,
        with expected_reads, the view a job of that many reads repays
        (pa_index_prepare_ex: the neighbour bits only above the break-even;
        a later call with more reads to come, or None, makes them)."""
        if expected_reads is None:
            _check(lib().pa_index_prepare(self._h, _stream(stream)))
        else:
            _check(lib().pa_index_prepare_ex(self._h, max(0, min(int(expected_reads), 2 ** 64 - 1)), _stream(stream)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pa_index_free(self._h)
            self._h = None

    __del__ = close

    def info(self) -> IndexInfo:
        inf = IndexInfo()
        _check(lib().pa_index_get_info(self._h, ctypes.byref(inf)))
        return inf

    @property
    def n_kmers(self) -> int:
        return int(self.info().n_kmers)

    def lookup(self, kmers: Sequence[str], stream=None) -> Tuple[np.ndarray, np.ndarray]:
        n = len(kmers)
        cls = np.zeros(n, dtype=np.int64)
        size = np.zeros(n, dtype=np.uint32)
        if n == 0:
            return cls, size
        lens = {len(x) for x in kmers}
        if len(lens) != 1:
            for i, km in enumerate(kmers):
                c, s = self.lookup([km], stream)
                cls[i], size[i] = c[0], s[0]
            return cls, size
        kl = lens.pop()
        blob = "".join(kmers).encode("utf-8", errors="replace") if kl else b""
        if len(blob) != n * kl:  # non-ASCII text cannot be a k-mer
            return np.full(n, -1, dtype=np.int64), size
        _check(lib().pa_index_lookup(self._h, blob, n, kl, _ptr(cls), _ptr(size), _stream(stream)))
        return cls, size

    def class_genomes(self, cls: int) -> list:
        n = U32(0)
        _check(lib().pa_index_class_genomes(self._h, int(cls), None, 0, ctypes.byref(n), None))
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        _check(lib().pa_index_class_genomes(self._h, int(cls), _ptr(out), out.size, ctypes.byref(n), None))
        return [int(x) for x in out[:n.value]]

    # pa_kmer_hit (include/pa.h)
    HIT_DTYPE = np.dtype([("query", np.uint32), ("genome", np.uint32), ("position", np.uint64)])

    def positions(self, kmers: Sequence[str], reverse: bool = False, stream=None) -> np.ndarray:
        """Every occurrence of the k-mers in the genomes (pa_index_positions):
        a HIT_DTYPE array sorted by (query, strand, genome, position); `query`
        carries PA_POS_RC_BIT for a reverse-complement hit (reverse=True)."""
        n = len(kmers)
        empty = np.zeros(0, dtype=self.HIT_DTYPE)
        if n == 0:
            return empty
        lens = {len(x) for x in kmers}
        if len(lens) != 1:  # mixed lengths: only k-long ones can be keys; query numbers restored
            sel = [i for i, x in enumerate(kmers) if len(x) == self.k]
            h = self.positions([kmers[i] for i in sel], reverse, stream)
            rcb = np.uint32(PA_POS_RC_BIT)
            h["query"] = np.asarray(sel, dtype=np.uint32)[h["query"] & ~rcb] | (h["query"] & rcb)
            return h
        kl = lens.pop()
        blob = "".join(kmers).encode("utf-8", errors="replace") if kl else b""
        if kl == 0 or len(blob) != n * kl:  # non-ASCII text cannot be a k-mer
            return empty
        flags = PA_POS_REVERSE if reverse else 0
        nh = U64(0)
        cap = 4096
        while True:
            out = np.zeros(cap, dtype=self.HIT_DTYPE)
            _check(lib().pa_index_positions(self._h, blob, n, kl, flags, out.ctypes.data_as(P), cap,
                                            ctypes.byref(nh), _stream(stream)))
            if nh.value <= cap:
                return out[:nh.value]
            cap = int(nh.value)

    def extsim_stats(self, group_of: Sequence[int], n_groups: int):
        g = np.ascontiguousarray(group_of, dtype=np.uint32)
        total = np.zeros(n_groups, dtype=np.uint64)
        uniq = np.zeros(n_groups, dtype=np.uint64)
        inter = np.zeros(n_groups * n_groups, dtype=np.uint64)
        _check(lib().pa_index_extsim_stats(self._h, _ptr(g), n_groups, _ptr(total), _ptr(uniq), _ptr(inter), None))
        return total, uniq, inter.reshape(n_groups, n_groups)

    def profile_enable(self, on: bool = True):
        _check(lib().pa_profile_enable(self._h, 1 if on else 0))

    PROF_KERNELS = ("k_quality_masks", "k_align_lane", "k_align_lane_na", "k_align_fast", "k_align_exact",
                    "k_align_lane_rc", "k_rc_seeds")

    def profile_read_kernels(self) -> dict:
        """{kernel: (summed ms, launches)} of the align passes since the last
        call (pa_profile_read_kernels: HIP events around each launch)."""
        ms = np.zeros(len(self.PROF_KERNELS), dtype=np.float64)
        nl = np.zeros(len(self.PROF_KERNELS), dtype=np.uint64)
        _check(lib().pa_profile_read_kernels(self._h, _ptr(ms), _ptr(nl)))
        return {k: (float(ms[i]), int(nl[i])) for i, k in enumerate(self.PROF_KERNELS)}

    def profile_read(self) -> Tuple[float, int, int]:
        ms = ctypes.c_double(0)
        nl = U64(0)
        dr = U64(0)
        _check(lib().pa_profile_read(self._h, ctypes.byref(ms), ctypes.byref(nl), ctypes.byref(dr)))
        return float(ms.value), int(nl.value), int(dr.value)


class Reads:
    """A device-resident read batch (pa_reads)."""

    def __init__(self, handle, device: int):
        self._h = handle
        self.device = device
        n = U64(0)
        nb = U64(0)
        ml = U32(0)
        _check(lib().pa_reads_info(self._h, ctypes.byref(n), ctypes.byref(nb), ctypes.byref(ml)))
        self.n, self.n_bases, self.max_len = int(n.value), int(nb.value), int(ml.value)

    @classmethod
    def upload(cls, seq: np.ndarray, qual: np.ndarray, off: np.ndarray, device: Optional[int] = None,
               stream=None) -> "Reads":
        device = default_device() if device is None else int(device)
        seq = np.ascontiguousarray(seq, dtype=np.uint8).reshape(-1)
        qual = np.ascontiguousarray(qual, dtype=np.uint8).reshape(-1)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        h = P()
        _check(lib().pa_reads_upload(device, _ptr(seq), _ptr(qual), _ptr(off), len(off) - 1, _stream(stream),
                                     ctypes.byref(h)))
        return cls(h, device)

    @classmethod
    def synthesize(cls, index: Index, n_reads: int, read_len: int, first_read: int = 0, seed: int = 2,
                   sub_rate: float = 0.005, stream=None, rc_rate: float = 0.0, foreign_rate: float = 0.0) -> "Reads":
        h = P()
        if rc_rate or foreign_rate:
            _check(lib().pa_reads_synthesize_mix(index.handle, n_reads, read_len, first_read, seed, sub_rate, rc_rate,
                                                 foreign_rate, _stream(stream), ctypes.byref(h)))
        else:
            _check(lib().pa_reads_synthesize(index.handle, n_reads, read_len, first_read, seed, sub_rate,
                                             _stream(stream), ctypes.byref(h)))
        return cls(h, index.device)

    def effective(self, params: "Params", stream=None) -> Tuple["Params", int]:
        """(the filters an align of this batch applies, the batch's smallest
        quality byte): pa_params_effective."""
        out = Params()
        q = I32(0)
        _check(lib().pa_params_effective(self._h, ctypes.byref(params), ctypes.byref(out), ctypes.byref(q),
                                         _stream(stream)))
        return out, int(q.value)

    def download(self, first: int = 0, count: Optional[int] = None):
        count = self.n - first if count is None else count
        off = np.zeros(count + 1, dtype=np.uint64)
        _check(lib().pa_reads_download(self._h, first, count, None, None, _ptr(off), None))
        nb = int(off[-1])
        seq = np.zeros(max(nb, 1), dtype=np.uint8)
        qual = np.zeros(max(nb, 1), dtype=np.uint8)
        _check(lib().pa_reads_download(self._h, first, count, _ptr(seq), _ptr(qual), _ptr(off), None))
        return seq[:nb], qual[:nb], off

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            lib().pa_reads_free(self._h)
            self._h = None

    __del__ = close


class Result:
    """Device accumulators of PseudoAlignment counters (pa_result)."""

    def __init__(self, index: Index):
        h = P()
        _check(lib().pa_result_create(index.handle, ctypes.byref(h)))
        self._h = h
        self.n_genomes = index.n_genomes

    @property
    def handle(self):
        return self._h

    def reset(self, stream=None):
        _check(lib().pa_result_reset(self._h, _stream(stream)))

    def fetch(self, stream=None):
        st = Stats()
        G = self.n_genomes
        u = np.zeros(max(G, 1), dtype=np.uint64)
        a = np.zeros(max(G, 1), dtype=np.uint64)
        f = np.zeros(max(G, 1), dtype=np.uint64)
        _check(lib().pa_result_fetch(self._h, ctypes.byref(st), _ptr(u), _ptr(a), _ptr(f), _stream(stream)))
        stats = np.array([st.unique_mapped_reads, st.ambiguous_mapped_reads, st.unmapped_reads,
                          st.filtered_quality_reads, st.filtered_quality_kmers, st.filtered_hr_kmers],
                         dtype=np.uint64)
        return stats, u[:G], a[:G], f[:G]

    def device_view(self):
        s = P()
        ns = U64(0)
        m = P()
        nm = U64(0)
        _check(lib().pa_result_device_view(self._h, ctypes.byref(s), ctypes.byref(ns), ctypes.byref(m),
                                           ctypes.byref(nm)))
        return int(s.value or 0), int(ns.value), int(m.value or 0), int(nm.value)

    @property
    def n_sum(self) -> int:
        return 6 + 2 * self.n_genomes

    def copy_out(self, sum_dst_ptr: int, min_dst_ptr: int, stream=None) -> None:
        """D2D copy of [stats|unique|ambiguous] and [first_key] into caller device buffers."""
        _check(lib().pa_result_copy_out(self._h, sum_dst_ptr or None, min_dst_ptr or None, _stream(stream)))

    def load(self, stats: np.ndarray, unique: np.ndarray, ambiguous: np.ndarray, first_key: np.ndarray) -> None:
        """Overwrite the counters from host arrays (pa_result_load): the
        host SUM / MIN of read shards."""
        sb = np.ascontiguousarray(np.concatenate([stats, unique, ambiguous]).astype(np.uint64))
        mb = np.ascontiguousarray(np.asarray(first_key, dtype=np.uint64))
        assert sb.size == self.n_sum and mb.size == self.n_genomes
        _check(lib().pa_result_load(self._h, _ptr(sb), _ptr(mb) if mb.size else None))

    def copy_in(self, sum_src_ptr: int, min_src_ptr: int, stream=None) -> None:
        _check(lib().pa_result_copy_in(self._h, sum_src_ptr or None, min_src_ptr or None, _stream(stream)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pa_result_free(self._h)
            self._h = None

    __del__ = close


class Comm:
    """An RCCL communicator of the job's ranks (pa_comm_init), for
    pa_counters_reduce.  Rank 0 makes the id (``unique_id()``); every rank
    passes the same bytes."""

    def __init__(self, device: int, nranks: int, rank: int, uid: bytes):
        if len(uid) != PA_COMM_ID_BYTES:
            raise ValueError("communicator id must be PA_COMM_ID_BYTES bytes")
        h = P()
        buf = ctypes.create_string_buffer(bytes(uid), PA_COMM_ID_BYTES)
        _check(lib().pa_comm_init(int(device), int(nranks), int(rank), ctypes.cast(buf, P), ctypes.byref(h)))
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(PA_COMM_ID_BYTES)
        _check(lib().pa_comm_unique_id(ctypes.cast(buf, P)))
        return buf.raw

    @property
    def handle(self):
        return self._h

    @property
    def n_ranks(self) -> int:
        """Ranks the communicator spans (pa_comm_count -> ncclCommCount)."""
        n = I32(0)
        _check(lib().pa_comm_count(self._h, ctypes.byref(n)))
        return int(n.value)

    def close(self):
        if getattr(self, "_h", None):
            lib().pa_comm_free(self._h)
            self._h = None

    __del__ = close


def counters_reduce(result: "Result", comm, stream=None) -> None:
    """In-place SUM / MIN all-reduce of a pa_result over RCCL (pa_counters_reduce);
    ``comm`` is a Comm or a raw ncclComm_t pointer."""
    h = comm.handle if isinstance(comm, Comm) else P(int(comm))
    _check(lib().pa_counters_reduce(result.handle, h, _stream(stream)))


def align(index: Index, reads: Reads, params: Params, read_index_base: int, result: Result, stream=None) -> None:
    _check(lib().pa_align(index.handle, reads.handle, ctypes.byref(params), int(read_index_base), result.handle,
                          _stream(stream)))


def align_fastq_file(index: Index, path: str, params: Params, read_index_base: int, result: Result,
                     threads: Optional[int] = None, window_bytes: int = 0, stream=None) -> Optional[int]:
    """pa_align_fastq_file: the FASTQ file parsed on the device and aligned in
    windows; returns the number of records, or None when the file is outside
    the device-parsed subset of the grammar (``result`` then holds a partial
    sum: reset it and take the exact path)."""
    n = U64(0)
    if window_bytes <= 0:
        env = os.environ.get("PA_STREAM_WINDOW")
        window_bytes = int(env) if env and env.isdigit() else 0
    st = lib().pa_align_fastq_file(index.handle, os.fsencode(path), ctypes.byref(params), int(read_index_base),
                                   result.handle, int(threads or ingest_threads()), int(window_bytes),
                                   _stream(stream), ctypes.byref(n))
    if st == PA_ENOTCANON:
        return None
    _check(st)
    return int(n.value)


class IdSet:
    """Read-id hashes of a FASTQ byte range (pa_align_fastq_range), for
    idsets_disjoint; freed by close()."""

    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            lib().pa_idset_free(self._h)
            self._h = None

    __del__ = close


def align_fastq_range(index: Index, path: str, offset: int, length: int, params: Params, read_index_base: int,
                      result: Result, threads: Optional[int] = None, window_bytes: int = 0, stream=None,
                      want_ids: bool = True):
    """pa_align_fastq_range: the records of bytes [offset, offset + length) of a
    plain FASTQ file (cut on record boundaries) parsed and aligned on the
    index's device; returns (records, IdSet or None), or None when the range
    is outside the device-parsed subset of the grammar (the caller then takes
    the exact path for the whole file)."""
    n = U64(0)
    h = P()
    if window_bytes <= 0:
        env = os.environ.get("PA_STREAM_WINDOW")
        window_bytes = int(env) if env and env.isdigit() else 0
    st = lib().pa_align_fastq_range(index.handle, os.fsencode(path), int(offset), int(length), ctypes.byref(params),
                                    int(read_index_base), result.handle, int(threads or ingest_threads()),
                                    int(window_bytes), _stream(stream), ctypes.byref(n),
                                    ctypes.byref(h) if want_ids else None)
    if st == PA_ENOTCANON:
        return None
    _check(st)
    return int(n.value), (IdSet(h) if want_ids else None)


def idsets_disjoint(sets: Sequence[IdSet], device: int = 0) -> bool:
    """pa_idsets_disjoint: no read-id hash in two of the sets."""
    arr = (P * max(len(sets), 1))(*[s.handle for s in sets])
    d = I32(0)
    _check(lib().pa_idsets_disjoint(arr, len(sets), int(device), ctypes.byref(d)))
    return bool(d.value)


NO_ORDER = 0xFFFFFFFFFFFFFFFF  # pa_index_dumpref: a description no k-mer holds


def index_dumpref(index: "Index", keep: Optional[np.ndarray], desc_of: np.ndarray, desc_json: List[str], fd: int,
                  threads: Optional[int] = None):
    """pa_index_dumpref: the dumpref "Kmers" object written to ``fd``; returns
    per-description (unique_kmers, multi_mapping_kmers, first-appearance rank,
    last genome) arrays and the number of k-mers written."""
    nd = len(desc_json)
    names = (ctypes.c_char_p * max(nd, 1))(*[d.encode("ascii") for d in desc_json])
    uniq = np.zeros(max(nd, 1), dtype=np.uint64)
    multi = np.zeros(max(nd, 1), dtype=np.uint64)
    order = np.zeros(max(nd, 1), dtype=np.uint64)
    last = np.zeros(max(nd, 1), dtype=np.uint32)
    desc_of = np.ascontiguousarray(desc_of, dtype=np.uint32)
    keep = None if keep is None else np.ascontiguousarray(keep, dtype=np.uint8)
    nk = U64(0)
    _check(lib().pa_index_dumpref(index.handle, _ptr(keep), _ptr(desc_of), nd, names, int(fd),
                                  int(threads or ingest_threads()), _ptr(uniq), _ptr(multi), _ptr(order), _ptr(last),
                                  ctypes.byref(nk)))
    return uniq[:nd], multi[:nd], order[:nd], last[:nd], int(nk.value)


class FastqPrefetch:
    """pa_fastq_prefetch_start: a plain FASTQ file moved into device memory on a
    background native thread (so the copy overlaps the FASTA parse and the index
    build); consumed by align_fastq_prefetched, freed by close()."""

    def __init__(self, path: str, device: Optional[int] = None, threads: Optional[int] = None,
                 window_bytes: int = 0) -> None:
        self.handle = P()
        self.path = path
        self.device = default_device() if device is None else int(device)
        if window_bytes <= 0:
            env = os.environ.get("PA_STREAM_WINDOW")
            window_bytes = int(env) if env and env.isdigit() else 0
        _check(lib().pa_fastq_prefetch_start(os.fsencode(path), self.device, int(threads or ingest_threads()),
                                             int(window_bytes), ctypes.byref(self.handle)))

    @classmethod
    def adopt(cls, handle, path: str) -> "FastqPrefetch":
        """A prefetch already started through the C ABI (main.py starts one at
        entry, before the imports): this object owns and frees it."""
        self = cls.__new__(cls)
        self.handle = P(handle.value if hasattr(handle, "value") else handle)
        self.path = path
        self.device = default_device()
        return self

    def close(self) -> None:
        if self.handle:
            lib().pa_fastq_prefetch_free(self.handle)
            self.handle = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def align_fastq_prefetched(index: Index, prefetch: FastqPrefetch, params: Params, read_index_base: int,
                           result: Result, stream=None) -> Optional[int]:
    """pa_align_fastq_prefetched: like align_fastq_file on a prefetched file;
    None when the file is outside the device-parsed subset of the grammar."""
    n = U64(0)
    st = lib().pa_align_fastq_prefetched(index.handle, prefetch.handle, ctypes.byref(params), int(read_index_base),
                                         result.handle, _stream(stream), ctypes.byref(n))
    if st == PA_ENOTCANON:
        return None
    _check(st)
    return int(n.value)


def align_detail(index: Index, reads: Reads, params: Params, stream=None):
    n = reads.n
    types = np.zeros(max(n, 1), dtype=np.uint8)
    qf = np.zeros(max(n, 1), dtype=np.uint32)
    hr = np.zeros(max(n, 1), dtype=np.uint32)
    off = np.zeros(n + 1, dtype=np.uint64)
    total = U64(0)
    _check(lib().pa_align_detail(index.handle, reads.handle, ctypes.byref(params), _ptr(types), _ptr(qf), _ptr(hr),
                                 _ptr(off), None, 0, ctypes.byref(total), _stream(stream)))
    lists = np.zeros(max(int(total.value), 1), dtype=np.uint32)
    if total.value:
        _check(lib().pa_align_detail(index.handle, reads.handle, ctypes.byref(params), _ptr(types), _ptr(qf),
                                     _ptr(hr), _ptr(off), _ptr(lists), lists.size, ctypes.byref(total),
                                     _stream(stream)))
    return types[:n], qf[:n], hr[:n], off, lists[:int(total.value)]
