"""FASTA / FASTQ record containers with the reference's acceptance grammar.

Drop-in for src/records.py.  The grammar (src/records.py:141-199, 212-302) is:

* FASTA: a line starting with ``>`` and at least one description character
  (anything but line breaks / non-tab whitespace), then a genome section of
  ACGTN and whitespace, non-empty, running up to the next line that starts
  with ``>`` or to the end of the text.  Whitespace is removed from genomes.
* FASTQ: exactly four lines per record -- ``@id``, ACGT sequence, ``+`` with
  optional dots, qualities from ``!`` to ``~`` -- each record followed by the
  next ``@`` line or the end of the text (one final line break allowed).
* Records that do not fit are skipped by the scan; then, in this order:
  a duplicate FASTQ id raises DuplicateRecordError (as records are created),
  no record raises NoRecordsInData, any non-whitespace character outside a
  record raises UnparsedDataError, and (FASTQ) a sequence/quality length
  mismatch raises InvalidRecordData.

FASTQ containers keep the reads column-wise (ids, and the sequence and quality
bytes concatenated with uint64 offsets) so that a batch can be handed to the
GPU without materialising one Python object per read; Records are built on
iteration.  Parity with the reference on its own edge cases is pinned by
tests/golden/parser_cases.json.

Both containers first hand the text to the native multi-threaded parser of
libpa.so (csrc/pa_ingest.cpp), which accepts exactly the canonical subset of
this grammar and yields the same records; any other text (and every text the
reference rejects) is parsed by the regular expressions below.
"""

from __future__ import annotations

import re
from collections import namedtuple
from typing import Dict, Iterator, List, Sequence, Tuple

import numpy as np

UNPARSED_SNIPPET_LEN = 20

Section = namedtuple("Section", ["name", "data"])


class NoRecordsInData(Exception):
    def __init__(self, message: str = "No valid records found in the data.") -> None:
        super().__init__(message)


class InvalidRecordData(Exception):
    def __init__(self, message: str = "") -> None:
        super().__init__(message)


class DuplicateRecordError(Exception):
    def __init__(self, message: str = "Duplicate records found for the unique index.") -> None:
        super().__init__(message)


class UnparsedDataError(Exception):
    def __init__(self, message: str = "Unparsed data found in the input.") -> None:
        super().__init__(message)


class _LazyText:
    """ASCII bytes of a section not yet decoded into a str (a slice of the
    native parser's column): a genome is decoded on first access, so the
    dumpalign CLI -- whose index is built from the parser's packed bytes --
    never decodes 100 MB of genome text it does not read."""

    __slots__ = ("buf", "lo", "hi")

    def __init__(self, buf, lo: int, hi: int) -> None:
        self.buf, self.lo, self.hi = buf, lo, hi

    def text(self) -> str:
        return self.buf[self.lo:self.hi].tobytes().decode("ascii")


class Record:
    """A parsed record: ``identifier`` is the first section's data; sections by name."""

    __slots__ = ("identifier", "_sections")

    def __init__(self, sections: Sequence[Section]) -> None:
        if len(sections) == 0:
            raise InvalidRecordData("The data given to construct record has no sections.")
        self.identifier: str = sections[0].data
        self._sections: Dict[str, str] = {}
        for s in sections:
            if s.name in self._sections:
                raise InvalidRecordData(f"Section header: {s.name} has appeared twice in the given data.")
            self._sections[s.name] = s.data

    def __getitem__(self, key: str) -> str:
        v = self._sections[key]
        if type(v) is _LazyText:
            v = self._sections[key] = v.text()
        return v

    def _materialize(self) -> Dict[str, str]:
        for k in self._sections:
            self[k]
        return self._sections

    def __str__(self) -> str:
        return "\n".join(f"{k}: {v}" for k, v in self._materialize().items())

    __repr__ = __str__

    def __getstate__(self):
        return {"identifier": self.identifier, "sections": self._materialize()}

    def __setstate__(self, state):
        if "_Record__sections" in state:  # pickled by the reference (src/records.py:74-90: name-mangled dict)
            self.identifier = state["identifier"]
            self._sections = dict(state["_Record__sections"])
            return
        self.identifier = state["identifier"]
        self._sections = state["sections"]


# header text: any run of non-whitespace, tab or space characters
_TEXT = r"(?:\S|[\t ])+"
_FASTA_RE = re.compile(r"^>(" + _TEXT + r")\r?\n([ACGTN\s]+?)(?=\r?\n>|(?:\r?\n)?\Z)", re.MULTILINE)
_FASTQ_RE = re.compile(r"^@(" + _TEXT + r")\r?\n([ACGT]+)\r?\n\+(\.*)\r?\n([!-~]+)(?=\r?\n@|(?:\r?\n)?\Z)",
                       re.MULTILINE)
_WS_RE = re.compile(r"\s")


def _first_unparsed(data: str, spans: List[Tuple[int, int]]) -> int:
    """Index of the first non-whitespace character outside every span, or -1."""
    pos = 0
    for s, e in spans + [(len(data), len(data))]:
        if s > pos:
            gap = data[pos:s]
            stripped = gap.lstrip()
            if stripped:
                return pos + (len(gap) - len(stripped))
        pos = max(pos, e)
    return -1


def _raise_unparsed(data: str, spans: List[Tuple[int, int]]) -> None:
    i = _first_unparsed(data, spans)
    if i >= 0:
        raise UnparsedDataError(f"Unparsed data found at index {i}: {data[i:i + UNPARSED_SNIPPET_LEN]}...")


class RecordContainer:
    """Base container: parse_records(text) then iterate Records."""

    SECTION_NAMES: Tuple[str, ...] = ()

    def __init__(self) -> None:
        self._records: List[Record] = []

    def parse_records(self, data: str) -> None:  # pragma: no cover - abstract
        raise NotImplementedError

    def __iter__(self) -> Iterator[Record]:
        return iter(self._records)

    def __len__(self) -> int:
        return len(self._records)


def _native_columns(kind: int, data):
    """Columns from the native multi-threaded parser (pa_parse_text), or None
    when the text is outside its canonical subset (then the regex grammar below
    decides, exactly as the reference)."""
    import pa_native
    return pa_native.parse_text(kind, data)


class FASTARecordContainer(RecordContainer):
    """Genomes: sections ``description`` and ``genome`` (src/records.py:212-233)."""

    SECTION_NAMES = ("description", "genome")

    def load_columns(self, cols) -> None:
        """Records from native parser columns (pa_native.SeqColumns).  The
        concatenated genome bytes are kept (``packed``): an index of exactly
        these records is built from them without concatenating again."""
        seq, off = cols.seq, cols.off
        for i, name in enumerate(cols.names):
            genome = _LazyText(seq, int(off[i]), int(off[i + 1]))  # (decoded on first access)
            self._records.append(Record([Section("description", name), Section("genome", genome)]))
        self._packed = (seq, np.asarray(off, dtype=np.uint64), list(self._records))

    def packed_genomes(self, records: Sequence[Record]):
        """(bytes, offsets) of ``records`` concatenated, if they are exactly this
        container's natively parsed records in order; else None."""
        p = getattr(self, "_packed", None)
        if p is None or len(records) != len(p[2]) or any(a is not b for a, b in zip(records, p[2])):
            return None
        return p[0], p[1]

    def parse_records(self, data: str) -> None:
        if not self._records:
            cols = _native_columns(0, data)
            if cols is not None:
                self.load_columns(cols)
                return
        self._parse_regex(data)

    def _parse_regex(self, data: str) -> None:
        spans = []
        for m in _FASTA_RE.finditer(data):
            spans.append(m.span())
            desc = m.group(1).strip()
            genome = _WS_RE.sub("", m.group(2))
            self._records.append(Record([Section("description", desc), Section("genome", genome)]))
        if not self._records:
            raise NoRecordsInData
        _raise_unparsed(data, spans)


class FASTAQRecordContainer(RecordContainer):
    """Reads: sections identifier/sequence/space/quality_sequence (src/records.py:245-302).

    Column-wise storage: ``ids`` (list of str), ``seq``/``qual`` (uint8 arrays),
    ``offsets`` (uint64, n+1).  Space sections are kept only when non-empty.
    """

    SECTION_NAMES = ("identifier", "sequence", "space", "quality_sequence")

    def __init__(self) -> None:
        super().__init__()
        self._ids: List[str] = []
        self._id_view = None  # native parse: pa_native.IdBlob, materialised on first use of .ids
        self.seq = np.zeros(0, dtype=np.uint8)
        self.qual = np.zeros(0, dtype=np.uint8)
        self.offsets = np.zeros(1, dtype=np.uint64)
        self._spaces: Dict[int, str] = {}

    @property
    def ids(self) -> List[str]:
        if self._id_view is not None:
            self._ids = self._id_view.tolist()
            self._id_view = None
        return self._ids

    @ids.setter
    def ids(self, value: List[str]) -> None:
        self._ids, self._id_view = value, None

    def id_sequence(self):
        """The ids as a sequence, without materialising a native blob."""
        return self._id_view if self._id_view is not None else self._ids

    def load_columns(self, cols) -> None:
        """Reads from native parser columns (pa_native.SeqColumns) into an empty
        container (the parser has checked that the ids are unique)."""
        assert len(self) == 0
        self._ids, self._id_view = [], cols.names
        self.seq, self.qual, self.offsets = cols.seq, cols.qual, cols.off

    def parse_records(self, data: str) -> None:
        if len(self) == 0:
            cols = _native_columns(1, data)
            if cols is not None:
                self.load_columns(cols)
                return
        self._parse_regex(data)

    def _parse_regex(self, data: str) -> None:
        ids: List[str] = list(self.ids)
        seen = set(ids)
        seqs: List[str] = []
        quals: List[str] = []
        spans = []
        base = len(ids)
        for m in _FASTQ_RE.finditer(data):
            spans.append(m.span())
            rid = m.group(1).strip()
            if rid in seen:
                raise DuplicateRecordError(f"Duplicate record found with unique index: {rid}")
            seen.add(rid)
            ids.append(rid)
            seqs.append(m.group(2))
            if m.group(3):
                self._spaces[base + len(seqs) - 1] = m.group(3)
            quals.append(m.group(4))
        if not ids:
            raise NoRecordsInData
        _raise_unparsed(data, spans)
        for i, (s, q) in enumerate(zip(seqs, quals)):
            if len(s) != len(q):
                raise InvalidRecordData(f"Mismatch in record {base + i + 1} between nucleotide length: {len(s)} "
                                        f"and PHRED section lengths: {len(q)}")
        self._append(ids[base:], seqs, quals)

    def _append(self, ids: List[str], seqs: List[str], quals: List[str]) -> None:
        lens = np.fromiter((len(s) for s in seqs), dtype=np.uint64, count=len(seqs))
        off = np.zeros(len(seqs) + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        seq = np.frombuffer("".join(seqs).encode("ascii"), dtype=np.uint8)
        qual = np.frombuffer("".join(quals).encode("ascii"), dtype=np.uint8)
        if self.ids:
            off = off + self.offsets[-1]
            self.offsets = np.concatenate([self.offsets[:-1], off])
            self.seq = np.concatenate([self.seq, seq])
            self.qual = np.concatenate([self.qual, qual])
        else:
            self.offsets, self.seq, self.qual = off, seq, qual
        self.ids.extend(ids)

    def add_reads(self, ids: Sequence[str], seq: np.ndarray, qual: np.ndarray, offsets: np.ndarray) -> None:
        """Bulk-load already validated reads (ids unique, ACGT, qualities 33-126)."""
        seen = set(self.ids)
        for rid in ids:
            if rid in seen:
                raise DuplicateRecordError(f"Duplicate record found with unique index: {rid}")
            seen.add(rid)
        off = np.asarray(offsets, dtype=np.uint64)
        if self.ids:
            off = off - off[0] + self.offsets[-1]
            self.offsets = np.concatenate([self.offsets[:-1], off])
            self.seq = np.concatenate([self.seq, np.asarray(seq, dtype=np.uint8).reshape(-1)])
            self.qual = np.concatenate([self.qual, np.asarray(qual, dtype=np.uint8).reshape(-1)])
        else:
            self.offsets = off - off[0]
            self.seq = np.ascontiguousarray(seq, dtype=np.uint8).reshape(-1)
            self.qual = np.ascontiguousarray(qual, dtype=np.uint8).reshape(-1)
        self.ids.extend(ids)

    def __len__(self) -> int:
        return len(self._id_view) if self._id_view is not None else len(self._ids)

    def record(self, i: int) -> Record:
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return Record([Section("identifier", self.id_sequence()[i]), Section("sequence", self.seq[a:b].tobytes().decode()),
                       Section("space", self._spaces.get(i, "")),
                       Section("quality_sequence", self.qual[a:b].tobytes().decode())])

    def __iter__(self) -> Iterator[Record]:
        return (self.record(i) for i in range(len(self)))
