"""Synthetic FASTA/FASTQ workloads for the pseudo-alignment engine.

The reference ships no data (its RUN_LOG names files that are not in the repo,
SURVEY.md section 6), so every benchmark and most parity tests run on synthetic
genomes and reads shaped like BASELINE.json's configs:

* genomes are uniform i.i.d. ACGT, grouped into families whose members carry a
  per-base substitution rate against the family base (shared k-mers, so reads
  become ambiguous and unique reads get p-demoted);
* one conserved segment is copied into every genome (so ``--max-genomes``
  fires);
* a small fraction of positions start an ``N`` run (exercises the N skip of
  ``src/kmer.py:145``);
* reads are forward-strand substrings with substitution errors and raw-ASCII
  qualities from a clipped normal (quirk 5 of SURVEY.md section 8).

Everything is numpy, seeded, and returns ASCII ``uint8`` arrays so the same
bytes can be handed to the C-ABI (``pa_index_build`` / ``pa_reads_upload``) or
written out as FASTA/FASTQ text for the CLI.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def family_genomes(n_genomes: int, length: int, seed: int = 1, family_size: int = 5,
                   sub_rate: float = 0.01, conserved_len: int = 5000,
                   n_rate: float = 1e-4, n_run: int = 10) -> List[np.ndarray]:
    """Return ``n_genomes`` ASCII genomes (``uint8`` arrays of ``length`` bases)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    conserved_len = int(min(conserved_len, length // 2))
    conserved = ACGT[rng.integers(0, 4, size=conserved_len)] if conserved_len > 0 else None
    out: List[np.ndarray] = []
    base = None
    whole = np.empty(n_genomes * length, dtype=np.uint8)  # (views of one buffer, as family_genomes_fast)
    for g in range(n_genomes):
        if g % max(family_size, 1) == 0:
            base = ACGT[rng.integers(0, 4, size=length)]
        seq = whole[g * length:(g + 1) * length]
        seq[:] = base
        if sub_rate > 0:
            hit = np.flatnonzero(rng.random(length) < sub_rate)
            # substitute with one of the three other bases
            shift = rng.integers(1, 4, size=hit.size)
            code = (np.searchsorted(ACGT, seq[hit]) + shift) % 4
            seq[hit] = ACGT[code]
        if conserved is not None:
            at = int(rng.integers(0, length - conserved_len + 1))
            seq[at:at + conserved_len] = conserved
        if n_rate > 0 and n_run > 0:
            starts = np.flatnonzero(rng.random(length) < n_rate)
            for s in starts:
                seq[s:s + n_run] = ord("N")
        out.append(seq)
    return out


def family_genomes_fast(n_genomes: int, length: int, seed: int = 1, family_size: int = 5,
                        sub_rate: float = 0.01, conserved_len: int = 5000,
                        n_rate: float = 1e-4, n_run: int = 10, near_dup_every: int = 0,
                        near_dup_sub: float = 0.0003) -> List[np.ndarray]:
    """Same family structure as family_genomes, generated with byte-sized draws
    (substitution and N-run positions drawn by count, not by a per-base test) so
    that multi-Gbp references (BASELINE config 5: 2000 x 4 Mbp) take seconds per
    Gbp.  A different random stream from family_genomes: C2-C4 keep theirs.

    ``near_dup_every`` = f > 0 makes every f-th family (families f-1, 2f-1, ...)
    a family of near-duplicates: its members carry ``near_dup_sub`` substitutions
    per base against the family base instead of ``sub_rate``.  Two members then
    share ~(1 - 2 near_dup_sub)^k of their k-mers (0.98 at k = 31 and 0.03 %),
    above the EXTSIM threshold 0.95, so the similarity filter
    (src/kmer.py:188-263) keeps one member of such a family and drops the rest;
    members of the other families (1 % apart: ~0.54 shared) are all kept."""
    rng = np.random.Generator(np.random.PCG64(seed))
    conserved_len = int(min(conserved_len, length // 2))
    conserved = ACGT[rng.integers(0, 4, size=conserved_len, dtype=np.uint8)] if conserved_len > 0 else None
    out: List[np.ndarray] = []
    base = None
    fam = max(family_size, 1)
    # the genomes are views of one buffer, back to back (pa_native.concat then
    # hands it to the index build without a copy)
    whole = np.empty(n_genomes * length, dtype=np.uint8)
    for g in range(n_genomes):
        if g % fam == 0:
            base = rng.integers(0, 4, size=length, dtype=np.uint8)
        f = g // fam
        rate = near_dup_sub if (near_dup_every > 0 and f % near_dup_every == near_dup_every - 1) else sub_rate
        codes = base.copy()
        if rate > 0:
            hit = rng.integers(0, length, size=int(rng.binomial(length, rate)))
            codes[hit] = (codes[hit] + rng.integers(1, 4, size=hit.size, dtype=np.uint8)) & 3
        seq = whole[g * length:(g + 1) * length]
        np.take(ACGT, codes, out=seq)
        if conserved is not None:
            at = int(rng.integers(0, length - conserved_len + 1))
            seq[at:at + conserved_len] = conserved
        if n_rate > 0 and n_run > 0:
            for s in rng.integers(0, length, size=int(rng.binomial(length, n_rate))):
                seq[s:s + n_run] = ord("N")
        out.append(seq)
    return out


def sample_reads(genomes: Sequence[np.ndarray], n_reads: int, read_len: int, seed: int = 2,
                 err_rate: float = 0.005, qual_mean: float = 60.0, qual_sd: float = 8.0,
                 qual_min: int = 35, qual_max: int = 74) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Sample fixed-length forward-strand reads.

    Returns ``(seq, qual, origin)`` where ``seq``/``qual`` are ``(n_reads, read_len)``
    ASCII arrays and ``origin`` the source genome index of every read.  ``N`` bases
    of the source are replaced by random bases (the FASTQ grammar only allows
    ACGT in reads, ``src/records.py:262``).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.array([len(g) for g in genomes], dtype=np.int64)
    ok = np.flatnonzero(lens >= read_len)
    if ok.size == 0:
        raise ValueError("no genome is at least one read long")
    origin = ok[rng.integers(0, ok.size, size=n_reads)]
    starts = (rng.random(n_reads) * (lens[origin] - read_len + 1)).astype(np.int64)
    seq = np.empty((n_reads, read_len), dtype=np.uint8)
    for g in np.unique(origin):
        rows = np.flatnonzero(origin == g)
        idx = starts[rows, None] + np.arange(read_len)[None, :]
        seq[rows] = genomes[g][idx]
    nmask = seq == ord("N")
    if nmask.any():
        seq[nmask] = ACGT[rng.integers(0, 4, size=int(nmask.sum()))]
    if err_rate > 0:
        emask = rng.random(seq.shape) < err_rate
        ne = int(emask.sum())
        if ne:
            code = (np.searchsorted(ACGT, seq[emask]) + rng.integers(1, 4, size=ne)) % 4
            seq[emask] = ACGT[code]
    q = np.clip(np.rint(rng.normal(qual_mean, qual_sd, size=seq.shape)), qual_min, qual_max)
    qual = q.astype(np.uint8)
    return seq, qual, origin


def fasta_text(headers: Sequence[str], genomes: Sequence[np.ndarray], width: int = 0) -> str:
    parts = []
    for h, g in zip(headers, genomes):
        s = bytes(g).decode("ascii")
        if width and width > 0:
            s = "\n".join(s[i:i + width] for i in range(0, len(s), width))
        parts.append(f">{h}\n{s}\n")
    return "".join(parts)


def fastq_text(ids: Sequence[str], seq: np.ndarray, qual: np.ndarray) -> str:
    parts = []
    for i, rid in enumerate(ids):
        parts.append(f"@{rid}\n{bytes(seq[i]).decode('ascii')}\n+\n{bytes(qual[i]).decode('ascii')}\n")
    return "".join(parts)


def bgzf_bytes(data: bytes, level: int = 6, block: int = 65280) -> bytes:
    """``data`` as a BGZF file (what ``bgzip`` writes: gzip members of at most
    64 KiB of text, each recording its compressed size in a "BC" extra field,
    then the empty end-of-file member).  Python's gzip reads it as any
    multi-member gzip file; libpa inflates its members in parallel."""
    import struct
    import zlib
    out = []

    def member(chunk: bytes) -> bytes:
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        bsize = 12 + 6 + len(comp) + 8  # header + BC subfield + data + trailer
        hdr = struct.pack("<4BIBBH", 0x1F, 0x8B, 8, 4, 0, 0, 0xFF, 6) + struct.pack("<BBHH", 66, 67, 2, bsize - 1)
        return hdr + comp + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk) & 0xFFFFFFFF)

    for i in range(0, len(data), block):
        out.append(member(data[i:i + block]))
    out.append(member(b""))
    return b"".join(out)


def write_bgzf(path: str, data: bytes, level: int = 6, workers: int = 1) -> None:
    """Write ``data`` as BGZF (bgzf_bytes), compressing slices on ``workers``
    processes for multi-GB files."""
    if workers <= 1 or len(data) < (64 << 20):
        with open(path, "wb") as f:
            f.write(bgzf_bytes(data, level))
        return
    from concurrent.futures import ProcessPoolExecutor
    step = 65280 * 1024
    pieces = [data[i:i + step] for i in range(0, len(data), step)]
    with ProcessPoolExecutor(max_workers=workers) as ex, open(path, "wb") as f:
        parts = list(ex.map(_bgzf_piece, [(p, level) for p in pieces]))
        for p in parts:
            f.write(p)
        f.write(bgzf_bytes(b"", level))


def write_gzip(path: str, data: bytes, level: int = 6, workers: int = 1, chunk: int = 1 << 20) -> None:
    """Write ``data`` as ONE gzip member (what `gzip` and pigz write, not BGZF):
    1 MiB slices deflated on ``workers`` threads, each with the previous 32 KiB
    as its dictionary and ended by a sync flush (pigz's layout), so the slices
    join into one deflate stream; CRC-32 and size in the trailer."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    mv = memoryview(data)
    n = len(data)
    starts = list(range(0, n, chunk)) or [0]

    def piece(i):
        s = starts[i]
        kw = {"zdict": bytes(mv[max(0, s - 32768):s])} if s else {}
        co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, zlib.Z_DEFAULT_STRATEGY, **kw)
        last = i == len(starts) - 1
        return co.compress(mv[s:s + chunk]) + co.flush(zlib.Z_FINISH if last else zlib.Z_SYNC_FLUSH)

    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        parts = list(ex.map(piece, range(len(starts))))
    with open(path, "wb") as f:
        f.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff")
        for p in parts:
            f.write(p)
        f.write(struct.pack("<II", zlib.crc32(mv) & 0xFFFFFFFF, n & 0xFFFFFFFF))


def _bgzf_piece(args) -> bytes:
    data, level = args
    full = bgzf_bytes(data, level)
    return full[:-28]  # (without the end-of-file member: 28 bytes)
