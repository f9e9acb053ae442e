"""Host inflate of ".gz" input (csrc/pa_gz.cpp, csrc/pa_pgz.cpp) against
Python's gzip, which is what the reference reads such files with
(src/data_file.py:123-125: gzip.open(...).read()).

Ordinary gzip files (one deflate stream per member) are inflated in parallel:
chunks of compressed bytes find their first block by search and decode over a
window of markers, resolved once the previous chunk is known.  The text must
equal gzip.decompress byte for byte for any chunk size and thread count --
compression levels 1-9, incompressible and highly repetitive data, stored
blocks, several members, full flushes, the empty file -- and damaged or
truncated data must be refused (PA_ENOTCANON), never returned.  CPU only: no
device is touched."""

import gzip
import os
import zlib

import numpy as np
import pytest

import pa_native as N
import synth


def _fastq(n, seed):
    gens = synth.family_genomes(2, 20000, seed=seed, family_size=2, sub_rate=0.01, conserved_len=100)
    seq, qual, _ = synth.sample_reads(gens, n, 150, seed=seed + 1, err_rate=0.01)
    return synth.fastq_text([f"r{i}" for i in range(n)], seq, qual).encode()


def _cases():
    rng = np.random.default_rng(5)
    t = _fastq(20000, 3)
    out = [(f"fastq_l{lvl}", gzip.compress(t, compresslevel=lvl), t) for lvl in (1, 6, 9)]
    r = bytes(rng.integers(0, 256, 700_000, dtype=np.uint8))  # incompressible: stored blocks
    out.append(("random", gzip.compress(r, 6), r))
    m = bytes(rng.choice(list(b"AAAAAAAAAAAB"), 1_500_000))  # long matches, high ratio
    out.append(("repetitive", gzip.compress(m, 9), m))
    out.append(("two_members", gzip.compress(t[:1_000_000], 6) + gzip.compress(t[1_000_000:], 1), t))
    co = zlib.compressobj(6, zlib.DEFLATED, 31)
    z = co.compress(t[:500_000]) + co.flush(zlib.Z_FULL_FLUSH) + co.compress(t[500_000:]) + co.flush()
    out.append(("full_flush", z, t))
    out.append(("empty", gzip.compress(b"", 6), b""))
    out.append(("tiny", gzip.compress(b"@r\nACGT\n+\nIIII\n", 6), b"@r\nACGT\n+\nIIII\n"))
    return out


CASES = _cases()


@pytest.mark.parametrize("chunk_kb", ["64", "256", "4096"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_inflate_equals_python_gzip(case, chunk_kb, tmp_path, monkeypatch):
    monkeypatch.setenv("PA_PGZ_CHUNK_KB", chunk_kb)
    name, blob, want = case
    p = tmp_path / f"{name}.gz"
    p.write_bytes(blob)
    assert gzip.decompress(blob) == want
    for threads in (1, 3, 8):
        got = N.gz_inflate_file(str(p), len(want) + 64, threads=threads)
        assert got == want, (name, threads)


def test_ratio_above_the_speculative_cap(tmp_path, monkeypatch):
    """Text at ~1000:1: chunks started by the header search are held to 16-64 M
    symbols (pa_pgz.cpp phase B, the batch's host-memory bound), stop there and
    leave their range to the next batch's first chunk -- the text is still
    exact, on any thread count."""
    monkeypatch.setenv("PA_PGZ_CHUNK_KB", "64")
    line = b"@r\n" + b"A" * 4000 + b"\n+\n" + b"I" * 4000 + b"\n"
    want = line * 12_000  # 96 MB
    blob = gzip.compress(want, 9)
    assert len(want) > 500 * len(blob)
    p = tmp_path / "ratio.gz"
    p.write_bytes(blob)
    for threads in (1, 8):
        assert N.gz_inflate_file(str(p), len(want), threads=threads) == want


def test_damaged_and_truncated_data_refused(tmp_path, monkeypatch):
    monkeypatch.setenv("PA_PGZ_CHUNK_KB", "128")
    blob = CASES[1][1]
    bad = bytearray(blob)
    bad[len(bad) // 2] ^= 0x55
    crc = bytearray(blob)
    crc[-6] ^= 1  # the trailer's CRC-32
    for name, data in (("flipped", bytes(bad)), ("truncated", blob[:len(blob) * 2 // 3]), ("crc", bytes(crc)),
                       ("trailing", blob + b"junk")):
        p = tmp_path / f"{name}.gz"
        p.write_bytes(data)
        with pytest.raises(N.PaError):
            N.gz_inflate_file(str(p), 1 << 28, threads=8)


def test_not_gzip_refused(tmp_path):
    p = tmp_path / "plain.gz"
    p.write_bytes(b"@r\nACGT\n+\nIIII\n")
    with pytest.raises(N.PaError):
        N.gz_inflate_file(str(p), 1 << 20, threads=4)


@pytest.mark.parametrize("pgz", ["1", "0"])
def test_exact_capacity(tmp_path, monkeypatch, pgz):
    """A text of exactly `cap` bytes fits (the zlib path knows its end only
    after one more read), one byte more is refused as too large -- parallel
    (PA_PGZ=1) and zlib (PA_PGZ=0) paths alike."""
    monkeypatch.setenv("PA_PGZ", pgz)
    t = _fastq(3000, 9)
    p = tmp_path / "x.gz"
    p.write_bytes(gzip.compress(t, 6))
    assert N.gz_inflate_file(str(p), len(t), threads=4) == t
    with pytest.raises((N.PaError, ValueError)):
        N.gz_inflate_file(str(p), len(t) - 1, threads=4)
