"""Device-parsed FASTQ files (pa_align_fastq_file, csrc/pa_fastq.hip) against
the exact path (FASTAQFile(path).container + align_reads_from_container,
src/data_file.py:134-158, src/records.py:245-302, src/kmer.py:600-620).

Every file is aligned both ways through the drop-in API; the summaries must be
identical (key order included), and files outside the device-parsed subset of
the grammar must fall back to the exact path -- which raises the reference's
own errors.  Small windows (PA_STREAM_WINDOW) make records straddle window
boundaries (the carried tail).  The prefetched form (pa_fastq_prefetch_start +
pa_align_fastq_prefetched: the file moved to the device on a background
thread while the index is built, as the dumpalign CLI does) is held to the
same bar, with small copy chunks so that the pinned ring wraps."""

import gzip
import json
import os

import numpy as np
import pytest

import pa_native as N
import synth
from data_file import FASTAQFile
from kmer import KmerReference, PseudoAlignment
from records import FASTARecordContainer

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ref():
    if N.device_count() < 1:
        pytest.fail("no HIP device visible (no CPU fallback exists)")
    gens = synth.family_genomes(8, 30000, seed=5, family_size=4, sub_rate=0.02, conserved_len=800)
    c = FASTARecordContainer()
    c.parse_records(synth.fasta_text([f"g{i} test genome" for i in range(len(gens))], gens, width=70))
    return gens, KmerReference(31, c)


def reads_text(gens, n, seed, lens=(150,), ids=None, plus="+", nl="\n", final_nl=True):
    rng = np.random.default_rng(seed)
    parts = []
    for i in range(n):
        L = int(lens[i % len(lens)])
        seq, qual, _ = synth.sample_reads(gens, 1, L, seed=seed * 1000 + i, err_rate=0.02)
        rid = ids[i] if ids is not None else f"r{i} len={L}"
        parts.append(f"@{rid}{nl}{bytes(seq[0]).decode()}{nl}{plus}{nl}{bytes(qual[0]).decode()}")
    return nl.join(parts) + (nl if final_nl else "")


def both_ways(ref_obj, path, **kw):
    a = PseudoAlignment(ref_obj)
    a.align_reads_from_file(path, **kw)
    b = PseudoAlignment(ref_obj)
    b.align_reads_from_container(FASTAQFile(path).container, **kw)
    return a, b


PARAMS = [dict(), dict(m=2, p=0), dict(min_read_quality=58, min_kmer_quality=60, max_genomes=2),
          dict(min_read_quality=20, min_kmer_quality=25, max_genomes=10)]  # (C3 literal: elided thresholds)


@pytest.mark.parametrize("window", [0, 65536])
@pytest.mark.parametrize("kw", PARAMS)
def test_streamed_equals_exact(ref, tmp_path, monkeypatch, window, kw):
    gens, r = ref
    monkeypatch.setenv("PA_STREAM_WINDOW", str(window))
    p = tmp_path / "reads.fq"
    p.write_text(reads_text(gens, 3000, seed=11, lens=(150, 100, 31, 20, 176, 250)))
    a, b = both_ways(r, str(p), **kw)
    assert getattr(a, "_streamed_records", None) == 3000  # the device path was taken
    assert json.dumps(a.get_summary(), indent=4) == json.dumps(b.get_summary(), indent=4)


def test_streamed_reads_dict_and_gz(ref, tmp_path, monkeypatch):
    gens, r = ref
    monkeypatch.setenv("PA_STREAM_WINDOW", "65536")
    text = reads_text(gens, 1500, seed=12, final_nl=False)
    p = tmp_path / "reads.fq.gz"
    with gzip.open(p, "wt") as f:
        f.write(text)
    a, b = both_ways(r, str(p), m=1, p=1)
    assert getattr(a, "_streamed_records", None) == 1500
    assert a.get_summary() == b.get_summary()
    assert a.reads == b.reads  # per-read results: the file parsed again on demand


@pytest.mark.parametrize("variant", ["crlf", "plus_id", "blank_end", "lead_space_id"])
def test_outside_subset_falls_back(ref, tmp_path, variant):
    gens, r = ref
    if variant == "crlf":
        text = reads_text(gens, 200, seed=13, nl="\r\n")
    elif variant == "plus_id":
        text = reads_text(gens, 200, seed=13, plus="+")
        text = text.replace("\n+\n", "\n+ \n", 1)
    elif variant == "blank_end":
        text = reads_text(gens, 200, seed=13) + "\n"
    else:
        text = reads_text(gens, 200, seed=13, ids=[f" r{i}" for i in range(200)])
    p = tmp_path / "reads.fq"
    p.write_bytes(text.encode())
    a = PseudoAlignment(r)
    try:
        a.align_reads_from_file(str(p))
    except Exception as e:  # the exact path's verdict: the reference's exception
        with pytest.raises(type(e)):
            FASTAQFile(str(p))
        return
    assert getattr(a, "_streamed_records", None) is None
    b = PseudoAlignment(r)
    b.align_reads_from_container(FASTAQFile(str(p)).container)
    assert a.get_summary() == b.get_summary()


def test_duplicate_id_raises_reference_error(ref, tmp_path):
    gens, r = ref
    ids = [f"r{i}" for i in range(100)]
    ids[77] = "r3"
    p = tmp_path / "dup.fq"
    p.write_text(reads_text(gens, 100, seed=14, ids=ids))
    with pytest.raises(Exception) as ei:
        PseudoAlignment(r).align_reads_from_file(str(p))
    assert "Duplicate" in type(ei.value).__name__ or "uplicate" in str(ei.value)


def test_empty_and_bad_extension(ref, tmp_path):
    _, r = ref
    p = tmp_path / "empty.fq"
    p.write_text("")
    with pytest.raises(Exception):
        PseudoAlignment(r).align_reads_from_file(str(p))
    with pytest.raises(Exception) as ei:
        PseudoAlignment(r).align_reads_from_file(str(tmp_path / "reads.txt"))
    assert type(ei.value).__name__ == "InvalidExtensionError"


@pytest.mark.parametrize("window,chunk", [(0, 0), (65536, 4096), (65536, 100000)])
@pytest.mark.parametrize("kw", PARAMS)
def test_prefetched_equals_exact(ref, tmp_path, monkeypatch, window, chunk, kw):
    gens, r = ref
    monkeypatch.setenv("PA_STREAM_WINDOW", str(window))
    if chunk:
        monkeypatch.setenv("PA_PREFETCH_CHUNK", str(chunk))
    p = tmp_path / "reads.fq"
    p.write_text(reads_text(gens, 3000, seed=15, lens=(150, 100, 31, 20, 176, 250)))
    pf = N.FastqPrefetch(str(p))
    a = PseudoAlignment(r)
    a.align_reads_from_file(str(p), prefetch=pf, **kw)
    assert not pf.handle  # consumed and freed
    assert getattr(a, "_streamed_records", None) == 3000
    b = PseudoAlignment(r)
    b.align_reads_from_container(FASTAQFile(str(p)).container, **kw)
    assert json.dumps(a.get_summary(), indent=4) == json.dumps(b.get_summary(), indent=4)


def test_prefetch_too_large_takes_the_windowed_stream(ref, tmp_path, monkeypatch):
    """A file above the prefetch limit (a quarter of the free device memory;
    lowered here) is aligned by the windowed stream instead, same results."""
    gens, r = ref
    monkeypatch.setenv("PA_PREFETCH_MAX_BYTES", "1000")
    monkeypatch.setenv("PA_STREAM_WINDOW", "65536")
    p = tmp_path / "reads.fq"
    p.write_text(reads_text(gens, 2000, seed=19))
    a = PseudoAlignment(r)
    a.align_reads_from_file(str(p), prefetch=N.FastqPrefetch(str(p)), m=2, p=0)
    assert getattr(a, "_streamed_records", None) == 2000
    b = PseudoAlignment(r)
    b.align_reads_from_container(FASTAQFile(str(p)).container, m=2, p=0)
    assert a.get_summary() == b.get_summary()


def test_prefetched_outside_subset_and_gz(ref, tmp_path, monkeypatch):
    gens, r = ref
    monkeypatch.setenv("PA_PREFETCH_CHUNK", "8192")
    p = tmp_path / "reads.fq"
    p.write_bytes(reads_text(gens, 300, seed=16, nl="\r\n").encode())
    a = PseudoAlignment(r)
    a.align_reads_from_file(str(p), prefetch=N.FastqPrefetch(str(p)))
    assert getattr(a, "_streamed_records", None) is None  # the exact path
    b = PseudoAlignment(r)
    b.align_reads_from_container(FASTAQFile(str(p)).container)
    assert a.get_summary() == b.get_summary()
    ids = [f"r{i}" for i in range(300)]
    ids[250] = "r3"
    d = tmp_path / "dup.fq"
    d.write_text(reads_text(gens, 300, seed=17, ids=ids))
    with pytest.raises(Exception) as ei:
        PseudoAlignment(r).align_reads_from_file(str(d), prefetch=N.FastqPrefetch(str(d)))
    assert "uplicate" in type(ei.value).__name__ + str(ei.value)
    g = tmp_path / "reads.fq.gz"
    with gzip.open(g, "wt") as f:
        f.write(reads_text(gens, 10, seed=18))
    with pytest.raises(N.PaUnsupported):
        N.FastqPrefetch(str(g))


@pytest.mark.parametrize("kind", ["plain_text_named_gz", "crc_corrupt_gz", "truncated_gz"])
def test_bad_gzip_takes_the_reference_error(ref, tmp_path, kind):
    """A ".fq.gz" that is not gzip data, or a damaged one, gives the exact path's
    verdict (src/data_file.py:117-128: gzip.open(...).read()), not a libpa error."""
    gens, r = ref
    text = reads_text(gens, 400, seed=20).encode()
    p = tmp_path / "reads.fq.gz"
    if kind == "plain_text_named_gz":
        p.write_bytes(text)
    else:
        blob = bytearray(gzip.compress(text))
        if kind == "crc_corrupt_gz":
            blob[-8] ^= 0xFF  # the CRC-32 of the trailer
        else:
            blob = blob[:len(blob) * 2 // 3]
        p.write_bytes(bytes(blob))
    with pytest.raises(Exception) as want:
        FASTAQFile(str(p))
    with pytest.raises(type(want.value)):
        PseudoAlignment(r).align_reads_from_file(str(p))


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_file_past_4_gib(ref, tmp_path):
    """A FASTQ file larger than 2^32 bytes through the device parse (prefetched
    and windowed): line-feed offsets stay window-relative, so records past 4 GiB
    parse like the rest.  The file is K copies of one block of records (ids made
    unique per copy), so its summary is K times the block's, key order equal."""
    gens, r = ref
    block_text = reads_text(gens, 4000, seed=21, lens=(150, 100, 176))
    lines = block_text.split("\n")
    K = (2 ** 32 + 2 ** 27) // len(block_text) + 1
    p = tmp_path / "big.fq"
    with open(p, "w") as f:
        for j in range(K):
            out = list(lines)
            for i in range(0, len(out) - 1, 4):
                out[i] = "@b" + str(j) + "_" + out[i][1:]
            f.write("\n".join(out))
    assert os.path.getsize(p) > 2 ** 32
    one = tmp_path / "block.fq"
    one.write_text(block_text)
    b = PseudoAlignment(r)
    b.align_reads_from_container(FASTAQFile(str(one)).container)
    want = b.get_summary()
    for prefetch in (True, False):
        a = PseudoAlignment(r)
        a.align_reads_from_file(str(p), prefetch=N.FastqPrefetch(str(p)) if prefetch else None)
        assert getattr(a, "_streamed_records", None) == 4000 * K
        got = a.get_summary()
        assert list(got["Summary"]) == list(want["Summary"])
        assert got["Statistics"] == {k: v * K for k, v in want["Statistics"].items()}
        assert got["Summary"] == {g: {k: v * K for k, v in c.items()} for g, c in want["Summary"].items()}
    os.unlink(p)


@pytest.mark.parametrize("window", [0, 65536, 200000])
def test_streamed_bgzf_equals_exact(ref, tmp_path, monkeypatch, window):
    """A BGZF .fq.gz (bgzip's format: src/data_file.py:117-128 reads it as any
    gzip file) through the device stream, its members inflated on host threads
    (pa_gz.cpp) window by window: the summary equals the exact path's."""
    gens, r = ref
    monkeypatch.setenv("PA_STREAM_WINDOW", str(window))
    text = reads_text(gens, 4000, seed=23, lens=(150, 100, 31, 176)).encode()
    p = tmp_path / "reads.fq.gz"
    p.write_bytes(synth.bgzf_bytes(text, level=1))
    for kw in (dict(), dict(m=2, p=0, min_read_quality=58, min_kmer_quality=60, max_genomes=2)):
        a, b = both_ways(r, str(p), **kw)
        assert getattr(a, "_streamed_records", None) == 4000
        assert json.dumps(a.get_summary(), indent=4) == json.dumps(b.get_summary(), indent=4)
