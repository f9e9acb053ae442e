"""CPU-only tests of the host side: the C ABI library loads and exports every
symbol of include/pa.h, the FASTA/FASTQ grammar matches the reference, the CLI
flag handling matches src/main.py.  No kernel is launched here."""

import ctypes
import gzip
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import pa_native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")
GOLD = os.path.join(REPO, "tests", "golden")


def header_functions():
    text = open(os.path.join(REPO, "include", "pa.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pa_[a-z_]+)\s*\(", text)))


def test_header_matches_binding_table():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_every_symbol():
    lib = ctypes.CDLL(N.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], stdout=subprocess.PIPE, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(header_functions()) <= exported


def test_library_has_gfx950_code_object():
    blob = open(N.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_no_device_fails_loudly_without_gpu():
    if N.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(N.PaDeviceError):
        N.Index(["ACGT"], 3)


def test_version_and_error_string():
    assert b"gfx950" in N.lib().pa_version()
    assert isinstance(N.lib().pa_last_error(), bytes)


def test_header_constants_match_binding():
    text = open(os.path.join(REPO, "include", "pa.h")).read()
    for name in ("PA_NB_READS_PER_KBASE", "PA_NB_READS_PER_KBASE_2W", "PA_NB_READS_PER_KBASE_3W", "PA_MAX_K",
                 "PA_COMPACT_READS_PER_BASE"):
        m = re.search(rf"#define {name} (\d+)", text)
        assert m and int(m.group(1)) == getattr(N, name), name
    for name in ("PA_BUILD_DEFER_TILES", "PA_BUILD_COMPACT"):
        m = re.search(rf"#define {name} (\d+)u", text)
        assert m and int(m.group(1)) == getattr(N, name), name


def test_compact_table_policy(tmp_path):
    """The CLI's job gets the compact k-mer table below PA_COMPACT_READS_PER_BASE
    reads per genome base (reads counted high: one per 64 bytes of the FASTQ,
    4x that for gzip, split over the shards); no reads file: the default table."""
    import main
    genomes = [{"genome": "ACGT" * 2500}, {"genome": "A" * 10000}]  # 20 000 bases
    fq = tmp_path / "r.fq"
    fq.write_bytes(b"x" * (64 * 59999))  # ~60 k reads < 3 x 20 000
    assert main.compact_for_job(str(fq), genomes)
    fq.write_bytes(b"x" * (64 * 60000))
    assert not main.compact_for_job(str(fq), genomes)
    assert main.compact_for_job(str(fq), genomes, shards=2)
    gz = tmp_path / "r.fq.gz"
    gz.write_bytes(b"x" * (16 * 60000))
    assert not main.compact_for_job(str(gz), genomes)
    assert not main.compact_for_job(None, genomes)
    assert not main.compact_for_job(str(tmp_path / "missing.fq"), genomes)


def test_library_built_from_this_checkout():
    """pa_version() carries the SHA-256 of the sources, header and flags it was
    built from (build_native.source_hash); it must be this checkout's, so the
    GPU evidence is tied to HEAD's sources."""
    import build_native
    have = build_native.library_hash(N.lib().pa_version().decode())
    assert len(have) == 64
    assert have == build_native.source_hash()


PARSER = json.load(open(os.path.join(GOLD, "parser_cases.json")))


@pytest.mark.parametrize("kind", ["fasta", "fastq"])
def test_parser_grammar_golden(kind):
    import records as R
    cls = R.FASTARecordContainer if kind == "fasta" else R.FASTAQRecordContainer
    for text, exp in PARSER[kind]:
        c = cls()
        try:
            c.parse_records(text)
            got = {"records": [{"identifier": r.identifier, "sections": {n: r[n] for n in cls.SECTION_NAMES}}
                               for r in c]}
        except Exception as e:  # noqa: BLE001
            got = {"error": type(e).__name__, "message": str(e)}
        assert got == exp, repr(text)


def test_fastq_columns(tmp_path):
    import records as R
    from data_file import FASTAQFile, FASTAFile, InvalidExtensionError, NoRecordsInDataFile
    c = R.FASTAQRecordContainer()
    c.parse_records("@a\nACGT\n+\nIIII\n@b\nGG\n+..\n#$\n")
    assert c.ids == ["a", "b"]
    assert c.offsets.tolist() == [0, 4, 6]
    assert bytes(c.seq) == b"ACGTGG" and bytes(c.qual) == b"IIII#$"
    recs = list(c)
    assert recs[1]["space"] == ".." and recs[1]["quality_sequence"] == "#$"
    p = tmp_path / "r.fq.gz"
    with gzip.open(p, "wt") as f:
        f.write("@x\nAC\n+\nII\n")
    assert FASTAQFile(str(p)).container.ids == ["x"]
    with pytest.raises(InvalidExtensionError):
        FASTAFile(str(tmp_path / "g.fasta"))
    q = tmp_path / "e.fa"
    q.write_text("junk\n")
    with pytest.raises(NoRecordsInDataFile):
        FASTAFile(str(q))


def _cli(*args):
    return subprocess.run([sys.executable, os.path.join(PKG, "main.py"), *args], stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=120)


def test_cli_errors_before_any_gpu_work(tmp_path):
    r = _cli("-t", "bogus")
    assert r.returncode != 0 and "Unsupported task" in r.stderr
    r = _cli("-t", "dumpalign", "-g", "x.fa")
    assert r.returncode != 0 and "For task 'dumpalign'" in r.stderr
    r = _cli("-t", "reference", "-g", "x.fa", "-k", "3", "-r", "o.kdb", "--reads", "r.fq")
    assert r.returncode != 0 and "For task 'reference'" in r.stderr
    r = _cli("-t", "dumpalign", "-g", str(tmp_path / "missing.fa"), "-k", "3", "--reads", str(tmp_path / "m.fq"))
    assert r.returncode != 0 and "does not exist" in r.stderr
    bad = tmp_path / "g.txt"
    bad.write_text(">g\nACGT\n")
    fq = tmp_path / "r.fq"
    fq.write_text("@r\nACGT\n+\nIIII\n")
    r = _cli("-t", "dumpalign", "-g", str(bad), "-k", "3", "--reads", str(fq))
    assert r.returncode != 0 and "Invalid file extension" in r.stderr


def test_cli_argument_defaults_and_coercion():
    import main
    a = main.parse_arguments(["-t", "dumpalign", "-g", "g.fa", "-k", "5", "--reads", "r.fq"])
    assert a.min_read_quality is None and a.min_kmer_quality is None and a.max_genomes is None
    assert a.unique_threshold is None and a.ambiguous_threhold is None
    a = main.parse_arguments(["-t", "dumpalign", "-g", "g.fa", "-k", "5", "--reads", "r.fq", "-m", "0", "-p", "0",
                              "--max-genomes", "0"])
    assert a.unique_threshold == 0 and a.max_genomes == 0


def test_synth_shapes():
    import synth
    g = synth.family_genomes(7, 1000, seed=1, family_size=3, sub_rate=0.02, conserved_len=100, n_rate=1e-3)
    assert len(g) == 7 and all(x.size == 1000 for x in g)
    assert set(np.unique(np.concatenate(g)).tolist()) <= set(b"ACGTN")
    s, q, o = synth.sample_reads(g, 50, 80, seed=2)
    assert s.shape == (50, 80) and set(np.unique(s).tolist()) <= set(b"ACGT")
    assert q.min() >= 35 and q.max() <= 74


# ---- native ingest (csrc/pa_ingest.cpp) == the regex grammar on its subset -------

def _records_of(c, kind):
    import records as R
    cls = R.FASTARecordContainer if kind == 0 else R.FASTAQRecordContainer
    return [(r.identifier, [r[n] for n in cls.SECTION_NAMES]) for r in c]


def _regex(kind, text):
    import records as R
    c = R.FASTARecordContainer() if kind == 0 else R.FASTAQRecordContainer()
    try:
        c._parse_regex(text)
    except Exception as e:  # noqa: BLE001
        return type(e).__name__
    return _records_of(c, kind)


def _native(kind, text, threads):
    import records as R
    cols = N.parse_text(kind, text, threads=threads)
    if cols is None:
        return None
    c = R.FASTARecordContainer() if kind == 0 else R.FASTAQRecordContainer()
    c.load_columns(cols)
    return _records_of(c, kind)


def _random_fasta(rng):
    parts = []
    for g in range(int(rng.integers(1, 5))):
        hdr = "".join(rng.choice(list("ab c\tXY_:|>1"), size=int(rng.integers(1, 8))))
        body = "".join(rng.choice(list("ACGTN"), size=int(rng.integers(1, 200))))
        w = int(rng.integers(5, 70))
        body = "\n".join(body[i:i + w] for i in range(0, len(body), w))
        parts.append(f">{hdr}\n{body}\n")
    return "".join(parts)


def _random_fastq(rng):
    parts = []
    for r in range(int(rng.integers(1, 6))):
        n = int(rng.integers(1, 40))
        rid = "".join(rng.choice(list("ab c\t1_:"), size=int(rng.integers(1, 6))))
        seq = "".join(rng.choice(list("ACGT"), size=n))
        q = "".join(chr(int(x)) for x in rng.integers(33, 127, size=n))
        parts.append(f"@{rid}\n{seq}\n+\n{q}\n")
    return "".join(parts)


POOL = list("ACGTNacgtn>@+.!~ \t\n\r\x0b\x0c\x1c") + ["\r\n", "\n\n", "é", "\x00"]


def _mutate(rng, text):
    t = list(text)
    for _ in range(int(rng.integers(0, 3))):
        op = int(rng.integers(0, 4))
        i = int(rng.integers(0, len(t) + 1))
        if op == 0:
            t.insert(i, str(rng.choice(POOL)))
        elif op == 1 and t:
            del t[min(i, len(t) - 1)]
        elif op == 2 and t:
            t[min(i, len(t) - 1)] = str(rng.choice(POOL))
        else:
            t = list("".join(t).replace("\n", "\r\n"))
    return "".join(t)


@pytest.mark.parametrize("kind", [0, 1])
def test_native_parser_matches_regex_grammar(kind):
    """Differential check: wherever the native parser accepts a text, the regex
    grammar accepts it with the same records; it rejects (None) everything else
    the grammar rejects.  Random canonical texts plus random mutations."""
    rng = np.random.Generator(np.random.PCG64(123 + kind))
    accepted = rejected = 0
    for it in range(3000):
        base = _random_fasta(rng) if kind == 0 else _random_fastq(rng)
        if it % 7 == 3:
            base = base.rstrip("\n")
        if it % 11 == 5 and kind == 1:
            base = base + base  # duplicate ids
        text = base if it % 3 == 0 else _mutate(rng, base)
        nat = _native(kind, text, threads=1 + it % 4)
        ref = _regex(kind, text)
        if nat is None:
            rejected += 1
            continue
        accepted += 1
        assert nat == ref, repr(text)
    assert accepted > 800 and rejected > 300


@pytest.mark.parametrize("kind", [0, 1])
def test_native_parser_golden_cases(kind):
    name = "fasta" if kind == 0 else "fastq"
    for text, exp in PARSER[name]:
        nat = _native(kind, text, threads=2)
        if nat is not None:
            assert "records" in exp, repr(text)
            assert nat == [(r["identifier"], list(r["sections"].values())) for r in exp["records"]], repr(text)


def test_native_parse_file_large_multithread(tmp_path):
    """A multi-chunk FASTQ and FASTA through pa_parse_file (plain and .gz)."""
    import synth
    from data_file import FASTAQFile, FASTAFile
    gens = synth.family_genomes(3, 300000, seed=7, family_size=3, n_rate=1e-3, n_run=4)
    seq, qual, _ = synth.sample_reads(gens, 40000, 100, seed=8)
    fq = synth.fastq_text([f"r{i}" for i in range(len(seq))], seq, qual)
    fa = synth.fasta_text(["g0 a", "g1", "g2\t"], gens, width=61)
    (tmp_path / "r.fq").write_text(fq)
    (tmp_path / "g.fa").write_text(fa)
    with gzip.open(tmp_path / "r.fq.gz", "wt") as f:
        f.write(fq)
    for path in ("r.fq", "r.fq.gz"):
        cols = N.parse_file(N.PA_FASTQ, str(tmp_path / path), threads=8)
        assert cols is not None
        assert list(cols.names) == [f"r{i}" for i in range(len(seq))]
        assert cols.names[7] == "r7" and cols.names[-1] == f"r{len(seq) - 1}"
        assert np.array_equal(cols.seq, seq.reshape(-1)) and np.array_equal(cols.qual, qual.reshape(-1))
        assert cols.off.tolist() == list(range(0, 100 * len(seq) + 1, 100))
    c = FASTAQFile(str(tmp_path / "r.fq")).container
    assert c.ids[:3] == ["r0", "r1", "r2"] and np.array_equal(c.seq, seq.reshape(-1))
    cols = N.parse_file(N.PA_FASTA, str(tmp_path / "g.fa"), threads=8)
    assert list(cols.names) == ["g0 a", "g1", "g2"]
    for i, g in enumerate(gens):
        assert np.array_equal(cols.seq[int(cols.off[i]):int(cols.off[i + 1])], g)
    recs = list(FASTAFile(str(tmp_path / "g.fa")).container)
    assert [r.identifier for r in recs] == ["g0 a", "g1", "g2"] and recs[1]["genome"] == bytes(gens[1]).decode()
    # duplicate ids -> not canonical; the regex grammar raises the reference's error
    (tmp_path / "d.fq").write_text("@a\nAC\n+\nII\n@a\nAC\n+\nII\n")
    assert N.parse_file(N.PA_FASTQ, str(tmp_path / "d.fq")) is None
    import records as R
    with pytest.raises(R.DuplicateRecordError):
        FASTAQFile(str(tmp_path / "d.fq"))
    assert N.parse_file(N.PA_FASTQ, str(tmp_path / "missing.fq")) is None


@pytest.mark.parametrize("kind", [0, 1])
def test_native_parse_file_matches_universal_newlines(kind, tmp_path):
    """Files: the reference reads them as UTF-8 text with universal newlines
    (src/data_file.py:117-158); pa_parse_file must agree wherever it accepts."""
    import records as R
    rng = np.random.Generator(np.random.PCG64(555 + kind))
    path = tmp_path / "x"
    accepted = 0
    for it in range(1500):
        base = _random_fasta(rng) if kind == 0 else _random_fastq(rng)
        if it % 5 == 1:
            base = base.replace("\n", "\r\n")
        text = _mutate(rng, base) if it % 2 else base
        path.write_bytes(text.encode("utf-8"))
        cols = N.parse_file(kind, str(path), threads=1 + it % 4)
        if cols is None:
            continue
        accepted += 1
        c = R.FASTARecordContainer() if kind == 0 else R.FASTAQRecordContainer()
        c.load_columns(cols)
        with open(path, "r", encoding="utf-8") as f:
            assert _records_of(c, kind) == _regex(kind, f.read()), repr(text)
    assert accepted > 500


def test_reference_written_kdb_and_aln_load(monkeypatch, tmp_path):
    """Files saved by the reference CLI (tests/golden/config1*.kdb, config1.aln,
    made by make_golden.py) load through the restricted unpickler; their own
    dicts give the reference's dumpref / dumpalign output (no device needed:
    the index build is stubbed here, the GPU tests run the real one)."""
    import gzip as gz
    import hashlib
    import pickle

    import kmer
    monkeypatch.setattr(kmer.KmerReference, "_build", lambda self: setattr(self, "_view", None))
    cases = json.load(open(os.path.join(GOLD, "dumpref_cases.json")))["config1"]
    for name in ("config1", "config1_sim"):
        ref = kmer.KmerReference.load(os.path.join(GOLD, name + ".kdb"))
        assert isinstance(ref, kmer.KmerReference) and ref.kmer_len == 21
        text = json.dumps(ref.get_summary(), indent=4) + "\n"
        assert hashlib.sha256(text.encode()).hexdigest() == cases[name]["dumpref_r_sha256"]
        assert all(isinstance(g, kmer.Record) for g in ref.genomes)
    aln = kmer.PseudoAlignment.load(os.path.join(GOLD, "config1.aln"))
    assert json.dumps(aln.get_summary(), indent=4) + "\n" == cases["config1_aln"]["dumpalign_a"]
    assert all(isinstance(e["mapping_type"], kmer.ReadMappingType) for e in aln.reads.values())
    # anything but the classes such files hold is refused
    bad = tmp_path / "bad.kdb"
    with gz.open(bad, "wb") as f:
        f.write(b"cos\ngetcwd\n(tR.")
    with pytest.raises(pickle.UnpicklingError):
        kmer.KmerReference.load(str(bad))


def test_native_parse_file_bgzf(tmp_path):
    """BGZF ``.fq.gz`` / ``.fa.gz`` (bgzip's multi-member gzip, read by
    src/data_file.py:117-128 through gzip.open like any gzip file) inflated
    member-parallel by pa_gz.cpp: the same columns as the plain text; a member
    with a bad CRC-32, a truncated file or plain text named .gz fall back to the
    exact path (None), which raises the reference's own error."""
    import synth
    from data_file import FASTAQFile
    gens = synth.family_genomes(3, 200000, seed=9, family_size=3, n_rate=1e-3, n_run=4)
    seq, qual, _ = synth.sample_reads(gens, 30000, 120, seed=10)
    fq = synth.fastq_text([f"r{i}" for i in range(len(seq))], seq, qual).encode()
    fa = synth.fasta_text(["g0", "g1 x", "g2"], gens, width=70).encode()
    (tmp_path / "r.fq.gz").write_bytes(synth.bgzf_bytes(fq))
    (tmp_path / "g.fa.gz").write_bytes(synth.bgzf_bytes(fa, level=1))
    assert gzip.decompress((tmp_path / "r.fq.gz").read_bytes()) == fq
    for threads in (1, 3, 16):
        cols = N.parse_file(N.PA_FASTQ, str(tmp_path / "r.fq.gz"), threads=threads)
        assert cols is not None and len(cols.names) == len(seq)
        assert np.array_equal(cols.seq, seq.reshape(-1)) and np.array_equal(cols.qual, qual.reshape(-1))
    cols = N.parse_file(N.PA_FASTA, str(tmp_path / "g.fa.gz"), threads=4)
    for i, g in enumerate(gens):
        assert np.array_equal(cols.seq[int(cols.off[i]):int(cols.off[i + 1])], g)
    # damaged files: the exact path's verdict
    blob = bytearray(synth.bgzf_bytes(fq))
    blob[5000] ^= 0x55  # inside a member's deflate data (or its header): inflate or CRC fails
    (tmp_path / "bad.fq.gz").write_bytes(bytes(blob))
    (tmp_path / "cut.fq.gz").write_bytes(synth.bgzf_bytes(fq)[:100000])
    (tmp_path / "txt.fq.gz").write_bytes(fq)
    for name in ("bad.fq.gz", "cut.fq.gz", "txt.fq.gz"):
        assert N.parse_file(N.PA_FASTQ, str(tmp_path / name)) is None, name
        with pytest.raises(Exception):
            FASTAQFile(str(tmp_path / name))


def test_early_prefetch_sniffing_matches_the_prefetch_conditions(monkeypatch):
    """The CLI's entry-time FASTQ prefetch (main._early_reads_path) takes exactly
    the files the later prefetch would: every argparse spelling of the task and
    the reads, plain `.fq` only, not with streaming or prefetch turned off
    (a second, never-adopted prefetch otherwise held device memory)."""
    import main
    for v in ("PA_STREAM", "PA_PREFETCH"):
        monkeypatch.delenv(v, raising=False)
    f = main._early_reads_path
    assert f(["-t", "dumpalign", "-g", "g.fa", "-k", "31", "--reads", "r.fq"]) == "r.fq"
    assert f(["-tdumpalign", "--reads=r.fq"]) == "r.fq"
    assert f(["--task=dumpalign", "--reads", "r.fq"]) == "r.fq"
    assert f(["--task", "dumpalign", "--reads=x/r.fq"]) == "x/r.fq"
    assert f(["-t", "align", "--reads", "r.fq"]) is None
    assert f(["-t", "dumpalign", "--reads", "r.fq.gz"]) is None
    assert f(["-t", "dumpalign", "--reads", "r.fastq"]) is None
    assert f(["-t", "dumpalign"]) is None
    monkeypatch.setenv("PA_PREFETCH", "0")
    assert f(["-t", "dumpalign", "--reads", "r.fq"]) is None
    monkeypatch.setenv("PA_PREFETCH", "1")
    monkeypatch.setenv("PA_STREAM_WINDOW", "1048576")
    assert main._stream_window() == 1048576
