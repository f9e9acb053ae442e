"""GPU parity tests: libpa.so (HIP kernels) against the reference's golden
vectors and against the CPU restatement (oracle/) on seeded synthetic data.

Everything here calls through the C ABI (pa_native -> libpa.so) and needs an
MI355X; bit-exact equality is required everywhere (integer work).
"""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pa_native as N
import pa_oracle as O
import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


UNIT = load("unit_cases.json")
# the reference's demo configurations (src/RUN_LOG:28-84) and k = 96-159
DEMO = load("demo_cases.json")
CASES = UNIT + DEMO["cases"]
TYPE = {0: "DROPPED", 1: "UNMAPPED", 2: "UNIQUELY_MAPPED", 3: "AMBIGUOUSLY_MAPPED"}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if N.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X (no CPU fallback exists)")


def reads_of(reads):
    seq, off = N.concat([r[1] for r in reads])
    qual, _ = N.concat([r[2] for r in reads])
    return seq, qual, off


def summary_from_counters(idents, stats, uq, am, fk, ps):
    """get_summary from per-genome counters + first-appearance keys (as kmer.py does)."""
    st = {"unique_mapped_reads": int(stats[0]), "ambiguous_mapped_reads": int(stats[1]),
          "unmapped_reads": int(stats[2])}
    if ps["mrq"] is not None:
        st["filtered_quality_reads"] = int(stats[3])
    if ps["mkq"] is not None:
        st["filtered_quality_kmers"] = int(stats[4])
    if ps["mg"] is not None:
        st["filtered_hr_kmers"] = int(stats[5])
    counts, first = {}, {}
    for g in np.flatnonzero(fk != N.NO_FIRST_KEY):
        name = idents[g]
        c = counts.setdefault(name, [0, 0])
        c[0] += int(uq[g])
        c[1] += int(am[g])
        first[name] = min(first.get(name, 1 << 64), int(fk[g]))
    return {"Statistics": st, "Summary": {n: {"unique_reads": counts[n][0], "ambiguous_reads": counts[n][1]}
                                          for n in sorted(first, key=first.get)}}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_unit_cases(case):
    """Per-read results (exact kernel) and summaries (fast + exact kernels) vs the reference."""
    idents = [g[0] for g in case["genomes"]]
    index = N.Index([g[1] for g in case["genomes"]], case["k"])
    assert index.n_kmers == case["n_kmers"]
    # index: the genome set of every k-mer
    kms = [km for km, _ in case["kmer_sets"]]
    if kms:
        cls, size = index.lookup(kms)
        for (km, gl), c, s in zip(case["kmer_sets"], cls, size):
            assert c >= 0 and int(s) == len(gl), km
            assert index.class_genomes(int(c)) == gl, km
    seq, qual, off = reads_of(case["reads"])
    reads = N.Reads.upload(seq, qual, off)
    for res in case["results"]:
        ps = res["params"]
        prm = N.Params.make(ps["m"], ps["p"], ps["mrq"], ps["mkq"], ps["mg"])
        types, qf, hr, loff, lists = N.align_detail(index, reads, prm)
        for r, (rid, tname, glist, eqf, ehr) in enumerate(res["reads"]):
            assert TYPE[int(types[r])] == tname, (rid, ps)
            assert [idents[g] for g in lists[loff[r]:loff[r + 1]]] == glist, (rid, ps)
            assert (int(qf[r]), int(hr[r])) == (eqf, ehr), (rid, ps)
        result = N.Result(index)
        N.align(index, reads, prm, 0, result)
        stats, uq, am, fk = result.fetch()
        summ = summary_from_counters(idents, stats, uq, am, fk, ps)
        assert json.dumps(summ, indent=4) == res["summary_text"], ps


def test_dropin_api_on_reference_fixtures():
    """The reference's own test_kmer.py scenarios through the drop-in classes."""
    from kmer import KmerReference, PseudoAlignment, Read, ReadMappingType
    from records import FASTAQRecordContainer, FASTARecordContainer

    def fa(text):
        c = FASTARecordContainer()
        c.parse_records(text)
        return c

    def fq(text):
        c = FASTAQRecordContainer()
        c.parse_records(text)
        return c

    ref = KmerReference(4, fa(">Genome1\nATGCCTTTTCGGGG\n>Genome2\nGCCGTTTTCGGGGCTA\n>Genome3\nCCGG\n"
                              ">Genome4\nAAAAAAAAGGGCT\n>Genome5\nTTTTTTTTGCTAA\n"))
    rec = list(fq("@Read4\nATGCCGGGGCTAA\n+\nIIIIIIIIIIIII\n"))[0]
    assert Read(rec).pseudo_align(ref) == ReadMappingType.AMBIGUOUSLY_MAPPED
    assert Read(rec).pseudo_align(ref, p=5) == ReadMappingType.UNIQUELY_MAPPED
    r = Read(rec)
    r.pseudo_align(ref)
    assert [g.identifier for g in r.mapping.genomes_mapped_to] == ["Genome1", "Genome1", "Genome2"]
    with pytest.raises(ValueError):
        Read(rec).pseudo_align(ref, m=-1)
    with pytest.raises(TypeError):
        Read(rec).pseudo_align(ref, m=1.5)

    sample = fa(">Genome1\nAGCTAGCTAGCTAGCTAGCT\n>Genome2\nTGCATGCATGCATGCATGCA\n"
                ">Genome3\nAGCTTGCATGCAGCTAGCTA\n>Genome4\nCCGGAAGCTTGCATGCAGCTA\n")
    kref = KmerReference(3, sample)
    assert kref.get_kmer_references("AGC") and not kref.get_kmer_references("GGG")
    assert kref.n_kmers == len(kref.kmers)
    reads = fq("@Read1\nAGCTAGCT\n+\nIIIIIIII\n@Read2\nTGCATGCA\n+\n!!!!!!!!\n@Read3\nGGGGGGGG\n+\n!!IIIIII\n")
    pa = PseudoAlignment(kref)
    pa.align_reads_from_container(reads, min_read_quality=40, min_kmer_quality=50, max_genomes=2)
    s = pa.get_summary()["Statistics"]
    assert (s["filtered_quality_reads"], s["filtered_quality_kmers"], s["filtered_hr_kmers"]) == (1, 1, 5)
    pa = PseudoAlignment(kref)
    pa.align_reads_from_container(reads, min_read_quality=30, min_kmer_quality=30, max_genomes=3)
    s = pa.get_summary()["Statistics"]
    assert (s["unique_mapped_reads"], s["ambiguous_mapped_reads"], s["unmapped_reads"]) == (0, 2, 1)
    assert set(pa.reads) == {"Read1", "Read2", "Read3"}
    pa = PseudoAlignment(kref)
    pa.align_reads_from_container(reads, min_read_quality=40)
    assert "Read2" not in pa.reads  # dropped, not unmapped
    from kmer import AddingExistingRead
    with pytest.raises(AddingExistingRead):
        pa.align_reads_from_container(reads)


def test_config1_cli_stdout():
    """BASELINE config 1 through the drop-in CLI: stdout identical to the reference's."""
    for case in load("config1_cli.json"):
        cmd = [sys.executable, os.path.join(PKG, "main.py"), "-t", "dumpalign", "-g",
               os.path.join(GOLD, "config1.fa"), "-k", "21", "--reads", os.path.join(GOLD, "config1.fq")] + case["flags"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert r.stdout == case["stdout"], case["flags"]


def test_demo_k150_cli_stdout(tmp_path):
    """The reference's demo runs `dumpalign -k 150 --min-read-quality 59
    --min-kmer-quality 60 --max-genomes 2` (and `--max-genomes 0`,
    src/RUN_LOG:64-84) through the drop-in CLI on a mid-sized reference:
    stdout identical to the reference CLI's."""
    cli = DEMO["cli"]
    case = next(c for c in DEMO["cases"] if c["name"] == cli["case"])
    fa, fq = tmp_path / "mid.fa", tmp_path / "mid.fq"
    fa.write_text("".join(f">{h}\n{s}\n" for h, s in case["genomes"]))
    fq.write_text("".join(f"@{i}\n{s}\n+\n{q}\n" for i, s, q in case["reads"]))
    for run in cli["runs"]:
        cmd = [sys.executable, os.path.join(PKG, "main.py"), "-t", "dumpalign", "-g", str(fa), "-k", str(cli["k"]),
               "--reads", str(fq)] + run["flags"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert r.stdout == run["stdout"], run["flags"]


def test_align_without_reference_file_fails_like_the_reference(tmp_path):
    """`-t align -g -k --reads -a` without -r: the reference saves its k-mer
    reference to None (src/main.py:366-372), gzip.open raises a TypeError the
    CLI does not catch (src/main.py:401), and the process exits with status 1
    and a traceback before the alignment file is written."""
    aln = tmp_path / "out.aln"
    cmd = [sys.executable, os.path.join(PKG, "main.py"), "-t", "align", "-g", os.path.join(GOLD, "config1.fa"),
           "-k", "21", "--reads", os.path.join(GOLD, "config1.fq"), "-a", str(aln)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 1, r.stderr
    assert "Traceback" in r.stderr and "TypeError" in r.stderr
    assert not aln.exists()
    # (with -r the reference takes its -r branch, src/main.py:359-365: the
    # file must already exist -- the -g branch runs only without -r)


@pytest.mark.parametrize("case", load("extsim_cases.json"), ids=lambda c: c["name"])
def test_extsim_golden(case):
    from kmer import KmerReference, PseudoAlignment
    from records import FASTAQRecordContainer, FASTARecordContainer
    fa = FASTARecordContainer()
    fa.parse_records("".join(f">{h}\n{s}\n" for h, s in case["genomes"]))
    ref = KmerReference(case["k"], fa, filter_similar=True, similarity_threshold=case["threshold"])
    assert json.dumps(ref.similarity_info, indent=4) == case["similarity_text"]
    assert [g.identifier for g in ref.genomes] == case["kept"]
    assert ref.n_kmers == case["n_kmers"]
    fq = FASTAQRecordContainer()
    fq.parse_records("".join(f"@{i}\n{s}\n+\n{q}\n" for i, s, q in case["reads"]))
    pa = PseudoAlignment(ref)
    pa.align_reads_from_container(fq)
    assert json.dumps(pa.get_summary(), indent=4) == case["summary_text"]


# ---------------------------------------------------------------------------
# fast kernel vs the oracle on synthetic data
# ---------------------------------------------------------------------------

SYNTH = [
    # (n_genomes, genome_len, family, sub, k, n_reads, read_len, err, param sets)
    (12, 20000, 4, 0.02, 31, 6000, 150, 0.01, [dict(), dict(m=0, p=0), dict(p=-1), dict(m=3, p=4),
                                                dict(mrq=58, mkq=59, mg=3), dict(mrq=20, mkq=25, mg=10),
                                                dict(mg=1), dict(mg=0)]),
    (6, 8000, 3, 0.03, 21, 4000, 100, 0.02, [dict(), dict(m=0, p=0), dict(mkq=60), dict(mg=2)]),
    (8, 6000, 4, 0.05, 25, 3000, 60, 0.01, [dict(), dict(m=2, p=0)]),
    # 250-bp reads: the lane kernel's 256-window shape (NM = 4), with and without filters
    (10, 9000, 5, 0.02, 31, 2000, 250, 0.01, [dict(), dict(m=0, p=0), dict(mkq=58), dict(mrq=58, mg=2), dict(mg=1),
                                               dict(mrq=57), dict(m=3, p=0)]),
    (25, 40000, 5, 0.01, 31, 12000, 272, 0.01, [dict(), dict(m=0, p=-1), dict(mg=3), dict(m=2, p=0)]),
    (5, 7000, 5, 0.01, 32, 2000, 120, 0.01, [dict(), dict(m=0, p=0)]),  # 2-word keys, fast path
    (5, 7000, 5, 0.01, 45, 1500, 150, 0.01, [dict(), dict(m=0, p=0)]),
    (4, 5000, 2, 0.02, 64, 800, 150, 0.005, [dict(), dict(m=0, p=0)]),  # 3-word keys, wave kernel
    (5, 7000, 5, 0.01, 63, 1500, 150, 0.01, [dict(), dict(m=0, p=0), dict(mrq=58, mkq=59, mg=2)]),
    # the reference's own demo k (src/RUN_LOG:30, 39): 3- and 4-word keys on the wave kernel
    (4, 6000, 2, 0.02, 75, 1000, 150, 0.005, [dict(), dict(m=0, p=0), dict(mkq=58, mg=1)]),
    (4, 6000, 2, 0.02, 100, 1000, 150, 0.005, [dict(), dict(m=0, p=0)]),
    (4, 6000, 2, 0.02, 75, 800, 250, 0.005, [dict(), dict(m=0, p=0), dict(mrq=57, mkq=58, mg=1)]),  # 250 bp
    # three-word keys on the lane kernel (63 < k <= 95: neighbour summaries, sibling walks)
    (25, 40000, 5, 0.01, 75, 8000, 150, 0.015, [dict(), dict(m=0, p=0), dict(mg=2), dict(m=2, p=0), dict(mg=1),
                                                 dict(mrq=58, mkq=59, mg=2), dict(mkq=60)]),
    (12, 20000, 4, 0.02, 95, 3000, 150, 0.01, [dict(), dict(m=0, p=-1), dict(mg=3), dict(mkq=59)]),
    # k = 96 ... 159 (four- and five-word keys, the wave kernel): the reference's
    # demo k = 150 with its flags (src/RUN_LOG:64-84) on 150- and 200-bp reads
    (6, 8000, 3, 0.004, 101, 1500, 150, 0.003, [dict(), dict(m=0, p=0), dict(mrq=59, mkq=60, mg=2)]),
    (6, 8000, 3, 0.004, 127, 1500, 180, 0.003, [dict(), dict(mg=1), dict(mrq=59, mkq=60, mg=0)]),
    (6, 8000, 3, 0.004, 128, 1500, 200, 0.003, [dict(), dict(m=0, p=0), dict(mkq=60)]),
    (10, 8000, 5, 0.002, 150, 2000, 150, 0.002, [dict(), dict(mrq=59, mkq=60, mg=2), dict(mrq=59, mkq=60, mg=0),
                                                  dict(m=0, p=0)]),
    (10, 8000, 5, 0.002, 150, 1500, 200, 0.002, [dict(), dict(mrq=59, mkq=60, mg=2), dict(mrq=59, mkq=60, mg=0)]),
    (6, 8000, 3, 0.004, 159, 1500, 200, 0.003, [dict(), dict(m=2, p=-1), dict(mrq=59, mkq=60, mg=2)]),
    (3, 4000, 1, 0.0, 17, 1500, 40, 0.02, [dict(), dict(mkq=55)]),
    (70, 3000, 10, 0.01, 15, 3000, 80, 0.01, [dict(), dict(m=0, p=0)]),  # many genomes per class
    # families (1% apart) and 1.5% read errors: off-walk k-mers, sibling walks,
    # the lane kernel's bound decision under several (m, p)
    (25, 40000, 5, 0.01, 31, 20000, 150, 0.015, [dict(m=2, p=0), dict(m=10, p=10), dict(m=0, p=-1),
                                                  dict(m=1, p=0), dict(m=5, p=1)]),
    # C4-shaped: 500 genomes (hash decision path, LDS counters), k=31, 150 bp
    (500, 20000, 5, 0.01, 31, 20000, 150, 0.005, [dict(), dict(m=0, p=0), dict(mrq=58, mkq=59, mg=10)]),
    # more genomes than the per-workgroup LDS counters hold (global counters)
    (2100, 1500, 5, 0.01, 31, 8000, 150, 0.005, [dict(), dict(mg=3)]),
]


def _synthetic_case(ng, glen, fam, sub, k, nr, rl, err, seed):
    gens = synth.family_genomes(ng, glen, seed=seed, family_size=fam, sub_rate=sub,
                                conserved_len=min(500, glen // 4), n_rate=2e-4, n_run=5)
    seq, qual, _ = synth.sample_reads(gens, nr, rl, seed=seed + 1, err_rate=err)
    # ragged tail: some shorter reads (and a few shorter than k)
    lens = np.full(nr, rl, dtype=np.int64)
    lens[::7] = np.maximum(1, rl - 1 - (np.arange(len(lens[::7])) % (rl - 1)))
    off = np.zeros(nr + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    s = np.concatenate([seq[i, :lens[i]] for i in range(nr)])
    q = np.concatenate([qual[i, :lens[i]] for i in range(nr)])
    return gens, s, q, off


@pytest.mark.parametrize("cfg", SYNTH, ids=[f"G{c[0]}_k{c[4]}_L{c[6]}" for c in SYNTH])
def test_fast_kernel_vs_oracle(cfg):
    ng, glen, fam, sub, k, nr, rl, err, psets = cfg
    gens, s, q, off = _synthetic_case(ng, glen, fam, sub, k, nr, rl, err, seed=k * 101 + ng)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    assert index.n_kmers == oix.n_kmers
    reads = N.Reads.upload(s, q, off)
    idents = [f"g{i}" for i in range(ng)]
    for ps in psets:
        full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None}
        full.update(ps)
        base = 12345
        ores = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"],
                         mkq=full["mkq"], mg=full["mg"], read_base=base, detail=False)
        prm = N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"])
        result = N.Result(index)
        N.align(index, reads, prm, base, result)
        stats, uq, am, fk = result.fetch()
        assert stats.tolist() == ores.stats.tolist(), ps
        assert uq.tolist() == ores.unique.tolist(), ps
        assert am.tolist() == ores.ambiguous.tolist(), ps
        ofk = np.where(ores.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, ores.first_key)
        assert fk.tolist() == ofk.tolist(), ps
        # summaries identical, key order included
        assert summary_from_counters(idents, stats, uq, am, fk, full) == \
            O.summary_by_walk(oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"],
                                        mkq=full["mkq"], mg=full["mg"]), idents, full["mrq"], full["mkq"], full["mg"])


@pytest.mark.parametrize("k,L", [(31, 150), (45, 150), (75, 150), (31, 250), (63, 250)])
def test_chimeric_reads_of_two_genomes(k, L):
    """Reads carrying specific k-mers of two genomes of a family in every
    proportion -- a stretch of genome A with a stretch of its sibling B at the
    same coordinates spliced in (1..149 bases), some with a second splice or
    errors, some with an internal repeat -- against the oracle under m / p
    sets that put the lane kernel's two-genome decision (ns >= c + max(m, 1),
    noff + c - ns <= p) on both sides of its bounds, also under --max-genomes,
    --min-kmer-quality and --min-read-quality (raw-ASCII qualities ~N(60, 8))."""
    rng = np.random.default_rng(7 + k)
    gens = synth.family_genomes(8, 30000, seed=k, family_size=4, sub_rate=0.03, conserved_len=300)
    nr = 6000
    seq = np.empty((nr, L), dtype=np.uint8)
    for i in range(nr):
        fam = rng.integers(0, 2) * 4
        a, b = fam + rng.choice(4, 2, replace=False)
        st = int(rng.integers(0, 30000 - L))
        r = np.asarray(gens[a][st:st + L], dtype=np.uint8).copy()
        cut = int(rng.integers(1, L))
        if i % 2:
            r[cut:] = gens[b][st + cut:st + L]
        else:
            r[:cut] = gens[b][st:st + cut]
        if i % 5 == 0:  # a second splice back to A
            c2 = int(rng.integers(0, L))
            r[c2:] = gens[a][st + c2:st + L]
        if i % 3 == 0:  # sequencing errors
            for e in rng.integers(0, L, 2):
                if r[e] in b"ACGT":
                    r[e] = b"ACGT"[(b"ACGT".index(bytes([r[e]])) + 1) % 4]
        if i % 17 == 0 and k < 60:  # an internal repeat: one k-mer twice
            r[L - k:] = r[:k]
        seq[i] = r
    qual = np.clip(np.rint(rng.normal(60, 8, size=(nr, L))), 35, 74).astype(np.uint8)
    off = np.arange(nr + 1, dtype=np.uint64) * L
    s, q = seq.reshape(-1), qual.reshape(-1)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    reads = N.Reads.upload(s, q, off)
    for m, p, mrq, mkq, mg in ((1, 1, None, None, None), (0, 0, None, None, None), (2, 0, None, None, None),
                               (1, 5, None, None, None), (3, -1, None, None, None), (10, 10, None, None, None),
                               (1, 1, None, None, 2), (1, 0, None, 58, None), (1, 1, 57, 58, 3)):
        ores = oix.align(s.tobytes(), q.tobytes(), off, m=m, p=p, mrq=mrq, mkq=mkq, mg=mg, read_base=0, detail=False)
        result = N.Result(index)
        N.align(index, reads, N.Params.make(m, p, mrq, mkq, mg), 0, result)
        stats, uq, am, fk = result.fetch()
        assert stats.tolist() == ores.stats.tolist(), (m, p, mrq, mkq, mg)
        assert uq.tolist() == ores.unique.tolist(), (m, p, mrq, mkq, mg)
        assert am.tolist() == ores.ambiguous.tolist(), (m, p, mrq, mkq, mg)
        ofk = np.where(ores.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, ores.first_key)
        assert fk.tolist() == ofk.tolist(), (m, p, mrq, mkq, mg)


@pytest.mark.parametrize("k,L", [(31, 150), (75, 150), (31, 250)])
def test_chimeric_reads_without_neighbour_bits(k, L, monkeypatch):
    """The same without the neighbour bits (every mismatching window probed)."""
    monkeypatch.setenv("PA_NO_NB", "1")
    test_chimeric_reads_of_two_genomes(k, L)


@pytest.mark.parametrize("k", [63, 64, 75, 100, 127])
def test_non_acgt_anywhere_in_long_windows(k):
    """A non-ACGT base at any position of a window of k > 63 rules the window
    out (src/kmer.py's N k-mers): reads of two sibling genomes with one or a
    few N (or other) bytes placed at every offset, so that they fall past the
    first 64 positions of some windows (the wave kernel once tested only
    min(k, 64) of them)."""
    rng = np.random.default_rng(k)
    gens = synth.family_genomes(6, 20000, seed=k, family_size=3, sub_rate=0.01, conserved_len=200)
    L = 150
    reads = []
    for i in range(3000):
        g = int(rng.integers(0, 6))
        st = int(rng.integers(0, 20000 - L))
        r = np.asarray(gens[g][st:st + L], dtype=np.uint8).copy()
        for _ in range(1 + i % 3):
            r[(i * 7 + int(rng.integers(0, 5))) % L] = b"NNNRY"[i % 5]
        reads.append(r)
    seq = np.stack(reads)
    qual = np.full(seq.shape, ord("I"), dtype=np.uint8)
    off = np.arange(len(reads) + 1, dtype=np.uint64) * L
    s, q = seq.reshape(-1), qual.reshape(-1)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    for m, p in ((1, 1), (0, 0)):
        ores = oix.align(s.tobytes(), q.tobytes(), off, m=m, p=p, read_base=0, detail=False)
        result = N.Result(index)
        N.align(index, N.Reads.upload(s, q, off), N.Params.make(m, p, None, None, None), 0, result)
        stats, uq, am, fk = result.fetch()
        assert stats.tolist() == ores.stats.tolist(), (m, p)
        assert uq.tolist() == ores.unique.tolist(), (m, p)
        assert am.tolist() == ores.ambiguous.tolist(), (m, p)


@pytest.mark.parametrize("k", [31, 45, 75])
def test_repeats_and_genome_boundaries(k):
    """Genomes with tandem repeats (a 7-bp and a 40-bp unit, 12-20 copies) and
    a 300-bp segment copied elsewhere in the same genome and into a sibling,
    and reads from those regions (k-mers repeated inside a read and inside a
    genome: the local-repeat flags, quirk 3's distinct k-mers) and reads
    across the end of one genome and the start of the next (windows that lie
    in no genome, the walk's genome range), against the oracle."""
    rng = np.random.default_rng(100 + k)
    gens = [np.asarray(g, dtype=np.uint8).copy() for g in
            synth.family_genomes(6, 12000, seed=k + 1, family_size=3, sub_rate=0.02, conserved_len=200)]
    hot = []
    for gi, g in enumerate(gens):
        for unit_len, copies in ((7, 20), (40, 12)):
            unit = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), unit_len)
            at = int(rng.integers(500, 11000 - unit_len * copies))
            g[at:at + unit_len * copies] = np.tile(unit, copies)
            hot.append((gi, at))
        src = int(rng.integers(0, 11000))
        dst = int(rng.integers(0, 11000))
        g[dst:dst + 300] = g[src:src + 300].copy()
        hot.append((gi, dst))
        sib = (gi // 3) * 3 + (gi + 1) % 3
        gens[sib][src:src + 300] = g[src:src + 300]
    L = 150
    reads = []
    for i in range(4000):
        if i % 4 == 0:  # across a genome boundary
            g = int(rng.integers(0, 5))
            tail = int(rng.integers(1, L))
            r = np.concatenate([gens[g][len(gens[g]) - tail:], gens[g + 1][:L - tail]])
        else:
            gi, at = hot[int(rng.integers(0, len(hot)))]
            st = int(np.clip(at + rng.integers(-120, 300), 0, 12000 - L))
            r = gens[gi][st:st + L].copy()
            if i % 3 == 0:
                r[int(rng.integers(0, L))] = b"ACGT"[int(rng.integers(0, 4))]
        reads.append(np.asarray(r, dtype=np.uint8))
    seq = np.stack(reads)
    qual = np.full(seq.shape, ord("I"), dtype=np.uint8)
    off = np.arange(len(reads) + 1, dtype=np.uint64) * L
    s, q = seq.reshape(-1), qual.reshape(-1)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    assert index.n_kmers == oix.n_kmers
    for m, p in ((1, 1), (0, 0), (2, 5)):
        ores = oix.align(s.tobytes(), q.tobytes(), off, m=m, p=p, read_base=0, detail=False)
        result = N.Result(index)
        N.align(index, N.Reads.upload(s, q, off), N.Params.make(m, p, None, None, None), 0, result)
        stats, uq, am, fk = result.fetch()
        assert stats.tolist() == ores.stats.tolist(), (m, p, mrq, mkq, mg)
        assert uq.tolist() == ores.unique.tolist(), (m, p, mrq, mkq, mg)
        assert am.tolist() == ores.ambiguous.tolist(), (m, p, mrq, mkq, mg)
        ofk = np.where(ores.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, ores.first_key)
        assert fk.tolist() == ofk.tolist(), (m, p, mrq, mkq, mg)


NO_NB = [c for c in SYNTH if c[4] <= 95 and c[0] in (12, 25, 500, 70, 5)]


@pytest.mark.parametrize("cfg", NO_NB, ids=[f"G{c[0]}_k{c[4]}_L{c[6]}" for c in NO_NB])
def test_fast_kernel_vs_oracle_without_neighbour_bits(cfg, monkeypatch):
    monkeypatch.setenv("PA_NO_NB", "1")
    test_fast_kernel_vs_oracle(cfg)


SPLIT = [c for c in SYNTH if c[4] <= 31 and c[0] in (12, 25, 500)]


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("cfg", SPLIT, ids=[f"G{c[0]}_k{c[4]}_L{c[6]}" for c in SPLIT])
def test_fast_kernel_vs_oracle_with_split_neighbour_words(cfg, half, monkeypatch):
    """The neighbour words in two pieces (pa_device.h NbW: what a reference
    whose words find no single free range of the slab pool gets, C5 after
    EXTSIM); PA_NB_SPLIT=1 forces it, PA_NB_HALF=1 the 12-B present-only form."""
    monkeypatch.setenv("PA_NB_SPLIT", "1")
    if half:
        monkeypatch.setenv("PA_NB_HALF", "1")
    test_fast_kernel_vs_oracle(cfg)


def test_neighbour_bits_deferred_then_built(tmp_path):
    """A FASTQ file of few reads is aligned before the neighbour bits exist
    (index_prepare's reads_hint); the align that brings the reads past
    PA_NB_READS_PER_KBASE / 1000 per genome base builds them; results equal the oracle
    throughout."""
    from kmer import KmerReference, PseudoAlignment
    from records import FASTARecordContainer
    gens = synth.family_genomes(4, 15000, seed=41, family_size=2, sub_rate=0.01, conserved_len=300)
    c = FASTARecordContainer()
    c.parse_records(synth.fasta_text([f"d{i}" for i in range(4)], gens, width=60))
    ref = KmerReference(31, c)
    oix = O.OracleIndex(gens, 31)
    seq, qual, _ = synth.sample_reads(gens, 2000, 150, seed=42, err_rate=0.01)
    p = tmp_path / "few.fq"
    p.write_text(synth.fastq_text([f"f{i}" for i in range(2000)], seq, qual))
    pa = PseudoAlignment(ref)
    pa.align_reads_from_file(str(p), prefetch=N.FastqPrefetch(str(p)))
    assert getattr(pa, "_streamed_records", None) == 2000
    bytes_before = ref.index.info().device_bytes
    s, q, off = seq.reshape(-1), qual.reshape(-1), np.arange(0, 2001 * 150, 150, dtype=np.uint64)
    o = oix.align(s.tobytes(), q.tobytes(), off, read_base=0, detail=False)
    stats, *_ = pa._result.fetch()
    assert stats.tolist() == o.stats.tolist()
    # 300 k reads > 2.5 x 60 kb: this align builds the neighbour bits first
    seq2, qual2, _ = synth.sample_reads(gens, 300000, 150, seed=43, err_rate=0.01)
    s2, q2 = seq2.reshape(-1), qual2.reshape(-1)
    off2 = np.arange(0, 300001 * 150, 150, dtype=np.uint64)
    reads = N.Reads.upload(s2, q2, off2)
    res = N.Result(ref.index)
    N.align(ref.index, reads, N.Params.make(1, 1, None, None, None), 5000, res)
    assert ref.index.info().device_bytes > bytes_before  # the neighbour bits now exist
    o2 = oix.align(s2.tobytes(), q2.tobytes(), off2, read_base=5000, detail=False)
    st2, uq, am, fk = res.fetch()
    assert st2.tolist() == o2.stats.tolist() and uq.tolist() == o2.unique.tolist()
    assert am.tolist() == o2.ambiguous.tolist()


def test_detail_kernel_vs_oracle_per_read():
    gens, s, q, off = _synthetic_case(9, 6000, 3, 0.02, 27, 2500, 130, 0.01, seed=77)
    index = N.Index(gens, 27)
    oix = O.OracleIndex(gens, 27)
    reads = N.Reads.upload(s, q, off)
    for ps in (dict(m=1, p=1), dict(m=0, p=0, mrq=56, mkq=57, mg=4)):
        prm = N.Params.make(ps.get("m", 1), ps.get("p", 1), ps.get("mrq"), ps.get("mkq"), ps.get("mg"))
        types, qf, hr, loff, lists = N.align_detail(index, reads, prm)
        o = oix.align(s.tobytes(), q.tobytes(), off, m=ps.get("m", 1), p=ps.get("p", 1), mrq=ps.get("mrq"),
                      mkq=ps.get("mkq"), mg=ps.get("mg"))
        assert types.tolist() == o.types.tolist()
        assert qf.tolist() == o.qf.tolist() and hr.tolist() == o.hr.tolist()
        assert loff.tolist() == o.list_off.tolist()
        assert lists.tolist() == o.lists.tolist()


def test_batches_and_determinism():
    """Two half batches == one batch; repeated runs identical."""
    gens, s, q, off = _synthetic_case(8, 10000, 4, 0.02, 31, 4000, 150, 0.01, seed=5)
    index = N.Index(gens, 31)
    prm = N.Params.make(1, 1, None, None, None)
    full = N.Result(index)
    N.align(index, N.Reads.upload(s, q, off), prm, 0, full)
    a = full.fetch()
    N.align(index, N.Reads.upload(s, q, off), prm, 0, full)  # accumulate twice: counts double, keys same
    b = full.fetch()
    assert (b[0] == 2 * a[0]).all() and (b[1] == 2 * a[1]).all() and (b[3] == a[3]).all()
    half = N.Result(index)
    h = len(off) // 2
    N.align(index, N.Reads.upload(s[:int(off[h])], q[:int(off[h])], off[:h + 1]), prm, 0, half)
    N.align(index, N.Reads.upload(s[int(off[h]):], q[int(off[h]):], off[h:] - off[h]), prm, h, half)
    c = half.fetch()
    for x, y in zip(a, c):
        assert x.tolist() == y.tolist()


def test_synthesized_reads_parity():
    """Device-synthesized reads (bench workload) against the oracle on the downloaded bytes."""
    gens = synth.family_genomes(10, 30000, seed=3, family_size=5, sub_rate=0.01, conserved_len=1000)
    index = N.Index(gens, 31)
    reads = N.Reads.synthesize(index, 20000, 150, first_read=0, seed=2, sub_rate=0.005)
    s, q, off = reads.download()
    assert set(np.unique(s).tolist()) <= set(b"ACGT")
    assert q.min() >= 35 and q.max() <= 74
    oix = O.OracleIndex(gens, 31)
    for ps in (dict(), dict(mrq=58, mkq=59, mg=3)):
        full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        result = N.Result(index)
        N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 0, result)
        stats, uq, am, fk = result.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                      mg=full["mg"], detail=False)
        assert stats.tolist() == o.stats.tolist()
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist()


@pytest.mark.parametrize("read_len", [158, 159, 166, 176, 177, 250, 272, 300, 700, 1500])
def test_synthesized_long_reads_parity(read_len):
    """Device-synthesized reads longer than the 150-bp lane shape takes (the
    256-window shape from 129 windows or 177 bases on, the wave kernel past
    272 bases, the exact kernel past 256 windows) against the oracle."""
    gens = synth.family_genomes(20, 60000, seed=7, family_size=5, sub_rate=0.01, conserved_len=1000)
    index = N.Index(gens, 31)
    reads = N.Reads.synthesize(index, 30000, read_len, first_read=0, seed=3, sub_rate=0.008)
    s, q, off = reads.download()
    oix = O.OracleIndex(gens, 31)
    for ps in (dict(), dict(mrq=58, mg=3), dict(m=0, p=0)):
        full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        result = N.Result(index)
        N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 0, result)
        stats, uq, am, fk = result.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                      mg=full["mg"], detail=False)
        assert stats.tolist() == o.stats.tolist(), ps
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
        ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
        assert fk.tolist() == ofk.tolist(), ps


def test_edge_cases():
    # k <= 0 and k longer than every genome: empty index, every read unmapped
    for k in (0, -3, 50):
        index = N.Index(["ACGTACGTAC", "GGGGCCCC"], k)
        assert index.n_kmers == 0
        s, off = N.concat(["ACGTACGT", "A"])
        q, _ = N.concat(["IIIIIIII", "I"])
        res = N.Result(index)
        N.align(index, N.Reads.upload(s, q, off), N.Params.make(), 0, res)
        assert res.fetch()[0].tolist() == [0, 0, 2, 0, 0, 0]
    # k > PA_MAX_K fails loudly
    with pytest.raises(N.PaUnsupported):
        N.Index(["A" * 300], N.PA_MAX_K + 1)
    # invalid genome characters are rejected, like the FASTA grammar
    with pytest.raises(ValueError):
        N.Index(["ACGTX"], 3)
    # m < 0 is a ValueError at the ABI too
    index = N.Index(["ACGTACGT"], 3)
    s, off = N.concat(["ACGT"])
    with pytest.raises(ValueError):
        N.align(index, N.Reads.upload(s, s, off), N.Params.make(m=-1), 0, N.Result(index))
    # the largest supported k
    g = synth.family_genomes(3, 2000, seed=9, family_size=3, sub_rate=0.01, conserved_len=0, n_rate=0)
    index = N.Index(g, 159)
    oix = O.OracleIndex(g, 159)
    assert index.n_kmers == oix.n_kmers
    seq, qual, _ = synth.sample_reads(g, 300, 170, seed=10, err_rate=0.002)
    off = np.arange(301, dtype=np.uint64) * 170
    res = N.Result(index)
    N.align(index, N.Reads.upload(seq, qual, off), N.Params.make(), 0, res)
    o = oix.align(seq.tobytes(), qual.tobytes(), off, detail=False)
    assert res.fetch()[0].tolist() == o.stats.tolist()


@pytest.mark.parametrize("k", [160, 191, 192, 224, 255])
def test_long_k_vs_oracle(k):
    """k-mers of six to eight 64-bit key words (160 <= k <= PA_MAX_K): the
    reference takes any k (src/kmer.py:84-94); index size, per-k-mer genome
    lists and every read's outcome against the oracle, with and without the
    filters."""
    g = synth.family_genomes(4, 3000, seed=k, family_size=2, sub_rate=0.01, conserved_len=300, n_rate=1e-3)
    index = N.Index(g, k)
    oix = O.OracleIndex(g, k)
    assert index.n_kmers == oix.n_kmers
    L = k + 60
    seq, qual, _ = synth.sample_reads(g, 400, L, seed=k + 1, err_rate=0.002)
    off = np.arange(401, dtype=np.uint64) * L
    for prm in (dict(), dict(m=0, p=0), dict(mrq=53, mkq=58, mg=1)):
        res = N.Result(index)
        N.align(index, N.Reads.upload(seq, qual, off), N.Params.make(prm.get("m", 1), prm.get("p", 1), prm.get("mrq"),
                                                                       prm.get("mkq"), prm.get("mg")), 0, res)
        stats, uq, am, _ = res.fetch()
        o = oix.align(seq.tobytes(), qual.tobytes(), off, m=prm.get("m", 1), p=prm.get("p", 1), mrq=prm.get("mrq"),
                      mkq=prm.get("mkq"), mg=prm.get("mg"), detail=False)
        assert stats.tolist() == o.stats.tolist(), (k, prm)
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist()
    # the genome lists of k-mers taken from the genomes (and of absent ones)
    text = [x.tobytes().decode() if hasattr(x, "tobytes") else x for x in g]
    keys = [t[j:j + k] for t in text for j in (0, 777, len(t) - k)] + ["A" * k, "C" * k]
    cls, size = index.lookup(keys)
    for km, c, sz in zip(keys, cls, size):
        want = oix.lookup(km)
        got = index.class_genomes(int(c)) if c >= 0 else []
        assert got == want and int(sz) == len(want), (k, km[:20])


def _walk_adversarial_case(seed, n_genomes, k):
    """Genomes and reads aimed at the genome walk of the fast kernel: tandem
    repeats (a k-mer several times in one read), reads across the junction of
    two consecutive genomes (a walk could run on into the next genome), reads
    at the very start of the first genome, copies of one genome stretch in
    several genomes, and N runs next to repeats."""
    rng = np.random.Generator(np.random.PCG64(seed))
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    gens = []
    shared = acgt[rng.integers(0, 4, 400)]
    for g in range(n_genomes):
        parts = [acgt[rng.integers(0, 4, int(rng.integers(300, 900)))]]
        unit = acgt[rng.integers(0, 4, int(rng.integers(1, 9)))]
        parts.append(np.tile(unit, 200 // len(unit) + 1)[:int(rng.integers(40, 200))])  # tandem repeat
        parts.append(acgt[rng.integers(0, 4, 300)])
        if g % 3 == 0:
            parts.append(shared)  # one stretch in several genomes
        parts.append(np.full(int(rng.integers(1, 4)), ord("N"), dtype=np.uint8))
        parts.append(np.tile(unit, 20)[:60])
        parts.append(acgt[rng.integers(0, 4, int(rng.integers(200, 500)))])
        gens.append(np.concatenate(parts))
    reads = []
    cat = np.concatenate(gens)
    starts = np.cumsum([0] + [len(g) for g in gens])
    for i in range(3000):
        kind = i % 4
        L = int(rng.integers(k, 150)) if i % 5 else int(rng.integers(1, k + 3))
        if kind == 0:  # across the junction of genomes g and g+1
            g = int(rng.integers(0, n_genomes - 1))
            st = int(starts[g + 1]) - int(rng.integers(1, L + 1))
        elif kind == 1:  # the first bases of the first genome
            st = int(rng.integers(0, 4))
        else:
            st = int(rng.integers(0, len(cat) - L))
        r = cat[st:st + L].copy()
        bad = r == ord("N")
        r[bad] = acgt[rng.integers(0, 4, int(bad.sum()))]
        err = rng.random(L) < 0.01
        r[err] = acgt[rng.integers(0, 4, int(err.sum()))]
        reads.append(r)
    off = np.zeros(len(reads) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in reads])
    s = np.concatenate(reads)
    q = np.clip(rng.normal(60, 8, len(s)).round(), 35, 74).astype(np.uint8)
    return gens, s, q, off


@pytest.mark.parametrize("nb", ["nb", "no_nb"])
@pytest.mark.parametrize("n_genomes,k", [(6, 31), (12, 21), (90, 25), (5, 13)])
def test_walk_adversarial_vs_oracle(n_genomes, k, nb, monkeypatch):
    # no_nb: the tiles without neighbour bits (an index prepared for a file of
    # few reads, see index_prepare's reads_hint) -- every mismatch window probed
    if nb == "no_nb":
        monkeypatch.setenv("PA_NO_NB", "1")
    gens, s, q, off = _walk_adversarial_case(1000 + n_genomes + k, n_genomes, k)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    assert index.n_kmers == oix.n_kmers
    reads = N.Reads.upload(s, q, off)
    for ps in (dict(), dict(m=0, p=0), dict(p=3), dict(p=-1), dict(mg=2), dict(mrq=58, mkq=60)):
        full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        result = N.Result(index)
        N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 777, result)
        stats, uq, am, fk = result.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                      mg=full["mg"], read_base=777, detail=False)
        assert stats.tolist() == o.stats.tolist(), ps
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
        ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
        assert fk.tolist() == ofk.tolist(), ps


@pytest.mark.gpu
def test_full_size_shards_equal_one_pass():
    """C2-sized reference (50 x 2 Mbp): reads aligned as two shards with their
    global read bases (the multi-GPU split of pa_dist) accumulate to exactly the
    one-pass counters, first keys included; and a repeated pass is identical."""
    gens = synth.family_genomes(50, 2_000_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=5000,
                                n_rate=1e-4, n_run=10)
    index = N.Index(gens, 31)
    n = 2_000_000
    prm = N.Params.make(1, 1, None, None, 10)
    one = N.Result(index)
    reads = N.Reads.synthesize(index, n, 150, first_read=0, seed=2, sub_rate=0.005)
    N.align(index, reads, prm, 0, one)
    a = one.fetch()
    two = N.Result(index)
    for lo, hi in ((0, n // 2), (n // 2, n)):
        part = N.Reads.synthesize(index, hi - lo, 150, first_read=lo, seed=2, sub_rate=0.005)
        N.align(index, part, prm, lo, two)
    b = two.fetch()
    for x, y in zip(a, b):
        assert x.tolist() == y.tolist()
    again = N.Result(index)
    N.align(index, reads, prm, 0, again)
    for x, y in zip(a, again.fetch()):
        assert x.tolist() == y.tolist()
    assert int(a[0][0]) + int(a[0][1]) + int(a[0][2]) == n


@pytest.mark.gpu
@pytest.mark.parametrize("tpos_hi", ["1", "0"])
def test_large_reference_layout(monkeypatch, tpos_hi):
    """The layout of references too large for the default one (C5: 8 Gbp):
    table sized on the HyperLogLog distinct estimate at 1.43 slots per k-mer
    (load ~0.7, long probe chains), first occurrences as 33-bit concatenated
    positions (tpos_hi 1: bit 32 in the class word, C5's kept 4.8 Gbp) or
    genome-local (tpos_hi 0: references of >= 2^33 bases; first_pos) and
    present-only neighbour bits, no Bloom filter -- same index, same results as
    the oracle, the lane kernel on."""
    gens, s, q, off = _synthetic_case(20, 30000, 5, 0.01, 31, 8000, 150, 0.01, seed=4242)
    oix = O.OracleIndex(gens, 31)
    monkeypatch.setenv("PA_LAYOUT", "large")  # every choice the build makes for an 8 Gbp reference
    monkeypatch.setenv("PA_TPOS_HI", tpos_hi)
    index = N.Index(gens, 31)
    monkeypatch.delenv("PA_LAYOUT")
    monkeypatch.delenv("PA_TPOS_HI")
    info = index.info()
    assert index.n_kmers == oix.n_kmers
    assert info.table_slots < 2 * index.n_kmers  # sized on the estimate (default: 4 x windows)
    reads = N.Reads.upload(s, q, off)
    for ps in (dict(), dict(m=0, p=0, mrq=58, mkq=59, mg=3)):
        full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        result = N.Result(index)
        N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 0, result)
        stats, uq, am, fk = result.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                      mg=full["mg"], detail=False)
        assert stats.tolist() == o.stats.tolist(), ps
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps


@pytest.mark.parametrize("seed", range(12))
def test_pseudo_align_random_big_kmers_property(seed):
    """The reference's randomized property test (src/test_kmer.py:227-247, 364-421),
    seeded: the 31-mers of the 63-bp BigRead spread at random over 4 genomes
    joined by NN; the read is unique iff the specific-count margin is >= m and
    the total-count gap is <= p, recomputed from the index view -- and the GPU
    result equals the oracle's."""
    import random
    from kmer import KmerReference, Read, ReadMappingType, extract_kmers_from_genome
    from records import FASTAQRecordContainer, FASTARecordContainer
    fq = FASTAQRecordContainer()
    fq.parse_records("@BigRead\nAGCTAGCTAGAGGTCCTAATCCTAGCTAGCTAGCTAGCTAGCTAGCTGGTCATCAAAACCTTT\n+\n" + "I" * 63 + "\n")
    rec = list(fq)[0]
    rnd = random.Random(seed)
    k = 31
    genomes = {f">Genome{i + 1}": [] for i in range(4)}
    for _, km in extract_kmers_from_genome(k, rec["sequence"]):
        for g in rnd.sample(list(genomes), k=rnd.randint(1, 4)):
            genomes[g].append(km)
    if any(not s for s in genomes.values()):
        pytest.skip("a genome drew no k-mer")
    fa = FASTARecordContainer()
    fa.parse_records("".join(f"{name}\n{'NN'.join(seq)}\n" for name, seq in genomes.items()))
    ref = KmerReference(k, fa)
    m, p = 1, 1
    spec, total = {}, {}
    for km, gmap in ref.kmers.items():
        if len(gmap) == 1:
            g0 = next(iter(gmap))
            spec[g0] = spec.get(g0, 0) + len(gmap[g0])
        for g, pos in gmap.items():
            total[g] = total.get(g, 0) + len(pos)
    result = Read(rec).pseudo_align(ref, m=m, p=p)
    order = sorted(spec, key=spec.get, reverse=True)
    if not order:
        assert result == ReadMappingType.AMBIGUOUSLY_MAPPED
    else:
        top = spec[order[0]]
        second = spec[order[1]] if len(order) > 1 else 0
        if top - second >= m and not max(total.values()) - total[order[0]] > p:
            assert result == ReadMappingType.UNIQUELY_MAPPED
        else:
            assert result == ReadMappingType.AMBIGUOUSLY_MAPPED
    oix = O.OracleIndex([g["genome"] for g in fa], k)
    seq, off = O.concat([rec["sequence"]])
    qual, _ = O.concat([rec["quality_sequence"]])
    o = oix.align(seq, qual, off, m=m, p=p)
    assert int(o.types[0]) == result.value


@pytest.mark.parametrize("mrq,mkq", [(40, None), (None, 40), (40, 40), (41, 40), (40, 41), (20, 25), (0, 0)])
def test_quality_thresholds_no_read_can_fail(mrq, mkq, monkeypatch):
    """pa_align drops a quality threshold at or below the batch's smallest
    quality byte (no read or window mean can be below it, src/kmer.py:420, 587);
    the results equal the oracle's and the un-elided pass's, at the boundary
    (threshold == smallest byte) and one above it."""
    gens, s, q, off = _synthetic_case(10, 20000, 5, 0.01, 31, 5000, 150, 0.01, seed=91)
    q = np.maximum(q, 40).astype(np.uint8)  # smallest quality byte 40
    q[5 * 150 + 7] = 40
    index = N.Index(gens, 31)
    oix = O.OracleIndex(gens, 31)
    out = []
    for elide in ("1", "0"):
        if elide == "0":
            monkeypatch.setenv("PA_NO_QELIDE", "1")
        reads = N.Reads.upload(s, q, off)
        res = N.Result(index)
        N.align(index, reads, N.Params.make(1, 1, mrq, mkq, 10), 0, res)
        out.append([x.tolist() for x in res.fetch()])
    o = oix.align(s.tobytes(), q.tobytes(), off, m=1, p=1, mrq=mrq, mkq=mkq, mg=10, read_base=0, detail=False)
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    assert out[0] == out[1]
    assert out[0] == [o.stats.tolist(), o.unique.tolist(), o.ambiguous.tolist(), ofk.tolist()]


@pytest.mark.parametrize("k", [31, 45, 75])
@pytest.mark.parametrize("noanchor", ["1", "0", "1-nobloom"])
@pytest.mark.parametrize("ps", [dict(), dict(m=0, p=0), dict(mg=2), dict(mrq=58, mkq=60, mg=5), dict(p=-1)])
def test_unanchored_reads_vs_oracle(ps, noanchor, k, monkeypatch):
    """Reads with no seed in the index -- reverse-complemented reads (forward-only
    lookups) and reads of an unindexed organism, 1.5 % substitutions -- checked
    window by window by k_align_lane_na (k = 31) / k_align_lane_naw (two- and
    three-word keys, k = 45 / 75) (PA_LANE_NOANCHOR=1, the default with a
    Bloom filter; PA_NA_MIN=0 so that it takes them however few) or left to the
    wave kernel (0): both equal the oracle, with and without the Bloom filter."""
    monkeypatch.setenv("PA_LANE_NOANCHOR", noanchor[0])
    monkeypatch.setenv("PA_NA_MIN", "0")
    if noanchor.endswith("nobloom"):
        monkeypatch.setenv("PA_BLOOM_MB", "0")
    gens = synth.family_genomes(12, 30000, seed=61, family_size=4, sub_rate=0.01, conserved_len=800,
                                n_rate=2e-4, n_run=8)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    reads = N.Reads.synthesize(index, 20000, 150, first_read=0, seed=62, sub_rate=0.015, rc_rate=0.3,
                               foreign_rate=0.3)
    s, q, off = reads.download()
    full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
    res = N.Result(index)
    N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 99, res)
    stats, uq, am, fk = res.fetch()
    o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                  mg=full["mg"], read_base=99, detail=False)
    assert stats.tolist() == o.stats.tolist(), ps
    assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    assert fk.tolist() == ofk.tolist(), ps
    assert o.stats[2] > 5000  # many unmapped reads: the case under test


@pytest.mark.parametrize("ps", [dict(), dict(m=0, p=0), dict(mrq=53, mkq=58, mg=10), dict(mg=2), dict(mkq=61)],
                         ids=["default", "m0p0", "c3raw", "mg2", "mkq61"])
@pytest.mark.parametrize("rcwalk", ["1", "1-flat", "0"])
def test_reverse_strand_walk_vs_oracle(ps, rcwalk, monkeypatch):
    """Reads on the reverse strand (60 %), walked on it by k_align_lane_rc
    (PA_NA_RCWALK=1: the reverse-complement plane shows most of their windows
    absent; their seeds probed by k_rc_seeds over k_align_lane's per-wave
    queue segments, or -- "1-flat", PA_NA_SEG=0 -- over one flat queue) or
    checked window by window by k_align_lane_na (0), against
    genomes holding inverted repeats (a stretch followed later by its reverse
    complement: windows whose reverse complement IS a key, plane bit set) and
    palindromic runs; equal to the oracle (src/kmer.py:419-429)."""
    monkeypatch.setenv("PA_NA_MIN", "0")
    monkeypatch.setenv("PA_NA_RCWALK", rcwalk[0])
    monkeypatch.setenv("PA_NA_SEG", "0" if rcwalk.endswith("flat") else "1")
    gens = synth.family_genomes(10, 30000, seed=81, family_size=3, sub_rate=0.01, conserved_len=500,
                                n_rate=2e-4, n_run=8)
    comp = np.zeros(256, dtype=np.uint8)
    for a_, b_ in zip(b"ACGTN", b"TGCAN"):
        comp[a_] = b_
    rng = np.random.default_rng(82)
    for g in gens:  # inverted repeats: 20 stretches of 40-400 bases copied reverse-complemented further on
        for _ in range(20):
            ln = int(rng.integers(40, 400))
            a0 = int(rng.integers(0, len(g) - 2 * ln - 1))
            b0 = int(rng.integers(a0 + ln, len(g) - ln))
            g[b0:b0 + ln] = comp[g[a0:a0 + ln][::-1]]
        p0 = int(rng.integers(0, len(g) - 64))
        g[p0:p0 + 64] = np.frombuffer(b"ACGT" * 16, dtype=np.uint8)  # (ACGT)n is its own reverse complement
    index = N.Index(gens, 31)
    oix = O.OracleIndex(gens, 31)
    reads = N.Reads.synthesize(index, 30000, 150, first_read=0, seed=83, sub_rate=0.006, rc_rate=0.6,
                               foreign_rate=0.1)
    s, q, off = reads.download()
    full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
    res = N.Result(index)
    N.align(index, reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), 7, res)
    stats, uq, am, fk = res.fetch()
    o = oix.align(s.tobytes(), q.tobytes(), off, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                  mg=full["mg"], read_base=7, detail=False)
    assert stats.tolist() == o.stats.tolist(), ps
    assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    assert fk.tolist() == ofk.tolist(), ps
    assert o.stats[2] > 10000  # mostly unmapped reverse-strand reads: the case under test


@pytest.mark.parametrize("k", [3, 4, 5, 8, 11, 16, 21, 28, 31, 32, 33, 40, 47, 63, 64, 67, 75, 90, 95])
def test_quality_masks_every_k_vs_oracle(k):
    """k_quality_masks (the lane kernels' --min-read-quality / --min-kmer-quality
    pre-pass: 16-B chunks realigned to the read, the bytes k earlier by a second
    realignment templated on k >> 2) at every k residue and read length around
    its limits (k - 1 .. 176, and longer reads left to the wave kernel), with
    qualities in low and high runs so that both filters fire; equal to the oracle
    (src/kmer.py:394-408, 420-423, 587)."""
    rng = np.random.default_rng(700 + k)
    gens = synth.family_genomes(6, 6000, seed=k, family_size=3, sub_rate=0.01, conserved_len=300)
    nr = 4000
    seq, _, _ = synth.sample_reads(gens, nr, 200, seed=k + 1, err_rate=0.01)
    lens = rng.integers(max(1, k - 2), 181, nr)
    lens[:40] = np.arange(130, 170)[:40] + (k % 3)
    off = np.zeros(nr + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    s = np.concatenate([seq[i, :lens[i]] for i in range(nr)])
    q = rng.integers(45, 75, len(s)).astype(np.uint8)
    for st in rng.integers(0, len(s) - 40, len(s) // 60):  # low-quality runs
        q[st:st + rng.integers(3, 40)] = rng.integers(33, 45)
    index = N.Index(gens, k)
    oix = O.OracleIndex(gens, k)
    reads = N.Reads.upload(s, q, off)
    for mrq, mkq in ((55, None), (None, 54), (56, 52), (58, 60)):
        res = N.Result(index)
        N.align(index, reads, N.Params.make(1, 1, mrq, mkq, None), 7, res)
        got = [x.tolist() for x in res.fetch()]
        o = oix.align(s.tobytes(), q.tobytes(), off, m=1, p=1, mrq=mrq, mkq=mkq, mg=None, read_base=7, detail=False)
        ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
        assert got == [o.stats.tolist(), o.unique.tolist(), o.ambiguous.tolist(), ofk.tolist()], (mrq, mkq)
        assert (mrq is None or o.stats[3] > 0) and (mkq is None or o.stats[4] > 0)


@pytest.mark.parametrize("reduce", [False, True])
def test_compact_table_vs_oracle(reduce):
    """PA_BUILD_COMPACT (2 slots per genome window, the CLI's job table): the
    same counts as the oracle, with and without an EXTSIM-style rebuild
    (pa_index_reduce keeps the flag), and half the slots of the default table."""
    gens = synth.family_genomes(16, 40000, seed=91, family_size=4, sub_rate=0.01, conserved_len=700,
                                n_rate=2e-4, n_run=8)
    full = N.Index(gens, 31)
    index = N.Index(gens, 31, compact=True, defer_tiles=reduce)
    keep = list(range(0, 16, 2)) if reduce else list(range(16))
    if reduce:
        index.reduce(keep)
        full.close()
        full = N.Index([gens[i] for i in keep], 31)
    assert index.info().table_slots * 2 <= full.info().table_slots + 64
    kept = [gens[i] for i in keep]
    oix = O.OracleIndex(kept, 31)
    reads = N.Reads.synthesize(index, 40000, 150, first_read=0, seed=92, sub_rate=0.01, rc_rate=0.3,
                               foreign_rate=0.1)
    s, q, off = reads.download()
    for ps in (dict(), dict(mrq=58, mkq=60, mg=2), dict(m=0, p=0)):
        prm = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        res = N.Result(index)
        N.align(index, reads, N.Params.make(prm["m"], prm["p"], prm["mrq"], prm["mkq"], prm["mg"]), 5, res)
        stats, uq, am, fk = res.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=prm["m"], p=prm["p"], mrq=prm["mrq"], mkq=prm["mkq"],
                      mg=prm["mg"], read_base=5, detail=False)
        assert stats.tolist() == o.stats.tolist(), ps
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
        ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
        assert fk.tolist() == ofk.tolist(), ps
    full.close()
    index.close()


@pytest.mark.parametrize("lpos", ["1", "0"])
def test_build_list_places_vs_oracle(lpos, monkeypatch):
    """The genome lists of multi-genome k-mers appended by the places pass 1
    took (PA_BUILD_LPOS=1, no CAS in pass 2) or by pass 2's CASes (0): the
    same genome sets, so the same counts as the oracle, on families whose
    members share most k-mers and repeat some within a genome."""
    monkeypatch.setenv("PA_BUILD_LPOS", lpos)
    gens = synth.family_genomes(24, 30000, seed=93, family_size=6, sub_rate=0.005, conserved_len=2000,
                                n_rate=2e-4, n_run=8)
    for g in gens[:6]:  # repeats inside a genome: a stretch copied further on
        g[20000:20400] = g[1000:1400]
    index = N.Index(gens, 31)
    oix = O.OracleIndex(gens, 31)
    reads = N.Reads.synthesize(index, 30000, 150, first_read=0, seed=94, sub_rate=0.01)
    s, q, off = reads.download()
    for ps in (dict(), dict(mg=3), dict(m=0, p=0)):
        prm = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None, **ps}
        res = N.Result(index)
        N.align(index, reads, N.Params.make(prm["m"], prm["p"], prm["mrq"], prm["mkq"], prm["mg"]), 0, res)
        stats, uq, am, fk = res.fetch()
        o = oix.align(s.tobytes(), q.tobytes(), off, m=prm["m"], p=prm["p"], mrq=prm["mrq"], mkq=prm["mkq"],
                      mg=prm["mg"], read_base=0, detail=False)
        assert stats.tolist() == o.stats.tolist(), ps
        assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist(), ps
    index.close()
