"""Pin the CPU restatement (oracle/) against the reference's own outputs.

The golden vectors were produced by running the reference itself
(tests/golden/make_golden.py); these tests run on CPU only.
"""

import json
import os

import numpy as np
import pytest

import pa_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


UNIT = load("unit_cases.json")
# the reference's demo configurations (src/RUN_LOG:28-84: k = 75, k = 150 with
# --min-read-quality 59 --min-kmer-quality 60 --max-genomes 2 / 0) and k = 96-159
DEMO = load("demo_cases.json")


def _reads_arrays(reads):
    seq, off = O.concat([r[1] for r in reads])
    qual, _ = O.concat([r[2] for r in reads])
    return seq, qual, off


CASES = UNIT + DEMO["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_unit_cases(case):
    genomes = [g[1] for g in case["genomes"]]
    idents = [g[0] for g in case["genomes"]]
    ix = O.OracleIndex(genomes, case["k"])
    assert ix.n_kmers == case["n_kmers"]
    exp_sets = {km: gl for km, gl in case["kmer_sets"]}
    got = ix.export()
    if len(exp_sets) == case["n_kmers"]:
        assert got == exp_sets
    else:  # (demo cases hold a sample of the k-mers' sets)
        assert {km: got.get(km) for km in exp_sets} == exp_sets
    seq, qual, off = _reads_arrays(case["reads"])
    for res in case["results"]:
        ps = res["params"]
        out = ix.align(seq, qual, off, m=ps["m"], p=ps["p"], mrq=ps["mrq"], mkq=ps["mkq"], mg=ps["mg"])
        for r, (rid, tname, glist, qf, hr) in enumerate(res["reads"]):
            assert O.TYPE_NAMES[int(out.types[r])] == tname, (rid, ps)
            assert [idents[g] for g in out.genomes_of(r)] == glist, (rid, ps)
            assert int(out.qf[r]) == qf and int(out.hr[r]) == hr, (rid, ps)
        summ = O.summary_by_walk(out, idents, ps["mrq"], ps["mkq"], ps["mg"])
        assert summ == res["summary"]
        assert json.dumps(summ, indent=4) == res["summary_text"]


def test_oracle_extract_kmers_known_answer():
    # src/test_kmer.py:291-303: windows of AGCTAGCTAGCT with k=3
    ix = O.OracleIndex(["AGCTAGCTAGCT"], 3)
    assert sorted(ix.export()) == ["AGC", "CTA", "GCT", "TAG"]


EXTSIM = load("extsim_cases.json")


@pytest.mark.parametrize("case", EXTSIM, ids=[c["name"] for c in EXTSIM])
def test_oracle_extsim(case):
    idents = [g[0] for g in case["genomes"]]
    seqs = [g[1] for g in case["genomes"]]
    ix = O.OracleIndex(seqs, case["k"])
    kept, info = O.extsim(idents, [len(s) for s in seqs], ix, case["threshold"])
    assert json.dumps(info, indent=4) == case["similarity_text"]
    assert [idents[i] for i in kept] == case["kept"]
    ix2 = O.OracleIndex([seqs[i] for i in kept], case["k"])
    assert ix2.n_kmers == case["n_kmers"]
    seq, qual, off = _reads_arrays(case["reads"])
    out = ix2.align(seq, qual, off)
    summ = O.summary_by_walk(out, [idents[i] for i in kept])
    assert json.dumps(summ, indent=4) == case["summary_text"]


def test_oracle_first_key_matches_walk_order():
    """The (read << 20 | position) first-appearance keys reproduce the walk order."""
    case = next(c for c in UNIT if c["name"] == "rand_k11_1")
    idents = [g[0] for g in case["genomes"]]
    ix = O.OracleIndex([g[1] for g in case["genomes"]], case["k"])
    seq, qual, off = _reads_arrays(case["reads"])
    out = ix.align(seq, qual, off, m=0, p=0)
    walk = O.summary_by_walk(out, idents)
    keys = {}
    for g, fk in enumerate(out.first_key):
        if fk != np.iinfo(np.uint64).max:
            keys[idents[g]] = min(keys.get(idents[g], fk), fk)
    assert list(walk["Summary"].keys()) == sorted(keys, key=keys.get)


def test_oracle_parallel_shards_equal_single_thread():
    """bench.py's multi-thread CPU baseline: sharded counters == one pass."""
    import synth
    gens = synth.family_genomes(6, 6000, seed=4, family_size=3, sub_rate=0.02, conserved_len=300)
    seq, qual, _ = synth.sample_reads(gens, 3001, 100, seed=5, err_rate=0.01)
    off = np.arange(3002, dtype=np.uint64) * 100
    ix = O.OracleIndex(gens, 21)
    for kw in (dict(), dict(m=0, p=0, mrq=58, mkq=59, mg=2)):
        one = ix.align(seq.tobytes(), qual.tobytes(), off, read_base=9, detail=False, **kw)
        par = O.align_counts_parallel(ix, seq.reshape(-1), qual.reshape(-1), off, 4, read_base=9, **kw)
        assert par.stats.tolist() == one.stats.tolist()
        assert par.unique.tolist() == one.unique.tolist()
        assert par.ambiguous.tolist() == one.ambiguous.tolist()
        assert par.first_key.tolist() == one.first_key.tolist()


# ---- dumpref (src/kmer.py:300-329) --------------------------------------------------

DUMPREF = load("dumpref_cases.json")


def _fasta_genomes(path):
    """(description, sequence) of a FASTA file, through the drop-in parser."""
    from data_file import FASTAFile
    return [(r["description"], r["genome"]) for r in FASTAFile(path).container]


@pytest.mark.parametrize("case", DUMPREF["cases"], ids=[c["name"] for c in DUMPREF["cases"]])
def test_oracle_dumpref_cases(case):
    gold = json.loads(case["stdout"])
    kept = None
    if case["filter"] is not None:
        kept = {i for i, v in gold["Similarity"].items() if v["kept"] == "yes"}
    out = O.dumpref_summary(case["genomes"], case["k"], kept, gold.get("Similarity"))
    assert json.dumps(out, indent=4) + "\n" == case["stdout"]


def test_oracle_dumpref_config1():
    import hashlib
    genomes = _fasta_genomes(os.path.join(GOLD, "config1.fa"))
    text = json.dumps(O.dumpref_summary(genomes, 21), indent=4) + "\n"
    g = DUMPREF["config1"]["config1"]
    assert len(text) == g["length"] and hashlib.sha256(text.encode()).hexdigest() == g["sha256"]
    # EXTSIM at 0.3 drops genomes: kept set from the oracle's own EXTSIM pass
    seqs = [s for _, s in genomes]
    idx = O.OracleIndex(seqs, 21)
    kept_i, info = O.extsim([d for d, _ in genomes], [len(s) for s in seqs], idx, 0.3)
    assert len(kept_i) < len(genomes)
    kept = {genomes[i][0] for i in kept_i}
    text = json.dumps(O.dumpref_summary(genomes, 21, kept, info), indent=4) + "\n"
    g = DUMPREF["config1"]["config1_sim"]
    assert len(text) == g["length"] and hashlib.sha256(text.encode()).hexdigest() == g["sha256"]


LOOKUP = load("lookup_cases.json")


@pytest.mark.parametrize("case", LOOKUP, ids=[c["name"] for c in LOOKUP])
def test_oracle_lookup_cases(case):
    """get_kmer_references / get_kmer_and_reverse_references / __getitem__ of
    the reference (src/kmer.py:284-298, 331-351) vs the oracle's dict."""
    kept = [case["genomes"][i][1] for i in range(len(case["genomes"]))
            if case["genomes"][i][0] in set(case["kept_identifiers"])] if case["filter"] else [g[1] for g in case["genomes"]]
    kmers = O.kmer_dict(kept, case["k"])
    for q, fwd, both, none in case["queries"]:
        assert [list(x) for x in O.kmer_references(kmers, q)] == fwd, q
        assert [list(x) for x in O.kmer_references(kmers, q, reverse=True)] == both, q
        assert (not fwd) == none, q
