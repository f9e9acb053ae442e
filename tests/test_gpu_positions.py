"""Device k-mer positions (pa_index_positions): KmerReference.get_kmer_references,
__getitem__ and get_kmer_and_reverse_references (src/kmer.py:284-298, 331-351)
against the reference's outputs (tests/golden/lookup_cases.json, made by running
the reference) and against the oracle's restatement of its dict on larger
seeded references."""

import json
import os

import numpy as np
import pytest

import pa_native as N
import pa_oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLD, "lookup_cases.json")) as f:
    LOOKUP = json.load(f)


def _fa(genomes):
    from records import FASTARecordContainer
    c = FASTARecordContainer()
    c.parse_records("".join(f">{h}\n{s}\n" for h, s in genomes))
    return c


@pytest.mark.parametrize("case", LOOKUP, ids=[c["name"] for c in LOOKUP])
def test_dropin_lookups_vs_reference(case):
    from kmer import KmerReference
    kw = {} if case["filter"] is None else {"filter_similar": True, "similarity_threshold": case["filter"]}
    ref = KmerReference(case["k"], _fa(case["genomes"]), **kw)
    assert [g.identifier for g in ref.genomes] == case["kept_identifiers"]
    gi = {id(g): i for i, g in enumerate(ref.genomes)}
    for q, fwd, both, none in case["queries"]:
        got = ref.get_kmer_references(q)
        assert [[gi[id(g)], sorted(p)] for g, p in got.items()] == fwd, q
        got = ref.get_kmer_and_reverse_references(q)
        assert [[gi[id(g)], sorted(p)] for g, p in got.items()] == both, q
        assert (ref[q] is None) == none, q


def _random_genomes(rng, n, length, n_rate=0.002):
    out = []
    for i in range(n):
        g = rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=length + int(rng.integers(-length // 4, 1)))
        if i % 3 == 1 and i > 0:  # shared stretches: k-mers in several genomes
            src = out[i - 1]
            a = int(rng.integers(0, len(src) // 2))
            m = min(len(g), len(src) - a) // 2
            g[:m] = np.frombuffer(src.encode(), dtype=np.uint8)[a:a + m]
        g[rng.random(len(g)) < n_rate] = ord("N")
        out.append(bytes(g).decode())
    return out


@pytest.mark.parametrize("k", [31, 21, 32, 45, 64, 100])
def test_positions_batched_vs_oracle(k):
    rng = np.random.default_rng(k)
    seqs = _random_genomes(rng, 12, 6000)
    seqs[4] = seqs[4][:k - 1]  # shorter than k: no windows
    seqs[7] = "N" * 50
    index = N.Index(seqs, k)
    kmers = O.kmer_dict(seqs, k)
    keys = list(kmers)
    pick = [keys[int(i)] for i in rng.integers(0, len(keys), 1500)]
    queries = pick + [O.reverse_complement(q) for q in pick[:500]]
    queries += ["".join(rng.choice(list("ACGT"), k)) for _ in range(200)]
    queries += ["N" * k, "a" * k, "ACGT" * (k // 4 + 3), pick[0][:-1], pick[1]]
    for reverse in (False, True):
        hits = index.positions(queries, reverse=reverse)
        got = {}
        for q, g, p in hits.tolist():
            got.setdefault(q & 0x7FFFFFFF, {}).setdefault(g, []).append(p)
        for qi, q in enumerate(queries):
            want = O.kmer_references(kmers, q, reverse)
            # hits come sorted by (strand, genome, position); the dict order is
            # forward genomes then the reverse complement's new ones
            mine = got.get(qi, {})
            assert sorted((g, sorted(p)) for g, p in mine.items()) == sorted(want), (k, reverse, qi)
        strands = hits["query"] >> 31
        assert reverse or not strands.any()
    index.close()


def test_positions_many_hits_and_empty():
    # a homopolymer genome: one k-mer, ~100 k positions (more than the first
    # device hit buffer holds: the scan runs again with room for all)
    seqs = ["A" * 100_000, "ACGT" * 10, "", "A" * 40]
    index = N.Index(seqs, 31)
    h = index.positions(["A" * 31])
    assert len(h) == (100_000 - 30) + (40 - 30)
    assert (h["genome"][:100_000 - 30] == 0).all() and (h["position"][:100_000 - 30] == np.arange(100_000 - 30)).all()
    assert (h["genome"][100_000 - 30:] == 3).all()
    assert len(index.positions([])) == 0
    assert len(index.positions(["T" * 31], reverse=True)) == len(h)
    assert (index.positions(["T" * 31], reverse=True)["query"] >> 31 == 1).all()
    index.close()
