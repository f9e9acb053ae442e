"""The restricted oracle (ora_index_build_restricted) against the full oracle.

BASELINE configs 4 and 5 (1 and 8 Gbp) are too large for the full CPU index
(~609 B per k-mer in the reference; ~90 GB and ~0.7 TB
for the oracle), so their full-size GPU parity tests (tests/test_gpu_scale.py)
check libpa against an oracle index restricted to the k-mers of the aligned
read sample -- or of chosen genomes, for the EXTSIM statistics -- whose genome
lists come from streaming the whole reference (src/kmer.py:135-150).  Here,
on references the full oracle holds, the restricted one must give the same
answers: per-read types, filter counters and genomes_mapped_to lists for
every parameter set, per-k-mer genome lists, and the EXTSIM rows of the seed
genomes (src/kmer.py:152-177, 206-207).  CPU only.
"""

import numpy as np
import pytest

import pa_oracle as O
import synth

PARAMS = [dict(), dict(m=0, p=0), dict(m=3, p=-1), dict(mrq=53, mkq=58, mg=10), dict(mg=1), dict(mg=3, p=0)]


def _reads(gens, n, L, seed=2, err=0.01):
    seq, qual, _ = synth.sample_reads(gens, n, L, seed=seed, err_rate=err)
    # a tenth reverse-complemented (mostly absent forward k-mers) and a tenth random
    rng = np.random.default_rng(seed)
    rc = rng.random(n) < 0.1
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in zip(b"ACGT", b"TGCA"):
        comp[a] = b
    seq[rc] = comp[seq[rc][:, ::-1]]
    rnd = rng.random(n) < 0.1
    seq[rnd] = synth.ACGT[rng.integers(0, 4, size=(int(rnd.sum()), L))]
    off = np.arange(n + 1, dtype=np.uint64) * L
    return seq.reshape(-1), qual.reshape(-1), off


@pytest.fixture(scope="module")
def ref():
    gens = synth.family_genomes(30, 100_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=3000,
                                n_rate=1e-3, n_run=10)
    return gens, O.OracleIndex(gens, 31, threads=4)


def test_restricted_align_equals_full(ref):
    gens, full = ref
    s, q, off = _reads(gens, 6000, 150)
    rest = O.OracleIndex.restricted(gens, 31, (s, off), threads=4)
    assert 0 < rest.n_kmers <= full.n_kmers
    for ps in PARAMS:
        a = full.align(s.tobytes(), q.tobytes(), off, **ps)
        b = rest.align(s.tobytes(), q.tobytes(), off, **ps)
        for f in ("types", "qf", "hr", "list_off", "lists", "stats", "unique", "ambiguous", "first_key"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), (ps, f)


def test_restricted_lists_equal_full_and_thread_independent(ref):
    gens, full = ref
    s, q, off = _reads(gens, 500, 150, seed=5)
    r1 = O.OracleIndex.restricted(gens, 31, (s, off), threads=1)
    r7 = O.OracleIndex.restricted(gens, 31, (s, off), threads=7)
    e1, e7 = r1.export(), r7.export()
    assert e1 == e7
    text = s.tobytes().decode()
    for i in range(0, 500, 7):
        for w in range(0, 120, 13):
            km = text[i * 150 + w:i * 150 + w + 31]
            assert r1.lookup(km) == full.lookup(km), km
            assert e1.get(km, []) == full.lookup(km)


def test_restricted_extsim_rows_equal_full(ref):
    gens, full = ref
    idents = [f"g{i}" for i in range(len(gens))]
    idents[7] = idents[3]  # two records, one identifier group (src/kmer.py:162-176)
    gid = {}
    group_of = [gid.setdefault(x, len(gid)) for x in idents]
    seeds = [0, 1, 2, 3, 4, 7, 12, 29]
    rest = O.OracleIndex.restricted(gens, 31, [gens[i] for i in seeds], threads=3)
    ft, fu, fi = full.extsim_stats(group_of, len(gid))
    rt, ru, ri = rest.extsim_stats(group_of, len(gid))
    for a in sorted({group_of[i] for i in seeds}):
        assert rt[a] == ft[a] and ru[a] == fu[a], a
        assert np.array_equal(ri[a], fi[a]), a
        assert np.array_equal(ri[:, a], fi[:, a]), a


@pytest.mark.parametrize("k", [1, 15, 33, 65, 151, 0, -2])
def test_restricted_any_k(k):
    gens = synth.family_genomes(6, 3000, seed=3, family_size=3, sub_rate=0.02, conserved_len=200,
                                n_rate=1e-2, n_run=3)
    s, q, off = _reads(gens, 300, 100, seed=9, err=0.02)
    full = O.OracleIndex(gens, k, threads=2)
    rest = O.OracleIndex.restricted(gens, k, (s, off), threads=3)
    for ps in (dict(), dict(m=0, p=0, mkq=58, mg=2)):
        a = full.align(s.tobytes(), q.tobytes(), off, **ps)
        b = rest.align(s.tobytes(), q.tobytes(), off, **ps)
        assert np.array_equal(a.types, b.types) and np.array_equal(a.lists, b.lists), (k, ps)
        assert np.array_equal(a.stats, b.stats) and np.array_equal(a.first_key, b.first_key), (k, ps)
