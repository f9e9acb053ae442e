"""pa_index_reduce: an index rebuilt in place over some of its genomes (the
EXTSIM rebuild, src/kmer.py:232-263) equals an index built from those genomes'
text -- the same k-mers, genome sets and align counters -- for one-, two- and
three-word keys; bad genome lists are refused and leave the index intact."""

import numpy as np
import pytest

import pa_native as N
import synth

pytestmark = pytest.mark.gpu


def _fetch(index, reads, prm):
    res = N.Result(index)
    N.align(index, reads, prm, 0, res)
    out = [a.tolist() for a in res.fetch()]
    res.close()
    return out


@pytest.mark.parametrize("k,inplace", [(31, False), (45, False), (75, False), (31, True)])
def test_reduce_equals_build_of_kept(k, inplace, monkeypatch):
    """inplace: the path taken when the gathered codes do not fit beside the
    old index (PA_REDUCE_INPLACE=1 forces it): the kept runs compacted inside
    the old codes buffer, overlapping ones through a bounce buffer."""
    if inplace:
        monkeypatch.setenv("PA_REDUCE_INPLACE", "1")
    gens = synth.family_genomes(12, 60_000, seed=5, family_size=4, sub_rate=0.01, conserved_len=800)
    sel = [0, 1, 3, 4, 5, 8, 11]
    red = N.Index(gens, k, defer_tiles=True)
    red.reduce(sel)
    ref = N.Index([gens[i] for i in sel], k)
    a, b = red.info(), ref.info()
    assert red.n_genomes == len(sel) and a.n_genomes == len(sel)
    assert (a.n_kmers, a.n_multi_classes, a.class_genome_entries, a.total_windows) == \
           (b.n_kmers, b.n_multi_classes, b.class_genome_entries, b.total_windows)
    # genome sets of k-mers from every original genome (dropped ones' k-mers: absent or re-homed)
    rng = np.random.default_rng(1)
    kms = []
    for g in gens:
        for p in rng.integers(0, len(g) - k, 40):
            kms.append(bytes(g[p:p + k]).decode())
    ca, _ = red.lookup(kms)
    cb, _ = ref.lookup(kms)
    assert [(-1 if c < 0 else tuple(red.class_genomes(int(c)))) for c in ca] == \
           [(-1 if c < 0 else tuple(ref.class_genomes(int(c)))) for c in cb]
    reads = N.Reads.synthesize(ref, 20_000, 150, first_read=0, seed=3, sub_rate=0.01, rc_rate=0.1, foreign_rate=0.1)
    for prm in (N.Params.make(), N.Params.make(0, 0), N.Params.make(1, 1, None, None, 2)):
        assert _fetch(red, reads, prm) == _fetch(ref, reads, prm)
    for h in (reads, red, ref):
        h.close()


def test_reduce_refuses_bad_lists():
    gens = synth.family_genomes(5, 20_000, seed=2)
    idx = N.Index(gens, 31)
    n = idx.n_kmers
    with pytest.raises(ValueError):
        idx.reduce([2, 1])
    with pytest.raises(ValueError):
        idx.reduce([0, 5])
    assert idx.n_kmers == n and idx.n_genomes == 5  # untouched
    idx.reduce([1, 2, 3])
    assert idx.n_genomes == 3
    idx.close()


@pytest.mark.parametrize("inject", ["bounce", "copy"])
def test_reduce_in_place_failure_leaves_no_stale_index(inject, monkeypatch):
    """the in-place path must fail before it changes anything (the
    bounce buffer is taken first) or release the index (a copy failed
    mid-compaction) -- never return half-compacted codes behind the old genome
    offsets.  PA_REDUCE_INJECT makes the bounce allocation / a copy fail."""
    monkeypatch.setenv("PA_REDUCE_INPLACE", "1")
    monkeypatch.setenv("PA_REDUCE_INJECT", inject)
    gens = synth.family_genomes(6, 40_000, seed=4, family_size=3, sub_rate=0.01, conserved_len=500)
    idx = N.Index(gens, 31)
    before = idx.info()
    sel = np.asarray([0, 2, 3, 5], dtype=np.uint32)
    st = N.lib().pa_index_reduce(idx.handle, sel.ctypes.data_as(N.P), len(sel), 0, None)
    assert st == N.PA_ENOMEM
    after = idx.info()
    if inject == "bounce":  # nothing changed: the old index is whole and still aligns
        assert (after.n_genomes, after.n_kmers, after.total_windows) == \
               (before.n_genomes, before.n_kmers, before.total_windows)
        reads = N.Reads.synthesize(idx, 2000, 150, seed=3)
        assert _fetch(idx, reads, N.Params.make())[0][2] < 2000  # (most reads map)
        reads.close()
    else:  # released: an empty index, nothing left that describes the old genomes
        assert after.n_genomes == 0 and after.n_kmers == 0 and after.table_slots == 0
        with pytest.raises(ValueError, match="released"):
            N.Result(idx)
    idx.close()
    monkeypatch.delenv("PA_REDUCE_INJECT")
    ok = N.Index(gens, 31, defer_tiles=True)
    ok.reduce(sel)
    assert ok.n_genomes == 4
    ok.close()
