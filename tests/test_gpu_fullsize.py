"""GPU parity at the FULL size of BASELINE configs 4 and 5.

The full CPU index of these references does not fit host memory (C4: 1 Gbp,
~90 GB as the oracle holds it; C5: 8 Gbp, ~0.7 TB), so the oracle here is
restricted to the k-mers that matter (oracle/pa_oracle.c,
ora_index_build_restricted, pinned against the full oracle by
tests/test_oracle_restricted.py): the k-mers of the aligned read sample, or of
chosen genomes, each with exactly the genome list the full build gives it --
the whole reference is streamed in FASTA order (src/kmer.py:135-150).  So the
table sizing, Bloom filter form and neighbour-bit width that the full size
selects on the device are checked against the reference's decisions on the
same bytes:

* C4 (BASELINE configs[3]): the bench's 500 x 2 Mbp reference and the first
  500 k of its device-synthesized reads; statistics, per-genome counts and
  first-appearance keys bit for bit, for four parameter sets;
* C5 (BASELINE configs[4]): the bench's 2000 x 4 Mbp reference with
  near-duplicate families, EXTSIM at 0.95 on the device, checked
  - row by row for 17 genomes (three whole families and two more): total and
    unique k-mers and the intersections with every other genome
    (src/kmer.py:152-177, 206-207), and the greedy scores of the dropped ones;
  - by the greedy outcome's shape (1200 kept: one member of every
    near-duplicate family, every member of the others);
  then the index of the 1200 kept genomes against the oracle on the first
  300 k device-synthesized reads (src/kmer.py:232-263, 410-480).

These tests take minutes (genome synthesis and the oracle's reference scan
dominate), so they print their progress.
"""

import json
import sys
import time

import numpy as np
import pytest

import pa_native as N
import pa_oracle as O
import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = O.host_threads()
K = 31


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if N.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X (no CPU fallback exists)")


def _say(*a):
    print("[fullsize]", *a, file=sys.stderr, flush=True)


def _pack(gens):
    off = np.zeros(len(gens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(g) for g in gens], dtype=np.uint64)
    return np.concatenate(gens), off


def _views(buf, off):
    return [buf[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]


def _check(case, ps, base=0):
    """One pass of pa_align over the case's reads == the restricted oracle, bit for bit."""
    index, oix = case.index, case.oix
    s, q, off = case.host
    full = {"m": 1, "p": 1, "mrq": None, "mkq": None, "mg": None}
    full.update(ps)
    res = N.Result(index)
    N.align(index, case.reads, N.Params.make(full["m"], full["p"], full["mrq"], full["mkq"], full["mg"]), base, res)
    stats, uq, am, fk = res.fetch()
    res.close()
    o = O.align_counts_parallel(oix, s, q, off, THREADS, m=full["m"], p=full["p"], mrq=full["mrq"], mkq=full["mkq"],
                                mg=full["mg"], read_base=base)
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    assert stats.tolist() == o.stats.tolist(), ps
    assert uq.tolist() == o.unique.tolist(), ps
    assert am.tolist() == o.ambiguous.tolist(), ps
    assert fk.tolist() == ofk.tolist(), ps
    return stats


_LIVE = []  # cases still holding device memory (module fixtures end only with the module)


class _Full:
    """A device index of a packed reference, `n_reads` synthesized reads (the
    bench's, seed 2) and the restricted oracle over their k-mers."""

    def __init__(self, packed, n_reads, defer=False):
        t0 = time.perf_counter()
        self.index = N.Index(None, K, packed=packed, defer_tiles=defer)
        self.index.prepare()
        info = self.index.info()
        _say(f"device index {time.perf_counter() - t0:.1f} s: {info.n_kmers} k-mers, "
             f"{info.table_slots} slots, {info.table_bytes / 2**30:.1f} GiB table")
        self.reads = N.Reads.synthesize(self.index, n_reads, 150, first_read=0, seed=2, sub_rate=0.005)
        self.host = self.reads.download()
        t0 = time.perf_counter()
        s, _, off = self.host
        self.oix = O.OracleIndex.restricted(packed, K, (s, off), threads=THREADS)
        _say(f"restricted oracle {time.perf_counter() - t0:.1f} s: {self.oix.n_kmers} read k-mers in the reference")
        _LIVE.append(self)

    def close(self):
        if self.index is None:
            return
        self.reads.close()
        self.index.close()
        self.reads = self.index = self.oix = None
        _LIVE.remove(self)


# ---- C4: 500 x 2 Mbp ----------------------------------------------------------------

@pytest.fixture(scope="module")
def c4_full():
    t0 = time.perf_counter()
    gens = synth.family_genomes(500, 2_000_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=5000,
                                n_rate=1e-4, n_run=10)  # bench.py CONFIGS["c4"]
    packed = _pack(gens)
    del gens
    _say(f"C4 genomes {time.perf_counter() - t0:.1f} s")
    case = _Full(packed, 500_000)
    yield case
    case.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("ps", [dict(), dict(m=0, p=0), dict(mrq=53, mkq=58, mg=10), dict(mg=3)],
                         ids=["default", "m0p0", "c3raw", "mg3"])
def test_c4_full_size(c4_full, ps):
    stats = _check(c4_full, ps)
    assert int(stats[0] + stats[1] + stats[2] + stats[3]) == 500_000
    _say("C4", ps, [int(x) for x in stats])


# ---- C5: EXTSIM over 2000 x 4 Mbp, then the 1200 kept ---------------------------------

C5_ROWS = list(range(0, 10)) + list(range(1995, 2000)) + [1000, 1503]  # families 0, 1 (near-dup), 399 (near-dup)


@pytest.fixture(scope="module")
def c5_full():
    import kmer
    for case in list(_LIVE):  # C4's index (~100 GB) would leave C5's build too little HBM
        case.close()
    t0 = time.perf_counter()
    gens = synth.family_genomes_fast(2000, 4_000_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=5000,
                                     n_rate=1e-4, n_run=10, near_dup_every=2)  # bench.py CONFIGS["c5"]
    buf, off = _pack(gens)
    del gens
    views = _views(buf, off)
    _say(f"C5 genomes {time.perf_counter() - t0:.1f} s")
    t0 = time.perf_counter()
    index = N.Index(None, K, packed=(buf, off), defer_tiles=True)
    idents = [f"genome_{i}" for i in range(2000)]
    group_of = list(range(2000))
    gpu_stats = index.extsim_stats(group_of, 2000)
    keep, info = kmer.extsim_filter(index, idents, [len(v) for v in views], 0.95)
    index.close()
    _say(f"C5 device build + EXTSIM {time.perf_counter() - t0:.1f} s: kept {len(keep)}")
    t0 = time.perf_counter()
    oix = O.OracleIndex.restricted((buf, off), K, [views[i] for i in C5_ROWS], threads=THREADS)
    ora_stats = oix.extsim_stats(group_of, 2000)
    oix = None
    _say(f"C5 restricted oracle (EXTSIM rows) {time.perf_counter() - t0:.1f} s")
    kept = [i for i, x in enumerate(idents) if x in keep]
    kbuf, koff = _pack([views[i] for i in kept])
    del buf, views
    case = _Full((kbuf, koff), 300_000, defer=True)
    case.extsim = dict(idents=idents, keep=keep, info=info, kept=kept, gpu=gpu_stats, ora=ora_stats)
    yield case
    case.close()


@pytest.mark.timeout(1200)
def test_c5_full_extsim_rows(c5_full):
    e = c5_full.extsim
    (gt, gu, gi), (ot, ou, oi) = e["gpu"], e["ora"]
    for a in C5_ROWS:
        assert gt[a] == ot[a] and gu[a] == ou[a], a
        assert np.array_equal(gi[a], oi[a]), a
        assert np.array_equal(gi[:, a], oi[:, a]), a
    info = e["info"]
    for a in C5_ROWS:
        rec = info[e["idents"][a]]
        if rec["kept"] == "no":
            b = e["idents"].index(rec["similar_to"])
            assert b in C5_ROWS
            score = int(oi[a, b]) / min(int(ot[a]), int(ot[b]))
            assert json.dumps(rec["similarity_score"]) == json.dumps(score)
    # the greedy outcome: one member per near-duplicate family, all members of the others
    assert len(e["kept"]) == 1200
    kept = set(e["kept"])
    for f in range(400):
        members = kept & set(range(5 * f, 5 * f + 5))
        assert len(members) == (1 if f % 2 == 1 else 5), f


@pytest.mark.timeout(900)
@pytest.mark.parametrize("ps", [dict(), dict(m=0, p=0), dict(mrq=53, mkq=58, mg=10), dict(mg=2)],
                         ids=["default", "m0p0", "c3raw", "mg2"])
def test_c5_full_size_align(c5_full, ps):
    info = c5_full.index.info()
    assert info.n_genomes == 1200
    assert info.table_slots < 2 * info.total_windows  # the large layout: sized on the distinct estimate
    stats = _check(c5_full, ps)
    assert int(stats[0] + stats[1] + stats[2] + stats[3]) == 300_000
    _say("C5", ps, [int(x) for x in stats])
