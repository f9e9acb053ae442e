#!/usr/bin/env python3
"""Find the reads of tests/test_gpu_parity.py::test_chimeric_reads_of_two_genomes
whose GPU result differs from the oracle (chunk bisection), and print how they
were made and their per-read outcome under PA_NO_LANE=1.
    python scripts/chim_debug.py K M P"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd"),
                os.path.join(R, "oracle")]
import pa_native as N  # noqa: E402
import pa_oracle as O  # noqa: E402
import synth  # noqa: E402

k, m, p = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(7 + k)
gens = synth.family_genomes(8, 30000, seed=k, family_size=4, sub_rate=0.03, conserved_len=300)
L, nr = 150, 6000
seq = np.empty((nr, L), dtype=np.uint8)
how = []
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
    c2 = None
    if i % 5 == 0:
        c2 = int(rng.integers(0, L))
        r[c2:] = gens[a][st + c2:st + L]
    errs = []
    if i % 3 == 0:
        for e in rng.integers(0, L, 2):
            if r[e] in b"ACGT":
                r[e] = b"ACGT"[(b"ACGT".index(bytes([r[e]])) + 1) % 4]
                errs.append(int(e))
    rep = False
    if i % 17 == 0 and k < 60:
        r[L - k:] = r[:k]
        rep = True
    seq[i] = r
    how.append(dict(a=int(a), b=int(b), st=st, cut=cut, c2=c2, errs=errs, rep=rep, b_tail=bool(i % 2)))
qual = np.full((nr, L), ord("I"), dtype=np.uint8)
index = N.Index(gens, k)
oix = O.OracleIndex(gens, k)
prm = N.Params.make(m, p, None, None, None)


def run(lo, hi, env=None):
    for kk, v in (env or {}).items():
        os.environ[kk] = v
    s = seq[lo:hi].reshape(-1)
    q = qual[lo:hi].reshape(-1)
    off = np.arange(hi - lo + 1, dtype=np.uint64) * L
    res = N.Result(index)
    N.align(index, N.Reads.upload(s, q, off), prm, 0, res)
    st, uq, am, fk = res.fetch()
    o = oix.align(s.tobytes(), q.tobytes(), off, m=m, p=p, read_base=0, detail=False)
    for kk in (env or {}):
        del os.environ[kk]
    return (st.tolist(), uq.tolist(), am.tolist()), (o.stats.tolist(), o.unique.tolist(), o.ambiguous.tolist())


bad = []
for c0 in range(0, nr, 200):
    g, o = run(c0, c0 + 200)
    if g != o:
        for i in range(c0, c0 + 200):
            g1, o1 = run(i, i + 1)
            if g1 != o1:
                bad.append(i)
for i in bad:
    g1, o1 = run(i, i + 1)
    g2, _ = run(i, i + 1, {"PA_NO_LANE": "1"})
    det = oix.align(seq[i].tobytes(), qual[i].tobytes(), np.array([0, L], dtype=np.uint64), m=m, p=p, detail=True)
    print("read", i, how[i])
    print("  gpu", g1[0], [j for j, v in enumerate(g1[1]) if v], [j for j, v in enumerate(g1[2]) if v])
    print("  ora", o1[0], [j for j, v in enumerate(o1[1]) if v], [j for j, v in enumerate(o1[2]) if v])
    print("  no-lane", g2[0], [j for j, v in enumerate(g2[1]) if v])
    print("  oracle detail", det.types if hasattr(det, "types") else det)
print("bad reads", len(bad))
