"""Device memory pool (csrc/pa_mem.cpp): the large buffers of a closed index
or read batch stay in the library's slabs and are carved again -- best fit,
split, coalesced -- by the next build; pa_mem_trim gives idle slabs back.

Each case runs in a child process because the pool's threshold is read once per
process: with PA_POOL_MIN_MB=1 nearly every device buffer of libpa.so goes
through the pool, so an index built from reused, split and coalesced ranges
must still align bit-exactly like the oracle (the EXTSIM flow: the index of all
genomes closed, the index of the kept ones built in its memory).
"""

import os
import subprocess
import sys

import pytest

import pa_native as N

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")

CHILD = r"""
import sys
sys.path[:0] = [PKG, ORACLE]
import numpy as np
import pa_native as N
import pa_oracle as O
import synth

T = O.host_threads()


def check(index, genomes, n_reads, seed):
    reads = N.Reads.synthesize(index, n_reads, 150, first_read=0, seed=seed, sub_rate=0.01, rc_rate=0.3)
    s, q, off = reads.download()
    res = N.Result(index)
    N.align(index, reads, N.Params.make(1, 1), 0, res)
    stats, uq, am, fk = res.fetch()
    res.close()
    reads.close()
    oix = O.OracleIndex(genomes, 31, threads=T)
    o = O.align_counts_parallel(oix, s, q, off, T, m=1, p=1, mrq=None, mkq=None, mg=None, read_base=0)
    ofk = np.where(o.first_key == np.iinfo(np.uint64).max, N.NO_FIRST_KEY, o.first_key)
    assert stats.tolist() == o.stats.tolist()
    assert uq.tolist() == o.unique.tolist() and am.tolist() == o.ambiguous.tolist()
    assert fk.tolist() == ofk.tolist()


gens = synth.family_genomes(40, 300_000, seed=3, family_size=4, sub_rate=0.01, conserved_len=2000,
                            n_rate=1e-4, n_run=10)
a = N.Index(gens, 31)
check(a, gens, 200_000, 5)
a.close()
kept = gens[::3]                      # a smaller index in the first one's memory
b = N.Index(kept, 31)
check(b, kept, 200_000, 6)
c = N.Index(gens[1::2], 31)            # a second live index: new ranges beside b's
check(c, gens[1::2], 100_000, 7)
b.close()
c.close()
released = N.mem_trim()
import os
assert (released == 0) if os.environ.get("PA_POOL") == "0" else (released > 0), released
d = N.Index(kept, 31)                  # after the trim: fresh slabs
check(d, kept, 100_000, 8)
d.close()
print("POOL-OK", released)
"""


def _run(env_extra):
    code = CHILD.replace("PKG", repr(PKG)).replace("ORACLE", repr(os.path.join(REPO, "oracle")))
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "POOL-OK" in r.stdout, r.stdout[-2000:]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if N.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X (no CPU fallback exists)")


def test_pool_every_buffer_reused_split_and_trimmed():
    _run({"PA_POOL_MIN_MB": "1"})


def test_pool_off_same_results():
    _run({"PA_POOL": "0"})
