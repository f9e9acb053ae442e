"""The library's device memory pool (csrc/pa_mem.cpp) under the public async API.

Buffers of 256 MiB and more come from slabs the library keeps.  A freed
range must not be handed out again while work queued on a caller's stream can
still read it: pa_reads_free returns while an align on another stream is in
flight, and the next pa_reads_upload / synthesize must not overwrite those
reads mid-kernel.  The counters of the in-flight align must equal a
synchronous align of the same reads.
"""

import numpy as np
import pytest

import pa_native as N
import synth

pytestmark = pytest.mark.gpu


def _stats(res):
    stats, uq, am, fk = res.fetch()
    return stats.tolist(), uq.tolist(), am.tolist(), fk.tolist()


def test_free_reads_while_align_in_flight_then_reupload():
    import torch
    gens = synth.family_genomes(20, 200_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=2000)
    index = N.Index(gens, 31, device=0)
    n = 2_500_000  # 375 MB of bases: a pooled range
    prm = N.Params.make()
    want = N.Result(index)
    a = N.Reads.synthesize(index, n, 150, first_read=0, seed=2, sub_rate=0.005)
    N.align(index, a, prm, 0, want)
    a.close()
    torch.cuda.synchronize()

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = N.Result(index)
    a = N.Reads.synthesize(index, n, 150, first_read=0, seed=2, sub_rate=0.005, stream=s1)
    for _ in range(3):  # several passes queued, so the kernels are still running at the free
        got.reset(s1)
        N.align(index, a, prm, 0, got, s1)
    a.close()  # its range goes back to the pool only once the queued passes are done
    b = N.Reads.synthesize(index, n, 150, first_read=n, seed=7, sub_rate=0.02, stream=s2,
                           rc_rate=0.5, foreign_rate=0.3)
    torch.cuda.synchronize()
    assert _stats(got) == _stats(want)
    # the new batch is intact too: its align equals the same reads made alone
    r1 = N.Result(index)
    N.align(index, b, prm, n, r1)
    b.close()
    c = N.Reads.synthesize(index, n, 150, first_read=n, seed=7, sub_rate=0.02, rc_rate=0.5, foreign_rate=0.3)
    r2 = N.Result(index)
    N.align(index, c, prm, n, r2)
    torch.cuda.synchronize()
    assert _stats(r1) == _stats(r2)
    for h in (c, got, want, r1, r2, index):
        h.close()


def test_small_allocation_trims_idle_slabs():
    """Idle slabs count as free memory and are given back when the driver
    cannot meet an allocation: closing a large index leaves its ranges in the
    pool, and mem_trim then releases them (nothing held by live buffers)."""
    gens = synth.family_genomes(10, 400_000, seed=3, family_size=5, sub_rate=0.01, conserved_len=1000)
    index = N.Index(gens, 31, device=0)
    index.close()
    released = N.mem_trim(0)
    assert released >= 0
    assert N.mem_trim(0) == 0  # nothing idle left
