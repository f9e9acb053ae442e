"""The library's device memory pool (csrc/pa_mem.cpp) under the public async API.

Buffers of 256 MiB and more come from slabs the library keeps.  A freed
range must not be handed out again while work queued on a caller's stream can
still read it: pa_reads_free returns while an align on another stream is in
flight, and the next pa_reads_upload / synthesize must not overwrite those
reads mid-kernel.  The counters of the in-flight align must equal a
synchronous align of the same reads.
"""

import ctypes

import numpy as np
import pytest

import pa_native as N
import synth

pytestmark = pytest.mark.gpu


def _hip():
    """The HIP runtime libpa.so runs on (streams for the test; the runtime
    bundled with torch is a different one and sees no device libpa uses)."""
    h = ctypes.CDLL("libamdhip64.so.7")
    h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return h


def _stats(res):
    stats, uq, am, fk = res.fetch()
    return stats.tolist(), uq.tolist(), am.tolist(), fk.tolist()


def test_free_reads_while_align_in_flight_then_reupload():
    hip = _hip()
    gens = synth.family_genomes(20, 200_000, seed=1, family_size=5, sub_rate=0.01, conserved_len=2000)
    index = N.Index(gens, 31, device=0)
    n = 2_500_000  # 375 MB of bases: a pooled range
    prm = N.Params.make()
    want = N.Result(index)
    a = N.Reads.synthesize(index, n, 150, first_read=0, seed=2, sub_rate=0.005)
    N.align(index, a, prm, 0, want)
    a.close()
    assert hip.hipDeviceSynchronize() == 0

    s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s1)) == 0 and hip.hipStreamCreate(ctypes.byref(s2)) == 0
    s1, s2 = s1.value, s2.value
    got = N.Result(index)
    a = N.Reads.synthesize(index, n, 150, first_read=0, seed=2, sub_rate=0.005, stream=s1)
    for _ in range(3):  # several passes queued, so the kernels are still running at the free
        got.reset(s1)
        N.align(index, a, prm, 0, got, s1)
    a.close()  # its range goes back to the pool only once the queued passes are done
    b = N.Reads.synthesize(index, n, 150, first_read=n, seed=7, sub_rate=0.02, stream=s2,
                           rc_rate=0.5, foreign_rate=0.3)
    assert hip.hipDeviceSynchronize() == 0
    assert _stats(got) == _stats(want)
    # the new batch is intact too: its align equals the same reads made alone
    r1 = N.Result(index)
    N.align(index, b, prm, n, r1)
    b.close()
    c = N.Reads.synthesize(index, n, 150, first_read=n, seed=7, sub_rate=0.02, rc_rate=0.5, foreign_rate=0.3)
    r2 = N.Result(index)
    N.align(index, c, prm, n, r2)
    assert hip.hipDeviceSynchronize() == 0
    assert _stats(r1) == _stats(r2)
    for h in (c, got, want, r1, r2, index):
        h.close()
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)


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
