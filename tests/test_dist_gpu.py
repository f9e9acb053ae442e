"""Multi-rank product path on one device: the read-sharded reduction of
pa_dist with the HIP engine in the loop.

Two processes (gloo backend; both ranks on device 0, the only one on a test
box) each align their contiguous shard of the same reads with libpa.so --
global read indices as the read base -- and reduce their pa_result with
pa_dist.reduce_result (pa_result_copy_out -> all-reduce SUM / MIN ->
pa_result_copy_in).  Every rank's result must then give exactly the summary of
one process aligning all reads (Summary key order included), which the oracle's
per-read walk (src/kmer.py:622-657) also gives.  The RCCL form of the same
reduction (pa_counters_reduce, the C ABI) is checked on one rank: an identity.
"""

import os
import sys
import subprocess
import socket

import numpy as np
import pytest

import pa_dist
import pa_native as N
import pa_oracle as O
import synth

pytestmark = pytest.mark.gpu

WORLD = 2
PARAMS = [dict(), dict(m=0, p=0), dict(mrq=58, mkq=59, mg=3)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    gens = synth.family_genomes(10, 30000, seed=41, family_size=5, sub_rate=0.01, conserved_len=500)
    seq, qual, _ = synth.sample_reads(gens, 20000, 150, seed=42, err_rate=0.01)
    off = np.arange(20001, dtype=np.uint64) * 150
    return gens, seq.reshape(-1), qual.reshape(-1), off


def _prm(ps):
    return N.Params.make(ps.get("m", 1), ps.get("p", 1), ps.get("mrq"), ps.get("mkq"), ps.get("mg"))


def _worker(rank, port, out):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.cuda.set_device(0)
        gens, seq, qual, off = _data()
        n = len(off) - 1
        lo, hi = pa_dist.shard_range(n, rank, WORLD)
        index = N.Index(gens, 31, device=0)
        reads = N.Reads.upload(seq[int(off[lo]):int(off[hi])], qual[int(off[lo]):int(off[hi])],
                               off[lo:hi + 1] - off[lo], device=0)
        got = []
        for ps in PARAMS:
            res = N.Result(index)
            N.align(index, reads, _prm(ps), lo, res)
            sum_t, min_t = pa_dist.reduce_result(res, torch.device("cuda", 0))
            stats, uq, am, fk = res.fetch()  # written back: the job's counters
            blocks = (sum_t.cpu().numpy(), min_t.cpu().numpy())
            assert blocks[0].tolist() == np.concatenate([stats, uq, am]).astype(np.int64).tolist()
            got.append((blocks[0].tolist(), blocks[1].tolist()))
        out.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gpu_reduce_equals_one_process():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gens, seq, qual, off = _data()
    index = N.Index(gens, 31)
    reads = N.Reads.upload(seq, qual, off)
    oix = O.OracleIndex(gens, 31)
    idents = [f"genome {i}" for i in range(len(gens))]
    for i, ps in enumerate(PARAMS):
        one = N.Result(index)
        N.align(index, reads, _prm(ps), 0, one)
        stats, uq, am, fk = one.fetch()
        want_sum = np.concatenate([stats, uq, am]).astype(np.int64).tolist()
        for r in range(WORLD):  # every rank holds the job's counters
            assert res[r][i][0] == want_sum, (r, ps)
            assert res[r][i][1] == fk.astype(np.int64).tolist(), (r, ps)
        got = pa_dist.summary_from_blocks(np.array(res[0][i][0]), np.array(res[0][i][1]), idents, ps.get("mrq"),
                                          ps.get("mkq"), ps.get("mg"))
        o = oix.align(seq.tobytes(), qual.tobytes(), off, m=ps.get("m", 1), p=ps.get("p", 1), mrq=ps.get("mrq"),
                      mkq=ps.get("mkq"), mg=ps.get("mg"))
        want = O.summary_by_walk(o, idents, ps.get("mrq"), ps.get("mkq"), ps.get("mg"))
        assert got == want and list(got["Summary"]) == list(want["Summary"]), ps


def test_rccl_counters_reduce_single_rank():
    """pa_counters_reduce through the C ABI on a one-rank communicator: the
    collective runs (RCCL opened by libpa.so) and leaves the counters as they
    were.  In a fresh interpreter: this test process has mapped torch's
    bundled HIP runtime beside ROCm's by now (the gloo tests), and RCCL's own
    HSA lookups could then find the uninitialised one ("no ROCm-capable
    device", round 6) -- a product process uses one runtime."""
    if os.environ.get("PA_RCCL_TEST_CHILD") != "1":
        r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                            f"{os.path.abspath(__file__)}::test_rccl_counters_reduce_single_rank"],
                           env=dict(os.environ, PA_RCCL_TEST_CHILD="1"), stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-3000:]
        return
    gens, seq, qual, off = _data()
    index = N.Index(gens, 31)
    res = N.Result(index)
    N.align(index, N.Reads.upload(seq, qual, off), _prm({}), 0, res)
    before = res.fetch()
    comm = N.Comm(0, 1, 0, N.Comm.unique_id())
    N.counters_reduce(res, comm)
    after = res.fetch()
    comm.close()
    for a, b in zip(before, after):
        assert a.tolist() == b.tolist()
