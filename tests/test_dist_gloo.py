"""World-size-2 CPU (gloo) test of the read-sharded reduction in pa_dist.

Each rank aligns its contiguous shard of reads with GLOBAL read indices (here
with the CPU oracle standing in for the per-rank GPU pass, whose per-rank
counters the GPU tests pin to the oracle), packs the counters into the
sum / min blocks exactly as pa_result lays them out, and runs
pa_dist.reduce_blocks.  The reduced blocks must give the single-process
summary, Summary key order included.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pa_dist
import pa_oracle as O
import synth

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    gens = synth.family_genomes(6, 4000, seed=31, family_size=3, sub_rate=0.03, conserved_len=200)
    seq, qual, _ = synth.sample_reads(gens, 1500, 90, seed=32, err_rate=0.01)
    off = np.arange(1501, dtype=np.uint64) * 90
    return gens, seq.reshape(-1), qual.reshape(-1), off


def _blocks(res):
    G = res.unique.size
    s = np.concatenate([res.stats, res.unique, res.ambiguous]).astype(np.int64)
    fk = np.where(res.first_key == np.iinfo(np.uint64).max, np.uint64(pa_dist.NO_FIRST_KEY), res.first_key)
    return torch.from_numpy(s), torch.from_numpy(fk.astype(np.int64)), G


def _worker(rank, port, params, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        gens, seq, qual, off = _data()
        n = len(off) - 1
        lo, hi = pa_dist.shard_range(n, rank, WORLD)
        ix = O.OracleIndex(gens, 23)
        s_off = off[lo:hi + 1] - off[lo]
        res = ix.align(seq[int(off[lo]):int(off[hi])].tobytes(), qual[int(off[lo]):int(off[hi])].tobytes(), s_off,
                       read_base=lo, detail=False, **params)
        sum_t, min_t, _ = _blocks(res)
        pa_dist.reduce_blocks(sum_t, min_t)
        if rank == 0:
            out.put((sum_t.numpy().tolist(), min_t.numpy().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("params", [dict(), dict(m=0, p=0), dict(mrq=58, mkq=59, mg=2)])
def test_sharded_reduce_equals_single_process(params):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, params, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    sum_b, min_b = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gens, seq, qual, off = _data()
    full = O.OracleIndex(gens, 23).align(seq.tobytes(), qual.tobytes(), off, **params)
    idents = [f"genome {i}" for i in range(len(gens))]
    got = pa_dist.summary_from_blocks(np.array(sum_b), np.array(min_b), idents, params.get("mrq"), params.get("mkq"),
                                      params.get("mg"))
    want = O.summary_by_walk(full, idents, params.get("mrq"), params.get("mkq"), params.get("mg"))
    assert got == want
    assert list(got["Summary"]) == list(want["Summary"])


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 10_000_001):
        for w in (1, 2, 3, 8):
            rs = [pa_dist.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
