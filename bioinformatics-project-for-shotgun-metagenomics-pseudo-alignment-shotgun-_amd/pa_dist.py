"""Read-sharded multi-GPU pseudo-alignment (one process per GPU).

Reads are independent, so the data path needs no
exchange: every rank holds a replica of the index, aligns its own contiguous
shard of reads with global read indices [lo, hi), and the job ends with ONE
reduction of the counter blocks over RCCL (xGMI):

* sum block  = [6 statistics | G unique_reads | G ambiguous_reads]  -> SUM
* min block  = [G first-appearance keys (read << 20 | list position)] -> MIN

Both are int64 (counts and keys are < 2^63; an absent genome carries
PA_NO_FIRST_KEY = INT64_MAX so MIN ignores it).  Because the keys carry the
GLOBAL read index, the reduced keys order the Summary exactly as a single
process walking all reads would (quirk 9).  ~16*G + 48 bytes per rank: the
collective is latency-bound, bandwidth is irrelevant.
"""

from __future__ import annotations

import os
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

NO_FIRST_KEY = (1 << 63) - 1


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of n_total reads for `rank` of `world`."""
    return n_total * rank // world, n_total * (rank + 1) // world


def env_rank() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def default_backend(cuda_available: bool) -> str:
    """The backend of a multi-rank job: "nccl" (RCCL over xGMI on ROCm) on a
    GPU node, "gloo" for CPU rehearsals."""
    return "nccl" if cuda_available else "gloo"


def init_process_group(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (127.0.0.1 rendezvous)."""
    import torch
    import torch.distributed as dist
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = default_backend(torch.cuda.is_available())
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def reduce_blocks(sum_block, min_block, group=None) -> None:
    """In-place SUM / MIN all-reduce of the two counter blocks (torch int64 tensors)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(sum_block, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(min_block, op=dist.ReduceOp.MIN, group=group)


def reduce_result(result, device, stream=None, group=None, write_back: bool = True):
    """All-reduce a pa_result's counter blocks over torch.distributed and return
    them as (sum_block, min_block) int64 tensors on `device`.

    The blocks are copied out of the result (pa_result_copy_out, stream-ordered
    on `stream`), reduced -- in place on the device over RCCL for the "nccl"
    backend, through host tensors for "gloo" (CPU rehearsals, several ranks on
    one device) -- and, with `write_back`, copied back into the result
    (pa_result_copy_in), which then holds the job's counters."""
    import torch
    import torch.distributed as dist
    sum_t = torch.empty(result.n_sum, dtype=torch.int64, device=device)
    min_t = torch.empty(max(result.n_genomes, 1), dtype=torch.int64, device=device)
    if result.n_genomes == 0:
        min_t.fill_(NO_FIRST_KEY)
    result.copy_out(sum_t.data_ptr(), min_t.data_ptr() if result.n_genomes else 0, stream)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "gloo":
            torch.cuda.synchronize(device)
            sum_c, min_c = sum_t.cpu(), min_t.cpu()
            reduce_blocks(sum_c, min_c, group)
            sum_t.copy_(sum_c)
            min_t.copy_(min_c)
            torch.cuda.synchronize(device)
        else:
            reduce_blocks(sum_t, min_t, group)
    if write_back:
        result.copy_in(sum_t.data_ptr(), min_t.data_ptr() if result.n_genomes else 0, stream)
    return sum_t, min_t


def make_comm(device: int, group=None):
    """An RCCL communicator of the torch.distributed ranks for the C ABI's
    pa_counters_reduce: rank 0 makes the id, a broadcast shares it."""
    import torch.distributed as dist
    import pa_native as N
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    box = [N.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    return N.Comm(device, world, rank, box[0])


def reduce_result_capi(result, comm, stream=None) -> None:
    """The same reduction through libpa.so only (pa_counters_reduce: ncclSum /
    ncclMin in place on the result's device blocks) -- what an integrator
    without torch would call."""
    import pa_native as N
    N.counters_reduce(result, comm, stream)


def summary_from_blocks(sum_block: np.ndarray, min_block: np.ndarray, identifiers: Sequence[str],
                        mrq=None, mkq=None, mg=None) -> Dict:
    """PseudoAlignment.get_summary (src/kmer.py:622-657) from reduced blocks.

    Genomes sharing a FASTA header merge into one Summary key; keys are ordered
    by their first appearance."""
    G = len(identifiers)
    s = np.asarray(sum_block, dtype=np.int64)
    first = np.asarray(min_block, dtype=np.int64)[:G]
    stats = {"unique_mapped_reads": int(s[0]), "ambiguous_mapped_reads": int(s[1]), "unmapped_reads": int(s[2])}
    if mrq is not None:
        stats["filtered_quality_reads"] = int(s[3])
    if mkq is not None:
        stats["filtered_quality_kmers"] = int(s[4])
    if mg is not None:
        stats["filtered_hr_kmers"] = int(s[5])
    counts: Dict[str, list] = {}
    order: Dict[str, int] = {}
    for g in np.flatnonzero(first != NO_FIRST_KEY):
        name = identifiers[g]
        c = counts.setdefault(name, [0, 0])
        c[0] += int(s[6 + g])
        c[1] += int(s[6 + G + g])
        order[name] = min(order.get(name, NO_FIRST_KEY), int(first[g]))
    return {"Statistics": stats,
            "Summary": {n: {"unique_reads": counts[n][0], "ambiguous_reads": counts[n][1]}
                        for n in sorted(order, key=order.get)}}
