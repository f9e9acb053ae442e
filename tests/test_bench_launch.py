"""bench.py --gpus N starts its own N ranks.

The driver's scaling runs call ``python bench.py --gpus N``; without a torchrun
environment the parent starts the N rank processes itself, before anything
touches the GPU, and the line it prints is rank 0's, with ``n_gpus`` = the
ranks that ran.  On the 1-GPU test box both ranks share device 0 and reduce
over gloo (a test-only flag); the job's counters must then equal one process
aligning the same 2 x N global reads -- weak scaling with global read indices.
"""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")

SMALL = ["--config", "c2", "--reads-per-gpu", "200000", "--genome-len", "200000", "--steps", "2", "--warmup", "1",
         "--no-cpu-baseline", "--no-traffic", "--no-e2e"]


def test_launcher_fails_loudly_when_a_rank_fails():
    """A rank that dies after the rendezvous (a test flag) makes the whole job
    exit non-zero with no result line, the other rank stopped rather than left
    waiting in a collective -- never a silent 1-rank run.  CPU: gloo, and the
    dying rank exits before any device call."""
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--ranks-share-device", "--dist-backend", "gloo",
                        "--fail-rank", "1"] + SMALL, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert "--fail-rank" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_rank_world_mismatch_is_an_error():
    """A rank started with WORLD_SIZE != --gpus refuses to run."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_ranks_launched_by_bench_equal_one_process():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--ranks-share-device", "--dist-backend", "gloo"]
                       + SMALL, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["backend"] == "gloo"
    npg = line["config"]["reads_per_gpu"]
    assert npg == 200000 and line["value"] > 0

    # one process, the same index and the same 2 x npg global reads
    sys.path.insert(0, REPO)
    import bench
    import pa_native as N
    import synth
    cfg = dict(bench.CONFIGS["c2"], genome_len=200000)
    gens = synth.family_genomes(cfg["n_genomes"], cfg["genome_len"], seed=1, family_size=cfg["family"],
                                sub_rate=cfg["sub"], conserved_len=cfg["conserved"], n_rate=cfg["n_rate"],
                                n_run=cfg["n_run"])
    index = N.Index(gens, cfg["k"], device=0)
    res = N.Result(index)
    for rank in range(2):
        reads = N.Reads.synthesize(index, npg, cfg["read_len"], first_read=rank * npg, seed=2,
                                   sub_rate=cfg["read_err"])
        N.align(index, reads, N.Params.make(), rank * npg, res)
        reads.close()
    want = bench.counters_digest(res)
    assert line["job_counters"] == want
    assert sum(want["stats"][:4]) == 2 * npg
    res.close()
    index.close()


def test_default_is_the_north_star_job():
    """With no --config, bench.py measures the metric's configuration C4
    (BASELINE.json configs[3]): 500 x 2 Mbp genomes, k = 31, 150 bp reads, and
    the ranks of `--gpus 8` tile the north star's 500M reads exactly --
    contiguous, disjoint, in rank order -- while every other N keeps 62.5M reads
    per GPU (weak scaling)."""
    sys.path.insert(0, REPO)
    import bench
    ap_default = [a for a in open(BENCH).read().splitlines() if '"--config", default=' in a]
    assert ap_default and 'default="c4"' in ap_default[0]
    cfg = bench.CONFIGS["c4"]
    assert (cfg["n_genomes"], cfg["genome_len"], cfg["k"], cfg["read_len"]) == (500, 2_000_000, 31, 150)
    assert cfg["params"] == {} and cfg.get("rc_rate", 0) == 0 and cfg.get("foreign_rate", 0) == 0
    for world in (1, 2, 4, 8):
        spans = [bench.rank_reads(cfg, r, world) for r in range(world)]
        assert all(n == 62_500_000 for _, n in spans)
        assert spans[0][0] == 0
        assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        assert spans[-1][0] + spans[-1][1] == world * 62_500_000
    assert sum(n for _, n in (bench.rank_reads(cfg, r, 8) for r in range(8))) == 500_000_000


def test_eight_gpu_plan_is_the_north_star_over_rccl():
    """`bench.py --gpus 8` with the default config plans the north-star job:
    8 ranks x 62.5M reads (500M, contiguous global ranges), the torch
    reduction, and the nccl (RCCL) backend on a GPU node -- checked through the
    same job_plan the bench runs, and through `--plan` (no device call)."""
    sys.path.insert(0, REPO)
    import bench
    p = bench.job_plan("c4", 8, "torch", cuda_available=True)
    assert p["world"] == 8 and p["reduce"] == "torch" and p["backend"] == "nccl"
    assert [r["n"] for r in p["rank_reads"]] == [62_500_000] * 8
    assert [r["first"] for r in p["rank_reads"]] == [62_500_000 * i for i in range(8)]
    assert p["job_reads_per_step"] == 500_000_000
    assert bench.job_plan("c4", 2, "torch", cuda_available=False)["backend"] == "gloo"
    assert bench.job_plan("c4", 1, "torch", cuda_available=True)["backend"] is None
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--plan"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    q = json.loads(r.stdout.strip().splitlines()[-1])
    assert q["world"] == 8 and q["config"] == "c4" and q["job_reads_per_step"] == 500_000_000
    assert q["reduce"] == "torch" and q["backend"] in ("nccl", "gloo")  # (gloo here: this container has no GPU)


def test_counter_child_error_lines():
    """The counter child's failure keeps its own message: the profiler's log
    lines after it are dropped (a child's error was lost)."""
    sys.path.insert(0, REPO)
    import bench
    err = ("Traceback (most recent call last):\n  File \"bench.py\", line 1, in <module>\n"
           "pa_native.PaError: out of device memory (table)\n"
           "W20261017 12:53:42.739491 130735486295552 simple_timer.cpp:55] [rocprofv3] output generation :: 1.7 sec\n"
           "I20261017 12:53:42.739556 130735486295552 simple_timer.cpp:55] [rocprofv3] tool finalization :: 1.7 sec\n")
    s = bench.child_error_lines(err)
    assert "out of device memory" in s and "rocprofv3" not in s and "Traceback" in s


def test_kernel_short_names():
    """Counter rows are matched to kernels by their own mangled names (the
    length prefix keeps k_align_lane apart from k_align_lane_na)."""
    sys.path.insert(0, REPO)
    import bench
    names = {
        "_ZN12_GLOBAL__N_112k_align_laneILb0ELb0ELb0EEEvNS_9AlignArgsE.kd": "k_align_lane",
        "_ZN12_GLOBAL__N_115k_align_lane_naILb0ELb0ELb0EEEvNS_9AlignArgsE.kd": "k_align_lane_na",
        "_ZN12_GLOBAL__N_112k_align_fastILi1ELi2ELb1EEEvNS_9AlignArgsE.kd": "k_align_fast",
        "_ZN12_GLOBAL__N_113k_align_exactILi1EEEvNS_9ExactArgsE.kd": "k_align_exact",
        "_ZN2pa15k_quality_masksEPKhPKmmilljP15HIP_vector_typeIjLj4EEPh.kd": "k_quality_masks",
        "_ZN12_GLOBAL__N_110k_nb_buildEPKmPKjmiPKN3pad4SlotILi1EEENS4_7HomeCfgE": None,
    }
    for mangled, want in names.items():
        assert bench.kernel_short_name(mangled) == want, mangled


def test_roofline_models_are_bounds():
    """SURVEY.md 8(d)'s bytes (one slot per window) passed the peak
    over the measured pass, so the lines carry (a) the design's algorithmic
    bytes per read (a floor of the bytes moved) and (b) at N > 1 the fabric
    bytes per read an N = 1 counter pass measured (profiles/lines_per_read.json)
    -- both below the peak at round 5's measured C4 launch (14.733 ms)."""
    sys.path.insert(0, REPO)
    import bench
    cfg = bench.CONFIGS["c4"]
    d = bench.design_bytes_per_read(cfg, quality_applied=False)
    assert abs(d["bytes_per_read"] - (150 + 32 * (149 / 64 + 1) + 32 + 8 * 0.005 * 150)) < 1e-9
    assert bench.design_bytes_per_read(cfg, True)["parts"]["read"] == 300
    npg = cfg["reads_per_gpu"]
    assert d["bytes_per_read"] * npg / 14.733e-3 / 1e9 / bench.HBM_PEAK_GBS < 1.0
    rl = bench.multi_rank_roofline("c4", "k_align_lane", npg, 14.733, d["bytes_per_read"])
    assert rl["achieved_basis"].startswith("N > 1 LINES MODEL") and "profiles/" in rl["achieved_basis"]
    assert 0.3 < rl["frac"] <= 1.0
    rl2 = bench.multi_rank_roofline("no_such_config", "k_align_lane", npg, 14.733, d["bytes_per_read"])
    assert "design's algorithmic bytes" in rl2["achieved_basis"] and rl2["frac"] < 1.0
