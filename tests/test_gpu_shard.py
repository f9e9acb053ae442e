"""The dumpalign job read-sharded over GPUs (PA_GPUS=N, pa_shard.py; VERDICT
r5 item 6): one index replica per device, one byte range of the FASTQ file
each, the counters reduced on the host.  On the one-GPU test box the replicas
share device 0 (PA_GPUS_SHARE=1).  The CLI's stdout must be byte-identical to
the one-GPU run and to the reference's (src/main.py:289-310)."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pa_native as N
import synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd")
GOLD = os.path.join(REPO, "tests", "golden")
MAIN = os.path.join(PKG, "main.py")


def _cli(args, gpus=1):
    env = dict(os.environ, PA_CLI_TIMING="1")
    env.pop("PA_GPUS", None)
    if gpus > 1:
        env.update(PA_GPUS=str(gpus), PA_GPUS_SHARE="1")
    return subprocess.run([sys.executable, MAIN] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                          timeout=300, env=env)


def test_config1_cli_sharded_equals_reference():
    """BASELINE config 1, every golden flag set, two shards: the reference's stdout."""
    for case in json.load(open(os.path.join(GOLD, "config1_cli.json"))):
        r = _cli(["-t", "dumpalign", "-g", os.path.join(GOLD, "config1.fa"), "-k", "21", "--reads",
                  os.path.join(GOLD, "config1.fq")] + case["flags"], gpus=2)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "reads aligned (sharded)" in r.stderr, r.stderr[-2000:]
        assert r.stdout == case["stdout"], case["flags"]


def test_demo_k150_cli_sharded(tmp_path):
    """The reference's demo `dumpalign -k 150` with its quality flags
    (src/RUN_LOG:64-84), three shards: the reference's stdout."""
    demo = json.load(open(os.path.join(GOLD, "demo_cases.json")))
    cli = demo["cli"]
    case = next(c for c in demo["cases"] if c["name"] == cli["case"])
    fa, fq = tmp_path / "mid.fa", tmp_path / "mid.fq"
    fa.write_text("".join(f">{h}\n{s}\n" for h, s in case["genomes"]))
    fq.write_text("".join(f"@{i}\n{s}\n+\n{q}\n" for i, s, q in case["reads"]))
    for run in cli["runs"]:
        r = _cli(["-t", "dumpalign", "-g", str(fa), "-k", "150", "--reads", str(fq)] + run["flags"], gpus=3)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "reads aligned (sharded)" in r.stderr
        assert r.stdout == run["stdout"], run["flags"]


@pytest.fixture(scope="module")
def mid_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("shard")
    gens = synth.family_genomes(12, 150_000, seed=21, family_size=4, sub_rate=0.01, conserved_len=800)
    fa = d / "mid.fa"
    fa.write_text(synth.fasta_text([f"g{i} mid" for i in range(12)], gens, width=70))
    seq, qual, _ = synth.sample_reads(gens, 120_000, 150, seed=22, err_rate=0.01)
    fq = d / "mid.fq"
    fq.write_text(synth.fastq_text([f"m{i}" for i in range(120_000)], seq, qual))
    return str(fa), str(fq)


@pytest.mark.parametrize("flags", [[], ["-m", "2", "-p", "0"], ["--min-read-quality", "59",
                                                                 "--min-kmer-quality", "60", "--max-genomes", "2"]])
@pytest.mark.parametrize("gpus", [2, 4])
def test_sharded_cli_equals_one_gpu(mid_files, flags, gpus):
    fa, fq = mid_files
    args = ["-t", "dumpalign", "-g", fa, "-k", "31", "--reads", fq] + flags
    one = _cli(args)
    many = _cli(args, gpus=gpus)
    assert one.returncode == 0 and many.returncode == 0, many.stderr[-2000:]
    assert "reads aligned (sharded)" in many.stderr
    assert many.stdout == one.stdout


def test_duplicate_id_across_shards_fails_like_one_gpu(mid_files, tmp_path):
    """A read id repeated in the first and the last shard: the duplicate check
    across ranges sends the file to the exact path, which raises the
    reference's DuplicateRecordError (src/records.py:290-302) -- the same exit
    as the one-GPU run."""
    fa, fq = mid_files
    text = open(fq).read()
    first = text.split("\n", 1)[0]
    lines = text.split("\n")
    lines[-5] = first  # (the last record's header: the first record's id)
    dup = tmp_path / "dup.fq"
    dup.write_text("\n".join(lines))
    args = ["-t", "dumpalign", "-g", fa, "-k", "31", "--reads", str(dup)]
    one, many = _cli(args), _cli(args, gpus=2)
    assert one.returncode != 0 and many.returncode == one.returncode
    assert many.stderr.strip().splitlines()[-1] == one.stderr.strip().splitlines()[-1]
    assert many.stdout == one.stdout == ""


def test_api_replicas_and_per_read_results(mid_files):
    """pa_shard through the Python API: replicas on device 0, the sharded
    PseudoAlignment's summary and per-read results equal one pass's."""
    import pa_shard
    from data_file import FASTAFile
    from kmer import KmerReference, PseudoAlignment
    fa, fq = mid_files
    small = fq + ".small.fq"
    with open(fq) as f, open(small, "w") as g:
        for i, line in enumerate(f):
            if i >= 4 * 3000:
                break
            g.write(line)
    c = FASTAFile(fa).container
    refs = pa_shard.build_replicas(31, c, [0, 0, 0])
    pa = pa_shard.align_sharded(refs, small, 1, 1, None, 58, 3)
    assert pa is not None and len(pa._shards) == 3 and sum(x[2] for x in pa._shards) == 3000
    one = PseudoAlignment(KmerReference(31, c))
    one.align_reads_from_file(small, 1, 1, None, 58, 3)
    assert json.dumps(pa.get_summary(), indent=4) == json.dumps(one.get_summary(), indent=4)
    assert pa.reads == one.reads
