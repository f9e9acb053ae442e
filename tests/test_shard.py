"""pa_shard: the dumpalign job read-sharded over N GPUs (PA_GPUS=N).  CPU
tests of the byte-range cuts: every range starts at a record's '@' and holds
whole 4-line records, also when quality lines start with '@' or '+'
(src/records.py:245-302 allows both as quality characters)."""

import os

import numpy as np
import pytest

import pa_shard


def _fastq(path, n, seed, qual_start=None):
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for i in range(n):
            L = int(rng.integers(1, 60))
            s = "".join(rng.choice(list("ACGT"), L))
            q = "".join(chr(int(x)) for x in rng.integers(33, 127, L))
            if qual_start is not None and i % 2 == 0:
                q = qual_start + q[1:]
            f.write(f"@read_{i} desc\n{s}\n+\n{q}\n")


@pytest.mark.parametrize("qual_start", [None, "@", "+"])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_cuts_on_record_boundaries(tmp_path, n, qual_start):
    p = str(tmp_path / "r.fq")
    _fastq(p, 500, 7 + n, qual_start)
    data = open(p, "rb").read()
    shards = pa_shard.fastq_shards(p, n, probe=4096)
    assert shards is not None and 2 <= len(shards) <= n
    at = 0
    for off, ln in shards:
        assert off == at and ln > 0
        seg = data[off:off + ln]
        assert seg.startswith(b"@read_") and seg.endswith(b"\n")
        lines = seg.split(b"\n")[:-1]
        assert len(lines) % 4 == 0
        assert all(lines[i].startswith(b"@read_") and lines[i + 2] == b"+" for i in range(0, len(lines), 4))
        at += ln
    assert at == len(data)


def test_no_cut_in_tiny_or_empty_files(tmp_path):
    p = tmp_path / "one.fq"
    p.write_text("@a\nACGT\n+\nIIII\n")
    assert pa_shard.fastq_shards(str(p), 4) is None
    e = tmp_path / "empty.fq"
    e.write_text("")
    assert pa_shard.fastq_shards(str(e), 2) is None


def test_gpus_from_env(monkeypatch):
    monkeypatch.delenv("PA_GPUS", raising=False)
    monkeypatch.delenv("PA_GPUS_SHARE", raising=False)
    assert pa_shard.gpus_from_env() == (1, False)
    monkeypatch.setenv("PA_GPUS", "4")
    monkeypatch.setenv("PA_GPUS_SHARE", "1")
    assert pa_shard.gpus_from_env() == (4, True)
    assert pa_shard.devices_for(3, True) == [0, 0, 0]
