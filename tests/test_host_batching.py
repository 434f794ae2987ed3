"""Host-side batch planning of the CLI (no GPU): the count-matrix cap on files
per batch (the reference holds one genome's counts at a
time, kf2vec/main.py:301-357) and the up-front refusal of single files the
32-bit per-call offsets cannot hold."""
import os

import pytest

from kf2vecfsw_amd import main as M


def test_count_cap(monkeypatch):
    monkeypatch.delenv("KF_COUNT_BUDGET_MB", raising=False)
    assert M._count_cap(4 * 8192, None) == M.COUNT_BUDGET // (4 * 8192)          # k=7: 65,536 genomes
    assert M._count_cap(4 * 2098176, None) == 255                                # k=11: 8 MiB rows
    assert M._count_cap(4 * 2098176, 0.05) == 6
    assert M._count_cap(4 * 8390656, 0.001) == 1                                 # never 0
    monkeypatch.setenv("KF_COUNT_BUDGET_MB", "64")
    assert M._count_cap(4 * 2098176, 4.0) == 7


def test_batches_respect_bytes_and_files(tmp_path):
    paths = []
    for i, sz in enumerate([10, 10, 10, 10, 10, 500, 10, 10, 10]):
        p = tmp_path / f"f{i}.fna"
        p.write_bytes(b"A" * sz)
        paths.append(str(p))
    assert M._batches(paths, 1000) == [list(range(9))]
    assert M._batches(paths, 1000, max_files=4) == [[0, 1, 2, 3], [4, 5, 6, 7], [8]]
    assert M._batches(paths, 100, max_files=3) == [[0, 1, 2], [3, 4], [5], [6, 7, 8]]
    b = M._batches(paths, 1000, ramp=True, max_files=2)
    assert all(len(x) <= 2 for x in b) and sum(b, []) == list(range(9))


def test_refuse_huge_files(tmp_path):
    small = tmp_path / "a.fna"
    small.write_bytes(b">a\nACGT\n")
    M._refuse_huge_files([str(small)], "x")
    huge = tmp_path / "huge.fna"
    with open(huge, "wb") as f:
        f.truncate(1 << 32)   # sparse file: no disk blocks
    with pytest.raises(ValueError, match="huge.fna"):
        M._refuse_huge_files([str(small), str(huge)], "get_kmers -k 21")
    os.remove(huge)
