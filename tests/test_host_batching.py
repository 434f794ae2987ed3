"""Host-side batch planning of the CLI (no GPU): the count-matrix cap on files
per batch (the reference holds one genome's counts at a
time, kf2vec/main.py:301-357) and the up-front refusal of single files the
32-bit per-call offsets cannot hold."""
import os

import numpy as np
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


@pytest.mark.parametrize("world,expect", [(1, 16), (2, 8), (8, 2)])
def test_cli_host_threads_split_under_quota(monkeypatch, world, expect):
    """-p defaults to mp.cpu_count() (main.py:1031-1033),
    which on the GPU box is 256 against a 16-CPU cgroup quota.  Each process of a
    run gets min(-p, usable CPUs) split over the processes on the host: a -gpus N
    child (KF_SHARD "r,N"), a torchrun rank (LOCAL_WORLD_SIZE), or the single
    process (faked 16-CPU quota here)."""
    import argparse
    monkeypatch.setattr(M, "usable_cpus", lambda: (16, {"cgroup_cpu_quota": 16.0}))
    monkeypatch.setattr(M.mp, "cpu_count", lambda: 256)          # the box's nproc: -p's default and choices
    for var in ("KF_SHARD", "WORLD_SIZE", "RANK", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(var, raising=False)
    args = argparse.Namespace(p=M.build_parser().parse_args(["get_frequencies"]).p, gpus=1)
    assert args.p == 256
    if world == 1:
        assert M.cli_host_threads(args) == expect
    for r in range(world):                        # every -gpus N child (its parent passes -p through)
        monkeypatch.setenv("KF_SHARD", f"{r},{world}")
        child = M.build_parser().parse_args(
            M._child_argv(argparse.Namespace(input_dir="i", output_dir="o", k=7, p=256, pseudocount=False,
                                             raw_cnt=False, batch_gb=None)))
        assert child.p == 256 and M.cli_host_threads(child) == expect
    monkeypatch.delenv("KF_SHARD")
    monkeypatch.setenv("WORLD_SIZE", str(world))   # torchrun ranks on one node
    monkeypatch.setenv("LOCAL_WORLD_SIZE", str(world))
    for r in range(world):
        monkeypatch.setenv("RANK", str(r))
        assert M.cli_host_threads(args) == expect
    # -p below the quota is honoured, and a process never gets 0 threads
    assert M.host_threads(4, 1) == 4 and M.host_threads(4, 8) == 1 and M.host_threads(1, 16) == 1


@pytest.mark.parametrize("k", [3, 9, 13, 21, 31])
def test_fasta_pieces_count_every_window_once(tmp_path, oracle, k):
    """get_kmers' pieces of a large FASTA file (main.fasta_pieces, here with tiny
    pieces): counting every piece's bytes on its own and summing gives exactly
    the whole file's canonical k-mer counts (no window lost or counted twice),
    across line breaks, N runs, headers at and near the cuts, blank lines and
    stray '>' bytes inside sequence lines.  Oracle = the restatement of
    Jellyfish's counting (kf2vec/main.py:133-160)."""
    import gen
    rng = np.random.default_rng(k)
    for t in range(6):
        blob = gen.random_fasta(rng, int(rng.integers(2000, 20000)), max_records=int(rng.integers(1, 12)),
                                n_rate=0.01, lower=0.05, poly_rate=0.01)
        if t % 2:
            arr = np.frombuffer(blob, np.uint8).copy()
            pos = rng.integers(0, arr.size, 5)
            arr[pos[arr[pos] != 10]] = ord(">")          # stray '>' bytes (resets, or new headers at line starts)
            blob = arr.tobytes()
        if t == 4:
            blob = blob.replace(b"\n", b"\n\n\n")        # blank lines
        p = tmp_path / f"g{t}.fna"
        p.write_bytes(blob)
        for piece in (64, 97, 1000):
            parts = M.fasta_pieces(str(p), k, piece=piece)
            assert parts[0][0] == 0 and parts[-1][1] == len(blob) and len(parts) >= len(blob) // piece // 2
            assert all(a < e for a, e in parts)
            if k <= 11:
                whole, tot = oracle.count(blob, k)
                got, gt = np.zeros_like(whole), 0
                for a, e in parts:
                    c, t_ = oracle.count(blob[a:e], k)
                    got += c
                    gt += t_
                assert gt == tot and np.array_equal(got, whole), (t, piece)
            else:
                ek, ec = oracle.sparse_count(blob, k)
                acc = {}
                for a, e in parts:
                    kk, cc = oracle.sparse_count(blob[a:e], k)
                    for x, y in zip(kk.tolist(), cc.tolist()):
                        acc[x] = acc.get(x, 0) + y
                assert sorted(acc) == ek.tolist() and [acc[x] for x in ek.tolist()] == ec.tolist(), (t, piece)


def test_record_pieces_cut_at_headers(tmp_path, oracle):
    """get_chunks' parts of a large FASTA file (main.record_pieces, here with tiny
    parts): the parts tile the file, every part after the first starts at a
    header line, a record longer than a part stays whole, a '>' inside a line is
    no cut, and the oracle's get_chunks windows of the parts, concatenated in
    order, are the whole file's (kf2vec/main.py:726-838: windows never span a
    record)."""
    import gen
    rng = np.random.default_rng(77)
    recs = []
    for c in range(9):
        L = int(rng.choice([500, 9999, 10000, 23000, 61000]))
        seq = gen.random_seq(rng, L, lower=0.02)
        recs.append(b">ctg%d desc>x\n" % c + gen.wrap(seq, int(rng.choice([60, 80, 0])), crlf=c == 3))
    blob = b"text before any header\n" + b"".join(recs)
    p = tmp_path / "g.fna"
    p.write_bytes(blob)
    whole = oracle.chunk_windows(blob, "s")
    assert len(whole) > 10
    for piece in (1, 5000, 30000, 100000, len(blob)):
        parts = M.record_pieces(str(p), piece)
        assert parts[0][0] == 0 and parts[-1][1] == len(blob), piece
        assert all(parts[i][1] == parts[i + 1][0] and parts[i][0] < parts[i][1] for i in range(len(parts) - 1))
        for a, _ in parts[1:]:
            assert blob[a: a + 1] == b">" and blob[a - 1: a] == b"\n", (piece, a)
        for a, e in parts[:-1]:   # cut at the first header at or after a + piece
            assert e >= a + piece and b"\n>" not in blob[a + piece - 1: e - 1], (piece, a)
        if piece == 1:
            assert len(parts) == len(recs) + 1
        if piece >= len(blob):
            assert parts == [(0, len(blob))]
        got = []
        for a, e in parts:
            got += oracle.chunk_windows(blob[a:e], "s")
        assert got == whole, piece
    q = tmp_path / "nohdr.fna"
    q.write_bytes(b"ACGT" * 1000)
    assert M.record_pieces(str(q), 10) == [(0, 4000)]


def test_list_inputs_matches_reference_fnmatch(tmp_path):
    """main.list_inputs (a suffix test) picks the same files, in the same
    os.listdir order, as the reference's fnmatch over "*" + form
    (kf2vec/main.py:272-275), on names around the patterns."""
    import fnmatch
    names = ["a.fa", "b.FA", "c.fasta.gz", ".fa", "x.fq", "y.fastq", "z.fna~", "w.fa.fa", "v.fna", "u.fasta",
             "t.fq.txt", "sfa", "r.f", "q.fastqq", "p[1].fa", "o*.fna", "n?.fq"]
    for n in names:
        (tmp_path / n).write_bytes(b">x\nACGT\n")
    exp = [f for f in os.listdir(tmp_path) if True in (fnmatch.fnmatch(f, "*" + form) for form in M.FORMATS)]
    files, samples = M.list_inputs(str(tmp_path))
    assert files == exp and samples == [f.rsplit(".f", 1)[0] for f in exp]
